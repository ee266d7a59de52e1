# sort kernels with every load in flight (scatter at 3 or 4 waves/SIMD): parity on h3, then A/B bench
set -euo pipefail
OUT=gpurun_out/${1:-r02t}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in h3 h4; do
  SLO_LIB=sc-lego-loam_amd/variants/libslo_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_voxel.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_vox_$v.log 2>&1
  echo "$v: $(tail -1 $OUT/t_vox_$v.log)"
done
SLO_LIB=sc-lego-loam_amd/variants/libslo_h3.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -1 $OUT/t_par.log
bash tools/gpu_variants.sh ${1:-r02t}/v sc-lego-loam_amd/variants/libslo_base.so sc-lego-loam_amd/variants/libslo_h3.so sc-lego-loam_amd/variants/libslo_h4.so sc-lego-loam_amd/variants/libslo_base.so sc-lego-loam_amd/variants/libslo_h3.so sc-lego-loam_amd/variants/libslo_h4.so
