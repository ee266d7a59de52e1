# vg_reduce with the slice's point indices staged in LDS: voxel/parity on the variant, then A/B bench
set -euo pipefail
OUT=gpurun_out/${1:-r02u}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SLO_LIB=sc-lego-loam_amd/variants/libslo_r.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_voxel.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -1 $OUT/t_par.log
unset SLO_LIB
bash tools/gpu_variants.sh ${1:-r02u}/v sc-lego-loam_amd/variants/libslo_h3.so sc-lego-loam_amd/variants/libslo_r.so sc-lego-loam_amd/variants/libslo_h3.so sc-lego-loam_amd/variants/libslo_r.so
