# VoxelGrid scan / digit-width variants: voxel parity per variant, then A/B bench
set -euo pipefail
OUT=gpurun_out/${1:-r02q}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in scan s9 s10; do
  SLO_LIB=sc-lego-loam_amd/variants/libslo_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_voxel.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_vox_$v.log 2>&1
  echo "$v: $(tail -1 $OUT/t_vox_$v.log)"
done
bash tools/gpu_variants.sh ${1:-r02q}/v sc-lego-loam_amd/variants/libslo_head.so sc-lego-loam_amd/variants/libslo_scan.so sc-lego-loam_amd/variants/libslo_s9.so sc-lego-loam_amd/variants/libslo_s10.so sc-lego-loam_amd/variants/libslo_head.so sc-lego-loam_amd/variants/libslo_scan.so
