# candidate k (corner search prefetches its next x-window tile; fa_pick stages and collects with eight / four
# loads in flight; k2 adds vg_scan at 256 threads with its loads in flight): parity on k2, then A/B f / k / k2
set -euo pipefail
OUT=gpurun_out/${1:-r02y}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SLO_LIB=sc-lego-loam_amd/variants/libslo_k2.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_imu.py tests/test_gpu_ring.py tests/test_gpu_loop.py tests/test_gpu_voxel.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -1 $OUT/t_par.log
unset SLO_LIB
bash tools/gpu_variants.sh ${1:-r02y}/v sc-lego-loam_amd/variants/libslo_f.so sc-lego-loam_amd/variants/libslo_k.so sc-lego-loam_amd/variants/libslo_k2.so sc-lego-loam_amd/variants/libslo_f.so sc-lego-loam_amd/variants/libslo_k.so sc-lego-loam_amd/variants/libslo_k2.so
