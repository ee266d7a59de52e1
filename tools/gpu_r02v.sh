# ring VoxelGrid (fa_ring_ds) and projection with their loads in flight: parity on the combined variant, then A/B
set -euo pipefail
OUT=gpurun_out/${1:-r02v}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SLO_LIB=sc-lego-loam_amd/variants/libslo_rdi.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_imu.py tests/test_gpu_ring.py tests/test_gpu_wire.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -1 $OUT/t_par.log
unset SLO_LIB
bash tools/gpu_variants.sh ${1:-r02v}/v sc-lego-loam_amd/variants/libslo_r.so sc-lego-loam_amd/variants/libslo_rd.so sc-lego-loam_amd/variants/libslo_rdi.so sc-lego-loam_amd/variants/libslo_r.so sc-lego-loam_amd/variants/libslo_rd.so sc-lego-loam_amd/variants/libslo_rdi.so
