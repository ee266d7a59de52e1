# odometry Gauss-Newton iterations with each thread's query / index / matched-point loads issued four items at a
# time (variant o): parity on o, then A/B against the final build m
set -euo pipefail
OUT=gpurun_out/${1:-r02ab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SLO_LIB=sc-lego-loam_amd/variants/libslo_o.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_imu.py tests/test_gpu_ring.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -1 $OUT/t_par.log
unset SLO_LIB
bash tools/gpu_variants.sh ${1:-r02ab}/v sc-lego-loam_amd/variants/libslo_m.so sc-lego-loam_amd/variants/libslo_o.so sc-lego-loam_amd/variants/libslo_m.so sc-lego-loam_amd/variants/libslo_o.so
