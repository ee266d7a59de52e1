# IMU path: GPU parity (batched + single-scan), the non-IMU pipelines, graph vs eager
set -euo pipefail
OUT=gpurun_out/${1:-r02m}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_imu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_imu.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
timeout -k 10 200 python3 -u tools/graph_check.py 6 3 2 12 > $OUT/gc.log 2>&1
echo done
