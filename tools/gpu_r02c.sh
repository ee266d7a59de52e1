# round 2: C5 K=50 steady-state parity; default bench (100 timed steps,
# CPU baselines, one-stream leg); kernel trace cut to the timed window
set -euo pipefail
OUT=gpurun_out/r02c
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -k "c5_dense" -x -v -s --timeout 450 --timeout-method thread -p no:cacheprovider > $OUT/t_c5.log 2>&1
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 20 --profile-steps 0 --trace-marker > $OUT/kt.log 2>&1
python3 tools/trace_window.py $OUT/kt --json $OUT/window.json > $OUT/window.txt
echo done
