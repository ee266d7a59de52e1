#!/bin/bash
# Collect the round's measurements on the GPU box (run through gpurun):
#   1. bench.py (default config, with the CPU baseline)      -> gpurun_out/<tag>/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same bench command (minus the
#      CPU leg and the ICP batch; no warm-up and no instrumented pass: the
#      trace's mo_knn launches are exactly the bench's timed ones, so the
#      trace average checks roofline.avg_launch_us of the line in kt.log)                             -> gpurun_out/<tag>/kt/
#   3. rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE (separate passes, no trace
#      domains; MI355X_MICROARCH.md "rocprofv3 PMC slots")   -> gpurun_out/<tag>/pmc_*/
# then python3 tools/pmc_summary.py gpurun_out/<tag> profiles/<tag> (here).
# Every GPU step has its own time limit and the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--cpu-scans 0 --steps 8 --warmup 0 --profile-steps 0 --icp-jobs 0 $*"
echo "[profile] bench" && timeout -k 10 600 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -1 "$OUT/bench.json"
echo "[profile] kernel trace" && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/kt" -o kt -- python3 bench.py $SHORT > "$OUT/kt.log" 2>&1
echo "[profile] FETCH_SIZE" && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d "$OUT/pmc_fetch" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_fetch.log" 2>&1
echo "[profile] WRITE_SIZE" && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
    -d "$OUT/pmc_write" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_write.log" 2>&1
echo "[profile] done"
find "$OUT" -name "*.csv" | head -20
