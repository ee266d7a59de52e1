#!/bin/bash
# Collect the round's measurements on the GPU box (run through gpurun):
#   1. bench.py (default steady-state config, CPU baselines, one-stream leg)  -> gpurun_out/<tag>/bench.json
#   2. rocprofv3 --kernel-trace --stats of a shorter bench (no CPU / ICP legs,
#      no instrumented pass) with --trace-marker: the trace is cut to the timed
#      steps by tools/trace_window.py / tools/pmc_summary.py            -> gpurun_out/<tag>/kt/
#   3. rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE (separate passes, no trace
#      domains; MI355X_MICROARCH.md "rocprofv3 PMC slots"), same command  -> gpurun_out/<tag>/pmc_*/
# The summaries (tools/pmc_summary.py -> <tag>/summary/summary.json, tools/trace_window.py ->
# <tag>/window.json) are made on the box; copy them to profiles/<tag>/.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r02}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--cpu-scans 0 --single-steps 0 --steps 20 --profile-steps 0 --icp-jobs 0 --trace-marker $*"
echo "[profile] bench" && timeout -k 10 700 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
tail -c 400 "$OUT/bench.json"
echo "[profile] kernel trace" && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/kt" -o kt -- python3 bench.py $SHORT > "$OUT/kt.log" 2>&1
python3 tools/trace_window.py "$OUT/kt" --json "$OUT/window.json" > "$OUT/window.txt"
echo "[profile] FETCH_SIZE" && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d "$OUT/pmc_fetch" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_fetch.log" 2>&1
echo "[profile] WRITE_SIZE" && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
    -d "$OUT/pmc_write" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_write.log" 2>&1
# summaries on the box (the raw CSVs are too big to travel back), then drop the raw dirs
python3 tools/pmc_summary.py "$OUT" "$OUT/summary" > "$OUT/summary.txt"
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kt_kernel_stats_full_run.csv" \;
rm -rf "$OUT/kt" "$OUT/pmc_fetch" "$OUT/pmc_write"
echo "[profile] done"
