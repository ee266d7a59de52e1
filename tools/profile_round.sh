#!/bin/bash
# Collect the round's measurements on the GPU box (run through gpurun):
#   1. bench.py (default steady-state config, CPU baselines, one-stream leg)  -> gpurun_out/<tag>/bench.json
#      (skipped with NOBENCH=1)
#   2. rocprofv3 --kernel-trace --stats of a shorter bench (no CPU / ICP legs,
#      no instrumented pass) with --trace-marker: the trace is cut to the timed
#      steps by tools/trace_window.py / tools/pmc_summary.py            -> gpurun_out/<tag>/window.txt
#   3. rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, then the SQ occupancy /
#      stall counters (separate passes, no trace domains; MI355X_MICROARCH.md
#      "rocprofv3 PMC slots"), same command, counters collected only for the
#      kernels named by $PMC_KERNELS (every other dispatch runs unprofiled)
#                                                                        -> gpurun_out/<tag>/summary.txt, sq.txt
# The summaries are made on the box and the raw CSVs deleted at once (they do
# not fit the 64 MiB that travels back); copy them to profiles/<tag>/.
# Every GPU step has its own time limit, prints a heartbeat while it runs, and
# the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r03}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--cpu-scans 0 --single-steps 0 --modes-steps 0 --steps 12 --profile-steps 0 --icp-jobs 0 --extra none --trace-marker $*"
PMC_KERNELS=${PMC_KERNELS:-"spin|sleep|k_"}   # every libslo kernel (the config lines price each one ≥ 1 %)

# run "$@" under its own limit ($LIM s), printing a line every 30 s; returns its status
hb() {
  timeout -k 10 "$LIM" "$@" &
  local pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; kill -0 $pid 2>/dev/null && echo "  ... $(date +%T) running"; done
  wait $pid
}

if [ -z "${NOBENCH:-}" ]; then
  echo "[profile] bench"
  LIM=700 hb python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
  tail -c 400 "$OUT/bench.json"
fi
echo "[profile] kernel trace"
LIM=500 hb rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python3 bench.py $SHORT > "$OUT/kt.log" 2>&1
python3 tools/trace_window.py "$OUT/kt" --json "$OUT/window.json" > "$OUT/window.txt"
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kt_kernel_stats_full_run.csv" \;
# keep only the timed window's rows of the trace (pmc_summary.py reads them), drop the rest
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
sys.path.insert(0, "tools")
from pmc_summary import window
out = sys.argv[1]
src = glob.glob(os.path.join(out, "kt", "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(src)))
win = window(rows)
marks = [r for r in rows if "spin" in r["Kernel_Name"].lower() or "sleep" in r["Kernel_Name"].lower()][-2:]
with open(os.path.join(out, "kt_window.csv"), "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(sorted(marks + win, key=lambda r: int(r["Dispatch_Id"])))
PY
rm -rf "$OUT/kt" && mkdir -p "$OUT/kt" && mv "$OUT/kt_window.csv" "$OUT/kt/window_kernel_trace.csv"
head -25 "$OUT/window.txt"
echo "[profile] FETCH_SIZE"
LIM=600 hb rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$PMC_KERNELS" --output-format csv \
    -d "$OUT/pmc_fetch" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_fetch.log" 2>&1
echo "[profile] WRITE_SIZE"
LIM=600 hb rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$PMC_KERNELS" --output-format csv \
    -d "$OUT/pmc_write" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_summary.py "$OUT" "$OUT" > "$OUT/summary.txt"
rm -rf "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/kt"
head -30 "$OUT/summary.txt"
echo "[profile] SQ"
LIM=600 hb rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-include-regex "$PMC_KERNELS" --output-format csv \
    -d "$OUT/pmc_sq" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_sq.log" 2>&1
python3 tools/pmc_generic.py "$OUT/pmc_sq" > "$OUT/sq.txt"
rm -rf "$OUT/pmc_sq"
cat "$OUT/sq.txt"
echo "[profile] LDS"
# LDS-array busy cycles (SQ_LDS_IDX_ACTIVE) and bank-conflict cycles, for an LDS roofline of the LDS-resident sorts
LIM=600 hb rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES \
    --kernel-include-regex "spin|sleep|k_pc_finish|k_fa_ring_ds|k_pc_tail" --output-format csv \
    -d "$OUT/pmc_lds" -o pmc -- python3 bench.py $SHORT > "$OUT/pmc_lds.log" 2>&1
python3 tools/pmc_generic.py "$OUT/pmc_lds" > "$OUT/lds.txt"
rm -rf "$OUT/pmc_lds"
cat "$OUT/lds.txt"
echo "[profile] done"
