#!/bin/bash
# Quick A/B on the GPU box: the given pytest files (parity first), then short
# bench lines for the named configs (no CPU baseline, no one-stream legs).
#   tools/gpu_quick.sh <tag> "<pytest files>" "<configs: c3 c2 c5>" [extra bench args]
set -euo pipefail
TAG=$1; TESTS=$2; CONFIGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { tail -30 "$OUT/pytest.log"; exit 1; }
  tail -3 "$OUT/pytest.log"
fi
for c in $CONFIGS; do
  timeout -k 10 400 python3 bench.py --config "$c" --extra none --single-steps 0 --icp-jobs 0 --cpu-scans 0 \
    --steps 12 --warmup 3 "$@" > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  python3 - "$OUT/bench_$c.json" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
km = j["kernels_ms"]
tot = sum(v[0] for k, v in km.items() if not k.startswith("vg_sort:"))
print(sys.argv[1], "value", j["value"], "ms/step", j["ms_per_step"], "errors", j["stream_errors"], j["sort_guards"]["fallback_ranges"],
      j["sort_guards"]["inconsistent_steps"])
for k, v in list(km.items())[:14]:
    if not k.startswith("vg_sort:"):
        print(f"  {k:20s} {v[0]:8.2f} ms {v[1]:5d} {100 * v[0] / tot:5.1f}%  {j['kernels_algo_gbs'].get(k)} GB/s")
PY
done
