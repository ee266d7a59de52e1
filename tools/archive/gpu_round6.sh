#!/bin/bash
# round-6 GPU check: the full -m gpu suite, the C5 config line, then an A/B of
# experiment builds (SLO_LIB) on the C3 bench — each step under its own limit,
# stop at the first failure.  NOTEST=1 / NOC5=1 skip the first two.
set -o pipefail
OUT=gpurun_out/${1:-r06c}
shift
mkdir -p "$OUT"
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
fi
if [ -z "${NOC5:-}" ]; then
  timeout -k 10 400 python -u bench.py --extra none --single-steps 0 --icp-jobs 0 --modes-steps 0 --steps 12 --warmup 3 \
      --profile-steps 4 --cpu-scans 0 --config c5 --detail-out "$OUT/c5_detail.json" > "$OUT/c5.out" 2> "$OUT/c5.err" || exit $?
fi
i=0
for lib in "$@"; do
  i=$((i + 1))
  n=$i_$(basename "$lib" .so)
  SLO_LIB=$lib timeout -k 10 300 python -u bench.py --extra none --single-steps 0 --icp-jobs 0 --modes-steps 0 --cpu-scans 0 \
      --steps 40 ${BENCH_ARGS:-} --detail-out "$OUT/d_${i}_$n.json" > "$OUT/b_${i}_$n.out" 2> "$OUT/b_${i}_$n.err" || exit $?
  python3 -c "import json; d=json.loads(open('$OUT/b_${i}_$n.out').read().strip().splitlines()[-1]); print('$i $n', d['value'], d['roofline']['avg_launch_us'])"
done
