#!/bin/bash
# round 4 first GPU pass: f64 MFMA semantics, the bench-shape tests, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 60 ./tools/bin/mfma_f64_check 20000 > gpurun_out/r04a/mfma.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "bench_shape or argument_checks" -s > gpurun_out/r04a/new.log 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04a/all.log 2>&1 || exit 3
