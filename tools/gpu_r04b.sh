#!/bin/bash
# round 4: f64 MFMA rate, the MFMA Scan Context distance against the oracle
set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 60 ./tools/bin/mfma_f64_check 20000 > gpurun_out/r04b/mfma.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "sc_ or xsc or loop_fixture or pipeline_bit_exact" > gpurun_out/r04b/sc.log 2>&1 || exit 2
