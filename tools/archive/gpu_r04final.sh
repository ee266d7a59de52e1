#!/bin/bash
# round 4 close: the whole GPU suite, then the default bench (CPU baselines, C2 / C5 lines, ICP)
set -o pipefail
mkdir -p gpurun_out/r04close2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r04close2/tests.log 2>&1 || exit 2
./tools/gpu_bench.sh r04close2 || exit 3
