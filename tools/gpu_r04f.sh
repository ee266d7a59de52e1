#!/bin/bash
# round 4: the split back end (odometry | mapping contexts), then a short bench with the pipelined legs
set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 500 python -u -m pytest tests/test_gpu_modes.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04f/tests.log 2>&1 || exit 2
./tools/gpu_bench.sh r04f --extra none --cpu-scans 0 --icp-jobs 0 || exit 3
