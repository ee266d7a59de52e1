#!/bin/bash
# round 4: sharp points x-order in register slices — pipeline parity + mode S, stage timings, bench (no extras)
set -o pipefail
mkdir -p gpurun_out/r04af
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04af/tests.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/stage_profile.py > gpurun_out/r04af/stages.txt 2>&1 || exit 4
./tools/gpu_bench.sh r04af --extra none --cpu-scans 0 --icp-jobs 0 || exit 6
