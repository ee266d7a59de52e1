#!/bin/bash
# round 4: f64 MFMA rate probe, then the GPU suite (MFMA Scan Context distance, batched mapping VoxelGrids)
set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 60 ./tools/bin/mfma_f64_check 20000 > gpurun_out/r04c/mfma.log 2>&1 || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r04c/all.log 2>&1 || exit 2
