#!/bin/bash
# round 4: 32-bit finish items — VoxelGrid + pipeline parity, then the bench
set -o pipefail
mkdir -p gpurun_out/r04q
timeout -k 10 800 python -u -m pytest tests/test_gpu_voxel_pcl.py tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04q/tests.log 2>&1 || exit 2
./tools/gpu_bench.sh r04q --extra none --cpu-scans 0 --icp-jobs 0 || exit 6
