#!/bin/bash
# round 4: spent-depth ranges over 4 Ki heapsorted by a wave — VoxelGrid + pipeline parity (C5 included), bench with the C5 line
set -o pipefail
mkdir -p gpurun_out/r04s
timeout -k 10 800 python -u -m pytest tests/test_gpu_voxel_pcl.py tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04s/tests.log 2>&1 || exit 2
./tools/gpu_bench.sh r04s --extra c5 --cpu-scans 0 --icp-jobs 0 || exit 6
