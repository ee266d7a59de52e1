#!/bin/bash
# round 4: pc_write / pc_lrank occupancy — VoxelGrid parity, then the bench (no extras)
set -o pipefail
mkdir -p gpurun_out/r04w
timeout -k 10 500 python -u -m pytest tests/test_gpu_voxel_pcl.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04w/tests.log 2>&1 || exit 2
./tools/gpu_bench.sh r04w --extra none --cpu-scans 0 --icp-jobs 0 || exit 6
