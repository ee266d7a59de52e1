#!/bin/bash
# round 4: ring VoxelGrid at seven waves per SIMD (pool of 128) — VoxelGrid + pipeline parity, then the bench (no extras)
set -o pipefail
mkdir -p gpurun_out/r04ab
timeout -k 10 800 python -u -m pytest tests/test_gpu_voxel_pcl.py tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04ab/tests.log 2>&1 || exit 2
./tools/gpu_bench.sh r04ab --extra none --cpu-scans 0 --icp-jobs 0 || exit 6
