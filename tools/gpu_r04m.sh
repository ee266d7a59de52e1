#!/bin/bash
# round 4: four waves per ring VoxelGrid, few-stream surf search with split walks — parity, timings, bench
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 800 python -u -m pytest tests/test_gpu_voxel_pcl.py tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04m/tests.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/stage_profile.py > gpurun_out/r04m/stages.txt 2>&1 || exit 4
timeout -k 10 200 python -u tools/pipe_depth.py 220 6 > gpurun_out/r04m/depth.txt 2>&1 || exit 5
./tools/gpu_bench.sh r04m --extra none --cpu-scans 0 --icp-jobs 0 || exit 6
