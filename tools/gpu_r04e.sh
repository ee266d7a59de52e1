#!/bin/bash
# round 4: VoxelGrid / mode S / pipeline tests, then the default bench
set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "voxel or modes or bench_shape or pipeline_bit_exact" > gpurun_out/r04e/tests.log 2>&1 || exit 2
./tools/gpu_bench.sh r04e || exit 3
