#!/bin/bash
# round 4: the wave heapsort — VoxelGrid + pipeline parity, then ring / stage timings
set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 700 python -u -m pytest tests/test_gpu_voxel_pcl.py tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04j/tests.log 2>&1 || exit 2
SLO_LIB=sc-lego-loam_amd/variants/libslo_ring.so timeout -k 10 200 python -u tools/ring_diag.py > gpurun_out/r04j/ring.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/stage_profile.py > gpurun_out/r04j/stages.txt 2>&1 || exit 4
timeout -k 10 200 python -u tools/pipe_depth.py 220 6 > gpurun_out/r04j/depth.txt 2>&1 || exit 5
