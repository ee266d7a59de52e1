#!/bin/bash
# round 4: the Mode S odometry context skips transformFusion — mode S tests, stage timings, three-stage rate
set -o pipefail
mkdir -p gpurun_out/r04ac
timeout -k 10 500 python -u -m pytest tests/test_gpu_modes.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r04ac/tests.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/stage_profile.py > gpurun_out/r04ac/stages.txt 2>&1 || exit 4
timeout -k 10 200 python -u tools/pipe_depth.py 220 6 > gpurun_out/r04ac/depth.txt 2>&1 || exit 5
