#!/bin/bash
# round 4: few-stream surf search (8 lanes per query) — parity, stage timings, ring waves per ring at 170 streams
set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04l/tests.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/stage_profile.py > gpurun_out/r04l/stages.txt 2>&1 || exit 4
timeout -k 10 200 python -u tools/pipe_depth.py 220 6 > gpurun_out/r04l/depth.txt 2>&1 || exit 5
for v in "" variants/libslo_rw2.so variants/libslo_rw4.so; do
  echo "== lib ${v:-default}" >> gpurun_out/r04l/rw.txt
  SLO_LIB=${v:+sc-lego-loam_amd/$v} timeout -k 10 120 python -u tools/ring_diag.py 170 >> gpurun_out/r04l/rw.txt 2>&1 || exit 6
done
