#!/bin/bash
# round 4: global levels past log2(stride / 64 Ki): 9 and 12 — bench (no extras) each; VoxelGrid parity on the variant
set -o pipefail
mkdir -p gpurun_out/r04z
SLO_LIB=sc-lego-loam_amd/variants/libslo_x12.so timeout -k 10 500 python -u -m pytest tests/test_gpu_voxel_pcl.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04z/tests.log 2>&1 || exit 2
for v in variants/libslo_x9.so variants/libslo_x12.so; do
  tag=${v:-default}; tag=${tag##*/}
  SLO_LIB=${v:+sc-lego-loam_amd/$v} timeout -k 10 400 python -u bench.py --extra none --cpu-scans 0 --icp-jobs 0 --single-steps 0 \
    > gpurun_out/r04z/bench_$tag.json 2> gpurun_out/r04z/bench_$tag.err || exit 3
  echo "$tag done"
done
