#!/bin/bash
# round 4: the partner table at f/2 (half the LDS) — VoxelGrid + pipeline parity; bench at finish32 occupancy 5 (default) and 6
set -o pipefail
mkdir -p gpurun_out/r04aa
timeout -k 10 800 python -u -m pytest tests/test_gpu_voxel_pcl.py tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04aa/tests.log 2>&1 || exit 2
for v in "" variants/libslo_o6.so; do
  tag=${v:-default}; tag=${tag##*/}
  SLO_LIB=${v:+sc-lego-loam_amd/$v} timeout -k 10 400 python -u bench.py --extra none --cpu-scans 0 --icp-jobs 0 --single-steps 0 \
    > gpurun_out/r04aa/bench_$tag.json 2> gpurun_out/r04aa/bench_$tag.err || exit 3
  echo "$tag done"
done
