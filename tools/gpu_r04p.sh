#!/bin/bash
# round 4: 32-bit finish items (parity + bench), then mo_knn's query-order cell 4 m / 2 m / 8 m (MO_PERM_INV variants)
set -o pipefail
./tools/gpu_r04o.sh || exit $?
mkdir -p gpurun_out/r04n
for v in variants/libslo_p2.so variants/libslo_p8.so; do
  tag=${v##*/}
  SLO_LIB=sc-lego-loam_amd/$v timeout -k 10 400 python -u bench.py --extra none --cpu-scans 0 --icp-jobs 0 --single-steps 0 \
    --steps 30 > gpurun_out/r04n/bench_$tag.json 2> gpurun_out/r04n/bench_$tag.err || exit 3
  echo "$tag done"
done
