# PCL-order VoxelGrid check: its GPU tests, then the microbench (tools/vg_bench.py) at 40 and 170 streams
# with the sort's error counters; tag = $1
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_voxel_pcl.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for S in 40 170; do
  timeout -k 10 300 python3 tools/vg_bench.py --streams $S --which map,raw > $OUT/vgb_$S.log 2>&1 || { tail -8 $OUT/vgb_$S.log; exit 1; }
  echo "== S=$S"; grep -v amdgpu.ids $OUT/vgb_$S.log | grep -E '^(map|raw) 0' | sed 's/"pcl_work.*vg_stats/vg_stats/' | cut -c1-900
done
