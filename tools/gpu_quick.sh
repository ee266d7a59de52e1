# quick GPU check of the VoxelGrid sort: PCL-order tests, a pipeline parity case, the microbench; tag = $1
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_voxel_pcl.py \
    "tests/test_gpu_parity.py::test_pipeline_bit_exact" tests/test_gpu_voxel.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python3 tools/vg_bench.py --streams 170 > $OUT/vgb.log 2>&1 || { tail -20 $OUT/vgb.log; exit 1; }
grep -v amdgpu.ids $OUT/vgb.log | head -4
