# PCL-order sort: tests on the default build, then the VoxelGrid microbench per
# experiment build (sc-lego-loam_amd/variants/libslo_<name>.so); tag = $1, names = $2..
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_voxel_pcl.py \
    "tests/test_gpu_parity.py::test_pipeline_bit_exact" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=sc-lego-loam_amd/variants/libslo_$v.so; fi
  SLO_LIB=$L timeout -k 10 300 python3 tools/vg_bench.py --streams 170 > $OUT/vgb_$v.log 2>&1 || { tail -20 $OUT/vgb_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/vgb_$v.log | grep -E '^(map|raw) 0' | cut -c1-900
done
