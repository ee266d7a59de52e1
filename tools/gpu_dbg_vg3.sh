# the PCL-order tests against an experiment build; tag = $1, build = $2
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SLO_LIB=sc-lego-loam_amd/variants/libslo_$2.so timeout -k 10 600 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_voxel_pcl.py > $OUT/pytest.log 2>&1 || true
grep -E "PASSED|FAILED|Error|assert" $OUT/pytest.log | head -20
