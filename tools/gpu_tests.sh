# run pytest selections on the GPU box: tools/gpu_tests.sh <tag> <pytest args...>
# (log in gpurun_out/<tag>/pytest.log; every test under its own 300 s limit)
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 ${GPU_T:-1000} python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -5 $OUT/pytest.log
