# Final check of the round's build: the whole -m gpu suite, smoke(), then the round's profile (tools/profile_round.sh)
set -euo pipefail
TAG=${1:-r02g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_gpu.log 2>&1
tail -1 $OUT/t_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
bash tools/profile_round.sh $TAG
