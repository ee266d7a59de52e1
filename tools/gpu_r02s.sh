# End-of-round check of the final build: the whole -m gpu suite, then the round's profile (tools/profile_round.sh)
set -euo pipefail
OUT=gpurun_out/${1:-r02e}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_gpu.log 2>&1
tail -2 $OUT/t_gpu.log
bash tools/profile_round.sh ${1:-r02e}
