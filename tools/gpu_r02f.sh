# full GPU suite after the body-frame keyframe ring + pose-graph wiring
set -euo pipefail
OUT=gpurun_out/r02f
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/t_all.log 2>&1
timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 > $OUT/b.json 2> $OUT/b.err
echo done
