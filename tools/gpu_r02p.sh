# Re-entry check of HEAD (the whole -m gpu suite), then the VoxelGrid variants A/B (tools/gpu_r02q.sh)
set -euo pipefail
OUT=gpurun_out/${1:-r02p}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_gpu.log 2>&1
tail -3 $OUT/t_gpu.log
bash tools/gpu_r02q.sh
