# pose-graph pipeline test; context count / stagger sweep at steady state
set -euo pipefail
OUT=gpurun_out/r02g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_posegraph.py -x -v -s --timeout 350 --timeout-method thread -p no:cacheprovider > $OUT/t_pg.log 2>&1
Q="--cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 --profile-steps 0"
for v in "--groups 3" "--groups 4" "--groups 4 --stagger" "--groups 6" "--groups 8"; do
  tag=$(echo $v | tr -d ' -')
  timeout -k 10 300 python3 bench.py $Q $v > $OUT/b_$tag.json 2> $OUT/b_$tag.err
done
echo done
