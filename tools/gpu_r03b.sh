# round 3: GPU suite, then the bench in PCL order and in the stable order
set -euo pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for vo in 0 1; do
  timeout -k 10 300 python3 bench.py --cpu-scans 0 --icp-jobs 0 --steps 40 --single-steps 50 --voxel-order $vo \
      --roofline-kernel mo_knn --roofline-also fa_search_corner > $OUT/bench_vo$vo.json 2> $OUT/bench_vo$vo.err
  python3 -c "import json; d=json.load(open('$OUT/bench_vo$vo.json')); print('vo $vo', d['value'], d['ms_per_step'], d.get('single_stream',{}).get('value'))"
done
