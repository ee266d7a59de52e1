# tests given as arguments first (if any), then a short bench per voxel order
# listed in $VOS (default "0"); tag = $1
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for vo in ${VOS:-0}; do
  timeout -k 10 400 python3 bench.py --cpu-scans 0 --icp-jobs 0 --steps 40 --single-steps 50 --voxel-order $vo \
      --roofline-kernel mo_knn --roofline-also fa_search_corner > $OUT/bench_vo$vo.json 2> $OUT/bench_vo$vo.err
  python3 - <<PY
import json
d = json.load(open('$OUT/bench_vo$vo.json'))
print('vo $vo', d['value'], d['ms_per_step'], d.get('single_stream', {}).get('value'))
km = d['kernels_ms']
for k, v in sorted(km.items(), key=lambda kv: -kv[1][0])[:14]:
    print('   ', k, v)
PY
done
