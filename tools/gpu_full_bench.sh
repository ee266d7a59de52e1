# the default bench line (what the driver runs), then a summary; tag = $1
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
python3 - <<PY
import json
d = json.load(open('$OUT/bench.json'))
print(d['value'], d['ms_per_step'], d.get('single_stream', {}).get('value'))
print(json.dumps(d['roofline'])[:1500])
print(json.dumps(d['cpu_baseline']))
km = d['kernels_ms']
for k, v in sorted(km.items(), key=lambda kv: -kv[1][0])[:16]:
    print('   ', k, v)
PY
