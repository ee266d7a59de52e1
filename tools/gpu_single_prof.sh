# one stream: per-kernel device time and launch counts of 8 instrumented steps (2 mapping steps); tag = $1
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --streams 1 --groups 1 --cpu-scans 0 --icp-jobs 0 --profile-steps 8 \
    --steps 40 --single-steps 60 > $OUT/single.json 2> $OUT/single.err || { tail -5 $OUT/single.err; exit 1; }
python3 - <<PY
import json
d = json.load(open('$OUT/single.json'))
print(d['value'], d['ms_per_step'], d['single_stream'])
km = d['kernels_ms']
tot = sum(v[0] for k, v in km.items() if not k.startswith('vg_sort:'))
n = sum(v[1] for k, v in km.items() if not k.startswith('vg_sort:'))
print('kernel ms', round(tot, 3), 'launches', n)
for k, v in list(km.items())[:25]:
    print('   ', k, v)
PY
