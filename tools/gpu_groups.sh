# contexts per GPU: the bench's throughput at several --groups; tag = $1, group counts = $2..
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in "$@"; do
  timeout -k 10 400 python3 bench.py --groups $g --cpu-scans 0 --single-steps 0 --icp-jobs 0 --profile-steps 0 --steps 60 \
      > $OUT/g$g.json 2> $OUT/g$g.err || { tail -5 $OUT/g$g.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/g$g.json')); print('groups $g', d['value'], d['ms_per_step'])"
done
