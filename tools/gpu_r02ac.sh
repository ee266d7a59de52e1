# contexts per GPU on the final build: --groups 2 / 3 / 4 (40-step bench, no CPU legs), twice
set -euo pipefail
OUT=gpurun_out/${1:-r02ac}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for g in 2 3 4; do
    timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 --groups $g > $OUT/g${g}_$rep.json 2> $OUT/g${g}_$rep.err
    python3 -c "import json; d=json.load(open('$OUT/g${g}_$rep.json')); print('groups $g', d['value'], d['ms_per_step'])"
  done
done
