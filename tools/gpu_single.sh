# one-stream latency per experiment build: bench.py with one stream in one context; tag = $1, builds = $2..
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ $v = base ]; then L=""; else L=sc-lego-loam_amd/variants/libslo_$v.so; fi
  SLO_LIB=$L timeout -k 10 300 python3 bench.py --streams 1 --groups 1 --cpu-scans 0 --icp-jobs 0 --profile-steps 0 \
      --steps 40 --single-steps 60 > $OUT/single_$v.json 2> $OUT/single_$v.err || { tail -5 $OUT/single_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/single_$v.json')); print('$v', d['value'], d['ms_per_step'], d['single_stream'])"
done
