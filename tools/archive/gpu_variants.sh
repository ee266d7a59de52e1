# bench several libslo variants (SLO_LIB) back to back: tools/gpu_variants.sh <tag> <lib>...
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  n=$(basename $lib .so)
  SLO_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 ${BENCH_ARGS:-} > $OUT/$n.json 2> $OUT/$n.err
  python3 -c "import json,sys; d=json.load(open('$OUT/$n.json')); r=d['roofline']; print('$n', d['value'], r['avg_launch_us'], r['isolated']['avg_launch_us'], r['isolated']['frac'])"
done
echo done
