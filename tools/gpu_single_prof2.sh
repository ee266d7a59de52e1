# one stream, per-kernel device time, PCL vs stable VoxelGrid order; tag = $1
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for vo in 0 1; do
timeout -k 10 300 python3 bench.py --streams 1 --groups 1 --cpu-scans 0 --icp-jobs 0 --profile-steps 8 --voxel-order $vo \
    --steps 40 --single-steps 60 > $OUT/single_vo$vo.json 2> $OUT/single_vo$vo.err || { tail -5 $OUT/single_vo$vo.err; exit 1; }
python3 - <<PY
import json
d = json.load(open('$OUT/single_vo$vo.json'))
print('vo $vo', d['value'], d['ms_per_step'], d['single_stream']['latency_ms'])
km = d['kernels_ms']
print('   ', {k: v for k, v in km.items() if k.startswith('fa_') or k.startswith('ip_')})
PY
done
