# throughput vs streams per GPU / contexts: tools/gpu_sweep.sh <tag> "<streams>:<groups>" ...
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for sg in "$@"; do
  S=${sg%%:*}; G=${sg##*:}
  timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --profile-steps 0 --steps 40 --streams $S --groups $G > $OUT/s${S}_g${G}.json 2> $OUT/s${S}_g${G}.err
  python3 -c "import json; d=json.load(open('$OUT/s${S}_g${G}.json')); print('$S', '$G', d['value'], d['ms_per_step'], d['stream_errors'])"
done
echo done
