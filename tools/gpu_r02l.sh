# per-step HIP graphs: GPU suite (graphs on by default), then bench graphs vs eager with the one-stream leg
set -euo pipefail
OUT=gpurun_out/${1:-r02l}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 100 --icp-jobs 0 --steps 40 > $OUT/b_graph.json 2> $OUT/b_graph.err
timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 100 --icp-jobs 0 --steps 40 --no-graphs > $OUT/b_eager.json 2> $OUT/b_eager.err
for f in b_graph b_eager; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); r=d['roofline']; print('$f', d['value'], r['avg_launch_us'], r['isolated']['frac'], d['single_stream'])"; done
echo done
