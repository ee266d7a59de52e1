set -euo pipefail
D=gpurun_out/w22
mkdir -p $D
for g in 3 4; do
  timeout -k 10 300 python3 bench.py --cpu-scans 0 --icp-jobs 0 --groups $g > $D/g$g.json 2> $D/g$g.err
done
timeout -k 10 300 python3 bench.py --cpu-scans 0 --icp-jobs 0 --groups 4 --streams 640 > $D/g4s640.json 2> $D/g4s640.err
echo done
