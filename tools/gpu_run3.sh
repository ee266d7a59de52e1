set -euo pipefail
mkdir -p gpurun_out/w3
for S in 256 512 768 1024; do
  J=0; [ $S = 256 ] && J=64
  timeout -k 10 400 python3 bench.py --cpu-scans 0 --streams $S --icp-jobs $J > gpurun_out/w3/b$S.json 2> gpurun_out/w3/b$S.err
  tail -c 300 gpurun_out/w3/b$S.json
done
echo done
