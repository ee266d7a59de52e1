set -euo pipefail
mkdir -p gpurun_out/w8
for cfg in "512 3" "512 4" "640 2"; do
  set -- $cfg
  timeout -k 10 400 python3 bench.py --cpu-scans 0 --icp-jobs 0 --profile-steps 0 --streams $1 --groups $2 > gpurun_out/w8/b$1_g$2.json 2> gpurun_out/w8/b$1_g$2.err
  tail -c 200 gpurun_out/w8/b$1_g$2.json
done
echo done
