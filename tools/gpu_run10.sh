set -euo pipefail
mkdir -p gpurun_out/w21
timeout -k 10 400 python3 bench.py --cpu-scans 0 --icp-jobs 0 > gpurun_out/w21/b512.json 2> gpurun_out/w21/b512.err
echo done
