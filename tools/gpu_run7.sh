set -euo pipefail
mkdir -p gpurun_out/w12
timeout -k 10 400 python3 bench.py --cpu-scans 0 --icp-jobs 0 > gpurun_out/w12/stagger.json 2> gpurun_out/w12/stagger.err
timeout -k 10 400 python3 bench.py --cpu-scans 0 --icp-jobs 0 --no-stagger > gpurun_out/w12/lock.json 2> gpurun_out/w12/lock.err
echo done
