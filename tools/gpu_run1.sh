set -euo pipefail
mkdir -p gpurun_out/w1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/w1/gpu_tests.log 2>&1
timeout -k 10 400 python3 bench.py --cpu-scans 0 > gpurun_out/w1/b256.json 2> gpurun_out/w1/b256.err
timeout -k 10 400 python3 bench.py --cpu-scans 0 --streams 512 > gpurun_out/w1/b512.json 2> gpurun_out/w1/b512.err
echo done
