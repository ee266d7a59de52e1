set -euo pipefail
mkdir -p gpurun_out/w20
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/w20/gpu_tests.log 2>&1 || { tail -30 gpurun_out/w20/gpu_tests.log; exit 1; }
timeout -k 10 400 python3 bench.py --cpu-scans 0 > gpurun_out/w20/b512.json 2> gpurun_out/w20/b512.err
echo done
