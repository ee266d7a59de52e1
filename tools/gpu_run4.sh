set -euo pipefail
mkdir -p gpurun_out/w4
timeout -k 10 300 python -u -m pytest tests/test_gpu_loop.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w4/gpu_loop.log 2>&1 || { tail -30 gpurun_out/w4/gpu_loop.log; exit 1; }
timeout -k 10 400 python3 bench.py --cpu-scans 0 --streams 256 > gpurun_out/w4/b256.json 2> gpurun_out/w4/b256.err
echo done
