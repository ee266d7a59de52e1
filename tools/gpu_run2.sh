set -euo pipefail
mkdir -p gpurun_out/w2
timeout -k 10 400 python -u -m pytest tests/test_gpu_loop.py -x -v --timeout 300 --timeout-method thread > gpurun_out/w2/gpu_loop.log 2>&1 || { tail -40 gpurun_out/w2/gpu_loop.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/w2/gpu_tests.log 2>&1
echo done
