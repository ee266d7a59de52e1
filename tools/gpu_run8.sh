set -euo pipefail
mkdir -p gpurun_out/w18
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "7-5-2-10" --timeout 200 --timeout-method thread > gpurun_out/w18/c5.log 2>&1 || { tail -30 gpurun_out/w18/c5.log; exit 1; }
timeout -k 10 400 python3 bench.py --cpu-scans 0 --icp-jobs 0 --force-gather --streams 256 --steps 8 --warmup 4 > gpurun_out/w18/gather.json 2> gpurun_out/w18/gather.err
echo done
