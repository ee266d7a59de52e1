set -euo pipefail
mkdir -p gpurun_out/w19
timeout -k 10 400 python3 bench.py --cpu-scans 0 --icp-jobs 0 --force-gather --streams 256 --steps 8 --warmup 4 > gpurun_out/w19/gather.json 2> gpurun_out/w19/gather.err
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --cpu-scans 0 --icp-jobs 0 --force-gather --streams 256 --steps 8 --warmup 4 > gpurun_out/w19/trun.json 2> gpurun_out/w19/trun.err
echo done
