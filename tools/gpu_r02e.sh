# record exchange + cross-stream store on the device; corner search with the
# wave binary search; bench through the gather path (one-rank RCCL group)
set -euo pipefail
OUT=gpurun_out/r02e
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_xsc.py tests/test_gpu_parity.py -k "xsc or pipeline_bit_exact or node_mirrors or sc_loop" -x -v --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/t.log 2>&1
timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 > $OUT/b.json 2> $OUT/b.err
timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 --force-gather --profile-steps 0 > $OUT/bg.json 2> $OUT/bg.err
echo done
