# round 2, first GPU call: new GPU tests (device generator, VoxelGrid overflow),
# the full GPU suite, then the steady-state bench.
set -euo pipefail
OUT=gpurun_out/r02a
mkdir -p $OUT
nproc > $OUT/host.txt; python3 -c "import os;print(len(os.sched_getaffinity(0)))" >> $OUT/host.txt
cat /sys/fs/cgroup/cpu.max >> $OUT/host.txt 2>/dev/null || true
grep -m1 "model name" /proc/cpuinfo >> $OUT/host.txt || true
ldd --version | head -1 >> $OUT/host.txt || true
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_gen.py tests/test_gpu_voxel.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t_new.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_all.log 2>&1
timeout -k 10 500 python3 bench.py --icp-jobs 0 > $OUT/bench.json 2> $OUT/bench.err
echo done
