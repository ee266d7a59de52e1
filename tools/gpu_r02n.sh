# chunked cross-stream K-NN: xsc GPU test, store micro-bench old vs new at 1 and 8 ranks' sizes
set -euo pipefail
OUT=gpurun_out/${1:-r02n}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_xsc.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_xsc.log 2>&1
for n in 512 4096; do
  timeout -k 10 200 python3 -u tools/xsc_bench.py $n 512 64 >> $OUT/xsc.log 2>&1
  SLO_LIB=sc-lego-loam_amd/variants/libslo_oldxsc.so timeout -k 10 200 python3 -u tools/xsc_bench.py $n 512 64 | sed 's/^/old: /' >> $OUT/xsc.log 2>&1
done
cat $OUT/xsc.log
echo done
