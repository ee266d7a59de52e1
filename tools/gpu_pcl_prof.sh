# PCL-order sort: microbench with work counters, then SQ counters of its kernels; tag = $1
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/vg_bench.py --streams 170 > $OUT/vgb.log 2>&1 || { tail -20 $OUT/vgb.log; exit 1; }
grep -v amdgpu.ids $OUT/vgb.log | head -4
bash tools/gpu_pmc_vg.sh $1
