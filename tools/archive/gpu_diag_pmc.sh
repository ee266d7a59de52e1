# diagnostic PMC passes over the timed window of a short steady-state bench
# (bench.py --trace-marker, cut by pmc_generic.py).
#   tools/gpu_diag_pmc.sh <tag> [name-filter] ["COUNTERS OF PASS 1" "COUNTERS OF PASS 2" ...]
# One rocprofv3 run per pass (at most 8 SQ_ counters each).
set -euo pipefail
OUT=gpurun_out/${1:-diag}
FILT=${2:-}
shift 2 || shift $#
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 12 --profile-steps 0 --trace-marker"
if [ $# -eq 0 ]; then
  set -- "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum"
fi
i=0
for pass in "$@"; do
  i=$((i + 1))
  echo "[pmc] pass $i: $pass"
  timeout -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o pmc -- python3 $B > $OUT/p$i.log 2>&1
  python3 tools/pmc_generic.py $OUT/p$i $FILT > $OUT/p$i.txt
  rm -rf $OUT/p$i
done
echo done
