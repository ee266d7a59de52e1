# diagnostic PMC passes over the timed window of a short steady-state bench
# (one pass per counter group; bench.py --trace-marker, cut by pmc_generic.py)
set -euo pipefail
OUT=gpurun_out/${1:-diag}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 12 --profile-steps 0 --trace-marker"
timeout -s KILL 500 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o pmc -- python3 $B > $OUT/sq.log 2>&1
timeout -s KILL 500 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o pmc -- python3 $B > $OUT/tcc.log 2>&1
python3 tools/pmc_generic.py $OUT/sq > $OUT/sq.txt
python3 tools/pmc_generic.py $OUT/tcc > $OUT/tcc.txt
rm -rf $OUT/sq $OUT/tcc
echo done
