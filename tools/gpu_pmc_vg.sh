# SQ counters of the VoxelGrid sort kernels on the microbench (map cloud, 170 streams); tag = $1
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/p1 -o p1 --output-format csv -- python3 tools/vg_bench.py --streams 170 --reps 1 --which map > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM -d $OUT/p2 -o p2 --output-format csv -- python3 tools/vg_bench.py --streams 170 --reps 1 --which map > $OUT/p2.log 2>&1
python3 tools/pmc_generic.py $OUT/p1 pc_ > $OUT/pmc.txt
python3 tools/pmc_generic.py $OUT/p2 pc_ >> $OUT/pmc.txt
cat $OUT/pmc.txt
