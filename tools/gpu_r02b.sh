# round 2: C2 / long-C3 parity (+ the whole GPU suite after the corner-grid
# change); context-count sweep at steady state; kernel trace of the timed
# window only (--roctx + --selected-regions)
set -euo pipefail
OUT=gpurun_out/r02b
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "c2_sc_off or c3_steady" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not c2_sc_off and not c3_steady" > $OUT/t_all.log 2>&1
Q="--cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 --profile-steps 0"
for g in 1 3; do
  timeout -k 10 300 python3 bench.py $Q --groups $g > $OUT/b_g$g.json 2> $OUT/b_g$g.err
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --selected-regions --output-format csv -d $OUT/kt -o kt -- python3 bench.py $Q --steps 12 --roctx > $OUT/kt.log 2>&1
echo done
