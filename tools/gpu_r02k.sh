# LDS-staged mo_knn regions: parity (pipelines, steady state), diag counters, timing
set -euo pipefail
OUT=gpurun_out/${1:-r02k}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "pipeline_bit_exact or c3_steady or c2_sc_off or c5 or node_mirrors or ragged" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
SLO_LIB=sc-lego-loam_amd/variants/libslo_knndiag.so timeout -k 10 300 python3 -u tools/knn_diag.py 32 210 40 > $OUT/diag.log 2>&1
timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 > $OUT/b.json 2> $OUT/b.err
echo done
