# hand-written segmented VoxelGrid sort: parity (voxel, pipelines, steady state) + timing
set -euo pipefail
OUT=gpurun_out/${1:-r02j}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_voxel.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t_vox.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "pipeline_bit_exact or c3_steady or c2_sc_off or node_mirrors or sc_loop or ragged or front" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
timeout -k 10 300 python3 bench.py --cpu-scans 0 --single-steps 0 --icp-jobs 0 --steps 40 > $OUT/b.json 2> $OUT/b.err
echo done
