# hash-grid walks with unconditional entry loads (all of a step's loads in flight), local-map assembly and
# VoxelGrid bounds with eight loads per thread: parity on g2, then A/B (committed c0, g2, g4 = 5-NN unroll 4)
set -euo pipefail
OUT=gpurun_out/${1:-r02w}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SLO_LIB=sc-lego-loam_amd/variants/libslo_g2.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loop.py tests/test_gpu_voxel.py tests/test_gpu_posegraph.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -1 $OUT/t_par.log
export SLO_LIB=sc-lego-loam_amd/variants/libslo_g4.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "c3_steady or pipeline_bit_exact" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par4.log 2>&1
tail -1 $OUT/t_par4.log
unset SLO_LIB
bash tools/gpu_variants.sh ${1:-r02w}/v sc-lego-loam_amd/variants/libslo_c0.so sc-lego-loam_amd/variants/libslo_g2.so sc-lego-loam_amd/variants/libslo_g4.so sc-lego-loam_amd/variants/libslo_c0.so sc-lego-loam_amd/variants/libslo_g2.so sc-lego-loam_amd/variants/libslo_g4.so
