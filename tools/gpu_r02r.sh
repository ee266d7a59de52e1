# single-pass VoxelGrid scatter (decoupled look-back): voxel + pipeline parity on the variant, then A/B bench
set -euo pipefail
OUT=gpurun_out/${1:-r02r}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SLO_LIB=sc-lego-loam_amd/variants/libslo_osw.so
timeout -k 10 240 python3 -u -m pytest tests/test_gpu_voxel.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/t_vox.log 2>&1
tail -2 $OUT/t_vox.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loop.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -2 $OUT/t_par.log
unset SLO_LIB
BENCH_ARGS='--roofline-kernel mo_knn --roofline-also mo_knn' bash tools/gpu_variants.sh ${1:-r02r}/v sc-lego-loam_amd/variants/libslo_scan.so sc-lego-loam_amd/variants/libslo_osw.so sc-lego-loam_amd/variants/libslo_scan.so sc-lego-loam_amd/variants/libslo_osw.so
