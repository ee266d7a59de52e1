# LDS corner search + parallel gather: parity, then bench vs the previous build
set -euo pipefail
OUT=gpurun_out/${1:-r02o}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_imu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_par.log 2>&1
tail -2 $OUT/t_par.log
bash tools/gpu_variants.sh ${1:-r02o}/v sc-lego-loam_amd/libslo.so sc-lego-loam_amd/variants/libslo_head.so
