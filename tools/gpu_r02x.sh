# final candidate f (fa_points windows in LDS, vg_long gathers in flight, on top of g2): the whole -m gpu suite on
# the in-tree build (= f), an A/B against g2, then the round's profile (tools/profile_round.sh)
set -euo pipefail
TAG=${1:-r02f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/t_gpu.log 2>&1
tail -1 $OUT/t_gpu.log
bash tools/gpu_variants.sh $TAG/v sc-lego-loam_amd/variants/libslo_g2.so sc-lego-loam_amd/variants/libslo_f.so sc-lego-loam_amd/variants/libslo_g2.so sc-lego-loam_amd/variants/libslo_f.so
bash tools/profile_round.sh $TAG
