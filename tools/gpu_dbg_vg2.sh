# PCL-order sort error counters at 40 streams per experiment build; tag = $1, builds = $2..
set -euo pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ $v = base ]; then L=""; else L=sc-lego-loam_amd/variants/libslo_$v.so; fi
  SLO_LIB=$L timeout -k 10 300 python3 tools/vg_bench.py --streams 40 --which map --reps 1 > $OUT/vgb_$v.log 2>&1 || { tail -8 $OUT/vgb_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/vgb_$v.log | grep -E '^map 0' | sed 's/"pcl_work.*vg_stats/vg_stats/' | cut -c1-900
done
