set -o pipefail
mkdir -p gpurun_out/r06l
for v in sc-lego-loam_amd/libslo.so sc-lego-loam_amd/variants/libslo_fg2.so sc-lego-loam_amd/variants/libslo_nofork.so sc-lego-loam_amd/libslo.so; do
  n=$(basename $v .so)
  SLO_LIB=$v EAGER=0 SCANS=200 TRACE_OUT=gpurun_out/r06l/$n.json timeout -k 10 120 python -u tools/single_trace.py > gpurun_out/r06l/$n.log 2>&1 || exit $?
  echo "$n $(tail -1 gpurun_out/r06l/$n.log)"; grep flags gpurun_out/r06l/$n.log
done
