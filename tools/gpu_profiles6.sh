#!/bin/bash
# round-6: the no-assembly upper bound (experiment build, wrong results) against the
# library on C3, then the PMC profiles of C2, C5 and C4 (tools/profile_round.sh, no full bench)
set -o pipefail
NOTEST=1 NOC5=1 bash tools/gpu_round6.sh r06e sc-lego-loam_amd/libslo.so sc-lego-loam_amd/variants/libslo_noasm.so sc-lego-loam_amd/libslo.so || exit $?
for c in c2 c5 c4; do
  NOBENCH=1 bash tools/profile_round.sh r06$c --config $c || exit $?
done
