#!/bin/bash
# round-6: an A/B of experiment builds named in $AB (tools/archive/gpu_round6.sh), then the
# PMC profiles of the configs given (tools/profile_round.sh, no full bench)
set -o pipefail
if [ -n "${AB:-}" ]; then
  NOTEST=1 NOC5=1 bash tools/archive/gpu_round6.sh r06ab $AB || exit $?
fi
for c in ${*:-c2 c5 c4}; do
  NOBENCH=1 bash tools/profile_round.sh r06$c --config $c || exit $?
done
