#!/bin/bash
# round-6: the PMC profiles of C2, C5 and C4 (tools/profile_round.sh, no full bench)
set -o pipefail
for c in ${*:-c2 c5 c4}; do
  NOBENCH=1 bash tools/profile_round.sh r06$c --config $c || exit $?
done
