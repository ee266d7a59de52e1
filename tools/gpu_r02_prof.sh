set -euo pipefail
bash tools/profile_round.sh r02
bash tools/gpu_diag_pmc.sh r02diag
echo done
