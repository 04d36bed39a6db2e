set -eo pipefail
bash tools/gpu_round.sh r2b
bash tools/gpu_prof_round.sh r2b_prof
