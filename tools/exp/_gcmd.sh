set -eo pipefail
bash tools/gpu_prof_round.sh r2a
