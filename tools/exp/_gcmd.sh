set -eo pipefail
ROUNDS=1 timeout -k 10 1100 bash tools/exp/ab.sh ab26
