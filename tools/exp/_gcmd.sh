set -eo pipefail
ROUNDS=2 timeout -k 10 900 bash tools/exp/ab.sh ab27
