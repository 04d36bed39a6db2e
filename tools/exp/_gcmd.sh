set -eo pipefail
ROUNDS=2 timeout -k 10 600 bash tools/exp/ab_c1.sh c1r
