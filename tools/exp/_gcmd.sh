set -eo pipefail
timeout -k 10 900 bash tools/exp/drift.sh drift_final
