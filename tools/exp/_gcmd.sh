set -eo pipefail
bash tools/rehearse_world2.sh
