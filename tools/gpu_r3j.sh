#!/bin/bash
# A/B of the headline list kernel before / after the body refactor
# (tools/exp/ab.sh: a_old = HEAD~ sources, b_new = this tree).
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd $root
ROUNDS=2 bash tools/exp/ab.sh r3j/ab
