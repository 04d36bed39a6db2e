#!/bin/bash
# Occupancy probe for LDS-hungry counting layouts: the shipped kernel vs the
# same kernel forced to one workgroup per CU (768 and 1024 threads).
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd $root
ROUNDS=2 bash tools/exp/ab.sh r3k/ab2
