#!/bin/bash
# Round 4: configs[1] -- deferred kernel workgroup size / pairwise sweep.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r4l; mkdir -p $out
cd $root
EXPDIR=$root/tfg---quantum-byzantine-agreement_amd/_build/exp ROUNDS=3 bash tools/exp/ab_c1.sh r4l/c1
