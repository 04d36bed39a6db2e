#!/bin/bash
# Occupancy (896 threads at 7 waves/SIMD, 640 threads), late-drain (with and
# without a 6-wave register cap) and compile-time queue variants of the fused
# kernel vs the shipped one; parity of every variant first.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd $root
mkdir -p gpurun_out/r3k
for so in p1_drainhi p2_drainlo; do
  QBA_LIB=$root/tfg---quantum-byzantine-agreement_amd/_build/exp/$so.so timeout -k 10 200 python -u tools/exp/parity11.py > gpurun_out/r3k/parity_$so.txt 2>&1
done
ROUNDS=2 bash tools/exp/ab.sh r3k/ab6
