#!/bin/bash
# Round 4: small-launch cost of the pair-bin kernel (synchronous 1e6 passes),
# and the main-kernel A/B of classic counting vs pair bins with the trims.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r4d; mkdir -p $out
cd $root
for so in tfg---quantum-byzantine-agreement_amd/_build/exp/*.so; do
  name=$(basename $so .so)
  for c in 1e6 1.25e8; do
    QBA_LIB=$so timeout -k 10 120 python -u tools/exp/pb_small.py $c 100 > $out/small_${name}_$c.txt 2>&1
    echo "$name $(tail -1 $out/small_${name}_$c.txt)" >> $out/small_summary.txt
  done
done
EXPDIR=$root/tfg---quantum-byzantine-agreement_amd/_build/exp ROUNDS=2 bash tools/exp/ab.sh r4d/ab
EXPDIR=$root/tfg---quantum-byzantine-agreement_amd/_build/exp ROUNDS=2 bash tools/exp/ab_c1.sh r4d/c1
