#!/bin/bash
# Round 4: pair-bin flush with wave-reduced lane totals -- small-launch cost
# against classic counting, and configs[1].
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r4e; mkdir -p $out
cd $root
for so in tfg---quantum-byzantine-agreement_amd/_build/exp/*.so; do
  name=$(basename $so .so)
  for c in 1e6 1e7 1.25e8; do
    QBA_LIB=$so timeout -k 10 120 python -u tools/exp/pb_small.py $c 100 > $out/small_${name}_$c.txt 2>&1
    echo "$name $(tail -1 $out/small_${name}_$c.txt)" >> $out/small_summary.txt
  done
done
EXPDIR=$root/tfg---quantum-byzantine-agreement_amd/_build/exp ROUNDS=2 bash tools/exp/ab_c1.sh r4e/c1
