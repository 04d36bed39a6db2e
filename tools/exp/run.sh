#!/bin/bash
# Time bench.py (n = 11 fused step) with every experiment build (GPU box),
# ROUNDS interleaved passes over the builds (default 3) to expose run-to-run noise.
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
out=$root/gpurun_out/exp; mkdir -p $out
for r in $(seq 1 ${ROUNDS:-3}); do
  for so in $root/tfg---quantum-byzantine-agreement_amd/_build/exp/*.so; do
    name=$(basename $so .so)
    QBA_LIB=$so timeout -k 10 120 python $root/bench.py --no-cpu-baseline --steps 40 > $out/$name.$r.json 2> $out/$name.$r.err || exit 1
    python -c "import json,sys; d=json.load(open('$out/$name.$r.json')); print('%-22s pass %d  %.3e entries/s  launch %.4f ms' % ('$name', $r, d['value'], d['roofline']['launch_ms']))"
  done
done
