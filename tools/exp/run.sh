#!/bin/bash
# Time bench.py (n = 11 fused step) with every experiment build (GPU box).
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
out=$root/gpurun_out/exp; mkdir -p $out
for so in $root/tfg---quantum-byzantine-agreement_amd/_build/exp/*.so; do
  name=$(basename $so .so)
  QBA_LIB=$so timeout -k 10 120 python $root/bench.py --no-cpu-baseline --steps 20 > $out/$name.json 2> $out/$name.err || exit 1
  python -c "import json,sys; d=json.load(open('$out/$name.json')); print('%-12s %.3e entries/s  kernel %.3f ms' % ('$name', d['value'], d['roofline']['launch_ms']))"
done
