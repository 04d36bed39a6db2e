#!/bin/bash
# configs[1] (n=11, 1e6 entries, K steps in one hipGraph) for every experiment
# build, ROUNDS interleaved passes, plus the per-kernel trace of one pass.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
out=$root/gpurun_out/${1:-ab_c1}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for so in ${EXPDIR:-$root/tfg---quantum-byzantine-agreement_amd/_build/exp}/*.so; do
    name=$(basename $so .so)
    QBA_LIB=$so timeout -k 10 120 python $root/bench.py --config 1 --steps 200 --warmup 50 --no-cpu-baseline > $out/$name.$r.json 2> $out/$name.$r.err
    python -c "import json; d=json.load(open('$out/$name.$r.json')); print('%-12s pass %d  %.2f us/step' % ('$name', $r, d['ms_per_step']*1e3))" | tee -a $out/summary.txt
  done
done
for so in ${EXPDIR:-$root/tfg---quantum-byzantine-agreement_amd/_build/exp}/*.so; do
  name=$(basename $so .so)
  QBA_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$name.prof -o k -- \
     python $root/bench.py --config 1 --steps 200 --warmup 50 --no-cpu-baseline > $out/$name.prof.log 2>&1
  python - "$out/$name.prof/k_kernel_stats.csv" "$name" <<'PY' | tee -a $out/summary.txt
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'qba_k' in r['Name']]
print(sys.argv[2], '  '.join('%s %s x %.2f us' % (r['Name'].split('(')[0].replace('void ', ''), r['Calls'], float(r['AverageNs']) / 1e3) for r in rows))
PY
done
