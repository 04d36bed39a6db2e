#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py for every experiment build (GPU box),
# ROUNDS interleaved passes: per-kernel device time of each build on one box.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
out=$root/gpurun_out/exp_prof${TAG}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for so in $root/tfg---quantum-byzantine-agreement_amd/_build/exp/*.so; do
    name=$(basename $so .so)
    QBA_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$name.$r -o k -- \
      python $root/bench.py --no-cpu-baseline --steps 40 "$@" > $out/$name.$r.json 2> $out/$name.$r.err
    python - "$out/$name.$r/k_kernel_stats.csv" "$name" "$r" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'qba_k_lists' in r['Name'] or 'qba_k_reduce' in r['Name'] or 'finalize' in r['Name']]
print(sys.argv[2], 'pass', sys.argv[3], '  '.join('%s %s x %.2f us' % (r['Name'].split('(')[0].replace('void ', ''), r['Calls'], float(r['AverageNs']) / 1e3) for r in rows))
PY
  done
done
