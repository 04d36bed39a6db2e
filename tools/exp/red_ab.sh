#!/bin/bash
# qba_k_reduce variants at the headline size: per build, the reduce kernel's
# average duration over a 50-step bench run (rocprofv3 kernel stats).
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
out=$root/gpurun_out/${1:-red_ab}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for so in ${EXPDIR}/*.so; do
    n=$(basename $so .so)
    QBA_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$n.$r -o k -- \
      python $root/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $out/$n.$r.json 2> $out/$n.$r.err
    python - "$out/$n.$r/k_kernel_stats.csv" "$n" "$r" "$out/$n.$r.json" <<'PY' | tee -a $out/summary.txt
import csv, json, sys
rows = {r['Name'].split('(')[0].replace('void ', ''): r for r in csv.DictReader(open(sys.argv[1]))}
red = [v for k, v in rows.items() if k.startswith('qba_k_reduce')][0]
lst = [v for k, v in rows.items() if k.startswith('qba_k_lists')][0]
d = json.load(open(sys.argv[4]))
print('%-10s pass %s  reduce %.2f us  list %.1f us  ms/step %.4f' % (sys.argv[2], sys.argv[3], float(red['AverageNs']) / 1e3, float(lst['AverageNs']) / 1e3, d['ms_per_step']))
PY
  done
done
