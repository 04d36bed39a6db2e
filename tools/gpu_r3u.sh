#!/bin/bash
# Slab-reduce tuning at the headline's 512 slab rows: rows per reduce
# workgroup 32 (shipped) / 16, and all rows in flight; mean qba_k_reduce and
# list-kernel time over launches 5-299 of a 300-launch trace, two passes.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3u2; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for so in $root/tfg---quantum-byzantine-agreement_amd/_build/exp/*.so; do
    name=$(basename $so .so)
    QBA_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/$name.$r -o t -- \
        python $root/bench.py --no-cpu-baseline --steps 300 --warmup 0 > $out/$name.$r.log 2>&1
    python - "$out/$name.$r" "$name" <<'PY' | tee -a $out/summary.txt
import csv, sys, statistics as st
from pathlib import Path
rows = []
for f in Path(sys.argv[1]).rglob("*kernel_trace.csv"):
    rows += list(csv.DictReader(open(f)))
def mean(k):
    L = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if k in r["Kernel_Name"])
    return st.mean((e - s) / 1e3 for s, e in L[5:300])
print("%-12s reduce %.2f us   list %.1f us" % (sys.argv[2], mean("qba_k_reduce"), mean("qba_k_lists")))
PY
  done
done
