#!/bin/bash
# configs[3] (batched n = 7) A/B of experiment builds made with N=7 tools/exp/build.sh
# into EXPDIR (default _build/exp7): ROUNDS interleaved bench.py --config 3 runs each.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
tag=${1:-ab_c3}
out=$root/gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for so in ${EXPDIR:-$root/tfg---quantum-byzantine-agreement_amd/_build/exp7}/*.so; do
    name=$(basename $so .so)
    QBA_LIB=$so timeout -k 10 200 python $root/bench.py --config 3 --no-cpu-baseline > $out/$name.$r.json 2> $out/$name.$r.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); \
print(f'{sys.argv[2]:16s} pass {sys.argv[3]}  {d[\"ms_per_step\"]:.4f} ms/step')" $out/$name.$r.json $name $r | tee -a $out/summary.txt
  done
done
