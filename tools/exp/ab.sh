#!/bin/bash
# A/B of experiment builds (tools/exp/build.sh) on the GPU box, clock-proof:
# per build one PMC pass (shader cycles per dispatch = GRBM_GUI_ACTIVE / 8,
# VALU / LDS counts) and one 300-launch kernel trace (driver window =
# launches 5-24, steady state = 200-299).  ROUNDS interleaved passes.
# Usage: tools/exp/ab.sh <tag> [bench args]
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
tag=${1:-ab}; shift || true
out=$root/gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-1}); do
  for so in ${EXPDIR:-$root/tfg---quantum-byzantine-agreement_amd/_build/exp}/*.so; do
    name=$(basename $so .so)
    QBA_LIB=$so timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
        SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv \
        -d $out/$name.$r.pmc -o p -- python $root/bench.py --no-cpu-baseline --steps 30 --warmup 0 "$@" > $out/$name.$r.pmc.log 2>&1
    QBA_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/$name.$r.tr -o t -- \
        python $root/bench.py --no-cpu-baseline --steps 300 --warmup 0 "$@" > $out/$name.$r.tr.log 2>&1
    python $root/tools/exp/ab.py $out/$name.$r $name | tee -a $out/summary.txt
    # the driver's command (window only, events around the 20 timed launches)
    QBA_LIB=$so timeout -k 10 120 python $root/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" \
        > $out/$name.$r.drv.json 2> $out/$name.$r.drv.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); \
print(f'{sys.argv[2]:24s} driver command {d[\"ms_per_step\"]*1e3:6.1f} us/step')" $out/$name.$r.drv.json $name \
        | tee -a $out/summary.txt
  done
done
