#!/bin/bash
# PMC passes for bench.py (one rocprofv3 run per counter group, as the
# MI355X guide prescribes).  Usage: tools/pmc.sh <outdir> <bench args...>
set -e
out=$1; shift
mkdir -p "${GRAFT_REPO_ROOT:-.}/$out"
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS_ATOMIC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $root/$out/p$i -o pmc -- \
      python $root/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $root/$out/p$i.log 2>&1
done
