#!/bin/bash
# SQ counter passes of bench.py for every experiment build (GPU box):
# tools/exp/pmc_exp.sh -> gpurun_out/exp_pmc/<build>/summary.txt
set -e
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for so in $root/tfg---quantum-byzantine-agreement_amd/_build/exp/*.so; do
  name=$(basename $so .so)
  out=$root/gpurun_out/exp_pmc/$name; mkdir -p $out
  i=0
  for grp in \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS_ATOMIC" \
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
    "SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    QBA_LIB=$so timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $out/p$i -o pmc -- \
        python $root/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/p$i.log 2>&1
  done
  python $root/tools/pmc_summary.py $out | grep -A30 "qba_k_lists<11, 1" | head -26 > $out/summary.txt
done
