#!/bin/bash
# Round 3: nibble-row lists.  Parity (packed tests, then the whole GPU suite),
# then the layouts A/B on the shipped build: per layout one PMC pass (cycles,
# VALU, LDS per dispatch) and one 300-launch kernel trace (driver window =
# launches 5-24, steady = 200-299), two interleaved rounds; configs[1] both
# layouts.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3g; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py -x -v --timeout 120 --timeout-method thread \
    > $out/packed_tests.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gpu_suite.txt 2>&1
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for lay in packed bytes; do
    timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
        SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv \
        -d $out/$lay.$r.pmc -o p -- python $root/bench.py --no-cpu-baseline --steps 30 --warmup 0 --layout $lay \
        > $out/$lay.$r.pmc.log 2>&1
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/$lay.$r.tr -o t -- \
        python $root/bench.py --no-cpu-baseline --steps 300 --warmup 0 --layout $lay > $out/$lay.$r.tr.log 2>&1
    python $root/tools/exp/ab.py $out/$lay.$r $lay | tee -a $out/summary.txt
  done
done
for lay in packed bytes; do
  timeout -k 10 200 python $root/bench.py --no-cpu-baseline --layout $lay > $out/bench_$lay.json 2> $out/bench_$lay.err
  timeout -k 10 200 python $root/bench.py --config 1 --steps 200 --warmup 5 --no-cpu-baseline --layout $lay \
      > $out/c1_$lay.json 2> $out/c1_$lay.err
done
