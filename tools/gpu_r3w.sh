#!/bin/bash
# Round 3 final pass on one GPU: parity (packed tests incl. batched, the whole
# GPU suite, smoke), configs[3] in both layouts, then the round profile
# (tools/gpu_prof_round.sh: driver-command kernel trace + trace check, PMC
# passes -> traffic json of this build, the driver's bench line, count-mode
# CLI at sizeL = 1e9) and the other configs' lines.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3w; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_hostcalls.py tests/test_gpu_deferred.py -x -v --timeout 120 --timeout-method thread \
    > $out/packed_tests.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gpu_suite.txt 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
for lay in packed bytes; do
  timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline --layout $lay > $out/c3_$lay.json 2> $out/c3_$lay.err
done
bash tools/gpu_prof_round.sh r3w/prof
timeout -k 10 300 python -u tools/prof_config0.py > $out/prof_config0.txt 2>&1
for c in 0 1 4; do
  timeout -k 10 300 python -u bench.py --config $c > $out/bench_config$c.json 2> $out/bench_config$c.err
done
