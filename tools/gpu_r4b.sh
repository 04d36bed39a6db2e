#!/bin/bash
# Round 4: pair-bin counting first pass -- parity of the packed / kernel
# tests (incl. the forced-wrap recount), the driver's bench command, and the
# A/B of the shipped round-3 list kernel (a_ship) against the pair bins (b_pb).
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r4b; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
    > $out/tests.txt 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
ROUNDS=2 bash tools/exp/ab.sh r4b/ab
