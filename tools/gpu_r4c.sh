#!/bin/bash
# Round 4: exact-mode device rows (protocol GPU tests + the n=11 / 1e6 run
# profile) and the configs[1] A/B of the deferred kernel variants.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r4c; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_protocol.py tests/test_gpu_deferred.py tests/test_gpu_packed.py tests/test_gpu_kernels.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > $out/protocol_tests.txt 2>&1
timeout -k 10 300 python -u tools/prof_protocol.py 11 1e6 3 5 > $out/protocol_1e6_device_rows.txt 2>&1
EXPDIR=$root/tfg---quantum-byzantine-agreement_amd/_build/exp_c1 ROUNDS=2 bash tools/exp/ab_c1.sh r4c/c1
EXPDIR=$root/tfg---quantum-byzantine-agreement_amd/_build/exp ROUNDS=2 bash tools/exp/ab.sh r4c/ab
