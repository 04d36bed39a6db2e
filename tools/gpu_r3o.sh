#!/bin/bash
# Deferred-reduction parts (4 reduce workgroups per bin row) on the wide
# small-launch path: deferred parity tests and configs[1].
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3o; mkdir -p $out
cd $root
timeout -k 10 300 python -u -m pytest tests/test_gpu_deferred.py -x -q --timeout 120 --timeout-method thread \
    > $out/deferred_tests.txt 2>&1
timeout -k 10 300 python -u bench.py --config 1 --no-cpu-baseline > $out/bench_config1.json 2> $out/bench_config1.err
