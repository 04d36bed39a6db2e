#!/bin/bash
# The 8-wave build (1024-thread list workgroups, pairwise closed sampler,
# SGPR-lean stores/keys): whole GPU suite, smoke, driver's bench command,
# configs[1] and [3], and an A/B against the 768-thread build (c_ship).
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3l; mkdir -p $out
cd $root
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/gpu_suite.txt 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err
timeout -k 10 300 python -u bench.py --config 1 --no-cpu-baseline > $out/bench_config1.json 2> $out/bench_config1.err
timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline > $out/bench_config3.json 2> $out/bench_config3.err
ROUNDS=2 bash tools/exp/ab.sh r3l/ab
