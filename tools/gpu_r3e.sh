#!/bin/bash
# round 3: GPU suite, configs[1] (overlapped reduction), protocol profiles
set -eo pipefail
out=gpurun_out/r3e; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u bench.py --config 1 > $out/bench_config1.json 2> $out/bench_config1.err
timeout -k 10 200 python -u tools/prof_protocol.py 11 1e6 3 3 > $out/prof_protocol.txt 2>&1
timeout -k 10 200 python -u tools/prof_config0.py > $out/prof_config0.txt 2>&1
