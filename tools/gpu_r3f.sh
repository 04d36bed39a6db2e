#!/bin/bash
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3f; mkdir -p $out
cd $root
timeout -k 10 200 python -u tools/prof_protocol.py 11 1e6 3 3 > $out/prof_protocol.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/c1trace -o t -- python $root/bench.py --config 1 --steps 50 --warmup 5 --no-cpu-baseline > $out/c1.json 2> $out/c1.err
