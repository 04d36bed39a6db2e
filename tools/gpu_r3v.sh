#!/bin/bash
# Two more samples of the driver's command on a fresh box (box-to-box spread of
# the shipped build), after the GPU suite as the driver runs it.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3v; mkdir -p $out
cd $root
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_suite.txt 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver_$i.json 2> $out/bench_driver_$i.err
done
