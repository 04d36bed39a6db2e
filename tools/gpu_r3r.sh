#!/bin/bash
# 2-rank rehearsal of `python bench.py --gpus 2` (the self-launching form the
# driver's SCALE run uses) on a one-GPU box: the ranks share device 0 and
# reduce over gloo; checks the launch, barrier, max-over-ranks timing and the
# single JSON line (the number is not a measurement).
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r3r; mkdir -p $out
cd $root
QBA_SHARE_DEVICE=1 QBA_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 \
  --per-gpu 2.5e7 > $out/bench_world2.json 2> $out/bench_world2.err
