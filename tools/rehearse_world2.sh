#!/bin/bash
# Rehearsal of bench.py's N-rank path on a one-GPU box: 2 ranks under
# torch.distributed.run share device 0 and reduce over gloo.  Checks the
# launch, barrier, max-over-ranks timing and the single JSON line; the
# number it prints is not a measurement (two ranks share one GPU).
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=$root/gpurun_out/world2; mkdir -p $out
cd $root
QBA_SHARE_DEVICE=1 QBA_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  --per-gpu 2.5e7 > $out/bench.json 2> $out/bench.err
