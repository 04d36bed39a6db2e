#!/bin/bash
# configs[1] with the 1024-thread build: wide kernel (123 workgroups) vs the
# narrow kernel on a wider grid for launches below 2M entries (s_small2m);
# parity of the narrow variant first.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd $root
mkdir -p gpurun_out/r3m
QBA_LIB=$root/tfg---quantum-byzantine-agreement_amd/_build/exp/s_small2m.so timeout -k 10 200 python -u tools/exp/parity11.py > gpurun_out/r3m/parity_s_small2m.txt 2>&1
ROUNDS=2 bash tools/exp/ab_c1.sh r3m/c1
