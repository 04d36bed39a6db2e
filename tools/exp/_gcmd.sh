set -eo pipefail
out=gpurun_out/c1t; mkdir -p $out
QBA_LIB=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp/t_timing.so timeout -k 10 200 python tools/exp/c1_timing.py > $out/timing2.txt 2>&1
