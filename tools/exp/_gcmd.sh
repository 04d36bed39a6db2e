set -eo pipefail
out=gpurun_out/ab19; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/n_small512.so timeout -k 10 200 python tools/exp/parity11.py > $out/parity_n_small512.txt 2>&1
ROUNDS=3 timeout -k 10 600 bash tools/exp/ab_c1.sh ab19c1
