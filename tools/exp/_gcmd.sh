set -eo pipefail
out=gpurun_out/ab25; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/b_640.so timeout -k 10 120 python tools/exp/parity11.py > $out/parity_b_640.txt 2>&1
QBA_LIB=$E/c_512.so timeout -k 10 120 python tools/exp/parity11.py > $out/parity_c_512.txt 2>&1
ROUNDS=2 timeout -k 10 1100 bash tools/exp/ab.sh ab25
