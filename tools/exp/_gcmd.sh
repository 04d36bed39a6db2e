set -eo pipefail
out=gpurun_out/ab17; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/l_tweak.so timeout -k 10 200 python tools/exp/parity11.py > $out/parity_l_tweak.txt 2>&1
ROUNDS=2 timeout -k 10 900 bash tools/exp/ab.sh ab17
ROUNDS=2 timeout -k 10 600 bash tools/exp/ab_c1.sh ab17c1
