set -eo pipefail
out=gpurun_out/ab24; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/b_r16.so timeout -k 10 120 python tools/exp/parity11.py > $out/parity_b_r16.txt 2>&1
ROUNDS=3 timeout -k 10 900 bash tools/exp/ab_c1.sh ab24c1
