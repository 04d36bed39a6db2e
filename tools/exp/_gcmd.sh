set -eo pipefail
out=gpurun_out/pre; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/b_pre.so timeout -k 10 200 python tools/exp/parity11.py > $out/parity_b_pre.txt 2>&1
ROUNDS=2 timeout -k 10 600 bash tools/exp/ab_c1.sh pre
ROUNDS=1 timeout -k 10 600 bash tools/exp/ab.sh pre_h
