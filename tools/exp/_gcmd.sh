set -eo pipefail
out=gpurun_out/ab23; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/b_fused2.so timeout -k 10 120 python tools/exp/parity11.py > $out/parity_b_fused2.txt 2>&1
ROUNDS=2 timeout -k 10 600 bash tools/exp/ab_c1.sh ab23c1
