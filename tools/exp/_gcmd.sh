set -eo pipefail
out=gpurun_out/ab18; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/m_bcast.so timeout -k 10 200 python tools/exp/parity11.py > $out/parity_m_bcast.txt 2>&1
ROUNDS=2 timeout -k 10 900 bash tools/exp/ab.sh ab18
