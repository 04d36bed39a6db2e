set -eo pipefail
out=gpurun_out/ab16; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
for b in a_new g_isq; do
  QBA_LIB=$E/$b.so timeout -k 10 200 python tools/exp/parity11.py > $out/parity_$b.txt 2>&1
done
ROUNDS=2 timeout -k 10 900 bash tools/exp/ab.sh ab16
