set -eo pipefail
out=gpurun_out/ab21; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
QBA_LIB=$E/b_fused.so timeout -k 10 120 python tools/exp/parity11.py > $out/parity_b_fused.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
ROUNDS=2 timeout -k 10 900 bash tools/exp/ab_c1.sh ab21c1
ROUNDS=1 timeout -k 10 600 bash tools/exp/ab.sh ab21
