set -eo pipefail
B=$PWD/tfg---quantum-byzantine-agreement_amd/_build
o=gpurun_out/r4dc2; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gpu_suite.txt 2>&1
ROUNDS=2 EXPDIR=$B/exp_dc11 timeout -k 10 400 bash tools/exp/ab.sh r4dc2/ab
ROUNDS=3 EXPDIR=$B/exp_dc11 timeout -k 10 400 bash tools/exp/ab_c1.sh r4dc2/c1
for r in 1 2; do for so in $B/exp_dc7/*.so; do
  n=$(basename $so .so)
  QBA_LIB=$so timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $o/c3_$n.$r.json 2> $o/c3_$n.$r.err
  python -c "import json; d=json.load(open('$o/c3_$n.$r.json')); print('$n pass $r', d['ms_per_step'], d['value'])" | tee -a $o/c3_summary.txt
done; done
