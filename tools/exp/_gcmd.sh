set -eo pipefail
out=gpurun_out/c1g; mkdir -p $out
E=$PWD/tfg---quantum-byzantine-agreement_amd/_build/exp
run() {  # name so grid
  QBA_LIB=$E/$2.so QBA_EXP_GRID=$3 timeout -k 10 120 python bench.py --config 1 --steps 200 --warmup 50 --no-cpu-baseline > $out/$1.json 2>/dev/null
  python -c "import json; d=json.load(open('$out/$1.json')); print('%-16s %.2f us/step' % ('$1', d['ms_per_step']*1e3))" | tee -a $out/summary.txt
}
for r in 1 2; do
run base.$r a_base ""
run wide_il256.$r b_wide_il 256
run wide_il512.$r b_wide_il 512
run nar_il256.$r c_nar_il 256
run nar_il512.$r c_nar_il 512
done
