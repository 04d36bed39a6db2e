set -eo pipefail
o=gpurun_out/r4c1pb; mkdir -p $o
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --config 1 --steps 200 --warmup 50 --no-cpu-baseline > $o/base.$r.json 2> $o/base.$r.err
  QBA_PB_MIN_ENTRIES=0 timeout -k 10 120 python bench.py --config 1 --steps 200 --warmup 50 --no-cpu-baseline > $o/pb.$r.json 2> $o/pb.$r.err
  python -c "import json; a=json.load(open('$o/base.$r.json')); b=json.load(open('$o/pb.$r.json')); print('pass $r base %.2f us  pairbins %.2f us  verif %s %s' % (a['ms_per_step']*1e3, b['ms_per_step']*1e3, a.get('verification'), b.get('verification')))" | tee -a $o/summary.txt
done
