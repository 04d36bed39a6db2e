set -eo pipefail
out=gpurun_out/b3; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ -k "batch or check_gather or exact or packet" > $out/pytest.log 2>&1
E=tfg---quantum-byzantine-agreement_amd/_build/exp
for so in a_head7 b_new7 b_new7 a_head7; do
QBA_LIB=$PWD/$E/$so.so timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $out/c3_$so.json 2>/dev/null
python -c "import json; d=json.load(open('$out/c3_$so.json')); print('config3 %-8s %.1f us/step  %.3g entries/s' % ('$so', d['ms_per_step']*1e3, d['value']))" | tee -a $out/summary.txt
done
