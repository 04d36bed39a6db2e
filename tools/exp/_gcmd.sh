set -eo pipefail
out=gpurun_out/sv3; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_workloads.py -k "statevector or ghz or program or register or circuit or resource" > $out/pytest.log 2>&1
timeout -k 10 200 python bench.py --config 4 > $out/c4.json 2>/dev/null
python -c "import json; d=json.load(open('$out/c4.json')); print('cx pass %.0f GB/s (%.2f ms) prep %.1f ms' % (d['value'], d['ms_per_step'], d['register_prep_ms']))" | tee -a $out/summary.txt
