set -eo pipefail
out=gpurun_out/sv; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "statevector or ghz or program" > $out/pytest_sv.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_workloads.py -k "register or circuit or resource" > $out/pytest_sv_workloads.log 2>&1
timeout -k 10 300 python -u bench.py --config 4 > $out/bench_config4.json 2> $out/bench_config4.err
