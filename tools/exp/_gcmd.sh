set -eo pipefail
out=gpurun_out/inv; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "invalid or gather" > $out/pytest.log 2>&1
