set -eo pipefail
out=gpurun_out/cg; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "check_gather or exact or packet" > $out/pytest.log 2>&1
