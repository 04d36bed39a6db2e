set -eo pipefail
mkdir -p gpurun_out/wl1
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/wl1/pytest.log 2>&1
