set -eo pipefail
mkdir -p gpurun_out/ab1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1/pytest.log 2>&1
bash tools/exp/ab.sh ab1
