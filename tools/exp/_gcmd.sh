set -eo pipefail
mkdir -p gpurun_out/p1
timeout -k 10 600 python -u -m pytest tests/test_protocol.py tests/test_countmode.py tests/test_mpi.py tests/test_gpu_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/p1/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --config 0 --steps 20 > gpurun_out/p1/config0.json 2> gpurun_out/p1/config0.err
