set -eo pipefail
out=gpurun_out/c0b; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_protocol.py tests/test_countmode.py tests/test_mpi.py tests/test_integration.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u tools/prof_config0.py > $out/prof_config0.txt 2>&1
timeout -k 10 300 python -u bench.py --config 0 --steps 50 > $out/config0.json 2> $out/config0.err
