set -eo pipefail
out=gpurun_out/pp; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ -k "protocol or mpi or integration or packet" > $out/pytest.log 2>&1
timeout -k 10 300 python -u tools/prof_protocol.py 11 1e6 3 3 > $out/prof_1e6.txt 2>&1
timeout -k 10 100 python -u tools/prof_config0.py > $out/prof_config0.txt 2>&1
