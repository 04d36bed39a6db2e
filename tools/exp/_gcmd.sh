set -eo pipefail
out=gpurun_out/r2d; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err
