set -eo pipefail
out=gpurun_out/r2h; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
timeout -k 10 300 python -u bench.py --config 1 > $out/bench_config1.json 2> $out/bench_config1.err
timeout -k 10 300 python -u bench.py --config 3 > $out/bench_config3.json 2> $out/bench_config3.err
