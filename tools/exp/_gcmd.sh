set -eo pipefail
out=gpurun_out/full2; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 200 python -u tools/prof_config0.py > $out/prof_config0.txt 2>&1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err
timeout -k 10 300 python -u bench.py --config 1 --steps 200 --no-cpu-baseline > $out/bench_config1.json 2> $out/bench_config1.err
