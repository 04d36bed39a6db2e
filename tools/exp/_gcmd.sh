set -eo pipefail
out=gpurun_out/r2d; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
bash tools/gpu_prof_round.sh r2d
timeout -k 10 200 python -u bench.py --mode sample --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_sample.json 2> $out/bench_sample.err
timeout -k 10 200 python -u bench.py --mode split --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_split.json 2> $out/bench_split.err
timeout -k 10 200 python -u bench.py --steps 200 --warmup 50 --no-cpu-baseline > $out/bench_steady.json 2> $out/bench_steady.err
timeout -k 10 200 python -u bench.py --config 1 > $out/bench_config1.json 2> $out/bench_config1.err
timeout -k 10 200 python -u bench.py --config 0 > $out/bench_config0.json 2> $out/bench_config0.err
