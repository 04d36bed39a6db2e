set -eo pipefail
out=gpurun_out/r2c; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
bash tools/gpu_prof_round.sh r2c_prof
for c in 1 3 4 0; do
  timeout -k 10 300 python -u bench.py --config $c > $out/bench_config$c.json 2> $out/bench_config$c.err
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --no-cpu-baseline > $out/bench_steady.json 2> $out/bench_steady.err
timeout -k 10 300 python -u bench.py --mode sample --steps 200 --warmup 50 --no-cpu-baseline > $out/bench_sample.json 2> $out/bench_sample.err
