set -eo pipefail
out=gpurun_out/r2b; mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --no-cpu-baseline > $out/bench_steady.json 2> $out/bench_steady.err
timeout -k 10 300 python -u bench.py --config 1 > $out/bench_config1.json 2> $out/bench_config1.err
timeout -k 10 300 python -u bench.py --config 3 > $out/bench_config3.json 2> $out/bench_config3.err
timeout -k 10 300 python -u bench.py --config 4 > $out/bench_config4.json 2> $out/bench_config4.err
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err
