set -eo pipefail
out=gpurun_out/w2; mkdir -p $out
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/b1.json 2> $out/b1.err
bash tools/rehearse_world2.sh
cp gpurun_out/world2/bench.json $out/world2.json; cp gpurun_out/world2/bench.err $out/world2.err
