#!/bin/bash
# Round 4: the tail-deferred pair-bin step -- deferred / packed parity, then
# the driver's command with the deferred step and with the synchronous step
# (QBA_BENCH_DEFER=0), interleaved, and a kernel trace of the deferred form.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/r4n; mkdir -p $out
cd $root
timeout -k 10 400 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_packed.py tests/test_bench.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/tests.txt 2>&1
for r in 1 2 3; do
  for d in 1 0; do
    QBA_BENCH_DEFER=$d timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_defer${d}_$r.json 2> $out/bench_defer${d}_$r.err
    python -c "import json; d=json.load(open('$out/bench_defer${d}_$r.json')); print('defer=$d run $r', d['ms_per_step'], d['verification'].get('counts_equal_golden'))" >> $out/summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench -- \
    python $root/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/trace_bench.json 2> $out/trace.log
python $root/tools/trace_check.py $out/trace $out/trace_bench.json > $out/trace_check.txt
