#!/bin/bash
# Round 4 pass on one GPU for the shipped build: the whole GPU suite, smoke,
# the driver's bench command under a rocprofv3 kernel trace (+ trace check),
# the PMC passes -> profiles/traffic_n11.json (HBM bytes and the issue
# counters bench.py turns into roofline.issue, keyed to this build), the
# driver's command itself, the other configs, the count-mode CLI at 1e9 and
# the exact-mode protocol profile.  Every GPU step has its own time limit;
# the chain stops at the first failure.
# Usage: tools/gpu_r4_final.sh <tag> [skip-suite]
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=${1:-r4f}
out=$root/gpurun_out/$tag; mkdir -p $out
cd $root
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_suite.txt 2>&1
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o bench -- \
    python $root/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $out/trace_bench.json 2> $out/trace.log
python $root/tools/trace_check.py $out/trace $out/trace_bench.json > $out/trace_check.txt
bash $root/tools/pmc.sh gpurun_out/$tag/pmc
python $root/tools/pmc_summary.py $out/pmc > $out/pmc_summary.txt
python $root/tools/pmc_traffic.py $out/pmc 125000000 11 > $out/traffic_n11.json
cp $out/traffic_n11.json $root/profiles/traffic_n11.json  # keyed to this build (bench.py checks the sha)
cd $root
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.json 2> $out/bench_driver.err
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver2.json 2> $out/bench_driver2.err
# the count-mode CLI before configs[4]: a process right after that one's 256 GiB
# teardown waits seconds for device memory (profiles/r4/micro)
timeout -k 10 300 python -u -m tfg---quantum-byzantine-agreement_amd.tfg 1e9 3 --parties 11 --mode count --seed 11 --timing > $out/cli_count_1e9.txt 2>&1
for c in 0 1 3 4; do
  timeout -k 10 300 python -u bench.py --config $c > $out/bench_config$c.json 2> $out/bench_config$c.err
done
timeout -k 10 300 python -u tools/prof_protocol.py 11 1e6 3 5 > $out/protocol_1e6.txt 2>&1
