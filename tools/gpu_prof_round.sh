#!/bin/bash
# Round profile on one GPU: kernel-trace stats of the driver's bench command,
# the PMC passes (tools/pmc.sh) -> traffic json for this build, the bench line
# itself (driver's command), and the count-mode CLI at sizeL = 1e9.
# Usage: tools/gpu_prof_round.sh <tag>
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=${1:-r2}
out=$root/gpurun_out/$tag; mkdir -p $out
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
timeout -k 10 300 python -u -m tfg---quantum-byzantine-agreement_amd.tfg 1e9 3 --parties 11 --mode count --seed 11 --timing > $out/cli_count_1e9.txt 2>&1
