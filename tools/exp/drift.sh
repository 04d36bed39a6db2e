#!/bin/bash
# Launch-time drift of the headline kernel after idle: per-launch kernel trace
# and a GRBM_GUI_ACTIVE pass (effective shader clock per dispatch), for the
# fused kernel and the sample-only kernel.  Usage: tools/exp/drift.sh <tag>
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
out=$root/gpurun_out/${1:-drift}
mkdir -p "$out"
cd "$root"
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$out/driver.json" 2> "$out/driver.err"
cd /tmp && export TMPDIR=/tmp
for mode in fused sample; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/tr_$mode" -o t -- \
      python "$root/bench.py" --steps 300 --warmup 0 --no-cpu-baseline --mode $mode > "$out/tr_$mode.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$out/pmc_$mode" -o p -- \
      python "$root/bench.py" --steps 120 --warmup 0 --no-cpu-baseline --mode $mode > "$out/pmc_$mode.log" 2>&1
  python "$root/tools/drift.py" "$out/tr_$mode" --pmc "$out/pmc_$mode" --first 80 > "$out/drift_$mode.txt"
done
