#!/bin/bash
# rocprofv3 kernel-trace stats (CSV) of bench.py + the PMC passes of tools/pmc.sh.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=${1:-prof}; shift || true
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o bench -- \
    python "$root/bench.py" --no-cpu-baseline "$@" > "$out/trace.log" 2>&1
bash "$root/tools/pmc.sh" "gpurun_out/$tag/pmc" "$@"
python "$root/tools/pmc_summary.py" "$out/pmc" > "$out/pmc_summary.txt"
