#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=$root/gpurun_out/${1:-run}
mkdir -p "$out"
cd "$root"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o bench -- python "$root/bench.py" --no-cpu-baseline > "$out/prof.log" 2>&1
