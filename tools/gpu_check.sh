#!/bin/bash
# One GPU call: parity tests, smoke, the headline bench and the other configs,
# rocprofv3 kernel-trace stats.  Every GPU step has its own time limit; the
# chain stops at the first failure.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=$root/gpurun_out/${1:-run}
mkdir -p "$out"
cd "$root"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
if [ -n "$CONFIGS" ]; then
  for c in 0 1 3 4; do
    timeout -k 10 300 python -u bench.py --config $c > "$out/bench_config$c.json" 2> "$out/bench_config$c.err"
  done
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o bench -- python "$root/bench.py" --no-cpu-baseline > "$out/prof.log" 2>&1
