#!/bin/bash
# One GPU call: parity tests, smoke, the headline bench, configs[1], and the
# rocprofv3 kernel-trace stats of both bench commands.  Every GPU step has its
# own time limit; the chain stops at the first failure.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=$root/gpurun_out/${1:-round}
mkdir -p "$out"
cd "$root"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 python -u bench.py --config 1 --steps 200 > "$out/bench_config1.json" 2> "$out/bench_config1.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o bench -- python "$root/bench.py" --no-cpu-baseline > "$out/prof.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_c1" -o bench -- python "$root/bench.py" --config 1 --steps 200 --no-cpu-baseline > "$out/prof_c1.log" 2>&1
