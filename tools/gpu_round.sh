#!/bin/bash
# One GPU call, steps chosen on the command line (run in the order given):
#   tools/gpu_round.sh <tag> [steps...]
#     tests   pytest -m gpu (whole GPU suite)       smoke   __graft_entry__.smoke()
#     bench   the driver's command (N=1, --steps 20 --warmup 5), twice
#     long    bench.py defaults (50 + 200 launches)  c0 c1 c3 c4   bench.py --config k
#     prof    rocprofv3 --kernel-trace --stats of the driver's command (+ tools/trace_check.py)
#     profc1  the same for --config 1        profc3  ... for --config 3
#     pmc     tools/pmc.sh passes of the headline + tools/pmc_traffic.py -> pmc/traffic.json
#     pmcset  copy that file to profiles/traffic_n11.json (later bench steps report its traffic)
#     ab      tools/exp/ab.sh over the experiment builds in _build/exp (ROUNDS=2)
#     cli     the count-mode CLI at sizeL = 1e9 in a fresh process
# Default: tests smoke bench prof.  Every GPU step has its own time limit; the
# chain stops at the first failure (set -e), so nothing runs after a fault.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
tag=${1:-round}; shift || true
steps=${*:-tests smoke bench prof}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd "$root"
export TMPDIR=/tmp
for s in $steps; do
  echo "== $s $(date +%T)"
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             > "$out/pytest.log" 2>&1; tail -3 "$out/pytest.log" ;;
    smoke) timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 ;;
    bench) for i in 1 2; do
             timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench_driver$i.json" \
               2> "$out/bench_driver$i.err"; done ;;
    long) timeout -k 10 300 python -u bench.py > "$out/bench_long.json" 2> "$out/bench_long.err" ;;
    c0|c1|c3|c4) timeout -k 10 400 python -u bench.py --config ${s#c} > "$out/bench_config${s#c}.json" \
                   2> "$out/bench_config${s#c}.err" ;;
    prof) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o bench \
             -- python "$root/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$out/prof_bench.json" \
             2> "$out/prof.log")
          python tools/trace_check.py "$out/prof" "$out/prof_bench.json" > "$out/trace_check.txt" ;;
    profc1) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_c1" \
               -o bench -- python "$root/bench.py" --config 1 --steps 200 --no-cpu-baseline > "$out/prof_c1.log" 2>&1) ;;
    profc3) (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_c3" \
               -o bench -- python "$root/bench.py" --config 3 --no-cpu-baseline > "$out/prof_c3.log" 2>&1) ;;
    pmc) timeout -k 10 600 bash tools/pmc.sh "gpurun_out/$tag/pmc"
         python tools/pmc_traffic.py "$out/pmc" 125000000 11 > "$out/pmc/traffic.json"
         python tools/pmc_summary.py "$out/pmc" > "$out/pmc/summary.txt" ;;
    pmcset) cp "$out/pmc/traffic.json" profiles/traffic_n11.json ;;  # the box's bench steps then report it
    ab) ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash tools/exp/ab.sh "$tag/ab" ;;
    cli) timeout -k 10 300 python -u -m tfg---quantum-byzantine-agreement_amd.tfg 1e9 3 --parties 11 --mode count \
           --seed 11 --timing > "$out/cli_count_1e9.txt" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
