set -eo pipefail
out=$PWD/gpurun_out/r2g; mkdir -p $out
root=$PWD
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o k -- \
    python $root/bench.py --config 4 > $out/bench_config4.json 2> $out/prof_c4.log
cd $root
bash tools/gpu_prof_round.sh r2g_prof
