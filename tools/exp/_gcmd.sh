set -eo pipefail
out=gpurun_out/ev; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
r=0; for m in step loop loop step; do r=$((r+1));
QBA_BENCH_EVENTS=$m timeout -k 10 120 python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/b_$m.$r.json 2>/dev/null
python -c "import json; d=json.load(open('$GRAFT_REPO_ROOT/$out/b_$m.$r.json')); print('events=$m pass $r: %.1f us/step launch %.1f' % (d['ms_per_step']*1e3, d['roofline']['launch_ms']*1e3))" | tee -a $GRAFT_REPO_ROOT/$out/summary.txt
done
QBA_BENCH_EVENTS=loop timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/trace -o b -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/trace.log 2>&1
