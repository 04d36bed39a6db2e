set -eo pipefail
mkdir -p gpurun_out/dab
export TMPDIR=/tmp
for r in 1 2 3 4; do for d in 0 1; do
  QBA_BENCH_DEFER=$d timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/dab/d$d.$r.json 2> gpurun_out/dab/d$d.$r.err
  python -c "import json;d=json.loads(open('gpurun_out/dab/d$d.$r.json').read().strip().splitlines()[-1]);print('defer=$d run $r',d['ms_per_step'])"
done; done
for d in 0 1; do
  (cd /tmp && QBA_BENCH_DEFER=$d timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dab/tr$d -o t -- python $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 300 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/dab/tr$d.log 2>&1)
done
