set -e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/split -o s -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --mode split > $GRAFT_REPO_ROOT/gpurun_out/split/log.txt 2>&1
