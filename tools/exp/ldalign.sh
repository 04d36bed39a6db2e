#!/bin/bash
# (historical) row-stride alignment sweep used to pick Engine.alloc_lists' 4 KiB
# row alignment; alloc_lists now fixes it, so this reruns the default only.
cd ${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/ld.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ld.json')); print('pass $r %.3e launch %.4f' % (d['value'], d['roofline']['launch_ms']))"
done
