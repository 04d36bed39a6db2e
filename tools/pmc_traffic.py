#!/usr/bin/env python3
"""profiles/traffic_n11.json from a tools/pmc.sh run: HBM bytes per launch of
the fused list kernel (median over dispatches), from the FETCH_SIZE and
WRITE_SIZE passes (rocprofv3 reports both in KiB).

gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts 64 B per
128-B request of a wide streaming read, so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane stores and is calibrated here for the kernel's 4-B-per-lane
row stores against the known list bytes written per launch ((n+1) B/entry).

    python tools/pmc_traffic.py <pmc dir> <entries per launch> <n> [mode] [layout]

layout "packed" (default: bench.py's default) writes (n+1)/2 B/entry, "bytes" (n+1).
"""
import csv
import hashlib
import json
import os
import statistics
import sys
from pathlib import Path

root, per, n = Path(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
mode = sys.argv[4] if len(sys.argv) > 4 else "fused"
layout = sys.argv[5] if len(sys.argv) > 5 else "packed"
vals = {}
for f in root.glob("p*/**/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        # the synchronous step's list kernel, or the deferred step's (bench.py's
        # default: the previous step's reduction in its tail)
        if r["Kernel_Name"].startswith((f"void qba_k_lists<{n}, 1", f"void qba_k_lists_pbdef<{n},")):
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
fetch = statistics.median(vals["FETCH_SIZE"]) * 1024 * 2
# the issue side of the same kernel (the other tools/pmc.sh passes): per-launch
# medians, summed over the chip; bench.py turns them into roofline.issue
ISSUE = ("GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_LDS_ATOMIC", "SQ_INSTS_SALU",
         "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
         "SQ_INSTS_VMEM_WR", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_INT32", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
         "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA",
         "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_BRANCH")
issue = {c: statistics.median(vals[c]) for c in ISSUE if c in vals}
write = statistics.median(vals["WRITE_SIZE"]) * 1024
known = (n + 1) * per // (2 if layout == "packed" else 1)
out = {"n": n, "per_launch_entries": per, "mode": mode, "layout": layout,
       "hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
       "write_calibration": {"known_list_bytes": known, "write_over_known": write / known},
       "algorithmic_bytes_per_launch": known,  # the lists written once (bench.py roofline.achieved)
       "metric_scale_bytes_per_launch": 2 * (n + 1) * per,  # BASELINE's 2(n+1) B per entry convention
       "source": str(root), "kernel": f"qba_k_lists<{n},1,*> / qba_k_lists_pbdef<{n},*>",
       "issue_counters_per_launch": issue,
       # the library the counters were read from: bench.py drops the figure for any other build
       "libqba_sha16": hashlib.sha256(open(os.environ.get("QBA_LIB", Path(__file__).resolve().parent.parent
                                                         / "tfg---quantum-byzantine-agreement_amd" / "_build"
                                                         / "libqba.so"), "rb").read()).hexdigest()[:16]}
print(json.dumps(out, indent=1))
