#!/usr/bin/env python3
"""Summarise one build of tools/exp/ab.sh: cycles and counters per dispatch of
the list kernel (PMC pass) and its launch times (kernel trace)."""
import csv
import statistics as st
import sys
from pathlib import Path

base, name = Path(sys.argv[1]), sys.argv[2]
K = "qba_k_lists"
entries = float(sys.argv[3]) if len(sys.argv) > 3 else 1.25e8
by = {}
for f in Path(str(base) + ".pmc").rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if K in r["Kernel_Name"]:
            by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
d = [by[k] for k in sorted(by)][3:]  # skip the first launches
med = lambda c: st.median(x[c] for x in d) if d else float("nan")  # noqa: E731
cyc = med("GRBM_GUI_ACTIVE") / 8
valu = med("SQ_INSTS_VALU") * 64 / entries
lds = med("SQ_INSTS_LDS") * 64 / entries
conf = med("SQ_LDS_BANK_CONFLICT") / max(med("SQ_LDS_IDX_ACTIVE"), 1)
ldsbusy = med("SQ_LDS_IDX_ACTIVE") / 256 / cyc
L = []
for f in Path(str(base) + ".tr").rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        if K in r["Kernel_Name"]:
            L.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
L.sort()
us = [(e - s) / 1e3 for s, e in L]
win = st.mean(us[5:25]) if len(us) >= 25 else float("nan")
steady = st.mean(us[200:300]) if len(us) >= 300 else float("nan")
# step = start to start of consecutive list kernels: the kernel, the reduce
# launch and the dispatch gaps between them
step = [(L[i + 1][0] - L[i][0]) / 1e3 for i in range(len(L) - 1)]
swin = st.mean(step[5:24]) if len(step) >= 25 else float("nan")
ssteady = st.mean(step[200:299]) if len(step) >= 299 else float("nan")
print(f"{name:24s} cycles/launch {cyc:9.0f}  VALU/entry {valu:6.1f}  LDS-instr/entry {lds:5.2f}  "
      f"LDS busy {ldsbusy:4.2f} conflicts {conf:4.2f}  |  us: window {win:6.1f}  steady {steady:6.1f}"
      f"  | step: window {swin:6.1f}  steady {ssteady:6.1f}")
