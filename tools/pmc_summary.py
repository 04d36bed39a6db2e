#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per kernel, counter values per dispatch (median)."""
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
vals = defaultdict(lambda: defaultdict(list))
for f in root.glob("p*/**/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {statistics.median(v):.6g}  (n={len(v)})")
