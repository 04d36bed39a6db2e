#!/usr/bin/env python3
"""Per-launch duration (and effective shader clock) of one kernel over a run.

    tools/drift.py <trace-dir> [--pmc <pmc-dir>] [--kernel qba_k_lists] [--first 60]

<trace-dir> holds a rocprofv3 ``*kernel_trace.csv``; <pmc-dir> a
``*counter_collection.csv`` of a ``--pmc GRBM_GUI_ACTIVE GRBM_COUNT`` pass of
the same command.  The effective clock of a dispatch is GRBM_GUI_ACTIVE / 8
(the counter sums the 8 XCDs) / its duration (MI355X_MICROARCH.md, "DVFS
give-back"; reads high below ~0.3 ms)."""
import argparse
import csv
import statistics
from pathlib import Path


def launches(d: Path, kernel: str):
    rows = []
    for f in d.rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    return rows


def pmc(d: Path, kernel: str):
    by = {}
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            key = int(r["Dispatch_Id"])
            e = by.setdefault(key, {"t": (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="?")
    ap.add_argument("--pmc")
    ap.add_argument("--kernel", default="qba_k_lists")
    ap.add_argument("--first", type=int, default=60)
    a = ap.parse_args()
    if a.trace:
        L = launches(Path(a.trace), a.kernel)
        us = [(e - s) / 1e3 for s, e in L]
        gaps = [(L[i + 1][0] - L[i][1]) / 1e3 for i in range(len(L) - 1)]
        print(f"{a.kernel}: {len(us)} launches")
        print("first launches (us):", " ".join(f"{x:.0f}" for x in us[: a.first]))
        print("gaps after them (us):", " ".join(f"{x:.0f}" for x in gaps[: a.first]))
        print(f"{'launches':>12s} {'mean_us':>8s} {'min':>6s} {'max':>6s}")
        for i in range(0, len(us), 25):
            blk = us[i:i + 25]
            print(f"{i:5d}-{i + len(blk) - 1:5d} {statistics.mean(blk):8.1f} {min(blk):6.0f} {max(blk):6.0f}")
    if a.pmc:
        P = pmc(Path(a.pmc), a.kernel)
        print(f"PMC dispatches: {len(P)}")
        print(f"{'#':>4s} {'dur_us':>7s} {'clk_GHz':>8s}")
        for i, e in enumerate(P):
            dur = (e["t"][1] - e["t"][0]) * 1e-9
            g = e.get("GRBM_GUI_ACTIVE")
            clk = g / 8 / dur / 1e9 if g else float("nan")
            if i < a.first or i % 10 == 0:
                print(f"{i:4d} {dur * 1e6:7.0f} {clk:8.3f}")


if __name__ == "__main__":
    main()
