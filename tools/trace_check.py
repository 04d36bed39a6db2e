#!/usr/bin/env python3
"""Cross-check bench.py's launch time against the rocprofv3 kernel trace of
the SAME command: the average device span of the last K (timed) steps --
first timed qba_k_lists start to last qba_k_reduce end, / K -- next to the
bench line's roofline.launch_ms.

    tools/trace_check.py <trace-dir> <bench-json> [K]"""
import csv
import json
import sys
from pathlib import Path


def main():
    d, bj = Path(sys.argv[1]), json.loads(Path(sys.argv[2]).read_text())
    k = int(sys.argv[3]) if len(sys.argv) > 3 else bj["steps"]
    rows = [r for f in d.rglob("*kernel_trace.csv") for r in csv.DictReader(open(f))]
    span = lambda name: sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))  # noqa: E731
                               for r in rows if name in r["Kernel_Name"])
    lists, red = span("qba_k_lists"), span("qba_k_reduce")
    lt = lists[-k:]
    # a synchronous step is list kernel + qba_k_reduce; a deferred step
    # (qba_k_lists_pbdef) reduces the step before in its own tail, and the
    # timed region ends with ONE flush (qba_k_reduce_def)
    deferred = len(red) < len(lists)
    rt = red[-1:] if deferred else red[-k:]
    per_step = (rt[-1][1] - lt[0][0]) / k / 1e3
    print(f"launches in trace: {len(lists)} list, {len(red)} reduce; timed steps: {k}"
          + (" (deferred: one flush)" if deferred else ""))
    print(f"qba_k_lists average over the timed steps: {sum(e - s for s, e in lt) / k / 1e3:.1f} us")
    print(f"qba_k_reduce average over the timed {'flush' if deferred else 'steps'}: "
          f"{sum(e - s for s, e in rt) / len(rt) / 1e3:.2f} us")
    print(f"device span per timed step (trace): {per_step:.1f} us")
    print(f"bench roofline.launch_ms: {bj['roofline']['launch_ms'] * 1e3:.1f} us "
          f"(ms_per_step {bj['ms_per_step'] * 1e3:.1f} us)")
    print(f"difference: {100 * (bj['roofline']['launch_ms'] * 1e3 / per_step - 1):+.2f} %")


if __name__ == "__main__":
    main()
