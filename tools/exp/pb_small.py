#!/usr/bin/env python3
"""Time synchronous fused passes (qba_sample_check_packed) at a given size
with the library QBA_LIB points to, and report qba_last_stats (stats[1] =
workgroups that recounted after a pair-bin wrap).

    QBA_LIB=... python tools/exp/pb_small.py [count] [passes]"""
import importlib
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
eng_mod = importlib.import_module("tfg---quantum-byzantine-agreement_amd.engine")


def main():
    count = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    eng = eng_mod.Engine(0)
    n = 11
    eng.prepare(n)
    p = eng.alloc_packed(n, count)
    c = eng.alloc_counts(n)
    for _ in range(20):
        eng.sample_check_packed(n, 5, 0, count, p, c)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(passes):
        eng.sample_check_packed(n, 5, 0, count, p, c)
    b.record()
    torch.cuda.synchronize()
    print(f"count {count}: {a.elapsed_time(b) * 1e3 / passes:.2f} us per synchronous pass; stats {list(eng.last_stats())}")
    eng.close()


if __name__ == "__main__":
    main()
