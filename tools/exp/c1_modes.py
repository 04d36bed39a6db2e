#!/usr/bin/env python3
"""configs[1]'s two per-pass modes (~9.0 / ~10.0 us): is the mode set per
process, per allocation or per replay?  Three allocation rounds in one
process (fresh list/count buffers each, the old ones kept alive so the
addresses differ), five timed replays of a 200-pass deferred graph each."""
import importlib
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
eng_mod = importlib.import_module("tfg---quantum-byzantine-agreement_amd.engine")
eng = eng_mod.Engine(0)
n, count, steps = 11, 1_000_000, 200
eng.prepare(n)
keep = []
SYNC_FIRST = len(sys.argv) > 1 and sys.argv[1] == "sync_first"
if SYNC_FIRST:  # as bench.py --config 1: the synchronous graph is captured and timed first
    lists0 = eng.alloc_packed(n, count)
    counts0 = eng.alloc_counts(n)
    f0 = lambda: eng.sample_check_packed(n, 5, 0, count, lists0, counts0)  # noqa: E731
    f0(); f0(); torch.cuda.synchronize()
    s0 = torch.cuda.Stream(); s0.wait_stream(torch.cuda.current_stream())
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g0, stream=s0):
            for _ in range(steps):
                f0()
    torch.cuda.synchronize()
    for _ in range(20):
        g0.replay()
    torch.cuda.synchronize()
    keep.append((lists0, counts0, g0))
for rnd in range(3):
    lists = eng.alloc_packed(n, count)
    counts = eng.alloc_counts(n)
    keep.append((lists, counts, torch.empty(int(rnd * 7 + 1) * 1 << 20, dtype=torch.uint8, device="cuda")))
    f = lambda: eng.sample_check_packed(n, 5, 0, count, lists, counts, deferred=True)  # noqa: E731
    f(); f(); eng.flush_deferred(); torch.cuda.synchronize()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(steps):
                f()
            eng.flush_deferred()
    torch.cuda.synchronize()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    out = []
    for r in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); g.replay(); b.record(); torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / steps)
    print(f"alloc round {rnd}: lists {lists.data_ptr():#x} counts {counts.H.data_ptr():#x}  us/pass "
          + " ".join(f"{x:.2f}" for x in out), flush=True)
