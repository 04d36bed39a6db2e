#!/usr/bin/env python3
"""Where a fresh process's count-mode 1e9 run spends its first seconds: the
engine (torch's device init + qba_init), prepare(11) (both circuits compiled
into the sampler program), and count_tables(1e9) cold then warm."""
import importlib
import sys
import time
from pathlib import Path

t = time.perf_counter()
import torch  # noqa: E402

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
eng_mod = importlib.import_module("tfg---quantum-byzantine-agreement_amd.engine")
print(f"import: {time.perf_counter() - t:.3f} s", flush=True)


def timed(label, f):
    torch.cuda.synchronize() if torch.cuda.is_initialized() else None
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    print(f"{label}: {time.perf_counter() - t0:.4f} s", flush=True)
    return r


eng = timed("Engine(0)", lambda: eng_mod.Engine(0))
timed("prepare(11)", lambda: eng.prepare(11))
timed("alloc_packed(2^27)", lambda: eng.alloc_packed(11, 1 << 27))
for k in range(3):
    timed(f"count_tables(11, 1e9) #{k}", lambda: eng.count_tables(11, 10 ** 9, 11))
