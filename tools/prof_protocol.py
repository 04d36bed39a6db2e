#!/usr/bin/env python3
"""Where an exact-mode protocol run spends its time (GPU box): wall per run,
the cumulative time / calls of every Engine method the host calls, and the
host functions with the most own time (cProfile).

    tools/prof_protocol.py [n] [sizeL] [nDishonest] [runs]     (default 11 1e6 3 3)"""
import cProfile
import importlib
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
PKG = "tfg---quantum-byzantine-agreement_amd"
from prof_config0 import Timed  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11
    size = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1_000_000
    nd = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    runs = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    protocol = importlib.import_module(f"{PKG}.protocol")
    eng = importlib.import_module(f"{PKG}.engine").Engine(0)
    protocol.run_local(n, size, nd, eng, seed=1)
    t0 = time.perf_counter()
    for s in range(runs):
        protocol.run_local(n, size, nd, eng, seed=2 + s)
    wall = (time.perf_counter() - t0) / runs
    te = Timed(eng)
    pr = cProfile.Profile()
    pr.enable()
    for s in range(runs):
        protocol.run_local(n, size, nd, te, seed=2 + s)
    pr.disable()
    print(f"n={n} sizeL={size} nDis={nd}: wall per run {wall * 1e3:.1f} ms")
    for k in sorted(te.t, key=te.t.get, reverse=True):
        print(f"  {k:20s} {te.n[k] / runs:7.1f} calls/run  {te.t[k] / runs * 1e3:8.2f} ms/run")
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    eng.close()


if __name__ == "__main__":
    main()
