#!/usr/bin/env python3
"""Where configs[0]'s protocol run (n=3, sizeL=1000, nDis=1) spends its time:
wall per run, and the cumulative time / calls of every Engine method the
host calls (GPU box)."""
import collections
import importlib
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
PKG = "tfg---quantum-byzantine-agreement_amd"


class Timed:
    def __init__(self, eng):
        self._e = eng
        self.t = collections.defaultdict(float)
        self.n = collections.Counter()

    def __getattr__(self, name):
        a = getattr(self._e, name)
        if not callable(a):
            return a

        def f(*x, **k):
            t0 = time.perf_counter()
            try:
                return a(*x, **k)
            finally:
                self.t[name] += time.perf_counter() - t0
                self.n[name] += 1
        return f


def main(runs=50):
    protocol = importlib.import_module(f"{PKG}.protocol")
    eng = importlib.import_module(f"{PKG}.engine").Engine(0)
    for s in range(5):
        protocol.run_local(3, 1000, 1, eng, seed=1 + s)
    t0 = time.perf_counter()
    for s in range(runs):
        protocol.run_local(3, 1000, 1, eng, seed=1 + s)
    wall = (time.perf_counter() - t0) / runs
    te = Timed(eng)
    t0 = time.perf_counter()
    for s in range(runs):
        protocol.run_local(3, 1000, 1, te, seed=1 + s)
    wall2 = (time.perf_counter() - t0) / runs
    print(f"wall per run: {wall * 1e3:.3f} ms (instrumented {wall2 * 1e3:.3f} ms)")
    for k in sorted(te.t, key=te.t.get, reverse=True):
        print(f"  {k:18s} {te.n[k] / runs:6.1f} calls/run  {te.t[k] / runs * 1e3:7.3f} ms/run")
    if "--cprofile" in sys.argv:  # where the host's own time goes (cProfile inflates it)
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for s in range(runs):
            protocol.run_local(3, 1000, 1, eng, seed=1 + s)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(40)
    eng.close()


if __name__ == "__main__":
    main()
