#!/usr/bin/env python3
"""Count-mode pass timing at large sizeL: count_tables chunk by chunk (wall
and last_stats per chunk), then the CLI run under cProfile."""
import cProfile
import importlib
import pstats
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
PKG = "tfg---quantum-byzantine-agreement_amd"
eng_mod = importlib.import_module(f"{PKG}.engine")


def main():
    eng = eng_mod.Engine(0)
    n = 11
    eng.prepare(n)
    p = eng.alloc_packed(n, 1 << 27)
    c = eng.alloc_counts(n)
    for k, cnt in enumerate([1 << 27, 1 << 27, 60_475_904, 125_000_000]):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.sample_check_packed(n, 11, k << 27, cnt, p, c)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        st = eng.last_stats()
        print(f"chunk {k} count {cnt}: {1e3 * (t1 - t0):.2f} ms  stats {list(st)}", flush=True)
    for _ in range(2):
        t0 = time.perf_counter()
        eng.count_tables(n, 10 ** 9, 11)
        print(f"count_tables 1e9: {time.perf_counter() - t0:.3f} s", flush=True)
    tfg = importlib.import_module(f"{PKG}.tfg")
    pr = cProfile.Profile()
    pr.enable()
    tfg.main(["1e9", "3", "--parties", "11", "--mode", "count", "--seed", "11", "--timing"])
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
