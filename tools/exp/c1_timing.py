"""Phase timestamps of qba_k_lists at configs[1] (experiment build with
-DQBA_EXP_TIMING -DQBA_SPREAD=0; QBA_LIB points at it).  Prints, per
workgroup, the spread of kernel-start skew, stage (tables + zero + barrier),
main loop + drain, flush, in microseconds (s_memrealtime, 100 MHz)."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, root)
eng_mod = importlib.import_module("tfg---quantum-byzantine-agreement_amd.engine")
n = 11
for N in [int(float(a)) for a in sys.argv[1:]] or (1_000_000, 2_000_000, 4_000_000):
    E = eng_mod.Engine(0)
    E.prepare(n)
    lists, counts = E.alloc_lists(n, N), E.alloc_counts(n)
    for _ in range(200):
        E.sample_check(n, 1, 0, N, lists, counts)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    E.sample_check(n, 1, 0, N, lists, counts)
    b.record()
    torch.cuda.synchronize()
    grid = min(-(-(N // 4) // (2 * 1024)), 512)  # qba_k_lists: QBA_LBLOCK threads, 2 quads each
    lib = ctypes.CDLL(os.environ["QBA_LIB"])
    buf = np.zeros(grid * 8, np.uint64)
    rc = lib.qba_exp_timing(E.ctx, n, grid, buf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    t = buf.reshape(grid, 8)[:, :4].astype(np.int64)
    hw = buf.reshape(grid, 8)[:, 4].astype(np.int64)
    xcc = buf.reshape(grid, 8)[:, 5].astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0
    def pct(x):
        return "min %6.2f  p50 %6.2f  max %6.2f" % (np.min(x), np.median(x), np.max(x))
    print(f"N={N} grid={grid} event(list+reduce)={a.elapsed_time(b)*1e3:.2f} us")
    print("  start skew   ", pct(us[:, 0]))
    print("  stage        ", pct(us[:, 1] - us[:, 0]))
    print("  main+drain   ", pct(us[:, 2] - us[:, 1]))
    print("  flush(issue) ", pct(us[:, 3] - us[:, 2]))
    print("  last end     ", "%6.2f" % us[:, 3].max())
    import collections
    cu = collections.Counter(zip(xcc & 0xF, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF))
    per = collections.Counter(cu.values())
    print("  workgroups per CU:", dict(sorted(per.items())), " distinct CUs:", len(cu),
          " per XCC:", dict(sorted(collections.Counter(xcc & 0xF).items())))
    E.close()
