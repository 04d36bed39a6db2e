"""Per-wave phase stamps of the deferred list kernel at configs[1]
(experiment build t_ts2: s_memrealtime at step start, after each quad's
sampling, before the row stores, at the main loop's end and after the final
drains).  Prints the spread over waves, us from the first step start."""
import ctypes
import importlib
import os
import sys

import numpy as np
import torch

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, root)
eng_mod = importlib.import_module("tfg---quantum-byzantine-agreement_amd.engine")
n, N = 11, int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000
E = eng_mod.Engine(0)
E.prepare(n)
p, c = E.alloc_packed(n, N), E.alloc_counts(n)
lib = ctypes.CDLL(os.environ["QBA_LIB"])
for rep in range(3):
    for _ in range(300):
        E.sample_check_packed(n, 1, 0, N, p, c, deferred=True)
    torch.cuda.synchronize()
    buf = np.zeros((4096 * 16, 8), np.uint64)
    assert lib.qba_exp_ts(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    t = buf[(buf[:, 1] != 0) & (buf[:, 6] != 0)].astype(np.int64)
    t0 = t[:, 1].min()
    us = (t - t0) / 100.0
    f = lambda x: "p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f" % (np.percentile(x, 10), np.median(x), np.percentile(x, 90), x.max())
    print(f"N={N} waves with a step: {len(t)}")
    for name, a, b in (("start", None, 1), ("quad 0 sampled", 1, 2), ("quad 1 sampled (+pushes q0)", 2, 4),
                       ("pushes q1 + pack", 4, 6), ("stores", 6, 7), ("final drains", 7, 0)):
        x = us[:, b] if a is None else us[:, b] - us[:, a]
        print(f"  {name:30s} {f(x)}")
    print("  end (after drains)            ", f(us[:, 0]))
E.flush_deferred()
E.close()
