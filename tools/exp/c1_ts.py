"""Per-workgroup timeline of the deferred list kernel at configs[1] (n=11,
1e6 entries, nibble rows): experiment build with s_memrealtime stamps
(QBA_LIB -> a build exporting qba_exp_ts, e.g. the round-5 t_ts variant).
Prints, over the list and reduce workgroups of the last deferred launch, the
spread of start, stage end, main end and end (us from the first start)."""
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
    buf = np.zeros(4096 * 4, np.uint64)
    assert lib.qba_exp_ts(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    t = buf.reshape(4096, 4).astype(np.uint64)
    used = t[:, 0] != 0
    t = t[used]
    red = (t[:, 3] >> np.uint64(63)) == 1
    t[:, 3] &= np.uint64((1 << 63) - 1)
    t0 = t[:, 0].min()
    us = (t.astype(np.int64) - int(t0)) / 100.0
    L, R = us[~red], us[red]
    f = lambda x: "min %5.2f p50 %5.2f max %5.2f" % (x.min(), np.median(x), x.max())
    print(f"N={N} list WGs {len(L)}, reduce WGs {len(R)}")
    print("  list start ", f(L[:, 0]), "| stage end ", f(L[:, 1]), "| main end ", f(L[:, 2]), "| end ", f(L[:, 3]))
    if len(R):
        print("  reduce start", f(R[:, 0]), "| end ", f(R[:, 3]))
    print("  last end %.2f us" % us[:, 3].max())
E.flush_deferred()
E.close()
