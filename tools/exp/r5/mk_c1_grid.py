#!/usr/bin/env python3
"""configs[1] variant: the deferred kernel at QPT (1 or 2) quads per
thread-step, its list grid forced to 2 workgroups per CU minus the reduce
workgroups when the launch would leave slots idle.
    mk_c1_grid.py <name> <qpt>   ->  /tmp/c1v/<name>/csrc"""
import shutil
import sys
from pathlib import Path

name, qpt = sys.argv[1], int(sys.argv[2])
src = Path(__file__).resolve().parents[3] / "tfg---quantum-byzantine-agreement_amd" / "csrc"
dst = Path("/tmp/c1v") / name / "csrc"
shutil.rmtree(dst.parent, ignore_errors=True)
shutil.copytree(src, dst)
p = dst / "qba_lists_kern.h"
s = p.read_text()
a = "(L.packed ? (wide ? (const void *)qba_k_lists_def<NP, S, 2, 1> : (const void *)qba_k_lists_def<NP, S, 1, 1>)"
b = f"(L.packed ? (wide ? (const void *)qba_k_lists_def<NP, S, {qpt}, 1> : (const void *)qba_k_lists_def<NP, S, 1, 1>)"
assert s.count(a) == 1
s = s.replace(a, b)
a = "dgrid = grid_for(ctx, kd, dlds, L.count, wide ? (L.packed ? 2 : QBA_GRID_QPT) : 1, &dcap, QBA_DBLOCK);"
b = f"dgrid = grid_for(ctx, kd, dlds, L.count, wide ? (L.packed ? {qpt} : QBA_GRID_QPT) : 1, &dcap, QBA_DBLOCK);"
assert s.count(a) == 1
s = s.replace(a, b)
a = "    if (dgrid < ctx->num_cus && ctx->num_cus + qba_def_wgs<NP>() <= dcap) dgrid = ctx->num_cus;"
b = ("    if (dgrid < dcap - qba_def_wgs<NP>() && L.count < (1u << 22)) dgrid = dcap - qba_def_wgs<NP>();")
assert s.count(a) == 1
s = s.replace(a, b)
p.write_text(s)
print(dst)
