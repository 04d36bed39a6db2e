"""BASELINE.md CPU plan, item 2: the build's Python restatement under a real
``mpiexec -n 4`` at configs[0] (n = 3, 1 dishonest, sizeL = 1000).

    mpiexec -n 4 python tests/mpi_cpu_baseline.py [--runs R]

TEST / BASELINE INFRASTRUCTURE (bench.py --config 0 starts it): each rank is
one party of the package's protocol host (protocol.Party over the ctypes
MPICH binding, the reference's own racy rounds) with the numpy OracleEngine in
place of the GPU, i.e. tfg.py's algorithm restated on the host CPU, one
process per party as `mpiexec -n 4 python tfg.py 1000 1` runs it.  Lists are
drawn on the host from the closed form (the reference's qsimov sampler is not
installable).  Rank 0 prints one JSON line: wall per protocol run (barrier to
barrier, max over ranks) and the whole R-run loop."""
import argparse
import importlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))
PKG = "tfg---quantum-byzantine-agreement_amd"

from oracle_engine import OracleEngine  # noqa: E402
import tfg_oracle as orc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--sizeL", type=int, default=1000)
    ap.add_argument("--dishonest", type=int, default=1)
    a = ap.parse_args()
    comm_mod = importlib.import_module(f"{PKG}.comm")
    protocol = importlib.import_module(f"{PKG}.protocol")
    MPI = comm_mod.mpi_world()
    if MPI is None:
        raise SystemExit("not an mpiexec launch")
    world = MPI.COMM_WORLD
    rank, size = world.Get_rank(), world.Get_size()
    n = size - 1
    eng = OracleEngine()
    lists = [orc.closed_form_lists(n, a.sizeL, np.random.default_rng(1000 + s)) for s in range(a.runs + 1)]
    per = []
    for s in range(a.runs + 1):  # run 0 warms the imports and caches
        world.Barrier()
        t0 = time.perf_counter()
        p = protocol.Party(world, a.sizeL, a.dishonest, eng, np.random.RandomState(s * 1000 + rank), None,
                           lists[s], s)
        p.tolerate_empty_vi = True
        p.run()
        world.Barrier()
        if s:
            per.append(time.perf_counter() - t0)
    mine = np.array(per, dtype=np.float64)
    if rank != 0:
        world.Send([mine, MPI.INT], dest=0, tag=31_000)  # raw bytes (as tfg.py ships int64 as MPI.INT)
        return
    worst = mine.copy()
    for r in range(1, size):
        buf = np.empty_like(mine)
        world.Recv([buf, MPI.INT], source=r, tag=31_000)
        worst = np.maximum(worst, buf)
    ms = float(np.median(worst)) * 1e3
    print(json.dumps({"ranks": size, "n": n, "sizeL": a.sizeL, "nDishonest": a.dishonest, "runs": a.runs,
                      "ms_per_run_median": ms, "ms_per_run_mean": float(worst.mean()) * 1e3,
                      "entries_per_s": a.sizeL / (ms * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
