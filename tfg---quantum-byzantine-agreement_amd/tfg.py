"""Command line of the engine, interface-compatible with the reference
(README.md:4):

    mpiexec -n <nParties+1> python -m tfg---quantum-byzantine-agreement_amd.tfg <sizeL> <nDishonest>

With mpi4py present every MPI rank runs one party (GPU = rank % visible
GPUs).  Without mpi4py the same run happens in-process on a LocalWorld
(``--parties N`` sets nParties, default 3).  ``--mode count`` evaluates the
protocol from device count histograms (canonical order), which is what makes
sizeL = 1e9 practical; the default ``exact`` mode reproduces tfg.py's own
set-order semantics.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

from . import comm as comm_mod
from . import countmode, protocol
from .engine import Engine


def _args(argv):
    ap = argparse.ArgumentParser(prog="tfg", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("sizeL", type=float)
    ap.add_argument("nDishonest", type=int)
    ap.add_argument("--parties", type=int, default=3, help="nParties for an in-process run")
    ap.add_argument("--mode", choices=["exact", "count"], default="exact")
    ap.add_argument("--seed", type=int, default=None, help="rank RNG seed and list seed")
    ap.add_argument("--quiet", action="store_true", help="print only the outcome")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    a = _args(sys.argv[1:] if argv is None else argv)
    size_l = int(a.sizeL)
    verbose = not a.quiet and size_l <= 100_000 and a.mode == "exact"
    log = print if verbose else None
    party_cls = countmode.CountParty if a.mode == "count" else protocol.Party
    mpi = comm_mod.mpi_world()
    if mpi is not None and mpi.COMM_WORLD.Get_size() > 1:
        import torch
        c = mpi.COMM_WORLD
        eng = Engine(c.Get_rank() % max(torch.cuda.device_count(), 1))
        rng = np.random if a.seed is None else np.random.RandomState(a.seed * 1000 + c.Get_rank())
        p = party_cls(c, size_l, a.nDishonest, eng, rng, log, None, a.seed or 0)
        res = p.run()
        if res is not None and not verbose:
            print("Decisions:", np.array(res["decisions"]))
            print("Dishonests:", np.array(res["dishonest"]))
            print("Success:", res["success"])
        return 0
    eng = Engine(0)
    seed = 0 if a.seed is None else a.seed
    run = protocol.run_local(a.parties, size_l, a.nDishonest, eng, seed=seed, log=log,
                             party_cls=party_cls, timeout=600)
    if not verbose:
        print("Decisions:", np.array(run.result["decisions"]))
        print("Dishonests:", np.array(run.result["dishonest"]))
        print("Success:", run.result["success"])
    if run.error:
        print(f"{run.error} (min of an empty V_i, tfg.py:306) on ranks {run.error_ranks}")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
