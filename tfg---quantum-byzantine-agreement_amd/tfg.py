"""Command line of the engine, interface-compatible with the reference
(README.md:4):

    mpiexec -n <nParties+1> python -m tfg---quantum-byzantine-agreement_amd.tfg <sizeL> <nDishonest>

Three launch shapes:

* ``mpiexec -n <n+1>`` -- one process per party, as the reference.  The MPI
  layer is mpi4py when importable, else the package's ctypes binding of
  MPICH (mpi.py).  Exact mode: every party owns a GPU engine (device =
  rank % visible GPUs).  Count mode: the first G = min(n+1, GPUs) ranks own
  a GPU each, sample + check their sizeL shard and sum the counts with one
  RCCL all-reduce (C ABI qba_allreduce_i64; the unique id travels over MPI).
  ``--rounds epoch`` gives the rounds barrier-epoch delivery (deterministic,
  = the golden fixtures); the default keeps the reference's own rounds.
* ``torchrun --nproc-per-node G ... --mode count`` -- G GPU owners, one per
  GPU; rank 0 runs all n+1 parties in-process (LocalWorld), the count pass is
  sharded over the G ranks (torch.distributed all-reduce over RCCL).
* plain ``python -m ...tfg`` -- all parties in-process on one GPU
  (``--parties N`` sets nParties, default 3).

``--mode count`` evaluates the protocol from device count histograms
(canonical order), which is what makes sizeL = 1e9 practical; the default
``exact`` mode reproduces tfg.py's own set-order semantics.  Without
``--seed`` the lists and every party's random choices are drawn from OS
entropy, as the reference's unseeded ``np.random``; with it runs repeat.
"""
from __future__ import annotations

import argparse
import os
import secrets
import sys
import time

import numpy as np

from . import comm as comm_mod
from . import countmode, protocol

RCCL_ID_TAG = 29_999


def _args(argv):
    ap = argparse.ArgumentParser(prog="tfg", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("sizeL", type=float)
    ap.add_argument("nDishonest", type=int)
    ap.add_argument("--parties", type=int, default=3, help="nParties for an in-process run")
    ap.add_argument("--mode", choices=["exact", "count"], default="exact")
    ap.add_argument("--rounds", choices=["reference", "epoch"], default="reference",
                    help="reference: tfg.py's own (racy) rounds; epoch: barrier-epoch delivery")
    ap.add_argument("--seed", type=int, default=None, help="rank RNG seed and list seed")
    ap.add_argument("--quiet", action="store_true", help="print only the outcome")
    ap.add_argument("--timing", action="store_true", help="print the wall time of the run")
    ap.add_argument("--wire", action="store_true",
                    help="in-process exact mode: send the lists in the reference's int64-per-bit wire layout "
                         "(tfg.py:142-161) instead of handing each rank its device row")
    return ap.parse_args(argv)


def _outcome(res, verbose):
    if res is not None and not verbose:
        print("Decisions:", np.array(res["decisions"]))
        print("Dishonests:", np.array(res["dishonest"]))
        print("Success:", res["success"])


class RcclLink:
    """How the GPU owners of an mpiexec count run form their all-reduce group:
    an RCCL communicator through the C ABI (qba_rccl_init), its unique id
    created on rank 0 and sent to the other owners over MPI."""

    @staticmethod
    def unique_id() -> bytes:
        from .engine import Engine
        return Engine.rccl_unique_id()

    @staticmethod
    def allreduce(eng, uid: bytes, owners: int, rank: int):
        eng.rccl_init(uid, owners, rank)
        return countmode.rccl_allreduce(eng)


def count_owners(world, mpi, ndev: int, make_engine, link=RcclLink):
    """Count mode under mpiexec: the first G = min(ranks,
    GPUs) ranks own a GPU each (device = rank % ndev) and shard the count pass
    (countmode.ShardCounter); for G > 1 rank 0 makes the group's unique id and
    sends it to owners 1..G-1 over MPI, and every owner joins the group; a
    one-element all-reduce of ones then checks that the group sums exactly G
    owners (ShardCounter.check_group).
    Returns (engine or None, CountParty keyword arguments).  make_engine and
    link are the seams the CPU test of G > 1 owners fills with the numpy engine
    and an all-reduce over MPI (tests/mpi_driver.py --owners)."""
    rank, size = world.Get_rank(), world.Get_size()
    g = min(size, ndev)
    eng = make_engine(rank % ndev) if rank < g else None
    kw = {}
    if g > 1 and rank < g:
        uid = np.frombuffer(link.unique_id() if rank == 0 else bytes(128), np.uint8).copy()
        if rank == 0:
            for r in range(1, g):
                world.Send([uid, mpi.INT], dest=r, tag=RCCL_ID_TAG)
        else:
            world.Recv([uid, mpi.INT], source=0, tag=RCCL_ID_TAG)
        kw["counter"] = countmode.ShardCounter(eng, rank, g, link.allreduce(eng, uid.tobytes(), g, rank))
        kw["counter"].check_group()  # the communicator must sum exactly the G owners
    return eng, kw


def _mpiexec(a, mpi, size_l, verbose, log) -> int:
    import torch
    from .engine import Engine
    world = mpi.COMM_WORLD
    rank, size = world.Get_rank(), world.Get_size()
    ndev = max(torch.cuda.device_count(), 1)
    # list seed: explicit, or drawn on rank 0 and shared (the lists must agree)
    seed = np.array([a.seed if a.seed is not None else secrets.randbits(62)], np.int64)
    if rank == 0:
        for r in range(1, size):
            world.Send([seed, mpi.INT], dest=r, tag=RCCL_ID_TAG - 1)
    else:
        world.Recv([seed, mpi.INT], source=0, tag=RCCL_ID_TAG - 1)
    list_seed = int(seed[0])
    rng = np.random if a.seed is None else np.random.RandomState(a.seed * 1000 + rank)
    comm = comm_mod.EpochComm(world) if a.rounds == "epoch" else world
    kw = {}
    if a.mode == "count":
        eng, kw = count_owners(world, mpi, ndev, Engine, RcclLink)
        cls = countmode.CountParty
    else:
        eng = Engine(rank % ndev)
        cls = protocol.Party
    t0 = time.perf_counter()
    res = cls(comm, size_l, a.nDishonest, eng, rng, log, None, list_seed, **kw).run()
    _outcome(res, verbose)
    if a.timing and rank == 0:
        print(f"wall {time.perf_counter() - t0:.3f} s ({a.mode} mode, {size} ranks)")
    return 0


def _torchrun(a, size_l, verbose, log) -> int:
    """G torch ranks = G GPU owners; rank 0 hosts the protocol in-process."""
    import torch
    from . import distributed
    from .engine import Engine
    if a.mode != "count":
        raise SystemExit("torchrun launches shard the count pass: use --mode count")
    rank, local, world = distributed.init()
    eng = Engine(local)
    seed = torch.tensor([a.seed if a.seed is not None else secrets.randbits(62)], dtype=torch.int64,
                        device=eng.device)
    torch.distributed.broadcast(seed, 0)
    list_seed = int(seed.item())
    counter = countmode.ShardCounter(eng, rank, world, countmode.torch_allreduce, owners={0})
    counter.check_group()
    if rank != 0:
        counter.tables(a.parties, size_l, list_seed)
        return 0
    t0 = time.perf_counter()
    rank_seed = a.seed if a.seed is not None else secrets.randbits(20)
    run = protocol.run_local(a.parties, size_l, a.nDishonest, eng, seed=rank_seed, log=log,
                             party_cls=countmode.CountParty, timeout=600, list_seed=list_seed,
                             party_kwargs={"counter": counter})
    _outcome(run.result, verbose)
    if a.timing:
        print(f"wall {time.perf_counter() - t0:.3f} s (count mode, sizeL sharded over {world} GPUs)")
    return 1 if run.error else 0


def main(argv=None) -> int:
    a = _args(sys.argv[1:] if argv is None else argv)
    size_l = int(a.sizeL)
    verbose = not a.quiet and size_l <= 100_000 and a.mode == "exact"
    log = print if verbose else None
    mpi = comm_mod.mpi_world()
    if mpi is not None and mpi.COMM_WORLD.Get_size() > 1:
        return _mpiexec(a, mpi, size_l, verbose, log)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return _torchrun(a, size_l, verbose, log)
    from .engine import Engine
    eng = Engine(0)
    seed = secrets.randbits(20) if a.seed is None else a.seed
    list_seed = secrets.randbits(62) if a.seed is None else a.seed
    party_cls = countmode.CountParty if a.mode == "count" else protocol.Party
    t0 = time.perf_counter()
    run = protocol.run_local(a.parties, size_l, a.nDishonest, eng, seed=seed, log=log,
                             party_cls=party_cls, timeout=600, list_seed=list_seed,
                             party_kwargs={"wire": True} if a.wire else None)
    _outcome(run.result, verbose)
    if a.timing:
        print(f"wall {time.perf_counter() - t0:.3f} s ({a.mode} mode, in-process, {a.parties + 1} ranks)")
    if run.error:
        print(f"{run.error} (min of an empty V_i, tfg.py:306) on ranks {run.error_ranks}")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
