"""One rank of a protocol fixture case under a real ``mpiexec`` launch.

    mpiexec -n <n+1> python tests/mpi_driver.py <case> [--rounds epoch|reference] [--mode exact|count]

TEST INFRASTRUCTURE: drives the product host (protocol.Party /
countmode.CountParty over the ctypes MPICH binding, mpi.py) with the numpy
OracleEngine in place of the GPU, on the injected lists and per-rank seeds of
tests/golden/protocol.json.  After the protocol, each rank sends its
accept/reject/sent counts, V_i and wire traffic to rank 0, which prints one
JSON line in the fixture's format.
"""
import argparse
import importlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
PKG = "tfg---quantum-byzantine-agreement_amd"

from oracle_engine import OracleEngine  # noqa: E402

STATS_TAG = 30_000  # above every protocol tag (EpochComm: 256 * epochs + 6 + 2|L|)


class MpiLink:
    """tfg.count_owners' group seam for the CPU test: the id is 128 random
    bytes; the all-reduce sums the owners' buffers over MPI point-to-point
    (owner 0 gathers, adds, sends the sum back) and checks that every owner
    joined with the id owner 0 made."""

    TAG = 30_100

    def __init__(self, world, mpi, owners):
        self.world, self.mpi, self.owners = world, mpi, owners

    def unique_id(self) -> bytes:
        import os
        return os.urandom(128)

    def allreduce(self, eng, uid, owners, rank):
        assert owners == self.owners
        world, mpi, ids = self.world, self.mpi, np.frombuffer(uid, np.uint8).copy()

        def run(flat):
            flat = np.ascontiguousarray(np.asarray(flat, dtype=np.int64))
            if rank != 0:
                world.Send([ids, mpi.INT], dest=0, tag=self.TAG)
                world.Send([flat, mpi.INT], dest=0, tag=self.TAG + 1)
                out = np.empty_like(flat)
                world.Recv([out, mpi.INT], source=0, tag=self.TAG + 2)
                return out
            total = flat.copy()
            for r in range(1, owners):
                other = np.empty_like(ids)
                world.Recv([other, mpi.INT], source=r, tag=self.TAG)
                assert np.array_equal(other, ids), f"owner {r} joined with another id"
                part = np.empty_like(flat)
                world.Recv([part, mpi.INT], source=r, tag=self.TAG + 1)
                total += part
            for r in range(1, owners):
                world.Send([total, mpi.INT], dest=r, tag=self.TAG + 2)
            return total
        return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--rounds", choices=["epoch", "reference"], default="epoch")
    ap.add_argument("--mode", choices=["exact", "count"], default="exact")
    ap.add_argument("--owners", type=int, default=0,
                    help="count mode: G shard owners set up by tfg.count_owners (the mpiexec GPU-owner "
                         "path) with the numpy engine and an all-reduce over MPI in place of RCCL")
    a = ap.parse_args()
    comm_mod = importlib.import_module(f"{PKG}.comm")
    protocol = importlib.import_module(f"{PKG}.protocol")
    countmode = importlib.import_module(f"{PKG}.countmode")
    golden = ROOT / "tests" / "golden"
    case = next(c for c in json.loads((golden / "protocol.json").read_text()) if c["name"] == a.case)
    lists = np.load(golden / "protocol_lists.npz")[a.case]
    MPI = comm_mod.mpi_world()
    if MPI is None:
        raise SystemExit("not an mpiexec launch")
    world = MPI.COMM_WORLD
    if world.Get_size() != case["n"] + 1:
        raise SystemExit(f"case {a.case} needs {case['n'] + 1} ranks")
    comm = comm_mod.EpochComm(world) if a.rounds == "epoch" else world
    rank = world.Get_rank()
    cls = countmode.CountParty if a.mode == "count" else protocol.Party
    eng, kw = OracleEngine(), {}
    if a.owners:
        tfg = importlib.import_module(f"{PKG}.tfg")
        eng, kw = tfg.count_owners(world, MPI, a.owners, lambda dev: OracleEngine(), MpiLink(world, MPI, a.owners))
        assert (eng is None) == (rank >= a.owners) and ("counter" in kw) == (a.owners > 1 and rank < a.owners)
    p = cls(comm, case["sizeL"], case["nDishonest"], eng, np.random.RandomState(case["seed"] * 1000 + rank),
            None, lists, case["seed"], **kw)
    p.tolerate_empty_vi = True
    res = p.run()
    vi = sorted(int(x) for x in p.Vi) if rank > 1 and not p.dishonest else []
    mine = np.array([p.stats.accept, p.stats.reject, p.stats.sent, int(p.empty_vi_error),
                     int(rank > 1 and not p.dishonest), getattr(comm, "sent_messages", 0),
                     getattr(comm, "sent_bytes", 0), len(vi)] + vi, dtype=np.int64)
    if rank != 0:
        world.Send([np.array([len(mine)], np.int64), MPI.INT], dest=0, tag=STATS_TAG)
        world.Send([mine, MPI.INT], dest=0, tag=STATS_TAG + 1)
        return
    rows = [mine]
    for src in range(1, world.Get_size()):
        ln = np.empty(1, np.int64)
        world.Recv([ln, MPI.INT], source=src, tag=STATS_TAG)
        buf = np.empty(int(ln[0]), np.int64)
        world.Recv([buf, MPI.INT], source=src, tag=STATS_TAG + 1)
        rows.append(buf)
    out = dict(res)
    out["accept"] = [int(r[0]) for r in rows]
    out["reject"] = [int(r[1]) for r in rows]
    out["sent"] = [int(r[2]) for r in rows]
    out["error_ranks"] = [i for i, r in enumerate(rows) if r[3]]
    out["error"] = "ValueError" if out["error_ranks"] else None
    out["V"] = {str(i): [int(x) for x in r[8:8 + int(r[7])]] for i, r in enumerate(rows) if r[4]}
    out["messages"] = int(sum(r[5] for r in rows))
    out["bytes"] = int(sum(r[6] for r in rows))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
