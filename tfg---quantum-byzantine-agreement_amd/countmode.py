"""Count-mode protocol: decisions from the device's count histograms.

At large sizeL the reference's packets are impractical (P as int64 index
lists is ~250 MB per packet at n=11, sizeL=1e9).  Count mode
keeps the protocol rounds, random-number order and acceptance rules of
tfg.py:166-363 exactly, but in CANONICAL ORDER (every party gathers P in
ascending index order) and with compact packets:

* the lists never leave the device: one ``qba_sample_check`` pass (chunked;
  sharded over the GPU owners by :class:`ShardCounter` when there are
  several, one all-reduce of the counts) yields
      H[u][g][x] = #{k in P_u : L_g[k] = x}
      C[u][g][h] = #{k in P_u : L_g[k] = L_h[k]}        P[u] = |P_u|
  with P_u = {k : L0[k] != L1[k], Lc[k] = u}  (tfg.py:182, 327);
* P travels as its value u (or "cleared"); a tuple L_g[P_u] travels as the
  descriptor (u, g), canonicalised so that equal tuples compare equal
  (C[u][g][h] = |P_u|), which preserves the reference's set de-duplication;
* consistent(v, L, w) (tfg.py:87-98) is exact from the counts:
      Cond1: all descriptors have the same length (|P_u| or 0),
      Cond2: H[u][g][v] == 0 for every tuple (values are always in [0, w)),
      Cond3: C[u][g][h] == 0 for every pair of distinct tuples.

tests/test_countmode.py checks decisions, V_i and accept/reject counts
against the reference run with sorted sets (tests/golden/protocol.json,
"canonical").
"""
from __future__ import annotations

import itertools
from typing import Optional

import numpy as np

from .protocol import Party, _dt, _recv_array

EMPTY = ()


class CountTables:
    """H, C, P of one run (host copies) and the descriptor algebra."""

    def __init__(self, n: int, flat: np.ndarray):
        self.n = n
        self.w = 1 << int(n).bit_length()
        w, g = self.w, n + 1
        h, c = w * g * w, w * g * g
        flat = np.asarray(flat, dtype=np.int64)
        self.H = flat[:h].reshape(w, g, w)
        self.C = flat[h:h + c].reshape(w, g, g)
        self.P = flat[h + c:h + c + w]
        self.flat = flat

    def desc(self, g: int, u: Optional[int]):
        """Canonical descriptor of tuple(L_g[j] for j in sorted(P_u))."""
        if u is None or self.P[u] == 0:
            return EMPTY
        full = self.P[u]
        rep = next(h for h in range(self.n + 1) if self.C[u, g, h] == full)
        return (int(u), int(rep))

    def length(self, d) -> int:
        return 0 if d == EMPTY else int(self.P[d[0]])

    def consistent(self, v, L) -> bool:
        it = iter(L)
        first = next(it)  # StopIteration on an empty L, as tfg.py:90
        n0 = self.length(first)
        if any(self.length(d) != n0 for d in it):
            return False
        descs = [d for d in L if d != EMPTY]
        if not descs:
            return True
        if len({d[0] for d in descs}) != 1:
            raise AssertionError("tuples over different P in one packet")
        v = int(v)
        # every list value lies in [0, w), so Cond2 can only fail through x == v
        if 0 <= v < self.w and any(self.H[u, g, v] != 0 for u, g in descs):
            return False
        return all(self.C[a[0], a[1], b[1]] == 0 for a, b in itertools.combinations(descs, 2))


class ShardCounter:
    """The count pass of one run with sizeL sharded over G GPU owners
    (SURVEY.md §7 H7, §8(e)).

    Owner r samples and checks the entries ``shard_bounds(sizeL, r, G)`` on
    its own GPU -- Philox is keyed by the GLOBAL entry index, so the shards'
    union is exactly the unsharded lists -- and the owners' int64 buffers
    [H | C | P] are summed by ONE all-reduce: torch.distributed (RCCL over
    xGMI on MI355X, gloo in the CPU tests) under torchrun, or the C ABI's
    qba_allreduce_i64 (RCCL) under mpiexec.  Injected lists are split the
    same way.  ``participates(rank)`` names the protocol ranks that own a
    shard (all owners must call :meth:`tables` together)."""

    def __init__(self, engine, rank: int, world: int, allreduce, owners=None):
        self.engine, self.rank, self.world = engine, rank, world
        self.allreduce = allreduce
        self._owners = owners

    def group_ranks(self) -> int:
        """A one-element int64 1 from every owner through this counter's own
        all-reduce (RCCL, torch.distributed or the test's MPI seam): how many
        owners the collective summed."""
        dev = getattr(self.engine, "device", None)
        if dev is not None:
            import torch
            one = torch.ones(1, dtype=torch.int64, device=dev)
        else:
            one = np.ones(1, np.int64)
        return int(np.asarray(self.allreduce(one)).reshape(-1)[0])

    def check_group(self) -> int:
        """group_ranks(), raising QbaError unless it is the owner count (a
        collective: every owner calls it, right after the group is formed)."""
        seen = self.group_ranks()
        if seen != self.world:
            from ._lib import QbaError
            raise QbaError(f"the count all-reduce summed {seen} owner(s), expected {self.world}")
        return seen

    def participates(self, party_rank: int) -> bool:
        return party_rank in self._owners if self._owners is not None else party_rank < self.world

    def tables(self, n: int, sizeL: int, seed: int, lists=None) -> np.ndarray:
        """Sum of every owner's [H | C | P]; raises on EVERY owner when any
        owner's count pass failed.  The buffer carries one extra int64, the
        number of owners that failed: an owner whose pass raised still joins
        the collective (with zero tables and its flag set), so no rank is
        left blocked in the all-reduce."""
        from .distributed import count_layout, shard_bounds
        first, count = shard_bounds(sizeL, self.rank, self.world)
        err = None
        try:
            if lists is not None:
                part = np.ascontiguousarray(np.asarray(lists)[:, first:first + count])
                flat = self.engine.count_tables(n, count, seed, lists=part, device_out=True)
            else:
                flat = self.engine.count_tables(n, count, seed, first=first, device_out=True)
        except Exception as e:  # noqa: BLE001 -- re-raised below, after the collective
            err, flat = e, None
        out = np.asarray(self.allreduce(self._flagged(flat, err is not None, count_layout(n)[3])))
        if out[-1] != 0:
            if err is not None:
                raise err
            from ._lib import QbaError
            raise QbaError(f"count pass failed on {int(out[-1])} of {self.world} shard owner(s)")
        return out[:-1]

    def _flagged(self, flat, failed: bool, size: int):
        """[flat | failed] in the form the all-reduce takes (device tensor for
        a GPU engine, host array otherwise); zero tables when the pass failed."""
        import torch
        dev = getattr(self.engine, "device", None)
        if isinstance(flat, torch.Tensor) or (flat is None and dev is not None):
            dev = flat.device if isinstance(flat, torch.Tensor) else dev
            body = flat if flat is not None else torch.zeros(size, dtype=torch.int64, device=dev)
            return torch.cat([body, torch.tensor([int(failed)], dtype=torch.int64, device=dev)])
        body = np.asarray(flat, dtype=np.int64) if flat is not None else np.zeros(size, np.int64)
        return np.concatenate([body, np.array([int(failed)], np.int64)])


def torch_allreduce(flat):
    """Sum over the torch.distributed group (RCCL / gloo); host numpy result."""
    import torch
    from .distributed import allreduce_counts
    t = flat if isinstance(flat, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(flat))
    if t.is_cuda and torch.distributed.get_backend() == "gloo":
        t = t.cpu()
    return allreduce_counts(t).cpu().numpy()


def rccl_allreduce(engine):
    """Sum over the C ABI's RCCL communicator (qba_rccl_init); host numpy result."""
    def run(flat):
        engine.allreduce_i64(flat)
        return flat.cpu().numpy()
    return run


class PRef:
    """The P object of a packet: P_u, mutable only by clear() (tfg.py:280)."""

    __slots__ = ("u",)

    def __init__(self, u: Optional[int]):
        self.u = u

    def clear(self):
        self.u = None


class CountParty(Party):
    """A rank of the count-mode protocol (same rounds and RNG use as Party)."""

    chunk = 1 << 27

    def __init__(self, *args, counter: Optional[ShardCounter] = None, **kw):
        super().__init__(*args, **kw)
        self.counter = counter

    def particle_comm(self):
        c, n = self.comm, self.n
        w, g = 1 << int(n).bit_length(), n + 1
        size = w * g * w + w * g * g + w
        flat = None
        if self.counter is not None and self.counter.participates(self.rank):
            flat = self.counter.tables(n, self.sizeL, self.seed, self.inject)  # collective over the owners
        if self.rank == 0:
            self.say("|W| =", self.w)
            if flat is None:
                flat = self.engine.count_tables(n, self.sizeL, self.seed, self.inject, self.chunk)
            self.tables = CountTables(n, flat)
            reqs = [c.Isend([self.tables.flat, _dt(c)], dest=r) for r in range(1, n + 1)]
            for r in reqs:
                r.Wait()
            return
        self.tables = CountTables(n, _recv_array(c, 0, None, size))

    def commander_setup(self):
        self.v = self.rng.randint(self.w)
        self.say("v =", self.v)

    def p_for(self, v):
        return PRef(int(v))

    def own_tuple(self, P):
        return self.tables.desc(self.rank, P.u)

    def check(self, v, L) -> bool:
        return self._tally(self.tables.consistent(v, L))

    def precheck(self, inbox):
        return [None] * len(inbox)  # the count tables are already on the host

    def add_own_and_check(self, P, v, L, pre=None) -> bool:
        L.add(self.own_tuple(P))
        return self.check(v, L)

    def send(self, dest, P, v, L):
        self.stats.sent += 1
        pairs = np.array([x for d in L for x in (d if d != EMPTY else (-1, -1))], dtype=np.int64)
        head = np.array([-1 if P.u is None else P.u, int(v), len(L)], dtype=np.int64)
        self.comm.Isend([head, _dt(self.comm)], dest=dest, tag=1).Wait()
        self.comm.Isend([pairs, _dt(self.comm)], dest=dest, tag=2).Wait()

    def recv(self, src):
        head = _recv_array(self.comm, src, 1, 3)
        pairs = _recv_array(self.comm, src, 2, 2 * int(head[2])).reshape(-1, 2)
        L = {EMPTY if a < 0 else (int(a), int(b)) for a, b in pairs.tolist()}
        return PRef(None if head[0] < 0 else int(head[0])), int(head[1]), L
