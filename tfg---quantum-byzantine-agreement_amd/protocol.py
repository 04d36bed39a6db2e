"""tfg.py-compatible protocol host (exact mode).

This mirrors the reference's operator interface -- the same function names,
argument meaning, message format, random-number call order and error
behaviour (tfg.py:87-363) -- while every per-element operation on the lists
runs in libqba's HIP kernels through :class:`~.engine.Engine`:

======================  ==========================  ===============================
reference               here                        device work
======================  ==========================  ===============================
generacionListas  :68   :func:`generacionListas`    qba_sample + qba_values_to_bits
measure_to_ints   :128  :func:`measure_to_ints`     qba_bits_to_values
isQCorrList       :327  :meth:`Party.commander_setup`  qba_isq_indices
P filter          :182  :meth:`Party.p_for`         qba_select_eq
own tuple    :189, :291 :meth:`Party.own_tuple`     qba_gather
consistent        :87   :func:`consistent`          qba_consistent (Cond1 on host)
======================  ==========================  ===============================

Exactness: the reference builds each tuple in its process's own CPython
set-iteration order, so the host keeps real Python sets and
performs the same list(P) -> wire -> set(buff) hops; the device receives the
resulting index orders.  With identical injected lists, rank seeds and
delivery order the decisions, V_i sets and accept/reject counts equal the
reference's (tests/test_protocol.py against tests/golden/protocol.json).

Rounds use the host's comm: real mpi4py under ``mpiexec``, or
:class:`~.comm.LocalWorld` threads (barrier-epoch delivery, comm.py).
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import threading
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np

from . import comm as comm_mod
from ._lib import call
from .resource import n_qubits


def _dt(comm):
    """MPI INT of the library that owns `comm` (tfg.py:110 declares MPI.INT)."""
    return comm_mod.mpi_of(comm).INT


# ---------------------------------------------------------------------------
# module-level functions with the reference's names
# ---------------------------------------------------------------------------
def generacionListas(nParties, size, nQubits, w, engine=None, seed=0, lists=None):
    """rawS: (n+1, nQubits*size) int64 bits, MSB first per value (tfg.py:68-84).

    Lists are drawn on the device (Philox keyed by entry index, ``seed``), or
    taken from ``lists`` (an injected (n+1, size) value array), then encoded
    to the reference's one-int64-per-bit wire layout on the device.
    """
    if engine is None:
        raise RuntimeError("generacionListas needs an Engine (no CPU fallback)")
    if lists is None:
        dev = engine.sample(nParties, seed, 0, size)
    else:
        arr = np.ascontiguousarray(lists, dtype=np.uint8)
        if arr.shape != (nParties + 1, size):
            raise ValueError(f"injected lists must have shape {(nParties + 1, size)}")
        dev = engine.to_device(arr)
    if hasattr(engine, "lists_to_bits"):  # every row encoded on the device, one copy to the host
        return engine.lists_to_bits(dev, nParties + 1, size, nQubits)
    return np.stack([engine.to_host(engine.values_to_bits(dev[g, :size], size, nQubits))
                     for g in range(nParties + 1)])


def measure_to_ints(raw, sizeL, nQubits, engine=None):
    """MSB-first nQubits-bit groups -> list of ints (tfg.py:128-129), on the device."""
    if engine is None:
        raise RuntimeError("measure_to_ints needs an Engine (no CPU fallback)")
    vals = engine.bits_to_values(engine.to_device(np.asarray(raw, dtype=np.int64)), sizeL, nQubits)
    return engine.to_host(vals).astype(np.int64).tolist()


def consistent(v, L, w, engine=None):
    """consistent(v, L, w) of tfg.py:87-98.

    Cond1 (equal lengths; StopIteration on an empty L, as ``next(iter(L))``)
    is host bookkeeping; Cond2 and Cond3 run in qba_consistent.
    """
    it = iter(L)
    length = len(next(it))
    if any(len(t) != length for t in it):
        return False
    if engine is None:
        raise RuntimeError("consistent needs an Engine (no CPU fallback)")
    rows = np.array([t.arr if isinstance(t, PTuple) else list(t) for t in L], dtype=np.int64).reshape(len(L), length)
    return engine.consistent_rows(rows, int(v), int(w))


def decide_order(Vi, v, is_comm):
    """tfg.py:303-306: the commander keeps its v, a lieutenant takes min(V_i)."""
    return v if is_comm else min(Vi)


# ---------------------------------------------------------------------------
# wire format of a (P, v, L) packet (tfg.py:199-263)
# ---------------------------------------------------------------------------
def _wire(x) -> np.ndarray:
    """int64 array of a set / tuple in its iteration order (the wire order)."""
    arr = getattr(x, "arr", None)
    if arr is not None:  # PSet / PTuple: the order is kept as the array itself
        return arr
    return np.fromiter(x, dtype=np.int64, count=len(x))


# ---------------------------------------------------------------------------
# P sets and L tuples as CPython 3.10 holds them, without the Python objects
# (qba_host_pyset_order / qba_host_pytuple_hash restate setobject.c and
# tuplehash; tests/test_protocol.py compares them with the live interpreter).
# A 31 K-element P (n = 11, sizeL = 1e6) then costs one native pass instead of
# a Python set build plus its conversion back to an array at every hop.
# ---------------------------------------------------------------------------
NATIVE_SETS = sys.version_info[:2] == (3, 10) and os.environ.get("QBA_PYTHON_SETS") != "1"


class PSet:
    """A packet's P: the int64 array of set(insertion sequence) in CPython's
    iteration order (tfg.py:182, 240, 327).  Supports what tfg.py does with
    P: len, iteration, clear (tfg.py:280) and its repr in the logs."""

    __slots__ = ("arr",)

    def __init__(self, order: np.ndarray):
        self.arr = order

    # set(seq) depends only on seq: a P re-sent to many ranks (or to one
    # rank by several) arrives as the same wire array, so the order of the
    # last few distinct sequences is kept (keyed by the bytes, verified by
    # comparison; the arrays are never written in place)
    # (one memo for the class: LocalWorld's thread scheduler runs ranks in
    # threads, so lookups and evictions hold _memo_lock)
    _memo: Dict[tuple, tuple] = {}
    _memo_lock = threading.Lock()
    _MEMO_MAX = 64

    @classmethod
    def build(cls, seq) -> "PSet":
        seq = np.ascontiguousarray(seq, dtype=np.int64)
        key = (len(seq), hash(seq.tobytes()))
        with cls._memo_lock:
            hit = cls._memo.get(key)
        if hit is not None and np.array_equal(hit[0], seq):
            return cls(hit[1])
        out = np.empty(max(len(seq), 1), np.int64)
        got = C.c_int64()
        call("qba_host_pyset_order", seq.ctypes.data, len(seq), out.ctypes.data, C.byref(got))
        order = out[:got.value]
        with cls._memo_lock:
            while len(cls._memo) >= cls._MEMO_MAX:
                cls._memo.pop(next(iter(cls._memo)))
            cls._memo[key] = (seq.copy(), order)
        return cls(order)

    def __len__(self) -> int:
        return len(self.arr)

    def __iter__(self):
        return iter(self.arr.tolist())

    def clear(self) -> None:
        self.arr = self.arr[:0]

    def __repr__(self) -> str:
        return "{" + ", ".join(map(str, self.arr.tolist())) + "}" if len(self.arr) else "set()"


class PTuple:
    """An L tuple held as its int64 array; hashes and compares as the Python
    tuple of the same ints, so a set of them orders and de-duplicates as
    tfg.py's set of tuples does (tfg.py:189, 260, 291)."""

    __slots__ = ("arr", "_h")

    def __init__(self, arr: np.ndarray):
        self.arr = arr
        h = C.c_int64()
        call("qba_host_pytuple_hash", arr.ctypes.data, len(arr), C.byref(h))
        self._h = h.value

    def __hash__(self) -> int:
        return self._h

    def __eq__(self, other) -> bool:
        if isinstance(other, PTuple):
            return self._h == other._h and len(self.arr) == len(other.arr) and bool(np.array_equal(self.arr, other.arr))
        if isinstance(other, tuple):
            return tuple(self.arr.tolist()) == other
        return NotImplemented

    def __len__(self) -> int:
        return len(self.arr)

    def __iter__(self):
        return iter(self.arr.tolist())

    def __repr__(self) -> str:
        return repr(tuple(self.arr.tolist()))


def make_pset(seq):
    """set(seq) as tfg.py builds it (PSet when the native restatement applies)."""
    if NATIVE_SETS:
        return PSet.build(seq)
    return set(np.asarray(seq, dtype=np.int64).tolist())


def make_tuple(arr: np.ndarray):
    """tuple(arr) as tfg.py builds it (PTuple when the native restatement applies)."""
    arr = np.ascontiguousarray(arr, dtype=np.int64)
    return PTuple(arr) if NATIVE_SETS else tuple(arr.tolist())


class WireCache:
    """Wire arrays of the P sets and L tuples a rank handles, built once per
    object: a packet's P and tuples are re-sent to n - 1 ranks and checked
    once, and every conversion of a 31 K-element set or tuple costs ~0.5 ms
    (n = 11, sizeL = 1e6).  Keyed by id(); the entry holds the object, so the
    id cannot be reused while it is cached; the party clears it once per
    round, so it holds at most one round's packets.  Tuples are immutable; the only
    mutation of a P set is a dishonest rank's ``P.clear()`` (tfg.py:280), which
    the length check catches."""

    def __init__(self):
        self._d: Dict[int, tuple] = {}

    def __call__(self, x) -> np.ndarray:
        e = self._d.get(id(x))
        if e is None or e[0] is not x or len(e[1]) != len(x):
            e = (x, _wire(x))
            self._d[id(x)] = e
        return e[1]

    def put(self, x, arr: np.ndarray) -> None:
        self._d[id(x)] = (x, arr)

    def clear(self) -> None:
        self._d.clear()


def send_pvl(comm, rank, dest, P, v, L, is_biz, log=None, wire=_wire):
    if log:
        log(f"[{'B' if is_biz else ''}{rank} -> {dest}] Sending", (P, (v, L)))
    msgs = [np.array(len(P), dtype=np.int64),
            wire(P),
            np.array(v, dtype=np.int64),
            np.array(len(L), dtype=np.int64)]
    for sub in L:
        msgs.append(np.array(len(sub), dtype=np.int64))
        msgs.append(wire(sub))
    dt = _dt(comm)
    reqs = [comm.Isend([m, dt], dest=dest, tag=t) for t, m in enumerate(msgs, start=1)]
    for r in reqs:
        r.Wait()
    if log:
        log(f"[{'B' if is_biz else ''}{rank} -> {dest}] Sent packet!")


def _recv_array(comm, src, tag, n):
    """Receive n int64 from src; tag None = ANY_TAG of the comm's library."""
    buf = np.empty(n, dtype=np.int64)
    mpi = comm_mod.mpi_of(comm)
    comm.Irecv([buf, mpi.INT], source=src, tag=mpi.ANY_TAG if tag is None else tag).Wait()
    return buf


def recv_pvl(comm, rank, src, wire: Optional["WireCache"] = None):
    """Receive one packet; P and L are rebuilt as sets from the wire order.

    Elements are Python ints (``tolist``): they hash as the reference's
    numpy int64 scalars do, so the sets iterate in the same order, and are
    several times cheaper to hash and convert.  A tuple's wire order is its
    own order, so the received buffer becomes its cached wire array (P's
    iteration order differs from the wire order: the set hop, tfg.py:209)."""
    n_p = int(_recv_array(comm, src, 1, 1)[0])
    P = make_pset(_recv_array(comm, src, 2, n_p))
    v = _recv_array(comm, src, 3, 1)[0]
    n_l = int(_recv_array(comm, src, 4, 1)[0])
    L = set()
    for i in range(n_l):
        ln = int(_recv_array(comm, src, 5 + 2 * i, 1)[0])
        buf = _recv_array(comm, src, 6 + 2 * i, ln)
        t = make_tuple(buf)
        if wire is not None and not NATIVE_SETS:
            wire.put(t, buf)
        L.add(t)
    return P, v, L


# ---------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------
@dataclass
class PartyStats:
    accept: int = 0
    reject: int = 0
    sent: int = 0


class _Locked:
    """Serialises an Engine shared by the threads of a LocalWorld."""

    def __init__(self, engine, lock):
        self._engine, self._lock = engine, lock

    def __getattr__(self, name):
        attr = getattr(self._engine, name)
        if not callable(attr):
            return attr

        def call(*a, **k):
            with self._lock:
                return attr(*a, **k)
        return call


class Party:
    """State of one rank: 0 = the QSD, 1 = commander, >= 2 = lieutenants."""

    def __init__(self, comm, sizeL, nDishonest, engine, rng, log=None, lists=None, seed=0, wire=None):
        self.comm = comm
        self.rank = comm.Get_rank()
        self.n = comm.Get_size() - 1
        self.nq = n_qubits(self.n)
        self.w = 2 ** self.nq
        self.sizeL = sizeL
        self.n_dis = nDishonest
        self.engine = engine
        self.rng = rng
        self.log = log
        self.inject = lists
        self.seed = seed
        self.Vi: set = set()
        self.stats = PartyStats()
        self.li = None  # device row of this rank's list
        self.lc = None  # device row of Lc (commander only)
        self.dishonest = False
        self.dishonest_ids = None
        self._p_cache: Dict[int, List[int]] = {}
        self.wire = WireCache()
        self.tolerate_empty_vi = False  # run_local: record the reference's ValueError
        self.empty_vi_error = False
        # In-process (LocalWorld) with a device engine, rank 0's list sends
        # carry the device rows themselves (comm.DeviceRow, accounted as the
        # wire messages): no lists -> int64-per-bit -> lists round trip.  The
        # reference's wire codec stays for real MPI ranks and wire=True runs.
        if wire is None:
            wire = not (isinstance(comm, comm_mod.LocalComm) and hasattr(engine, "lists_to_bits"))
        self.wire_lists = bool(wire)

    def say(self, *args):
        if self.log:
            self.log(*args)

    # tfg.py:101-125
    def dishonest_comm(self):
        c, n = self.comm, self.n
        if self.rank == 0:
            ids = self.rng.choice(np.arange(1, n + 1), self.n_dis, replace=False)
            reqs = [c.Isend([np.array(i in ids, dtype=np.int64), _dt(c)], dest=i) for i in range(1, n + 1)]
            for r in reqs:
                r.Wait()
            self.dishonest_ids = ids
            return ids
        self.dishonest = bool(_recv_array(c, 0, None, 1)[0])
        self.say(f"[{self.rank}] I'm {'dis' if self.dishonest else ''}honest")
        return self.dishonest

    # tfg.py:132-163
    def particle_comm(self):
        c, n, nq, sl = self.comm, self.n, self.nq, self.sizeL
        if self.rank == 0:
            self.say("|W| =", self.w)
            if self.wire_lists:
                raw = generacionListas(n, sl, nq, self.w, self.engine, self.seed, self.inject)
            else:  # the same messages, each carrying its device row (comm.DeviceRow)
                dev = self._device_lists()
                raw = [comm_mod.DeviceRow(dev[g, :sl], nq * sl) for g in range(n + 1)]
            reqs = [c.Isend([raw[0], _dt(c)], dest=1)]
            reqs += [c.Isend([raw[g], _dt(c)], dest=g) for g in range(1, n + 1)]
            for r in reqs:
                r.Wait()
            return
        buf = (lambda: np.empty(nq * sl, np.int64)) if self.wire_lists else (lambda: comm_mod.RowSlot(nq * sl))
        mine = buf()
        req = c.Irecv([mine, _dt(c)], source=0)  # posted first: gets rawS[0] at rank 1
        if self.rank == 1:
            extra = buf()
            c.Irecv([extra, _dt(c)], source=0).Wait()
            self.lc = self._decode(extra)
        req.Wait()
        self.li = self._decode(mine)

    def _device_lists(self):
        """generacionListas' lists (tfg.py:68-84) left on the device: sampled
        (Philox keyed by entry, ``seed``) or the injected value array."""
        n, sl = self.n, self.sizeL
        if self.inject is None:
            return self.engine.sample(n, self.seed, 0, sl)
        arr = np.asarray(self.inject)
        if arr.shape != (n + 1, sl):
            raise ValueError(f"injected lists must have shape {(n + 1, sl)}")
        # the wire carries nq bits per value (rawS, tfg.py:84; measure_to_ints,
        # tfg.py:128-129): the device rows hold what the wire run decodes
        arr = np.ascontiguousarray(arr.astype(np.int64) & ((1 << self.nq) - 1), dtype=np.uint8)
        return self.engine.to_device(arr)

    def _decode(self, raw):
        if isinstance(raw, comm_mod.RowSlot):  # in-process: the device row itself
            return raw.row
        if hasattr(self.engine, "bits_to_values_host"):  # straight from the receive buffer
            return self.engine.bits_to_values_host(raw, self.sizeL, self.nq)
        return self.engine.bits_to_values(self.engine.to_device(raw), self.sizeL, self.nq)

    # tfg.py:327-330
    def commander_setup(self):
        self.isq = make_pset(self.engine.isq_indices(self.li, self.lc))
        self.say("isQCorr = ", self.isq)
        self.v = self.rng.randint(self.w)
        self.say("v =", self.v)

    def p_for(self, v) -> set:
        """{x for x in isQCorr if Lc[x] == v} in isQCorr's iteration order (tfg.py:182)."""
        key = int(v)
        if key not in self._p_cache:
            self._p_cache[key] = np.asarray(self.engine.select_eq(_wire(self.isq), self.lc, key), dtype=np.int64)
        return make_pset(self._p_cache[key])

    def own_tuple(self, P) -> tuple:
        """tuple(Li[j] for j in P) in this process's iteration order of P (tfg.py:189, 291)."""
        return make_tuple(self.engine.gather(self.li, _wire(P)))

    def check(self, v, L) -> bool:
        ok = consistent(v, L, self.w, self.engine)
        return self._tally(ok)

    def _tally(self, ok: bool) -> bool:
        if ok:
            self.stats.accept += 1
        else:
            self.stats.reject += 1
        return ok

    def _packet_request(self, P, v, L):
        """(order, rows, v) of one received packet for the device check, and
        Cond1 (tfg.py:89-92: every received tuple as long as P)."""
        order = self.wire(P)
        received = list(L)
        same_len = all(len(t) == len(order) for t in received)
        return (order, [self.wire(t) for t in received] if same_len else [], v), same_len

    def precheck(self, inbox):
        """Device checks of a whole round's inbox in ONE round trip
        (qba_check_packets_host), before the packets are processed in order:
        a packet's check depends only on its own P, v and L and this rank's
        list (a dishonest rank's mutations in lieu_broadcast touch only the
        objects of the packet being re-sent), so checking them first changes
        nothing the reference observes.  None when the engine has no batched
        call (the CPU test engine) or for count mode."""
        batch = getattr(self.engine, "check_packets", None)
        if batch is None or not inbox:
            return [None] * len(inbox)
        reqs, lens = zip(*(self._packet_request(P, v, L) for P, v, L in inbox))
        return [(make_tuple(arr) if NATIVE_SETS else own, ok, same, arr)
                for (own, ok, arr), same in zip(batch(self.li, list(reqs), self.w), lens)]

    def add_own_and_check(self, P, v, L, pre=None) -> bool:
        """``L.add(tuple(Li[j] for j in P))`` then ``consistent(v, L, w)``
        (tfg.py:189-192, 291-294): the gather and Cond2/Cond3 run on the
        device (one launch per packet; a round's packets share one host
        round trip, see precheck); Cond1 and the set bookkeeping stay here."""
        if pre is not None:
            own, ok, same_len, arr = pre
            if not NATIVE_SETS:
                self.wire.put(own, arr)  # its wire array, if it is re-sent (no re-conversion)
            L.add(own)
            return self._tally(ok and same_len)
        fast = getattr(self.engine, "check_packet", None)
        if fast is None:  # engines without the fused call (the CPU test engine)
            L.add(self.own_tuple(P))
            return self.check(v, L)
        (order, rows, _), same_len = self._packet_request(P, v, L)
        own, ok = fast(self.li, order, rows, v, self.w)
        if NATIVE_SETS:
            own = make_tuple(np.array(own, dtype=np.int64))
        L.add(own)
        return self._tally(ok and same_len)

    def send(self, dest, P, v, L):
        self.stats.sent += 1
        send_pvl(self.comm, self.rank, dest, P, v, L, self.dishonest, self.log, self.wire)

    def recv(self, src):
        # the wire arrays of the received P / tuples stay cached until the
        # round is over (Party.run clears the cache at each round start and
        # comm_broadcast before its receive): a round's inbox is drained
        # first and its packets are checked and re-sent afterwards
        return recv_pvl(self.comm, self.rank, src, self.wire)

    # tfg.py:166-196
    def comm_broadcast(self):
        if self.rank == 1:
            v = self.v
            if self.dishonest:
                v1 = self.rng.randint(self.w)
                v2 = self.rng.randint(self.w)
                while v2 == v1:
                    v2 = self.rng.randint(self.w)
            for dest in range(2, self.n + 1):
                if self.dishonest:
                    v = v1 if dest <= int((self.n + 1) / 2) else v2
                self.send(dest, self.p_for(v), v, set())
        elif self.rank > 1:
            self.wire.clear()
            P, v, L = self.recv(1)
            ok = self.add_own_and_check(P, v, L)
            self.say(f"[{self.rank}] L = {L}")
            if ok:
                self.Vi.add(v)
                self.lieu_broadcast(P, v, L)

    # tfg.py:266-286
    def lieu_broadcast(self, P, v, L):
        for dest in range(2, self.n + 1):
            if dest == self.rank:
                continue
            go = 1
            if self.dishonest:
                action = self.rng.randint(4)
                if action == 0:
                    go = self.rng.randint(2)
                    self.say(f"The action for general {self.rank} is: maybe not sending inf {go}")
                elif action == 1:
                    v = self.rng.randint(self.n + 1)
                    self.say(f"The action for general {self.rank} is: sending order {v}")
                elif action == 2:
                    P.clear()
                    self.say(f"The action for general {self.rank} is: empty P {P}")
                else:
                    L.clear()
                    self.say(f"The action for general {self.rank} is: empy L {L}")
            if go:
                self.send(dest, P, v, L)

    # tfg.py:289-300
    def lieu_receive(self, P, v, L, rnd, pre=None):
        if self.add_own_and_check(P, v, L, pre) and v not in self.Vi and len(L) == rnd + 1:
            self.Vi.add(v)
            if rnd <= self.n_dis:
                self.lieu_broadcast(P, v, L)

    # tfg.py:309-363
    def run(self) -> Optional[dict]:
        c = self.comm
        self.dishonest_comm()
        self.particle_comm()
        self.v = None
        if self.rank == 1:
            self.commander_setup()
        self.comm_broadcast()
        c.Barrier()
        mpi = comm_mod.mpi_of(c)
        status = mpi.Status()
        for rnd in range(1, self.n_dis + 2):
            if self.rank > 1:
                self.wire.clear()  # the previous round's packets are done with
                inbox = []
                while c.Iprobe(source=mpi.ANY_SOURCE, status=status):
                    inbox.append(self.recv(status.Get_source()))
                for (P, v, L), pre in zip(inbox, self.precheck(inbox)):
                    self.lieu_receive(P, v, L, rnd, pre)
            c.Barrier()
        if self.rank > 1 and not self.dishonest:
            self.say(f"[{self.rank}] V{self.rank} = {self.Vi}")
        if self.rank != 0:
            try:
                d = decide_order(self.Vi, self.v, self.rank == 1)
            except ValueError:  # min(set()) on an empty V_i (tfg.py:306)
                if not self.tolerate_empty_vi:
                    raise
                self.empty_vi_error, d = True, -1
            c.Send([np.array(d, dtype=np.int64), _dt(c)], dest=0)
            return None
        result = np.empty(self.n, dtype=np.int64)
        for src in range(1, self.n + 1):
            result[src - 1] = _recv_array(c, src, None, 1)[0]
        ids = self.dishonest_ids
        honest = {int(result[i]) for i in range(self.n) if i + 1 not in ids}
        self.say("Decisions:", result)
        self.say("Dishonests:", ids)
        self.say("Success:", len(honest) == 1)
        return {"decisions": result.tolist(), "dishonest": sorted(int(x) for x in ids),
                "success": len(honest) == 1}


def QBA(sizeL, nDishonest, engine=None, comm=None, rng=None, log=print, lists=None, seed=0):
    """One rank of the protocol (tfg.py:309-363): call it on every rank.

    ``comm`` defaults to ``mpi4py.MPI.COMM_WORLD``; ``rng`` to ``np.random``
    (the reference's global generator); ``lists`` injects (n+1, sizeL) values
    in place of sampling.  Returns the result dict on rank 0, None elsewhere.
    """
    if comm is None:
        mpi = comm_mod.mpi_world()
        if mpi is None:
            raise RuntimeError("not an mpiexec launch (and no mpi4py): use run_local() for an in-process run")
        comm = mpi.COMM_WORLD
    party = Party(comm, sizeL, nDishonest, engine, rng if rng is not None else np.random, log, lists, seed)
    return party.run()


@dataclass
class LocalRun:
    result: Optional[dict]
    V: Dict[int, List[int]] = field(default_factory=dict)
    accept: List[int] = field(default_factory=list)
    reject: List[int] = field(default_factory=list)
    sent: List[int] = field(default_factory=list)
    messages: int = 0
    bytes: int = 0
    error: Optional[str] = None
    error_ranks: List[int] = field(default_factory=list)


_RS_POOL = threading.local()


def _rank_rng(seed: int, rank: int) -> np.random.RandomState:
    """The stream of ``np.random.RandomState(seed)`` without building one: a
    RandomState per (thread, rank) is reseeded (legacy MT19937 seeding, the
    same state as the constructor's, Gaussian cache cleared).  Constructing
    one costs ~0.15-0.2 ms -- four per configs[0] run, a fifth of its wall."""
    pool = getattr(_RS_POOL, "rs", None)
    if pool is None:
        pool = _RS_POOL.rs = {}
    rs = pool.get(rank)
    if rs is None:
        rs = pool[rank] = np.random.RandomState()
    rs.seed(seed)
    return rs


def run_local(n_parties: int, sizeL: int, nDishonest: int, engine, seed: int = 0,
              lists: Optional[np.ndarray] = None, log: Optional[Callable] = None,
              list_seed: Optional[int] = None, timeout: float = 120.0,
              party_cls=None, party_kwargs: Optional[dict] = None) -> LocalRun:
    """Run all n+1 ranks in-process on a LocalWorld.

    Rank r draws from ``np.random.RandomState(seed*1000 + r)`` (the fixtures'
    convention).  A lieutenant whose V_i is empty raises ValueError in
    decide_order exactly like the reference; here it is recorded in
    ``error``/``error_ranks`` and the run completes with decision -1.
    """
    world = comm_mod.LocalWorld(n_parties + 1, timeout=timeout)
    shared = _Locked(engine, threading.RLock())
    parties: List[Optional[Party]] = [None] * (n_parties + 1)

    def body(c):
        rs = _rank_rng(seed * 1000 + c.rank, c.rank)
        p = (party_cls or Party)(c, sizeL, nDishonest, shared, rs, log, lists,
                                 seed if list_seed is None else list_seed, **(party_kwargs or {}))
        p.tolerate_empty_vi = True
        parties[c.rank] = p
        return p.run()

    res = world.run(body)
    out = LocalRun(result=res[0], messages=world.sent_messages, bytes=world.sent_bytes)
    for p in parties:
        out.accept.append(p.stats.accept)
        out.reject.append(p.stats.reject)
        out.sent.append(p.stats.sent)
        if p.rank > 1 and not p.dishonest:
            out.V[p.rank] = sorted(int(x) for x in p.Vi)
    out.error_ranks = [p.rank for p in parties if p.empty_vi_error]
    if out.error_ranks:
        out.error = "ValueError"
    return out
