"""Process-group transport for the protocol host.

The reference runs one MPI process per party and talks through the mpi4py
point-to-point subset listed in SURVEY.md §2 (Isend/Irecv/Send/Recv/Iprobe/
Barrier, reference tfg.py:101-163, 199-263, 335-358).  This module offers:

* :func:`mpi_world` -- the real ``mpi4py.MPI`` module when it is importable
  (``mpiexec -n <n+1> python -m ...tfg <sizeL> <nDis>``);
* :class:`LocalWorld` -- an in-process world where every rank is a thread.
  It implements exactly the mpi4py calls the protocol uses, with MPI's
  matching rules (posted receives are matched in posting order, messages
  from one source are non-overtaking) and one deliberate, documented choice
  that removes the reference's round race:

      ``Iprobe`` only sees messages sent before the last ``Barrier`` the
      probing rank passed ("barrier-epoch delivery"), and among those it
      reports the one with the lowest (epoch, source, sequence).

  Direct receives (``Irecv``/``Recv`` with an explicit source) are never
  gated, so the commander -> lieutenant hand-off of step 3a works inside one
  epoch as it does under real MPI.

The same world backs the in-process CLI and the golden-fixture generator
(tests/golden/gen_golden.py runs the reference's own ``QBA`` on it), so both
sides of a parity test see the same delivery order.
"""
from __future__ import annotations

import threading
import types
from typing import Any, Callable, List, Optional

import numpy as np

ANY_SOURCE = -1
ANY_TAG = -1


class _Datatype:
    def __init__(self, name: str):
        self.name = name

    def __repr__(self) -> str:  # pragma: no cover - cosmetic
        return f"<Datatype {self.name}>"


INT = _Datatype("MPI_INT")


class Status:
    """Subset of ``mpi4py.MPI.Status``."""

    def __init__(self) -> None:
        self.source = ANY_SOURCE
        self.tag = ANY_TAG

    def Get_source(self) -> int:
        return self.source

    def Get_tag(self) -> int:
        return self.tag


class DeviceRow:
    """In-process payload of one of rank 0's list sends (tfg.py:142-161): the
    device row itself instead of the reference's one-int64-per-bit encoding
    of it.  It is accounted as the wire message it stands for -- ``nbytes``
    and ``size`` of the rawS row -- so a LocalWorld run reports the same
    messages and bytes as the wire run.  Received only into a RowSlot."""

    __slots__ = ("row", "nbytes", "size")

    def __init__(self, row, size: int, itemsize: int = 8):
        self.row, self.size, self.nbytes = row, int(size), int(size) * itemsize


class RowSlot:
    """Receive buffer of a DeviceRow message (``size`` wire items, as the
    np.empty(nq * sizeL) buffer it replaces); ``row`` after delivery."""

    __slots__ = ("row", "size")

    def __init__(self, size: int):
        self.row, self.size = None, int(size)


def _payload(buf):
    arr = buf[0] if isinstance(buf, (list, tuple)) else buf
    if isinstance(arr, DeviceRow):
        return arr
    return np.array(arr, copy=True)


class _Msg:
    __slots__ = ("src", "tag", "data", "epoch", "seq")

    def __init__(self, src, tag, data, epoch, seq):
        self.src, self.tag, self.data, self.epoch, self.seq = src, tag, data, epoch, seq


class _Posted:
    __slots__ = ("src", "tag", "buf", "done", "status")

    def __init__(self, src, tag, buf):
        self.src, self.tag, self.buf = src, tag, buf
        self.done = False
        self.status = Status()


def _matches(want_src, want_tag, src, tag) -> bool:
    return (want_src in (ANY_SOURCE, src)) and (want_tag in (ANY_TAG, tag))


def _deliver(post: _Posted, msg: _Msg) -> None:
    dst = post.buf[0] if isinstance(post.buf, (list, tuple)) else post.buf
    if isinstance(msg.data, DeviceRow) or isinstance(dst, RowSlot):
        if not (isinstance(msg.data, DeviceRow) and isinstance(dst, RowSlot)):
            raise TypeError("a device-row message is received into a RowSlot (and only such a message)")
        if msg.data.size > dst.size:
            raise RuntimeError(f"message truncated: {msg.data.size} items into a buffer of {dst.size}")
        dst.row = msg.data.row
        post.status.source, post.status.tag = msg.src, msg.tag
        post.done = True
        return
    flat = dst.reshape(-1)
    src = msg.data.reshape(-1)
    if src.size > flat.size:
        raise RuntimeError(f"message truncated: {src.size} items into a buffer of {flat.size}")
    flat[: src.size] = src
    post.status.source, post.status.tag = msg.src, msg.tag
    post.done = True


class Request:
    def __init__(self, world: "LocalWorld", post: Optional[_Posted]):
        self._world = world
        self._post = post

    def Test(self) -> bool:
        return self._post is None or self._post.done

    def Wait(self, status: Optional[Status] = None) -> None:
        if self._post is None:
            return
        w = self._world
        if w.coop:
            w._coop_wait(lambda: self._post.done)
        else:
            with w._cv:
                ok = w._cv.wait_for(lambda: self._post.done or w._failed, timeout=w.timeout)
                if w._failed:
                    raise RuntimeError("LocalWorld aborted by another rank")
                if not ok:
                    w._fail()
                    raise TimeoutError("LocalWorld receive timed out (protocol deadlock?)")
        if status is not None:
            status.source, status.tag = self._post.status.source, self._post.status.tag


class LocalComm:
    """One rank's view of a :class:`LocalWorld` (the ``COMM_WORLD`` subset)."""

    mpi = None  # set below: the in-process constants (LOCAL_MPI)

    def __init__(self, world: "LocalWorld", rank: int):
        self.world = world
        self.rank = rank
        self.epoch = 0

    def Get_size(self) -> int:
        return self.world.size

    def Get_rank(self) -> int:
        return self.rank

    # -- point to point -------------------------------------------------
    def Isend(self, buf, dest: int, tag: int = 0) -> Request:
        self.world._send(self.rank, dest, tag, _payload(buf), self.epoch)
        return Request(self.world, None)

    def Send(self, buf, dest: int, tag: int = 0) -> None:
        self.Isend(buf, dest, tag)

    def Irecv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG) -> Request:
        return Request(self.world, self.world._post(self.rank, source, tag, buf))

    def Recv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> None:
        self.Irecv(buf, source, tag).Wait(status)

    def Iprobe(self, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> bool:
        return self.world._probe(self.rank, source, tag, self.epoch, status)

    def Barrier(self) -> None:
        w = self.world
        if w.coop:
            gen = w._bar_gen
            w._bar_count += 1
            if w._bar_count == w.size:
                w._bar_count = 0
                w._bar_gen += 1
            else:
                w._coop_wait(lambda: w._bar_gen != gen)
        else:
            try:
                w._barrier.wait(timeout=w.timeout)
            except threading.BrokenBarrierError:
                w._fail()
                raise RuntimeError("LocalWorld barrier broken (a rank failed or timed out)")
        self.epoch += 1


def _greenlet():
    try:
        import greenlet  # type: ignore
        return greenlet
    except ImportError:
        return None


class LocalWorld:
    """An in-process MPI world of ``size`` ranks.

    Two schedulers, same delivery semantics (so the same results):
    * ``coop`` (default when the ``greenlet`` module is importable and
      QBA_LOCAL_THREADS is unset): every rank is a greenlet of ONE thread and
      a blocking call (an unmatched receive, a barrier) switches to the next
      runnable rank -- no thread wake-ups and no GIL hand-offs around the
      engine's device calls; a world where no rank can run is a deadlock
      (RuntimeError);
    * threads: one thread per rank (the rounds as concurrent processes),
      with ``timeout`` on every blocking call.
    """

    def __init__(self, size: int, timeout: float = 120.0, coop: Optional[bool] = None):
        if size < 1:
            raise ValueError("world size must be >= 1")
        import os
        if coop is None:
            coop = _greenlet() is not None and os.environ.get("QBA_LOCAL_THREADS") != "1"
        self.coop = bool(coop)
        self._waiting: List[Optional[Callable[[], bool]]] = [None] * size
        self._bar_count = 0
        self._bar_gen = 0
        self._sched = None
        self.size = size
        self.timeout = timeout
        self._cv = threading.Condition()
        self._barrier = threading.Barrier(size)
        self._unexpected: List[List[_Msg]] = [[] for _ in range(size)]
        self._posted: List[List[_Posted]] = [[] for _ in range(size)]
        self._seq = 0
        self._failed = False
        self.comms = [LocalComm(self, r) for r in range(size)]
        self.sent_messages = 0
        self.sent_bytes = 0

    # -- internals (all under self._cv) ---------------------------------
    def _fail(self) -> None:
        with self._cv:
            self._failed = True
            self._cv.notify_all()
        self._barrier.abort()

    def _send(self, src, dest, tag, data, epoch) -> None:
        if not 0 <= dest < self.size:
            raise ValueError(f"invalid destination rank {dest}")
        with self._cv:
            self._seq += 1
            self.sent_messages += 1
            self.sent_bytes += data.nbytes
            msg = _Msg(src, tag, data, epoch, self._seq)
            for i, post in enumerate(self._posted[dest]):
                if _matches(post.src, post.tag, src, tag):
                    del self._posted[dest][i]
                    _deliver(post, msg)
                    self._cv.notify_all()
                    return
            self._unexpected[dest].append(msg)

    def _post(self, rank, source, tag, buf) -> _Posted:
        post = _Posted(source, tag, buf)
        with self._cv:
            q = self._unexpected[rank]
            for i, msg in enumerate(q):  # arrival order == non-overtaking per source
                if _matches(source, tag, msg.src, msg.tag):
                    del q[i]
                    _deliver(post, msg)
                    return post
            self._posted[rank].append(post)
        return post

    def _probe(self, rank, source, tag, epoch, status) -> bool:
        with self._cv:
            best = None
            for msg in self._unexpected[rank]:
                if msg.epoch >= epoch or not _matches(source, tag, msg.src, msg.tag):
                    continue
                key = (msg.epoch, msg.src, msg.seq)
                if best is None or key < best[0]:
                    best = (key, msg)
            if best is None:
                return False
            if status is not None:
                status.source, status.tag = best[1].src, best[1].tag
            return True

    # -- cooperative scheduling (coop) ------------------------------------
    def _coop_wait(self, ready: Callable[[], bool]) -> None:
        """Block the calling rank's greenlet until ready() holds."""
        if ready():
            return
        r = _tls.comm.rank
        self._waiting[r] = ready
        self._sched.switch()
        if self._failed:
            raise RuntimeError("LocalWorld aborted by another rank")

    def _run_coop(self, fn) -> List[Any]:
        glet = _greenlet()
        results: List[Any] = [None] * self.size
        errors: List[Optional[BaseException]] = [None] * self.size
        self._sched = glet.getcurrent()

        def body(r: int) -> None:
            try:
                results[r] = fn(self.comms[r])
            except BaseException as exc:  # noqa: BLE001 - re-raised below
                errors[r] = exc
                self._failed = True

        lets = [glet.greenlet(lambda r=r: body(r), parent=self._sched) for r in range(self.size)]
        prev = getattr(_tls, "comm", None)
        try:
            while True:
                live = [r for r in range(self.size) if not lets[r].dead]
                if not live:
                    break
                ran = False
                for r in live:
                    w = self._waiting[r]
                    if w is not None and not (self._failed or w()):
                        continue
                    self._waiting[r] = None
                    _tls.comm = self.comms[r]
                    lets[r].switch()
                    ran = True
                if not ran:
                    self._failed = True
                    for r in live:
                        errors[r] = errors[r] or RuntimeError("LocalWorld deadlock: no rank can proceed")
                    break
        finally:
            _tls.comm = prev
        primary = [e for e in errors if e is not None and not _is_echo(e)]
        if primary:
            raise primary[0]
        echoes = [e for e in errors if e is not None]
        if echoes:
            raise echoes[0]
        return results

    # -- running ---------------------------------------------------------
    def run(self, fn: Callable[[LocalComm], Any]) -> List[Any]:
        """Run ``fn(comm)`` on every rank in its own thread; return per-rank results.

        The first exception raised by any rank is re-raised (after the other
        ranks are released) as-is, so protocol errors such as the reference's
        ``ValueError`` from ``min(set())`` surface unchanged.
        """
        if self.coop:
            return self._run_coop(fn)
        results: List[Any] = [None] * self.size
        errors: List[Optional[BaseException]] = [None] * self.size

        def body(r: int) -> None:
            _tls.comm = self.comms[r]
            try:
                results[r] = fn(self.comms[r])
            except BaseException as exc:  # noqa: BLE001 - re-raised below
                errors[r] = exc
                self._fail()
            finally:
                _tls.comm = None

        threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.size)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        # Prefer a rank's own error over the "aborted by another rank" echoes.
        primary = [e for e in errors if e is not None and not _is_echo(e)]
        if primary:
            raise primary[0]
        echoes = [e for e in errors if e is not None]
        if echoes:
            raise echoes[0]
        return results


def _is_echo(exc: BaseException) -> bool:
    return isinstance(exc, RuntimeError) and "LocalWorld" in str(exc)


_tls = threading.local()


def current_comm() -> Optional[LocalComm]:
    """The calling thread's rank inside :meth:`LocalWorld.run` (else None)."""
    return getattr(_tls, "comm", None)


def local_mpi_module() -> types.ModuleType:
    """A module object that quacks like ``mpi4py.MPI`` for threads of a LocalWorld.

    ``COMM_WORLD`` resolves to the calling thread's :class:`LocalComm`.
    """
    mod = types.ModuleType("MPI")
    mod.INT = INT
    mod.ANY_SOURCE = ANY_SOURCE
    mod.ANY_TAG = ANY_TAG
    mod.Status = Status

    def __getattr__(name: str):
        if name == "COMM_WORLD":
            comm = current_comm()
            if comm is None:
                raise RuntimeError("COMM_WORLD used outside LocalWorld.run")
            return comm
        raise AttributeError(name)

    mod.__getattr__ = __getattr__  # PEP 562
    return mod


def mpi_world():
    """The MPI module of an ``mpiexec`` launch: ``mpi4py.MPI`` when it is
    importable, else the ctypes MPICH binding (:mod:`.mpi`) when this process
    is a rank of an mpiexec launch; None otherwise (use :class:`LocalWorld`)."""
    try:
        from mpi4py import MPI  # type: ignore
        return MPI
    except ImportError:
        pass
    from . import mpi as mpi_ctypes
    if not mpi_ctypes.launched_by_mpiexec():
        return None
    try:
        return mpi_ctypes.load()
    except mpi_ctypes.MPIError:
        return None


# constants of the in-process world, as an MPI-module-like namespace
LOCAL_MPI = types.SimpleNamespace(INT=INT, ANY_SOURCE=ANY_SOURCE, ANY_TAG=ANY_TAG, Status=Status)
LocalComm.mpi = LOCAL_MPI


def mpi_of(comm):
    """The MPI namespace (INT, ANY_SOURCE, ANY_TAG, Status) that goes with a
    communicator: the protocol must pass the datatypes and wildcards of the
    library that owns the communicator (MPICH's ANY_SOURCE is -2, not -1)."""
    ns = getattr(comm, "mpi", None)
    if ns is not None:
        return ns
    from mpi4py import MPI  # type: ignore  # a real mpi4py communicator
    return MPI


class EpochComm:
    """Barrier-epoch delivery over a real MPI communicator.

    The reference's rounds race: a rank still draining
    ``Iprobe`` in round r can receive packets another rank sent in round r,
    so outcomes under mpiexec depend on timing.  This wrapper gives a real
    MPI run the same deterministic semantics as :class:`LocalWorld` (and as
    the golden fixtures): every message carries its sender's epoch (number of
    barriers passed) in the tag, ``tag + TAG_STRIDE * epoch``, and ``Iprobe``
    reports only messages of earlier epochs, lowest (epoch, source) first;
    within one (epoch, source) MPI's non-overtaking rule keeps the order.
    Receives with an explicit tag after a probe use the probed message's
    epoch; other explicit-tag receives the receiver's own (the protocol's
    direct hand-offs happen inside one epoch).  Opt-in (``--rounds epoch``):
    the default keeps the reference's own racy rounds."""

    TAG_STRIDE = 256
    HEAD_TAG = 1  # first message of every (P, v, L) packet (tfg.py:206)

    def __init__(self, inner, count_traffic: bool = True):
        self.inner = inner
        self.epoch = 0
        self._probed = {}
        self.sent_messages = 0
        self.sent_bytes = 0
        self._count = count_traffic
        m = mpi_of(inner)
        self.mpi = types.SimpleNamespace(INT=m.INT, ANY_SOURCE=m.ANY_SOURCE, ANY_TAG=m.ANY_TAG, Status=m.Status)

    def Get_rank(self) -> int:
        return self.inner.Get_rank()

    def Get_size(self) -> int:
        return self.inner.Get_size()

    def _tally(self, buf) -> None:
        if self._count:
            self.sent_messages += 1
            self.sent_bytes += (buf[0] if isinstance(buf, (list, tuple)) else buf).nbytes

    def Isend(self, buf, dest: int, tag: int = 0):
        self._tally(buf)
        return self.inner.Isend(buf, dest=dest, tag=tag + self.TAG_STRIDE * self.epoch)

    def Send(self, buf, dest: int, tag: int = 0) -> None:
        self._tally(buf)
        self.inner.Send(buf, dest=dest, tag=tag + self.TAG_STRIDE * self.epoch)

    def _tag(self, source, tag):
        if tag == self.mpi.ANY_TAG:
            return tag
        return tag + self.TAG_STRIDE * self._probed.get(source, self.epoch)

    def Irecv(self, buf, source=None, tag=None):
        source = self.mpi.ANY_SOURCE if source is None else source
        tag = self.mpi.ANY_TAG if tag is None else tag
        return self.inner.Irecv(buf, source=source, tag=self._tag(source, tag))

    def Recv(self, buf, source=None, tag=None, status=None) -> None:
        source = self.mpi.ANY_SOURCE if source is None else source
        tag = self.mpi.ANY_TAG if tag is None else tag
        self.inner.Recv(buf, source=source, tag=self._tag(source, tag), status=status)

    def Iprobe(self, source=None, tag=None, status=None) -> bool:
        source = self.mpi.ANY_SOURCE if source is None else source
        tag = self.HEAD_TAG if tag is None or tag == self.mpi.ANY_TAG else tag
        srcs = range(self.Get_size()) if source == self.mpi.ANY_SOURCE else [source]
        st = status if status is not None else self.mpi.Status()
        for e in range(self.epoch):
            for s in srcs:
                if self.inner.Iprobe(source=s, tag=tag + self.TAG_STRIDE * e, status=st):
                    self._probed[st.Get_source()] = e
                    return True
        return False

    def Barrier(self) -> None:
        self.inner.Barrier()
        self.epoch += 1
        # a probe's epoch only names the packet it found; after the barrier
        # every explicit-tag receive uses this rank's own epoch again
        self._probed.clear()
