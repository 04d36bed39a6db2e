"""mpi4py-free MPI transport: a ctypes binding to MPICH's ``libmpi.so``.

The reference runs under ``mpiexec -n <nParties+1> python tfg.py ...`` with
mpi4py (tfg.py:7).  mpi4py is not installed in this image, MPICH is
(``/opt/conda/lib/libmpi.so``, ``/opt/conda/bin/mpiexec``), so this module
binds the C library directly and exposes exactly the mpi4py subset the
protocol uses ("NCCL/collective call sites"):

=======================  ===========================  =========================
mpi4py                   here                         reference call sites
=======================  ===========================  =========================
``COMM_WORLD``           :data:`MPI.COMM_WORLD`       tfg.py:311-313
``Get_rank/Get_size``    ``Comm.Get_rank/Get_size``   tfg.py:311-313
``Isend([buf, INT])``    ``Comm.Isend``               tfg.py:110, 142, 145, 206-223
``Irecv([buf, INT])``    ``Comm.Irecv``               tfg.py:118, 152, 156, 234-257
``Send / Recv``          ``Comm.Send / Comm.Recv``    tfg.py:355, 358
``Iprobe``               ``Comm.Iprobe``              tfg.py:341
``Barrier``              ``Comm.Barrier``             tfg.py:335, 348
``Request.Wait``         ``Request.Wait``             tfg.py:113-114, 227-228 ...
``Status.Get_source``    ``Status.Get_source``        tfg.py:342
``INT / ANY_SOURCE``     MPICH's integer handles      tfg.py:110, 341
=======================  ===========================  =========================

Buffers follow mpi4py's ``[array, datatype]`` convention: the element count
is ``array.nbytes // datatype.size``.  The reference declares its int64
arrays as ``MPI.INT`` (so it sends twice as many 4-byte elements); that
round-trips the raw bytes, and it is kept as is.

Handles are MPICH's ABI (mpi.h of MPICH 3.x): ``MPI_Comm`` and
``MPI_Datatype`` are ``int``, ``MPI_Request`` is ``int``, ``MPI_Status`` is
five ints with the source and tag at indices 2 and 3, ``MPI_ANY_SOURCE`` is
-2 and ``MPI_ANY_TAG`` -1 (tests/test_mpi.py checks them against the
installed mpi.h).
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
from typing import Optional

import numpy as np

LIB_CANDIDATES = (os.environ.get("QBA_MPI_LIB", ""), "/opt/conda/lib/libmpi.so.12", "/opt/conda/lib/libmpi.so",
                  "libmpi.so.12", "libmpi.so")

# MPICH ABI constants (mpi.h)
COMM_WORLD_HANDLE = 0x44000000
ANY_SOURCE = -2
ANY_TAG = -1
SUCCESS = 0
_STATUS_IGNORE = C.c_void_p(1)


class Datatype:
    def __init__(self, name: str, handle: int, size: int):
        self.name, self.handle, self.size = name, handle, size

    def Get_size(self) -> int:
        return self.size

    def __repr__(self) -> str:  # pragma: no cover - cosmetic
        return f"<MPI datatype {self.name}>"


INT = Datatype("MPI_INT", 0x4C000405, 4)
LONG = Datatype("MPI_LONG", 0x4C000807, 8)
INT64_T = Datatype("MPI_INT64_T", 0x4C00083A, 8)
BYTE = Datatype("MPI_BYTE", 0x4C00010D, 1)


class _CStatus(C.Structure):
    _fields_ = [("count_lo", C.c_int), ("count_hi_and_cancelled", C.c_int), ("MPI_SOURCE", C.c_int),
                ("MPI_TAG", C.c_int), ("MPI_ERROR", C.c_int)]


class MPIError(RuntimeError):
    pass


_lib: Optional[C.CDLL] = None


def _load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    err = None
    for path in LIB_CANDIDATES:
        if not path:
            continue
        try:
            lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
            break
        except OSError as exc:  # try the next candidate
            err = exc
    else:
        raise MPIError(f"no MPICH libmpi.so found ({err})")
    i, p = C.c_int, C.c_void_p
    sig = {
        "MPI_Initialized": [C.POINTER(i)], "MPI_Init": [p, p], "MPI_Finalized": [C.POINTER(i)],
        "MPI_Finalize": [], "MPI_Comm_rank": [i, C.POINTER(i)], "MPI_Comm_size": [i, C.POINTER(i)],
        "MPI_Isend": [p, i, i, i, i, i, C.POINTER(i)], "MPI_Irecv": [p, i, i, i, i, i, C.POINTER(i)],
        "MPI_Send": [p, i, i, i, i, i], "MPI_Recv": [p, i, i, i, i, i, p],
        "MPI_Wait": [C.POINTER(i), p], "MPI_Test": [C.POINTER(i), C.POINTER(i), p],
        "MPI_Iprobe": [i, i, i, C.POINTER(i), p], "MPI_Barrier": [i],
        "MPI_Get_count": [p, i, C.POINTER(i)], "MPI_Abort": [i, i],
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes, fn.restype = args, C.c_int
    _lib = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != SUCCESS:
        raise MPIError(f"{what} failed with MPI error code {rc}")


def _init() -> C.CDLL:
    lib = _load()
    flag = C.c_int(0)
    _check(lib.MPI_Initialized(C.byref(flag)), "MPI_Initialized")
    if not flag.value:
        _check(lib.MPI_Init(None, None), "MPI_Init")
        atexit.register(_finalize)
    return lib


def _finalize() -> None:
    lib = _load()
    done = C.c_int(0)
    lib.MPI_Finalized(C.byref(done))
    if not done.value:
        lib.MPI_Finalize()


def _buffer(buf):
    """mpi4py-style [array, datatype] (or a bare array as bytes) -> (ptr, count, handle, keepalive)."""
    if isinstance(buf, (list, tuple)):
        arr, dt = buf[0], (buf[1] if len(buf) > 1 else BYTE)
    else:
        arr, dt = buf, BYTE
    if not isinstance(arr, np.ndarray):
        arr = np.asarray(arr)
    if not arr.flags.c_contiguous:
        raise MPIError("MPI buffers must be C-contiguous numpy arrays")
    if arr.nbytes % dt.size:
        raise MPIError(f"{arr.nbytes} bytes is not a whole number of {dt.name}")
    return C.c_void_p(arr.ctypes.data), arr.nbytes // dt.size, dt.handle, arr


class Status:
    """``mpi4py.MPI.Status`` subset."""

    def __init__(self) -> None:
        self._s = _CStatus()

    def Get_source(self) -> int:
        return self._s.MPI_SOURCE

    def Get_tag(self) -> int:
        return self._s.MPI_TAG

    def Get_count(self, datatype: Datatype = BYTE) -> int:
        n = C.c_int()
        _check(_load().MPI_Get_count(C.byref(self._s), datatype.handle, C.byref(n)), "MPI_Get_count")
        return n.value


def _status_ptr(status: Optional[Status]):
    return C.byref(status._s) if status is not None else _STATUS_IGNORE


class Request:
    def __init__(self, handle: C.c_int, keep) -> None:
        self._h = handle
        self._keep = keep  # the buffer must outlive the operation

    def Wait(self, status: Optional[Status] = None) -> None:
        _check(_load().MPI_Wait(C.byref(self._h), _status_ptr(status)), "MPI_Wait")
        self._keep = None

    def Test(self, status: Optional[Status] = None) -> bool:
        flag = C.c_int(0)
        _check(_load().MPI_Test(C.byref(self._h), C.byref(flag), _status_ptr(status)), "MPI_Test")
        if flag.value:
            self._keep = None
        return bool(flag.value)


class Comm:
    """``mpi4py.MPI.Comm`` subset over an MPICH communicator handle."""

    def __init__(self, handle: int) -> None:
        self.handle = handle

    @property
    def mpi(self) -> "_Module":
        """The constants that go with this communicator (comm.mpi_of)."""
        return load()

    def Get_rank(self) -> int:
        r = C.c_int()
        _check(_init().MPI_Comm_rank(self.handle, C.byref(r)), "MPI_Comm_rank")
        return r.value

    def Get_size(self) -> int:
        s = C.c_int()
        _check(_init().MPI_Comm_size(self.handle, C.byref(s)), "MPI_Comm_size")
        if self.handle == COMM_WORLD_HANDLE:
            check_world_size(s.value)
        return s.value

    def Isend(self, buf, dest: int, tag: int = 0) -> Request:
        ptr, count, dt, keep = _buffer(buf)
        h = C.c_int()
        _check(_init().MPI_Isend(ptr, count, dt, dest, tag, self.handle, C.byref(h)), "MPI_Isend")
        return Request(h, keep)

    def Irecv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG) -> Request:
        ptr, count, dt, keep = _buffer(buf)
        h = C.c_int()
        _check(_init().MPI_Irecv(ptr, count, dt, source, tag, self.handle, C.byref(h)), "MPI_Irecv")
        return Request(h, keep)

    def Send(self, buf, dest: int, tag: int = 0) -> None:
        ptr, count, dt, _ = _buffer(buf)
        _check(_init().MPI_Send(ptr, count, dt, dest, tag, self.handle), "MPI_Send")

    def Recv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> None:
        ptr, count, dt, _ = _buffer(buf)
        _check(_init().MPI_Recv(ptr, count, dt, source, tag, self.handle, _status_ptr(status)), "MPI_Recv")

    def Iprobe(self, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> bool:
        flag = C.c_int(0)
        _check(_init().MPI_Iprobe(source, tag, self.handle, C.byref(flag), _status_ptr(status)), "MPI_Iprobe")
        return bool(flag.value)

    def Barrier(self) -> None:
        _check(_init().MPI_Barrier(self.handle), "MPI_Barrier")

    def Abort(self, code: int = 1) -> None:
        _init().MPI_Abort(self.handle, code)


class _Module:
    """Module-like namespace with mpi4py.MPI's names (``from ... import MPI``)."""

    INT, LONG, INT64_T, BYTE = INT, LONG, INT64_T, BYTE
    ANY_SOURCE, ANY_TAG = ANY_SOURCE, ANY_TAG
    Status = Status
    Request = Request
    Comm = Comm

    def __init__(self) -> None:
        self.COMM_WORLD = Comm(COMM_WORLD_HANDLE)

    @staticmethod
    def Finalize() -> None:
        _finalize()


MPI: Optional[_Module] = None


def load() -> _Module:
    """The binding as an ``MPI`` namespace (MPI_Init on first communicator use)."""
    global MPI
    if MPI is None:
        _load()
        MPI = _Module()
    return MPI


def launched_by_mpiexec() -> bool:
    """True when this process is a rank of an MPICH mpiexec (Hydra/PMI)
    launch.  The binding is MPICH's ABI only (libmpi.so.12, integer handles):
    an Open MPI launch (OMPI_COMM_WORLD_SIZE) is not recognised here, and
    :func:`check_world_size` refuses a world whose size disagrees with the
    launcher's, instead of running N independent single-rank copies."""
    return any(k in os.environ for k in ("PMI_RANK", "PMI_SIZE", "PMI_FD", "MPI_LOCALRANKID"))


def check_world_size(size: int) -> None:
    """Fail loudly when MPI_Init produced a world that is not the one the
    launcher started (e.g. a singleton init under a foreign launcher)."""
    for key in ("PMI_SIZE", "OMPI_COMM_WORLD_SIZE"):
        want = os.environ.get(key)
        if want is not None and int(want) != size:
            raise MPIError(f"MPI_Comm_size is {size} but {key}={want}: this binding speaks MPICH's ABI "
                           "and was not launched by an MPICH mpiexec")
