"""ctypes loader of oracle/lib/liboracle.so (the C twin in sampler_ref.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product package.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parent / "lib" / "liboracle.so"
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise FileNotFoundError(f"{LIB} missing: run `make -C oracle`")
        _lib = C.CDLL(str(LIB))
        _lib.oracle_counts.restype = C.c_int64
        _lib.oracle_sample_counts.restype = C.c_int64
    return _lib


def _p(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def n_qubits(n: int) -> int:
    return int(n).bit_length()


def philox(ctr: np.ndarray, key: int) -> np.ndarray:
    ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
    out = np.zeros_like(ctr)
    lib().oracle_philox(_p(ctr), C.c_int64(len(ctr)), C.c_uint64(key), _p(out))
    return out


def _prog_args(prog: dict):
    desc = np.ascontiguousarray(prog["desc"], dtype=np.int32)
    pat = np.ascontiguousarray(prog["pat"], dtype=np.uint64)
    apat = np.ascontiguousarray(prog["apat"], dtype=np.uint64)
    thr = np.ascontiguousarray(prog["thr"], dtype=np.uint64)
    keep = (desc, pat, apat, thr)
    return keep, [C.c_int(int(prog["nfac"])), _p(desc), _p(pat), _p(apat), _p(thr)]


def sample(n: int, seed: int, first: int, count: int, prog_notq: dict, prog_q: dict,
           closed: bool = False) -> np.ndarray:
    """Lists of entries [first, first+count); `closed` selects the closed-form
    schedule the engine uses when its program flags say so (n <= 11)."""
    lists = np.zeros((n + 1, max(count, 1)), np.uint8)
    k0, a0 = _prog_args(prog_notq)
    k1, a1 = _prog_args(prog_q)
    lib().oracle_sample(C.c_int(n), C.c_uint64(seed), C.c_uint64(first), C.c_uint64(count),
                        C.c_int(int(closed)), *a0, *a1,
                        _p(lists), C.c_uint64(lists.shape[1]))
    return lists[:, :count]


def counts(lists: np.ndarray, n: int):
    lists = np.ascontiguousarray(lists, dtype=np.uint8)
    w = 1 << n_qubits(n)
    H = np.zeros((w, n + 1, w), np.int64)
    Cc = np.zeros((w, n + 1, n + 1), np.int64)
    P = np.zeros(w, np.int64)
    bad = lib().oracle_counts(C.c_int(n), _p(lists), C.c_uint64(lists.shape[1]),
                              C.c_uint64(lists.shape[1]), _p(H), _p(Cc), _p(P))
    return H, Cc, P, int(bad)


def sample_counts(n: int, seed: int, first: int, count: int, prog_notq: dict, prog_q: dict,
                  closed: bool = False):
    lists = np.zeros((n + 1, max(count, 1)), np.uint8)
    w = 1 << n_qubits(n)
    H = np.zeros((w, n + 1, w), np.int64)
    Cc = np.zeros((w, n + 1, n + 1), np.int64)
    P = np.zeros(w, np.int64)
    k0, a0 = _prog_args(prog_notq)
    k1, a1 = _prog_args(prog_q)
    lib().oracle_sample_counts(C.c_int(n), C.c_uint64(seed), C.c_uint64(first), C.c_uint64(count),
                               C.c_int(int(closed)), *a0, *a1, _p(lists), C.c_uint64(lists.shape[1]), _p(H), _p(Cc), _p(P))
    return lists[:, :count], H, Cc, P


def _counts_buffers(n: int, lead=()):
    w = 1 << n_qubits(n)
    return (np.zeros(lead + (w, n + 1, w), np.int64), np.zeros(lead + (w, n + 1, n + 1), np.int64),
            np.zeros(lead + (w,), np.int64))


def stream_counts(n: int, seed: int, first: int, count: int, prog_notq: dict, prog_q: dict,
                  closed: bool = False):
    """H, C, P, bad over entries [first, first+count) sampled and counted
    without storing the lists (any size)."""
    H, Cc, P = _counts_buffers(n)
    k0, a0 = _prog_args(prog_notq)
    k1, a1 = _prog_args(prog_q)
    lib().oracle_stream_counts.restype = C.c_int64
    bad = lib().oracle_stream_counts(C.c_int(n), C.c_uint64(seed), C.c_uint64(first), C.c_uint64(count),
                                     C.c_int(int(closed)), *a0, *a1, _p(H), _p(Cc), _p(P))
    return H, Cc, P, int(bad)


def stream_row_sums(n: int, seed: int, first: int, count: int, prog_notq: dict, prog_q: dict,
                    closed: bool = False) -> np.ndarray:
    """uint64 [n+1, 2]: per row g, (sum_k L_g[k], sum_k L_g[k] * (k+1)) over the
    lists of entries [first, first+count), k counted from 0 at `first`;
    sampled without storing the lists (any size)."""
    S = np.zeros((n + 1, 2), np.uint64)
    k0, a0 = _prog_args(prog_notq)
    k1, a1 = _prog_args(prog_q)
    lib().oracle_stream_row_sums(C.c_int(n), C.c_uint64(seed), C.c_uint64(first), C.c_uint64(count),
                                 C.c_int(int(closed)), *a0, *a1, _p(S))
    return S


def row_sums(lists: np.ndarray) -> np.ndarray:
    """The same checksum of lists held in memory (uint8 [rows, count])."""
    L = np.asarray(lists, dtype=np.uint64)
    k = np.arange(1, L.shape[1] + 1, dtype=np.uint64)
    return np.stack([L.sum(1), (L * k).sum(1)], axis=1).astype(np.uint64)


def batched_counts(n: int, seed_base: int, n_inst: int, count: int, prog_notq: dict, prog_q: dict,
                   closed: bool = False):
    """Per-instance H, C, P of n_inst independent runs (key seed_base + i,
    entries [0, count)), as [n_inst, ...] arrays."""
    H, Cc, P = _counts_buffers(n, (n_inst,))
    k0, a0 = _prog_args(prog_notq)
    k1, a1 = _prog_args(prog_q)
    lib().oracle_batched_counts(C.c_int(n), C.c_uint64(seed_base), C.c_int64(n_inst), C.c_uint64(count),
                                C.c_int(int(closed)), *a0, *a1, _p(H), _p(Cc), _p(P))
    return H, Cc, P


def threads() -> int:
    return int(lib().oracle_threads())
