"""CPU oracle: a plain restatement of the reference's hot-path functions.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this
module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker.

Every function cites the line of ``tfg.py`` (Carl0sGV/TFG---Quantum-
Byzantine-Agreement, mounted at /root/reference during development) whose
behaviour it restates.  Pinning: ``tests/test_oracle_golden.py`` checks each
function against the fixtures that ``tests/golden/gen_golden.py`` produced by
running the reference's own code (with a recording ``qsimov`` stub and the
in-process MPI world), and against the five captured reference logs.
"""
from __future__ import annotations

import itertools
from typing import Iterable, List, Sequence, Tuple

import numpy as np


# ---------------------------------------------------------------------------
# sizes: tfg.py:317-318
# ---------------------------------------------------------------------------
def n_qubits(n_parties: int) -> int:
    """nQubits = ceil(log2(nParties+1))  (tfg.py:317)."""
    return int(np.ceil(np.log2(n_parties + 1)))


def width(n_parties: int) -> int:
    """w = 2**nQubits  (tfg.py:318)."""
    return 2 ** n_qubits(n_parties)


# ---------------------------------------------------------------------------
# resource gate lists: tfg.py:15-40
# ---------------------------------------------------------------------------
def notq_gates(n: int) -> List[Tuple[str, int, int]]:
    """Gate list of notQCorrelated (tfg.py:15-22) as (name, target, control|-1)."""
    nq = n_qubits(n)
    size = (n + 1) * nq
    ops = [("H", t, -1) for t in range(nq, size)]
    ops += [("X", t, t + nq) for t in range(nq)]
    return ops


def q_gates(n: int, perm: Sequence[int]) -> List[Tuple[str, int, int]]:
    """Gate list of qCorrelated (tfg.py:25-40) for the drawn permutation ``perm``
    (``perm[g-1]`` = value given to group g, the shuffled ``rands`` of tfg.py:30-31)."""
    nq = n_qubits(n)
    size = (n + 1) * nq
    ops = [("H", t, -1) for t in range(nq)]
    for g in range(1, n + 1):
        bits = format(int(perm[g - 1]), f"0{nq}b")  # MSB first, tfg.py:34
        ops += [("X", g * nq + j, -1) for j in range(nq) if bits[j] == "1"]
    ops += [("X", t, t % nq) for t in range(nq, size)]
    return ops


# ---------------------------------------------------------------------------
# bit <-> value codec: tfg.py:81-84, 128-129
# ---------------------------------------------------------------------------
def measure_to_ints(raw: Sequence[int], size_l: int, nq: int) -> List[int]:
    """MSB-first nq-bit groups -> ints (tfg.py:128-129)."""
    out = []
    for i in range(size_l):
        v = 0
        for b in raw[i * nq:(i + 1) * nq]:
            v = 2 * v + int(b)
        out.append(v)
    return out


def lists_to_raw(lists: np.ndarray, nq: int) -> np.ndarray:
    """Inverse of measure_to_ints for every group: (n+1, sizeL) values ->
    (n+1, nq*sizeL) int64 bits, the ``rawS`` layout of tfg.py:81-84."""
    lists = np.asarray(lists, dtype=np.int64)
    shifts = np.arange(nq - 1, -1, -1, dtype=np.int64)
    bits = (lists[:, :, None] >> shifts[None, None, :]) & 1
    return bits.reshape(lists.shape[0], -1).astype(np.int64)


# ---------------------------------------------------------------------------
# checks: tfg.py:87-98, 182, 189, 291, 327
# ---------------------------------------------------------------------------
def consistent(v, L, w) -> bool:
    """The three conditions of tfg.py:87-98, restated.

    Cond1 raises StopIteration on an empty L exactly like ``next(iter(L))``.
    """
    tuples = list(L)
    if not tuples:
        raise StopIteration
    n0 = len(tuples[0])
    if any(len(t) != n0 for t in tuples[1:]):
        return False
    for t in tuples:
        for x in t:
            if not (0 <= x <= w) or x == v:
                return False
    for a, b in itertools.combinations(tuples, 2):
        for k in range(n0):
            if a[k] == b[k]:
                return False
    return True


def is_qcorr_indices(l0: np.ndarray, l1: np.ndarray) -> np.ndarray:
    """Sorted positions k with Li[k] != Lc[k]  (tfg.py:327; Li = group 0, Lc = group 1)."""
    return np.nonzero(np.asarray(l0) != np.asarray(l1))[0].astype(np.int64)


def p_filter(order: Iterable[int], lc: np.ndarray, v: int) -> List[int]:
    """Elements of ``order`` (the iteration order of isQCorr) with Lc[x]==v (tfg.py:182)."""
    return [int(x) for x in order if int(lc[x]) == v]


def gather(li: np.ndarray, order: Iterable[int]) -> Tuple[int, ...]:
    """tuple(Li[j] for j in P) in P's iteration order (tfg.py:189, 291)."""
    return tuple(int(li[j]) for j in order)


def decide_order(vi, v, is_comm):
    """tfg.py:303-306 (ValueError from min() on an empty set is preserved)."""
    if is_comm:
        return v
    return min(vi)


def success(decisions: Sequence[int], dishonest_ids: Sequence[int]) -> bool:
    """tfg.py:362-363: honest decisions form a singleton."""
    dis = set(int(d) for d in dishonest_ids)
    honest = {int(decisions[i]) for i in range(len(decisions)) if i + 1 not in dis}
    return len(honest) == 1


# ---------------------------------------------------------------------------
# count mode: histograms every packet's check reduces to
# ---------------------------------------------------------------------------
def counts(lists: np.ndarray, n: int):
    """H[u][g][x], C[u][g][h] (g<h, symmetrised, diagonal = |P_u|) and |P_u|.

    Only Q positions (L0 != L1, tfg.py:327) count; u = Lc[k] = L1[k].
    """
    lists = np.asarray(lists).astype(np.int64)
    w = width(n)
    q = lists[0] != lists[1]
    sub = lists[:, q]
    u = sub[1]
    H = np.zeros((w, n + 1, w), np.int64)
    for g in range(n + 1):
        np.add.at(H, (u, g, sub[g]), 1)
    psz = np.bincount(u, minlength=w).astype(np.int64)
    C = np.zeros((w, n + 1, n + 1), np.int64)
    for g in range(n + 1):
        for h in range(g + 1, n + 1):
            eq = sub[g] == sub[h]
            if eq.any():
                C[:, g, h] = np.bincount(u[eq], minlength=w)
                C[:, h, g] = C[:, g, h]
        C[:, g, g] = psz
    return H, C, psz


# ---------------------------------------------------------------------------
# closed-form sampler: used only to make test inputs
# ---------------------------------------------------------------------------
def closed_form_lists(n: int, size_l: int, rng: np.random.Generator) -> np.ndarray:
    """Lists with the reference's joint law, drawn with numpy (not Philox).

    not-Q position: L0 = L1 ~ U[0,w), L2..Ln iid U[0,w)       (tfg.py:15-22)
    Q position:     L0 = r ~ U[0,w), Lg = r XOR pi(g), pi a uniform
                    permutation of 1..n                        (tfg.py:25-40)
    isQ ~ Bernoulli(1/2)                                       (tfg.py:69)
    """
    w = width(n)
    out = np.empty((n + 1, size_l), np.uint8)
    isq = rng.integers(0, 2, size_l)
    for k in range(size_l):
        if isq[k]:
            r = rng.integers(w)
            perm = rng.permutation(n) + 1
            out[0, k] = r
            out[1:, k] = r ^ perm
        else:
            a = rng.integers(w)
            out[0, k] = out[1, k] = a
            out[2:, k] = rng.integers(0, w, n - 1)
    return out
