"""Closed-form sampler (n <= 11): host-built permutation stage tables and the
oracle's restatement of the schedule.  CPU only (no device calls).

The engine draws pi by forward Fisher-Yates over positions 1..n whose digit
string is the mixed-radix rank R = floor(F * n! / 2^32); R is split into three
table indices (A: positions 1..3 when n >= 8; B, C: the 8-byte window holding
the rest, composed with v_perm_b32).  These tests restate that composition in
Python and check it against the direct Fisher-Yates decode of every rank
(n <= 8) or of 20k ranks (n = 9..11).
"""
import math

import numpy as np
import pytest

import oracle_lib
from conftest import sub


def fy_decode(n, R):
    """Forward Fisher-Yates: digit of position i has radix n-i+1, first most significant."""
    perm = list(range(16))
    div = math.factorial(n)
    for i in range(1, n):
        div //= n - i + 1
        d, R = divmod(R, div)
        perm[i], perm[i + d] = perm[i + d], perm[i]
    return perm[: n + 1]


def tables(n):
    lib = sub("_lib")
    sizes = np.zeros(6, np.int32)
    lib.call("qba_perm_tables", n, None, 0, sizes.ctypes.data_as(lib._pi32))
    words = np.zeros(int(sizes[5]), np.uint32)
    lib.call("qba_perm_tables", n, words.ctypes.data, len(words), sizes.ctypes.data_as(lib._pi32))
    return sizes, words


def vperm(hi, lo, sel):
    """v_perm_b32 restricted to selector bytes 0..7 (byte b of {hi:lo})."""
    src = [(lo >> (8 * b)) & 0xFF for b in range(4)] + [(hi >> (8 * b)) & 0xFF for b in range(4)]
    return sum(src[(sel >> (8 * b)) & 0xFF] << (8 * b) for b in range(4))


def compose(n, sizes, words, R):
    ra, rb, rc, offb, offc, _ = (int(x) for x in sizes)
    iA, rest = divmod(R, rb * rc)
    iB, iC = divmod(rest, rc)
    q = [int(w) for w in words[4 * iA: 4 * iA + 4]]
    win = 1 if n >= 8 else 0
    w0, w1 = q[win], q[win + 1]
    sb = words[offb + 2 * iB: offb + 2 * iB + 2]
    y0, y1 = vperm(w1, w0, int(sb[0])), vperm(w1, w0, int(sb[1]))
    if rc > 1:  # C stores its hi selector only (its swaps stay in window bytes 4..7)
        y1 = vperm(y1, y0, int(words[offc + iC]))
    q[win], q[win + 1] = y0, y1
    return [(q[g // 4] >> (8 * (g % 4))) & 0xFF for g in range(n + 1)]


@pytest.mark.parametrize("n", list(range(1, 12)))
def test_stage_tables_compose_to_fisher_yates(n):
    sizes, words = tables(n)
    ra, rb, rc = (int(x) for x in sizes[:3])
    assert ra * rb * rc == math.factorial(n)
    assert int(sizes[5]) == 4 * ra + 2 * rb + rc  # A [ra][4], B [rb][2], C [rc] (hi selector)
    assert ra == (n * (n - 1) * (n - 2) if n >= 8 else 1)
    nf = math.factorial(n)
    ranks = range(nf) if nf <= 40320 else \
        [0, nf - 1] + list(np.random.default_rng(n).integers(0, nf, 20_000))
    for R in ranks:
        assert compose(n, sizes, words, int(R)) == fy_decode(n, int(R)), (n, R)


@pytest.mark.parametrize("n", list(range(1, 12)))
def test_stage_tables_are_permutations(n):
    """What the fused kernels rely on when they skip the per-entry equal-pair
    test (qba_count_pb / qba_count_d with DIST): every
    stage-A row holds 0..n once, every B selector permutes the 8 window bytes
    and every C hi selector the window's bytes 4..7, each fixing the bytes
    past n -- so each Q entry's values r ^ pi(g) are distinct.  qba_plan checks
    the same when it builds a program (check_perm_tables); this pins it on
    the exported tables."""
    sizes, words = tables(n)
    ra, rb, rc, offb, offc, _ = (int(x) for x in sizes)
    base = 4 if n >= 8 else 0
    b = lambda w, k: (int(w) >> (8 * k)) & 0xFF  # noqa: E731
    for i in range(ra):
        row = [b(words[4 * i + g // 4], g % 4) for g in range(n + 1)]
        assert sorted(row) == list(range(n + 1)), (n, i, row)

    def perm_ok(sel, lo, hi):
        assert sorted(sel) == list(range(lo, hi + 1)), sel
        assert all(sel[k - lo] == k for k in range(lo, hi + 1) if base + k > n), sel

    for i in range(rb):
        perm_ok([b(words[offb + 2 * i + k // 4], k % 4) for k in range(8)], 0, 7)
    for i in range(rc if rc > 1 else 0):
        perm_ok([b(words[offc + i], k) for k in range(4)], 4, 7)


def closed_entry_py(n, seed, e):
    """Python restatement of the closed-form schedule for one entry."""
    nq = oracle_lib.n_qubits(n)
    W = 1 << nq
    p, h = e >> 1, e & 1
    x = [int(v) for v in oracle_lib.philox(np.array([p & 0xFFFFFFFF, p >> 32, 0, 0], np.uint32), seed)[0]]
    w0, w1 = x[2 * h], x[2 * h + 1]
    if not w0 & 1:
        # group g >= 1: nibble g of the word pair (w1 low nibbles, w1 high
        # nibbles, w0 high nibbles, byte order); group 0 = group 1
        vals = [(w1 >> s) & (W - 1) for s in (8, 16, 24, 4, 12, 20, 28)] + \
               [(w0 >> s) & (W - 1) for s in (4, 12, 20, 28)]
        return [vals[0]] + vals[: n]
    nf = math.factorial(n)
    t32, t27 = (1 << 32) % nf, ((1 << 27) % nf) << 5
    ok = lambda F, t: (F * nf) & 0xFFFFFFFF >= t  # noqa: E731
    if ok(w1, t32):
        F = w1
    elif ok(w0 & ~31 & 0xFFFFFFFF, t27):
        F = w0 & ~31 & 0xFFFFFFFF
    else:
        a, F = 0, None
        while F is None:
            a += 1
            ys = [int(v) for v in oracle_lib.philox(
                np.array([p & 0xFFFFFFFF, p >> 32, 0x80000000 + a, h], np.uint32), seed)[0]]
            F = next((y for y in ys if ok(y, t32)), None)
    perm = fy_decode(n, (F * nf) >> 32)
    r = (w0 >> 1) & (W - 1)
    return [r ^ q for q in perm]


def test_closed_rank_fallbacks():
    """The 27-bit second candidate and the retry blocks are reached: find
    entries of each kind at n = 11 and check the oracle against the Python
    restatement there."""
    n, seed = 11, 5
    nf = math.factorial(n)
    t32, t27 = (1 << 32) % nf, ((1 << 27) % nf) << 5
    ctr = np.zeros((1 << 16, 4), np.uint32)
    ctr[:, 0] = np.arange(1 << 16)
    x = oracle_lib.philox(ctr, seed).astype(np.uint64)
    kinds = {}
    for p in range(1 << 16):
        for h in (0, 1):
            w0, w1 = int(x[p, 2 * h]), int(x[p, 2 * h + 1])
            if not w0 & 1:
                continue
            if (w1 * nf) & 0xFFFFFFFF >= t32:
                kinds.setdefault("w1", 2 * p + h)
            elif ((w0 & ~31 & 0xFFFFFFFF) * nf) & 0xFFFFFFFF >= t27:
                kinds.setdefault("w0", 2 * p + h)
            else:
                kinds.setdefault("retry", 2 * p + h)
    assert {"w1", "w0"} <= set(kinds)
    info = {"nfac": 0, "desc": np.zeros((0, 6), np.int32), "pat": np.zeros(1, np.uint64),
            "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    for e in kinds.values():
        got = oracle_lib.sample(n, seed, e, 1, info, info, closed=True)
        assert list(got[:, 0]) == closed_entry_py(n, seed, e)


@pytest.mark.parametrize("n", [1, 3, 7, 8, 11])
def test_oracle_closed_schedule(n):
    seed, first, count = 0xC0FFEE ^ n, (1 << 35) + 11, 300
    info = {"nfac": 0, "desc": np.zeros((0, 6), np.int32), "pat": np.zeros(1, np.uint64),
            "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    got = oracle_lib.sample(n, seed, first, count, info, info, closed=True)
    for k in range(count):
        assert list(got[:, k]) == closed_entry_py(n, seed, first + k), k


def test_oracle_closed_statistics():
    """n = 11: Q entries are r ^ pi (all distinct), not-Q entries have L0 == L1,
    marginals uniform."""
    n, count = 11, 200_000
    info = {"nfac": 0, "desc": np.zeros((0, 6), np.int32), "pat": np.zeros(1, np.uint64),
            "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    L = oracle_lib.sample(n, 99, 0, count, info, info, closed=True).astype(np.int64)
    q = L[0] != L[1]
    assert abs(q.mean() - 0.5) < 0.01
    srt = np.sort(L[:, q], axis=0)
    assert (np.diff(srt, axis=0) > 0).all()
    perm = L[:, q] ^ L[0, q]
    assert (np.sort(perm[1:], axis=0) == np.arange(1, n + 1)[:, None]).all()
    for g in range(n + 1):
        cnt = np.bincount(L[g], minlength=16)
        chi2 = ((cnt - count / 16) ** 2 / (count / 16)).sum()
        assert chi2 < 60, (g, chi2)


@pytest.mark.parametrize("n", [3, 7, 11])
def test_oracle_stream_and_batched_counts(n):
    """The streaming and batched count oracles (used as the checkers of the
    full-size GPU tests) equal counts() over materialised lists."""
    info = {"nfac": 0, "desc": np.zeros((0, 6), np.int32), "pat": np.zeros(1, np.uint64),
            "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    seed, first, count = 77 + n, (1 << 33) + 5, 20_003
    L = oracle_lib.sample(n, seed, first, count, info, info, closed=True)
    H, Cc, P, bad = oracle_lib.counts(L, n)
    H2, C2, P2, bad2 = oracle_lib.stream_counts(n, seed, first, count, info, info, closed=True)
    assert bad == bad2 == 0
    assert np.array_equal(H, H2) and np.array_equal(Cc, C2) and np.array_equal(P, P2)
    Hb, Cb, Pb = oracle_lib.batched_counts(n, 1000, 5, 3001, info, info, closed=True)
    for i in range(5):
        h, c, p, _ = oracle_lib.counts(oracle_lib.sample(n, 1000 + i, 0, 3001, info, info, closed=True), n)
        assert np.array_equal(Hb[i], h) and np.array_equal(Cb[i], c) and np.array_equal(Pb[i], p)
