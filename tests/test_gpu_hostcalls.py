"""GPU parity of the exact-order protocol's synchronous host-pointer calls on
both of their paths: inputs up to QBA_CS_MAX (16384) items / QBA_ZC_MAX
(1 MiB) staged run as single-workgroup launches over zero-copy pinned
memory; larger ones through the device kernels and one D2H.  Each case is
checked against the numpy restatement (oracle/tfg_oracle.py), across the
path boundary."""
import numpy as np
import pytest

import tfg_oracle as orc
from conftest import sub

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("count", [0, 1, 999, 16_383, 16_384, 16_385, 40_000])
def test_isq_and_select_host_forms(engine, count):
    rng = np.random.default_rng(count)
    l0 = rng.integers(0, 8, max(count, 1)).astype(np.uint8)[:count]
    l1 = np.where(rng.random(count) < 0.5, l0, rng.integers(0, 8, count)).astype(np.uint8)
    d0 = engine.to_device(l0 if count else np.zeros(1, np.uint8))
    d1 = engine.to_device(l1 if count else np.zeros(1, np.uint8))
    if count == 0:
        d0, d1 = d0[:0], d1[:0]
    isq = engine.isq_indices(d0, d1)
    assert np.array_equal(isq, orc.is_qcorr_indices(l0, l1))
    order = rng.permutation(count).astype(np.int64)
    for v in (0, 3, 7):
        assert engine.select_eq(order, d1, v).tolist() == orc.p_filter(order, l1, v)


@pytest.mark.parametrize("m", [5, 20_000])
def test_select_host_bad_index(engine, m):
    """An index outside Lc fails the call on both paths and leaves the context usable."""
    lc = engine.to_device(np.zeros(100, np.uint8))
    order = np.arange(m, dtype=np.int64) % 100
    order[m // 2] = 100
    with pytest.raises(sub("_lib").QbaError):
        engine.select_eq(order, lc, 0)
    assert engine.select_eq(np.arange(3, dtype=np.int64), lc, 0).tolist() == [0, 1, 2]


def _packet_ref(li, order, rows, v, w):
    own = orc.gather(li, order)
    L = set(tuple(int(x) for x in r) for r in rows) | {own}
    try:
        ok = orc.consistent(v, L, w)
    except StopIteration:
        ok = None
    return own, ok


@pytest.mark.parametrize("ln,m", [(1, 1), (250, 3), (3000, 11), (70_000, 1), (40, 70)])
def test_check_packets_both_paths(engine, ln, m):
    """Packets under the zero-copy bound (m <= 64, <= 1 MiB) and over it
    (70 000 x 2 int64; 70 tuples), honest and tampered, alone and as one
    round: own tuple and verdict equal the restatement's."""
    rng = np.random.default_rng(ln * 131 + m)
    w, size = 15, max(ln * 4, 64)
    li = rng.integers(0, w + 1, size).astype(np.uint8)
    dli = engine.to_device(li)
    reqs, refs = [], []
    for case in range(4):
        order = rng.choice(size, ln, replace=False).astype(np.int64)
        v = int(rng.integers(0, w + 1))
        own = li[order].astype(np.int64)
        rows = []
        for a in range(m):
            if case == 0:
                r = own.copy()  # the set collapses to {own}
            elif case == 1:
                r = (own + 1 + a) % (w + 1)
            else:
                r = rng.integers(0, w + 1, ln).astype(np.int64)
            if case == 3 and a == 0:
                r[ln // 2] = w + 5  # Cond2 violation
            rows.append(r)
        reqs.append((order, rows, v))
        refs.append(_packet_ref(li, order, rows, v, w))
    got = engine.check_packets(dli, reqs, w)
    for (own, ok, _), (rown, rok) in zip(got, refs):
        assert own == rown and ok == rok
    for (order, rows, v), (rown, rok) in zip(reqs, refs):
        own, ok = engine.check_packet(dli, order, rows, v, w)
        assert own == rown and ok == rok
    bad = (np.array([size], np.int64), [np.zeros(1, np.int64)], 0)
    with pytest.raises(sub("_lib").QbaError):
        engine.check_packets(dli, [bad], w)


@pytest.mark.parametrize("count,nq", [(1000, 2), (10_000, 4), (70_000, 2)])
def test_codec_host_forms_both_paths(engine, count, nq):
    """lists -> rawS (zero-copy write below 1 MiB, D2H above) and rawS -> list
    (zero-copy read / H2D), against the restatement's codec."""
    rng = np.random.default_rng(count)
    L = rng.integers(0, 1 << nq, (3, count)).astype(np.uint8)
    d = engine.to_device(L)
    raw = engine.lists_to_bits(d, 3, count, nq)
    assert np.array_equal(raw, orc.lists_to_raw(L, nq))
    back = engine.bits_to_values_host(raw[1], count, nq)
    assert np.array_equal(back.cpu().numpy()[:count], L[1])
