"""GPU parity of the nibble-row ("packed") list kernels -- qba_sample_packed,
qba_sample_check_packed, qba_check_counts_packed, qba_lists_pack/unpack --
against the C twin (oracle/sampler_ref.c) and the byte-layout kernels.

Layout (include/qba.h): byte b of row g = value of column 2b | value of
column 2b+1 << 4.  Lists and counts must be bit-identical to the byte layout's
on the same entries; the cases follow test_gpu_kernels.py's (ragged tails,
chunk and 2^33 splits, unaligned chunk starts, collisions, out-of-range
values) plus the layout's own edges (odd counts, nothing written past the last
byte)."""
import numpy as np
import pytest
import torch

import oracle_lib
import tfg_oracle as orc
from conftest import GOLDEN, sub

pytestmark = pytest.mark.gpu


def _unpack(p, count):
    return sub("engine").unpack_nibbles(p.cpu().numpy(), count)


def _ref(engine, n, seed, first, count):
    info = engine.prepare(n)
    return oracle_lib.sample(n, seed, first, count, info["notq"], info["q"], info["closed"])


def _same_counts(c, ref):
    H, C, P, _ = oracle_lib.counts(ref, n=ref.shape[0] - 1)
    gH, gC, gP = c.numpy()
    return np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)


@pytest.mark.parametrize("n,first,count", [(1, 0, 1001), (2, 7, 999), (3, 0, 4096), (4, 1, 30_001),
                                           (5, 3, 777), (6, 0, 30_000), (7, 1 << 33, 5003), (8, 2, 40_003),
                                           (9, 5, 40_000), (10, 0, 50_001), (11, 0, 100_003),
                                           (11, (1 << 40) + 5, 20_001), (12, 6, 9_999), (13, 99, 3000),
                                           (14, 0, 12_345), (15, 1, 8191)])
def test_packed_sample_and_counts_bit_exact(engine, n, first, count):
    seed = 0x5EED ^ (n << 20)
    ref = _ref(engine, n, seed, first, count)
    p = engine.sample_packed(n, seed, first, count)
    assert np.array_equal(_unpack(p, count), ref)
    p2, c = engine.sample_check_packed(n, seed, first, count)
    assert np.array_equal(_unpack(p2, count), ref)
    assert _same_counts(c, ref)
    assert _same_counts(engine.check_counts_packed(p2, n, count), ref)


@pytest.mark.parametrize("count", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 15, 16, 17, 31, 4099, 4100, 8197])
def test_packed_tiny_and_ragged(engine, count):
    """Tails (partial quads, a lone low nibble) and nothing written past byte
    (count + 1) // 2 of any row."""
    n, seed, first = 11, 2024, 10
    ref = _ref(engine, n, seed, first, count)
    buf = torch.zeros((n + 1, 4096 + (count + 1) // 2 // 4096 * 4096), dtype=torch.uint8, device=engine.device)
    p, c = engine.sample_check_packed(n, seed, first, count, packed=buf)
    torch.cuda.synchronize()
    assert np.array_equal(_unpack(p, count), ref)
    host = buf.cpu().numpy()
    nb = (count + 1) // 2
    assert not host[:, nb:].any()
    if count % 2:
        assert not (host[:, nb - 1] >> 4).any()  # the missing column's nibble
    assert _same_counts(c, ref)
    assert _same_counts(engine.check_counts_packed(p, n, count), ref)


@pytest.mark.parametrize("first", [999, 1000])
def test_packed_chunked_and_unaligned_chunk_starts(first):
    """Chunks of 40004 entries (qba_test_set_knobs): every chunk after the first starts at byte
    20002 * k, off the wide step's 4-byte alignment every other chunk, so the
    one-quad (byte-store) step runs for the cut and the wide one after it."""
    eng = sub("engine").Engine(0).set_test_knobs(chunk=40004)
    try:
        n, seed, count = 11, 31337, 160_021
        ref = _ref(eng, n, seed, first, count)
        p, c = eng.sample_check_packed(n, seed, first, count)
        assert np.array_equal(_unpack(p, count), ref)
        assert _same_counts(c, ref)
        assert np.array_equal(_unpack(eng.sample_packed(n, seed, first, count), count), ref)
        assert _same_counts(eng.check_counts_packed(p, n, count), ref)
    finally:
        eng.close()


@pytest.mark.parametrize("n,first,count", [(11, (1 << 33) - 4000, 12_008), (11, (1 << 33) - 4001, 12_008),
                                           (11, (1 << 34) - 3, 20_001), (11, (1 << 34) - 6, 20_001),
                                           (7, (3 << 33) - 8, 16), (7, (3 << 33) - 7, 16)])
def test_packed_split_at_counter_word(engine, n, first, count):
    """Even first: split at the 2^33 multiple (an even column); odd first: the
    per-entry path, no split.  Both bit-exact."""
    seed = 0xC0FFEE + n
    ref = _ref(engine, n, seed, first, count)
    p, c = engine.sample_check_packed(n, seed, first, count)
    assert np.array_equal(_unpack(p, count), ref)
    assert _same_counts(c, ref)


def test_pack_unpack_roundtrip(engine):
    n, count = 11, 50_001
    rng = np.random.default_rng(3)
    L = rng.integers(0, 16, (n + 1, count)).astype(np.uint8)
    d = torch.zeros((n + 1, 53_248), dtype=torch.uint8, device=engine.device)
    d[:, :count] = torch.from_numpy(L).to(engine.device)
    p = engine.pack(d, n + 1, count)
    assert np.array_equal(_unpack(p, count), L)
    back = engine.unpack(p, n + 1, count)
    assert np.array_equal(back[:, :count].cpu().numpy(), L)
    d[3, 17] = 16
    with pytest.raises(sub("_lib").QbaError):
        engine.pack(d, n + 1, count)


def test_packed_counts_on_fixture_lists(engine):
    """Check-only over packed injected fixture lists (tampered / uniform ones with
    collisions) vs the numpy restatement."""
    arrays = np.load(GOLDEN / "protocol_lists.npz")
    for name in arrays.files:
        L = arrays[name]
        n = L.shape[0] - 1
        if L.max() > 15:
            continue
        d = torch.zeros((n + 1, (L.shape[1] + 63) // 64 * 64), dtype=torch.uint8, device=engine.device)
        d[:, : L.shape[1]] = torch.from_numpy(L)
        c = engine.check_counts_packed(engine.pack(d, n + 1, L.shape[1]), n, L.shape[1])
        gH, gC, gP = c.numpy()
        H, C, P = orc.counts(L, n)
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P), name


def test_packed_out_of_range_and_collisions(engine):
    """n = 3 (w = 4): values in [w, 15] at Q entries are caught by the range
    test (stats) exactly as in the byte layout; lists full of collisions take
    the pair slow path."""
    n, count = 3, 50_001
    lists = engine.sample(n, 77, 0, count)
    torch.cuda.synchronize()
    L = lists[:, :count].cpu().numpy().copy()
    rng = np.random.default_rng(n)
    isq = np.nonzero(L[0] != L[1])[0]
    for k in rng.choice(isq, 7, replace=False):
        L[rng.integers(2, n + 1), k] = rng.integers(4, 16)
    d = torch.zeros_like(lists)
    d[:, :count] = torch.from_numpy(L)
    c = engine.check_counts_packed(engine.pack(d, n + 1, count), n, count)
    H, C, P, bad = oracle_lib.counts(L, n)
    assert bad == engine.last_stats()[0] >= 7
    gH, gC, gP = c.numpy()
    assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)
    n, count = 11, 30_001
    L = rng.integers(0, 4, (n + 1, count)).astype(np.uint8)
    d = torch.zeros((n + 1, 30_720), dtype=torch.uint8, device=engine.device)
    d[:, :count] = torch.from_numpy(L).to(engine.device)
    c = engine.check_counts_packed(engine.pack(d, n + 1, count), n, count)
    H, C, P, bad = oracle_lib.counts(L, n)
    gH, gC, gP = c.numpy()
    assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)


def test_packed_headline_size_equals_byte_layout(engine):
    """The bench workload (n = 11, 1.25e8 entries): the packed fused pass writes
    exactly the byte layout's lists (unpacked on the device) and its counts."""
    n, seed, count = 11, 0x5EED, 125_000_000
    engine.prepare(n)
    lists, cb = engine.sample_check(n, seed, 0, count)
    p, cp = engine.sample_check_packed(n, seed, 0, count)
    u = engine.unpack(p, n + 1, count)
    assert torch.equal(u[:, :count], lists[:, :count])
    for a, b in zip(cb.numpy(), cp.numpy()):
        assert np.array_equal(a, b)
    del lists, u
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,count", [(7, 3001), (7, 3000), (12, 777)])
def test_packed_batched_instances(engine, n, count):
    """Batched runs (configs[3] shape, scaled down) over nibble rows: instance i
    == an ordinary run with key base + i, lists and counts, odd and even counts,
    closed-form and table samplers."""
    n_inst, base = 37, 1000
    info = engine.prepare(n)
    lists, c = engine.sample_check_batched(n, base, n_inst, count, packed=True)
    torch.cuda.synchronize()
    for i in (0, 1, 17, 36):
        ref = oracle_lib.sample(n, base + i, 0, count, info["notq"], info["q"], info["closed"])
        assert np.array_equal(_unpack(lists[i], count), ref)
        H, C, P, bad = oracle_lib.counts(ref, n)
        assert np.array_equal(c.H[i].cpu().numpy(), H)
        assert np.array_equal(c.C[i].cpu().numpy(), C)
        assert np.array_equal(c.P[i].cpu().numpy(), P)


@pytest.mark.parametrize("packed", [True, False])
def test_pairbin_wrap_recount_exact(packed):
    """The fused n = 11 kernel counts in 8-bit pair bins (qba_lists_kern.h,
    QbaPB).  list_grid = 2 (qba_test_set_knobs) puts ~2e6 entries on each of two workgroups, so
    every pair bin wraps many times; the flush's lane-total test must see it
    and the workgroups recount their rows exactly (stats[1] = 2).  Lists and
    counts stay bit-exact against the C twin, for both row layouts."""
    eng = sub("engine").Engine(0).set_test_knobs(list_grid=2)
    try:
        n, seed, first, count = 11, 0xBADC0DE, 6, 4_000_003
        ref = _ref(eng, n, seed, first, count)
        if packed:
            p, c = eng.sample_check_packed(n, seed, first, count)
            got = _unpack(p, count)
        else:
            lists, c = eng.sample_check(n, seed, first, count)
            torch.cuda.synchronize()
            got = lists[:, :count].cpu().numpy()
        assert np.array_equal(got, ref)
        assert _same_counts(c, ref)
        st = eng.last_stats()
        assert st[0] == 0 and st[1] == 2, st
    finally:
        eng.close()


def test_pairbin_no_recount_at_bench_size(engine):
    """At the headline launch (1.25e8 entries, <= 2^18 per workgroup) no pair
    bin wraps: no workgroup recounts (stats[1] == 0), and the counts of the
    packed fused pass equal the pair-bin check of its rows and the classic
    check (32-bit bins) of the same rows unpacked to bytes."""
    n, seed, count = 11, 0x5EED, 125_000_000
    p, c = engine.sample_check_packed(n, seed, 0, count)
    st = engine.last_stats()
    assert st[0] == 0 and st[1] == 0, st
    c2 = engine.check_counts_packed(p, n, count)
    assert list(engine.last_stats()) == [0, 0]
    u = engine.unpack(p, n + 1, count)
    del p
    c3 = engine.check_counts(u, n, count)
    for a, b, d in zip(c.numpy(), c2.numpy(), c3.numpy()):
        assert np.array_equal(a, b) and np.array_equal(a, d)
    del u
    torch.cuda.empty_cache()


def _collided(n, count, seed):
    """Uniform n = 11 lists with equal pairs injected at a third of the
    Q-correlated entries (random groups g != h >= 2: L_h := L_g)."""
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 16, (n + 1, count)).astype(np.uint8)
    L[1] = np.where(rng.random(count) < 0.5, L[0], L[1])  # ~half not Q-correlated
    isq = np.nonzero(L[0] != L[1])[0]
    for k in rng.choice(isq, len(isq) // 3, replace=False):
        g, h = rng.choice(np.arange(2, n + 1), 2, replace=False)
        L[h, k] = L[g, k]
    return L


@pytest.mark.parametrize("force,count", [("pb_min=0", 30_001), ("pb_min=0", 8),
                                         ("pb_min=0", 1_000_003), ("list_grid=2", 5_000_001)])
def test_pairbin_check_counts_collisions_exact(force, count):
    """Cond3 (tfg.py:96-98) through the pair-bin counter: qba_check_counts_packed
    at n = 11 counts in pair bins (QbaUsePB), so injected equal pairs drive the
    counter's distinctness test and its equal-pair slow path (C[u][g][h] in B's
    upper lanes).  Small and ragged launches (pair bins forced below their
    threshold) and a wrapping one (two workgroups: recount, stats[1] == 2) are
    bit-exact against the numpy restatement; uniform lists over [0, 4) make
    every Q entry collide."""
    key, val = force.split("=")
    eng = sub("engine").Engine(0).set_test_knobs(**{key: int(val)})
    try:
        n = 11
        for L in (_collided(n, count, count), np.random.default_rng(5).integers(0, 4, (n + 1, count)).astype(np.uint8)):
            d = torch.zeros((n + 1, (count + 4095) // 4096 * 4096), dtype=torch.uint8, device=eng.device)
            d[:, :count] = torch.from_numpy(L).to(eng.device)
            c = eng.check_counts_packed(eng.pack(d, n + 1, count), n, count)
            gH, gC, gP = c.numpy()
            H, C, P = orc.counts(L, n)
            assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)
            offdiag = int(C.sum() - sum(C[:, g, g].sum() for g in range(n + 1)))
            assert offdiag > 0 or count < 64
            st = list(eng.last_stats())
            assert st == ([0, 2] if key == "list_grid" else [0, 0]), st
    finally:
        eng.close()


def test_slab_stream_switch_after_destruction(engine):
    """A counting call on stream A, A synchronised and destroyed, then counting
    calls (and deferred ones) on new streams B, which may reuse A's handle:
    the library never touches a previous stream -- a counting call on another
    stream than the previous one synchronises the device first -- and every
    result stays exact
    (qba_slab_order)."""
    n, seed, count = 11, 99, 200_003
    ref = _ref(engine, n, seed, 0, count)
    a = torch.cuda.Stream()
    with torch.cuda.stream(a):
        p, c = engine.sample_check_packed(n, seed, 0, count)
    a.synchronize()
    assert _same_counts(c, ref)
    del a
    import gc
    gc.collect()
    for _ in range(2):
        b = torch.cuda.Stream()
        with torch.cuda.stream(b):
            p2, c2 = engine.sample_check_packed(n, seed, 0, count)
            p3, c3 = engine.sample_check_packed(n, seed, 0, count, deferred=True)
            engine.flush_deferred()
        b.synchronize()
        assert _same_counts(c2, ref) and _same_counts(c3, ref)
        assert np.array_equal(_unpack(p3, count), ref)
        del b
        gc.collect()
    p4, c4 = engine.sample_check_packed(n, seed, 0, count)
    assert _same_counts(c4, ref)


def test_slab_stream_switch_with_work_in_flight(engine):
    """a counting call on stream B while stream A's large counting
    launch is still in flight (A not synchronised, then destroyed): the switch
    synchronises the device before B's launch reuses the shared slab, so A's
    counts and B's are both exact -- in both orders of n and size."""
    import gc
    n = 11
    for big, small in [((3, 0, 20_000_003), (4, 7, 300_001)), ((5, 1, 16_777_217), (6, 0, 50_000))]:
        a = torch.cuda.Stream()
        with torch.cuda.stream(a):
            pa, ca = engine.sample_check_packed(n, *big)         # left in flight
        b = torch.cuda.Stream()
        with torch.cuda.stream(b):
            pb, cb = engine.sample_check_packed(n, *small)
            pd, cd = engine.sample_check_packed(n, *small, deferred=True)
            engine.flush_deferred()
        del a
        gc.collect()
        torch.cuda.synchronize()
        s, f, c = big
        info = engine.prepare(n)
        H, C, P, _ = oracle_lib.stream_counts(n, s, f, c, info["notq"], info["q"], info["closed"])
        gH, gC, gP = ca.numpy()
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P), big
        ref = _ref(engine, n, *small)
        assert _same_counts(cb, ref) and _same_counts(cd, ref), small
        assert np.array_equal(_unpack(pd, small[2]), ref)
        del pa, pb, pd
        torch.cuda.empty_cache()


@pytest.mark.parametrize("packed", [True, False])
def test_pairbin_kernel_small_launches_bit_exact(packed):
    """The pair-bin kernel (picked for launches of >= 2^24 entries) forced on
    small and ragged launches with pb_min = 0 (qba_test_set_knobs): tails (partial quads,
    counted entry by entry into the pair bins), odd first columns and a
    chunked call, bit-exact against the C twin, no recount."""
    eng = sub("engine").Engine(0).set_test_knobs(pb_min=0)
    try:
        n = 11
        for first, count in [(0, 1), (0, 2), (3, 5), (0, 8), (1, 17), (10, 4099), (0, 100_003), (7, 2_000_001)]:
            seed = 0xFACE + count
            ref = _ref(eng, n, seed, first, count)
            if packed:
                p, c = eng.sample_check_packed(n, seed, first, count)
                got = _unpack(p, count)
            else:
                lists, c = eng.sample_check(n, seed, first, count)
                torch.cuda.synchronize()
                got = lists[:, :count].cpu().numpy()
            assert np.array_equal(got, ref), (first, count)
            assert _same_counts(c, ref), (first, count)
            assert list(eng.last_stats()) == [0, 0], (first, count)
    finally:
        eng.close()
