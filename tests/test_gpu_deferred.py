"""GPU parity of the deferred-reduction entry points (include/qba.h:
qba_sample_check_deferred / qba_sample_check_packed_deferred /
qba_flush_deferred).

A deferred call's counts are reduced by the NEXT deferred call's list kernel
(reduce workgroups ahead of its list workgroups, two alternating slab
buffers) or by the flush, with plain stores of every output word.  The counts
must be bit-identical to the synchronous calls' and to the C twin's, in every
way a caller can chain them: separate outputs, one reused output buffer,
accumulate, different n between calls, a synchronous call or an empty call in
between, launches that fill the chip (the synchronous fallback), chunked
calls, two streams, and a hipGraph replayed twice."""
import numpy as np
import pytest
import torch

import oracle_lib
from conftest import sub

pytestmark = pytest.mark.gpu


def _ref_counts(engine, n, seed, first, count):
    info = engine.prepare(n)
    ref = oracle_lib.sample(n, seed, first, count, info["notq"], info["q"], info["closed"])
    H, C, P, _ = oracle_lib.counts(ref, n=n)
    return H, C, P


def _eq(c, ref):
    gH, gC, gP = c.numpy()
    return np.array_equal(gH, ref[0]) and np.array_equal(gC, ref[1]) and np.array_equal(gP, ref[2])


def _call(engine, packed, n, seed, first, count, counts=None, accumulate=False, deferred=True):
    f = engine.sample_check_packed if packed else engine.sample_check
    return f(n, seed, first, count, counts=counts, accumulate=accumulate, deferred=deferred)[1]


@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("n", [1, 3, 7, 11, 13])
def test_deferred_chain_separate_outputs(engine, packed, n):
    """Four deferred calls into four output buffers, then the flush."""
    calls = [(0x5EED + k, 1000 * k + (k & 1), 20_000 + 777 * k) for k in range(4)]
    outs = [_call(engine, packed, n, s, f, c) for s, f, c in calls]
    engine.flush_deferred()
    torch.cuda.synchronize()
    for (s, f, c), o in zip(calls, outs):
        assert _eq(o, _ref_counts(engine, n, s, f, c)), (n, s, f, c)


@pytest.mark.parametrize("packed", [True, False])
def test_deferred_reused_buffer_and_accumulate(engine, packed):
    """configs[1]'s pattern: every pass into the same buffer (the last pass's
    counts remain), then a run that accumulates its passes."""
    n = 11
    buf = engine.alloc_counts(n)
    for k in range(5):
        _call(engine, packed, n, 77, 50_000 * k, 1_000_000, counts=buf)
    engine.flush_deferred()
    torch.cuda.synchronize()
    assert _eq(buf, _ref_counts(engine, n, 77, 200_000, 1_000_000))
    acc = engine.alloc_counts(n)
    parts = [(0, 30_001), (30_001, 12_000), (42_001, 99_999)]
    for i, (f, c) in enumerate(parts):
        _call(engine, packed, n, 9, f, c, counts=acc, accumulate=i > 0)
    engine.flush_deferred()
    torch.cuda.synchronize()
    assert _eq(acc, _ref_counts(engine, n, 9, 0, 142_000))


def test_deferred_mixed_with_sync_calls_and_n(engine):
    """A pending reduction is flushed by a synchronous counting call, by an
    empty call and by a deferred call of another n -- each into its own
    outputs -- and a stale pending call never overwrites later results."""
    a = _call(engine, True, 11, 1, 0, 40_000)
    b = engine.sample_check_packed(11, 2, 0, 40_000)[1]          # synchronous: flushes a
    c = _call(engine, True, 5, 3, 10, 30_000)
    d = _call(engine, False, 11, 4, 0, 25_000)                   # other n: c reduced on its own
    e = engine.alloc_counts(11)
    _call(engine, True, 11, 5, 0, 0, counts=e)                   # empty: flushes d, zeroes e
    f = _call(engine, True, 11, 6, 0, 33_333)
    engine.check_counts_packed(engine.sample_packed(11, 7, 0, 1000), 11, 1000)  # flushes f
    torch.cuda.synchronize()
    assert _eq(a, _ref_counts(engine, 11, 1, 0, 40_000))
    assert _eq(b, _ref_counts(engine, 11, 2, 0, 40_000))
    assert _eq(c, _ref_counts(engine, 5, 3, 10, 30_000))
    assert _eq(d, _ref_counts(engine, 11, 4, 0, 25_000))
    assert not any(x.any() for x in (e.H.cpu(), e.C.cpu(), e.P.cpu()))
    assert _eq(f, _ref_counts(engine, 11, 6, 0, 33_333))


def test_deferred_full_chip_fallback_and_chunks():
    """A launch whose list workgroups fill every resident slot takes the
    synchronous path (the pending call is flushed first); a chunked deferred
    call defers chunk by chunk (each later chunk reduces the one before)."""
    eng = sub("engine").Engine(0)
    try:
        n = 11
        a = _call(eng, True, n, 41, 0, 50_000)
        big = _call(eng, True, n, 42, 123, 12_000_000)  # > 512 workgroups' worth: fallback
        b = _call(eng, True, n, 43, 0, 50_000)
        eng.flush_deferred()
        torch.cuda.synchronize()
        assert _eq(a, _ref_counts(eng, n, 41, 0, 50_000))
        assert _eq(big, _ref_counts(eng, n, 42, 123, 12_000_000))
        assert _eq(b, _ref_counts(eng, n, 43, 0, 50_000))
    finally:
        eng.close()
    eng = sub("engine").Engine(0).set_test_knobs(chunk=40004)
    try:
        c = _call(eng, True, 11, 44, 999, 160_021)
        d = _call(eng, False, 11, 45, 1000, 120_013)
        eng.flush_deferred()
        torch.cuda.synchronize()
        assert _eq(c, _ref_counts(eng, 11, 44, 999, 160_021))
        assert _eq(d, _ref_counts(eng, 11, 45, 1000, 120_013))
    finally:
        eng.close()


def test_deferred_two_streams(engine):
    """A deferred call on another stream than the pending one: the pending
    reduction is flushed on its own stream and the new stream waits for it
    before reusing the slab."""
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for k in range(6):
        with torch.cuda.stream(s1 if k % 2 == 0 else s2):
            outs.append(_call(engine, True, 11, 100 + k, 0, 60_000 + k))
    with torch.cuda.stream(s2):
        engine.flush_deferred()
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        assert _eq(o, _ref_counts(engine, 11, 100 + k, 0, 60_000 + k))


def test_deferred_in_graph_replayed(engine):
    """configs[1]'s bench form: K deferred passes + the flush captured in one
    hipGraph; each replay reproduces the passes' counts."""
    n, K = 11, 6
    outs = [engine.alloc_counts(n) for _ in range(K)]
    packed = engine.alloc_packed(n, 1_000_000)
    for k in range(K):  # warm (programs, slab sizes) outside the capture
        engine.sample_check_packed(n, 7 + k, k * 1_000_000, 1_000_000, packed, outs[k], deferred=True)
    engine.flush_deferred()
    torch.cuda.synchronize()
    for o in outs:
        for t in (o.H, o.C, o.P):
            t.zero_()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for k in range(K):
                engine.sample_check_packed(n, 7 + k, k * 1_000_000, 1_000_000, packed, outs[k], deferred=True)
            engine.flush_deferred()
    for _ in range(2):
        for o in outs:
            for t in (o.H, o.C, o.P):
                t.fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        for k, o in enumerate(outs):
            assert _eq(o, _ref_counts(engine, n, 7 + k, k * 1_000_000, 1_000_000)), k


def test_deferred_stats(engine):
    """qba_last_stats after the flush is the stats of the last deferred call."""
    _call(engine, True, 11, 5, 0, 10_000)
    engine.flush_deferred()
    torch.cuda.synchronize()
    assert list(engine.last_stats()) == [0, 0]


def test_deferred_capture_boundaries(engine):
    """a pending deferred reduction never crosses a capture
    boundary.  (a) pending from before a capture -> the deferred call inside
    the capture fails with QBA_ESTATE; (b) pending at the end of a capture ->
    qba_flush_deferred outside fails and drops it; the ctx stays usable and
    the next eager calls are exact."""
    qe = sub("_lib").QbaError
    n, count = 11, 50_000
    packed = engine.alloc_packed(n, count)
    c = engine.alloc_counts(n)
    engine.sample_check_packed(n, 3, 0, count, packed, c, deferred=True)  # pending, eager
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with pytest.raises(qe):
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                engine.sample_check_packed(n, 4, 0, count, packed, c, deferred=True)
    engine.flush_deferred()  # the eager pending one, eagerly
    torch.cuda.synchronize()
    assert _eq(c, _ref_counts(engine, n, 3, 0, count))
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g2, stream=s):
            engine.sample_check_packed(n, 5, 0, count, packed, c, deferred=True)  # left pending
    with pytest.raises(qe):
        engine.flush_deferred()
    c2 = engine.alloc_counts(n)
    engine.sample_check_packed(n, 6, 0, count, packed, c2, deferred=True)
    engine.flush_deferred()
    torch.cuda.synchronize()
    assert _eq(c2, _ref_counts(engine, n, 6, 0, count))
    assert list(engine.last_stats()) == [0, 0]


def _stream_ref(engine, n, seed, first, count):
    info = engine.prepare(n)
    H, C, P, _ = oracle_lib.stream_counts(n, seed, first, count, info["notq"], info["q"], info["closed"])
    return H, C, P


@pytest.mark.parametrize("packed", [True, False])
def test_deferred_pairbin_tail_chain(engine, packed):
    """Large deferred calls (>= 2^24 entries: the pair-bin kernel) run the
    pending reduction in workgroups after their own (qba_k_lists_pbdef), and
    small deferred calls reduce a pair-bin call's slab: a mixed chain, each
    call into its own outputs, equal to the C twin."""
    n = 11
    calls = [(51, 7, 60_001), (52, 1000, 20_000_003), (53, 0, 17_000_000), (54, 5, 90_000), (55, 0, 16_777_216)]
    outs = [_call(engine, packed, n, s, f, c) for s, f, c in calls]
    engine.flush_deferred()
    torch.cuda.synchronize()
    for (s, f, c), o in zip(calls, outs):
        assert _eq(o, _stream_ref(engine, n, s, f, c)), (s, f, c)
    assert list(engine.last_stats()) == [0, 0]


@pytest.mark.parametrize("packed", [True, False])
def test_deferred_pairbin_tail_forced_small(packed):
    """The tail-deferred pair-bin kernel forced on small, ragged calls
    (pb_min = 0, qba_test_set_knobs): a chain of deferred calls, one
    accumulating."""
    eng = sub("engine").Engine(0).set_test_knobs(pb_min=0)
    try:
        n = 11
        calls = [(61, 0, 1), (62, 3, 4099), (63, 10, 250_001), (64, 0, 1_000_000)]
        outs = [_call(eng, packed, n, s, f, c) for s, f, c in calls]
        acc = eng.alloc_counts(n)
        for i, (f, c) in enumerate([(0, 30_001), (30_001, 70_000)]):
            _call(eng, packed, n, 65, f, c, counts=acc, accumulate=i > 0)
        eng.flush_deferred()
        torch.cuda.synchronize()
        for (s, f, c), o in zip(calls, outs):
            assert _eq(o, _ref_counts(eng, n, s, f, c)), (s, f, c)
        assert _eq(acc, _ref_counts(eng, n, 65, 0, 100_001))
    finally:
        eng.close()


def _bench():
    import importlib.util
    from conftest import ROOT
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def _rows_window(p, start, count):
    """Columns [start, start+count) of nibble rows p (device), unpacked on the host."""
    b0, b1 = start // 2, (start + count + 1) // 2
    u = sub("engine").unpack_nibbles(p[:, b0:b1].cpu().numpy(), 2 * (b1 - b0))
    return u[:, start - 2 * b0:start - 2 * b0 + count]


@pytest.mark.parametrize("seed,first,count,golden_shard", [
    (77, 1000, (1 << 24) + 12_345, None),          # >= 2^24: qba_k_lists_pbdef<11,2,1>, ragged tail
    (0x5EED, 0, 125_000_000, 0),                    # the bench step itself (rank 0's shard)
    (0x5EED, 5 * 125_000_000, 125_000_000, 5),      # rank 5's shard of sizeL = 1e9
])
def test_deferred_pairbin_rows_bit_exact(engine, seed, first, count, golden_shard):
    """the ROWS the timed kernel writes.  bench.py times
    qba_sample_check_packed_deferred at >= 2^24 entries, i.e. the pair-bin
    kernel with the previous call's reduction in its tail (qba_k_lists_pbdef).
    A deferred call runs first, so that reduction is live; then the rows of
    the big call are compared with the C twin (oracle_lib.sample, tfg.py:
    68-84, 128-129) over its first and last 4,099 entries and three windows
    inside, and their device checksums (bench.device_row_sums, every entry)
    with the C twin's -- at the bench's size with the recorded fixture of
    that shard (tests/golden/gen_config2_rows.py).  The counts of both calls
    are checked too (the pending call's against the C twin, the big call's
    against the configs[2] totals where recorded)."""
    n = 11
    info = engine.prepare(n)
    prior = _call(engine, True, n, 4242, 0, 20_000_000)            # pending reduction
    p, c = engine.sample_check_packed(n, seed, first, count, deferred=True)
    _call(engine, True, n, 4343, 0, 60_000)                          # reduces the big call
    engine.flush_deferred()
    torch.cuda.synchronize()
    assert list(engine.last_stats()) == [0, 0]
    rng = np.random.default_rng(count)
    starts = [0, count - 4099] + sorted(int(x) for x in rng.integers(4099, count - 70_000, 3))
    for s in starts:
        m = 4099 if s in (0, count - 4099) else 65_537
        ref = oracle_lib.sample(n, seed, first + s, m, info["notq"], info["q"], info["closed"])
        assert np.array_equal(_rows_window(p, s, m), ref), (first, s, m)
    sums = _bench().device_row_sums(p, n, count, True).cpu().numpy()
    if golden_shard is None:
        want = oracle_lib.stream_row_sums(n, seed, first, count, info["notq"], info["q"], info["closed"])
    else:
        from conftest import GOLDEN
        want = np.load(GOLDEN / "config2_rows_n11_5eed.npz")["S"][golden_shard]
    assert np.array_equal(sums, want.astype(np.int64))
    assert _eq(prior, _stream_ref(engine, n, 4242, 0, 20_000_000))
    if golden_shard is None:
        assert _eq(c, _stream_ref(engine, n, seed, first, count))
    elif golden_shard == 0:
        from conftest import GOLDEN
        z = np.load(GOLDEN / "config2_totals_n11_5eed.npz")
        assert _eq(c, (z["H_1"], z["C_1"], z["P_1"]))
    del p
    torch.cuda.empty_cache()
