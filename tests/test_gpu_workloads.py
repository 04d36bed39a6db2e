"""GPU tests at the BASELINE.json workloads themselves, and the full-joint
distribution tests of the sampler.

* configs[2]: n = 11, sizeL = 1e9 -- every one of the 8 GPU shards (1.25e8
  entries each, ``distributed.shard_bounds``) sampled and checked on this
  GPU, the summed counts equal to the C twin's streaming count over all 1e9
  entries; the last shard's lists spot-checked byte for byte;
* a real 2^31-entry launch-chunk crossing (one ``sample_check`` call of
  2^31 + 12,345 entries, no environment override) and ``count_tables`` over
  the same sizeL;
* configs[3]: 4096 independent n = 7 instances x 1e5 entries, counts of every
  instance against the C twin, lists of 16 instances;
* configs[4]: the largest fp64 GHZ register of the Q resource that fits the
  GPU (35 qubits = 256 GiB on an MI355X) and both full n = 7 circuits
  (24 qubits) gate by gate, supports exact and probabilities within 1e-12;
* the joint outcome distribution of the reference's circuits (tfg.py:68-84):
  at n = 2 and n = 3 a chi-square / total-variation test of >= 1e7 sampled
  entries over all w^(n+1) outcomes against the probabilities of a dense
  statevector simulation of the reference's gate lists (zero-probability
  outcomes must never appear); at n = 7 uniformity of pi over all 7! = 5040
  permutations and independence of r from pi.

The checkers are the oracle (C twin, dense numpy statevector); the sampler's
RNG is the engine's own (qsimov's is unpinned), so the
distribution tests are statistical with the thresholds written below.
"""
import math

import numpy as np
import pytest
import torch
from scipy import stats

import oracle_lib
import statevector as sv_oracle
from conftest import sub

pytestmark = pytest.mark.gpu

# fixed seeds: every statistical test below is deterministic; the thresholds
# are the ones a correct sampler passes with overwhelming probability
P_MIN = 1e-6        # chi-square p-value floor
TV_SLACK = 4.0      # TV must stay below TV_SLACK * sqrt(K / N)


def _windows(total, width=65_536):
    mid = total // 2 - width // 2
    return [(0, width), (mid, mid + width), (total - width, total)]


def _assert_counts(c, H, C, P, what):
    gH, gC, gP = c if isinstance(c, tuple) else c.numpy()
    assert np.array_equal(gH, H), f"{what}: H differs"
    assert np.array_equal(gC, C), f"{what}: C differs"
    assert np.array_equal(gP, P), f"{what}: P differs"


_C2_TOTALS = {}


def _config2_totals(info, n, seed, sizeL):
    """The C twin's streaming counts over all 1e9 entries (computed once)."""
    key = (n, seed, sizeL)
    if key not in _C2_TOTALS:
        _C2_TOTALS[key] = oracle_lib.stream_counts(n, seed, 0, sizeL, info["notq"], info["q"], info["closed"])
    return _C2_TOTALS[key]


@pytest.mark.parametrize("layout", ["packed", "bytes"])
def test_config2_sizeL_1e9_all_shards(engine, layout):
    """BASELINE configs[2]: n = 11, sizeL = 1e9 as 8 shards of 1.25e8 entries
    (the per-GPU workload of the 8-GPU run); counts summed over the shards
    (what the RCCL all-reduce produces) == the C twin over all 1e9 entries.
    "packed" runs exactly the kernel and layout bench.py times
    (qba_sample_check_packed: nibble rows, pair-bin counting); "bytes" the
    byte-row form of the same fused kernel."""
    dist = sub("distributed")
    n, sizeL, world, seed = 11, 10 ** 9, 8, 0x5EED
    info = engine.prepare(n)
    per = dist.shard_bounds(sizeL, 0, world)[1]
    packed = layout == "packed"
    lists = engine.alloc_packed(n, per) if packed else engine.alloc_lists(n, per)
    total = engine.alloc_counts(n)
    for r in range(world):
        first, count = dist.shard_bounds(sizeL, r, world)
        if packed:
            engine.sample_check_packed(n, seed, first, count, lists, total, accumulate=r > 0)
        else:
            engine.sample_check(n, seed, first, count, lists, total, accumulate=r > 0)
    torch.cuda.synchronize()
    # lists of the last shard, three windows, value for value
    first, count = dist.shard_bounds(sizeL, world - 1, world)
    for a, b in _windows(count):
        ref = oracle_lib.sample(n, seed, first + a, b - a, info["notq"], info["q"], info["closed"])
        got = (sub("engine").unpack_nibbles(lists[:, a // 2:(b + 1) // 2].cpu().numpy(), b - a) if packed
               else lists[:, a:b].cpu().numpy())
        assert np.array_equal(got, ref), (a, b)
    H, C, P, bad = _config2_totals(info, n, seed, sizeL)
    assert bad == 0
    _assert_counts(total, H, C, P, f"sizeL=1e9 ({layout})")
    # honest lists: every Q position collision-free, |P| ~ sizeL / 2
    assert C.sum() == P.sum() * (n + 1)
    assert abs(P.sum() - sizeL / 2) < 6 * math.sqrt(sizeL / 4)


def test_config2_single_shard_one_call(engine):
    """One 1.25e8-entry sample_check call (the headline's launch) == the C twin."""
    n, seed, first, count = 11, 4242, 3 * 125_000_000, 125_000_000
    info = engine.prepare(n)
    lists, c = engine.sample_check(n, seed, first, count)
    c2 = engine.check_counts(lists, n, count)  # the check-only kernel on the same lists
    torch.cuda.synchronize()
    H, C, P, bad = oracle_lib.stream_counts(n, seed, first, count, info["notq"], info["q"], info["closed"])
    assert bad == 0
    _assert_counts(c, H, C, P, "fused")
    _assert_counts(c2, H, C, P, "check-only")
    for a, b in _windows(count):
        ref = oracle_lib.sample(n, seed, first + a, b - a, info["notq"], info["q"], info["closed"])
        assert np.array_equal(lists[:, a:b].cpu().numpy(), ref), (a, b)
    del lists
    torch.cuda.empty_cache()


def test_chunk_crossing_2p31(engine):
    """2^31 + 12,345 entries in ONE call: the library splits it into launches
    of 2^31 entries (32-bit in-kernel offsets, u32 bins); lists around the
    boundary and counts must be unaffected.  count_tables over the same sizeL
    (host chunks of 2^27) gives the same counts."""
    n, seed, count = 11, 99, (1 << 31) + 12_345
    info = engine.prepare(n)
    lists, c = engine.sample_check(n, seed, 0, count)
    torch.cuda.synchronize()
    H, C, P, bad = oracle_lib.stream_counts(n, seed, 0, count, info["notq"], info["q"], info["closed"])
    assert bad == 0
    _assert_counts(c, H, C, P, "2^31 + 12345")
    edge = 1 << 31
    for a, b in [(edge - 70_001, edge + 12_345), (0, 4096)]:
        ref = oracle_lib.sample(n, seed, a, b - a, info["notq"], info["q"], info["closed"])
        assert np.array_equal(lists[:, a:b].cpu().numpy(), ref), (a, b)
    del lists, c
    torch.cuda.empty_cache()
    flat = engine.count_tables(n, count, seed)
    h, cc = H.size, C.size
    assert np.array_equal(flat[:h].reshape(H.shape), H)
    assert np.array_equal(flat[h:h + cc].reshape(C.shape), C)
    assert np.array_equal(flat[h + cc:], P)


@pytest.mark.parametrize("col", [0, 4])
def test_phi_span_crossing_unaligned_first(engine, col):
    """One call across a multiple of 2^33 entries (the launch split that keeps
    the Philox counter's high word uniform) with first % 8 != 0, into rows
    whose first column is 8-B aligned (col 0) or only 4-B aligned (col 4):
    the alignment chunks keep the later launches on the wide kernel and the
    lists / counts stay bit-exact against the C twin."""
    n, seed = 11, 0x5EED
    first, count = (1 << 33) - 1_000_003, 2_000_013
    info = engine.prepare(n)
    buf = engine.alloc_lists(n, count + 8)
    lists = buf[:, col:]
    _, c = engine.sample_check(n, seed, first, count, lists)
    torch.cuda.synchronize()
    ref = oracle_lib.sample(n, seed, first, count, info["notq"], info["q"], info["closed"])
    assert np.array_equal(lists[:, :count].cpu().numpy(), ref)
    H, C, P, bad = oracle_lib.counts(ref, n)
    assert bad == 0
    _assert_counts(c, H, C, P, f"2^33 crossing, column {col}")


@pytest.mark.parametrize("layout", ["bytes", "packed"])
def test_config3_full_batched(engine, layout):
    """BASELINE configs[3]: 4096 independent 7-party instances x sizeL = 1e5
    per GPU; every instance's counts vs the C twin, 16 instances' lists.
    "packed" is the nibble-row form bench.py --config 3 times."""
    n, n_inst, count, base = 7, 4096, 100_000, 0x5EED
    info = engine.prepare(n)
    packed = layout == "packed"
    lists, c = engine.sample_check_batched(n, base, n_inst, count, packed=packed)
    torch.cuda.synchronize()
    H, C, P = oracle_lib.batched_counts(n, base, n_inst, count, info["notq"], info["q"], info["closed"])
    _assert_counts(c, H, C, P, f"batched ({layout})")
    for i in np.linspace(0, n_inst - 1, 16).astype(int):
        ref = oracle_lib.sample(n, base + int(i), 0, count, info["notq"], info["q"], info["closed"])
        got = (sub("engine").unpack_nibbles(lists[i].cpu().numpy(), count) if packed
               else lists[i, :, :count].cpu().numpy())
        assert np.array_equal(got, ref), i
    del lists, c
    torch.cuda.empty_cache()


def test_config4_largest_register(engine):
    """BASELINE configs[4]: the largest GHZ register of the Q resource
    (tfg.py:38-39 on one bit of every group: H, then q-1 CX gates from it)
    whose fp64 statevector fits this GPU; support {0...0, 1...1} at 1/2."""
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    q = 1
    while (8 << (q + 1)) < free * 0.95:
        q += 1
    # the largest register that fits at all: one more qubit doubles the state past free memory
    assert (8 << q) <= free < (8 << (q + 2)), (q, free)
    if torch.cuda.get_device_properties(0).total_memory >= 256 << 30:  # MI355X, 288 GB HBM3E
        assert q == 35, (q, free)  # BASELINE configs[4]: 2^35 fp64 amplitudes = 256 GiB
    gates = np.array([(0, 0, -1)] + [(1, t, 0) for t in range(1, q)], np.int32)
    sv = torch.empty(1 << q, dtype=torch.float64, device=engine.device)
    engine.statevector(q, gates, out=sv)
    idx, prob = engine.support(sv, q, cap=16)
    assert list(idx) == [0, (1 << q) - 1], q
    assert np.max(np.abs(prob - 0.5)) < 1e-12
    del sv
    torch.cuda.empty_cache()


@pytest.mark.parametrize("perm", [[1, 2, 3, 4, 5, 6, 7], [4, 5, 6, 7, 1, 2, 3], [7, 3, 1, 6, 2, 5, 4]])
def test_config4_full_circuits_n7(engine, perm):
    """The largest n whose WHOLE resource fits as one dense state (n = 7, 24
    qubits): both circuits gate by gate; support and probabilities exact."""
    res = sub("resource")
    n = 7
    nq = res.n_qubits(n)
    N, W = (n + 1) * nq, 1 << nq
    shift = [N - (g + 1) * nq for g in range(n + 1)]
    for kind, gate in (("notq", res.notQCorrelated(n, nq)), ("q", res.qCorrelated(n, nq, perm=perm))):
        sv = engine.statevector(N, gate.triples())
        idx, prob = engine.support(sv, N, cap=1 << 22)
        if kind == "notq":
            fields = np.stack([(idx >> s) & (W - 1) for s in shift])
            assert len(idx) == W ** n and bool((fields[0] == fields[1]).all())
            assert np.max(np.abs(prob - float(W) ** -n)) < 1e-12
        else:
            pi = [0] + list(perm)
            want = np.sort([sum((r ^ pi[g]) << shift[g] for g in range(n + 1)) for r in range(W)])
            assert np.array_equal(np.sort(idx), want)
            assert np.max(np.abs(prob - 1.0 / W)) < 1e-12


# ---------------------------------------------------------------------------
# full-joint distribution of the sampled lists vs the reference's circuits
# ---------------------------------------------------------------------------
def _reference_joint(n):
    """P(L0..Ln) of one shot of tfg.py:68-84: isQ ~ Bernoulli(1/2); not-Q =
    the notQCorrelated circuit; Q = qCorrelated with pi uniform over all n!
    permutations -- each circuit simulated densely from its gate list (the
    lists equal the reference's, tests/test_oracle_golden.py)."""
    from itertools import permutations
    res = sub("resource")
    nq = res.n_qubits(n)
    N = (n + 1) * nq
    ops = lambda g: [(name, t, c) for name, t, c in g.ops]  # noqa: E731
    p_notq = sv_oracle.probabilities(sv_oracle.run(ops(res.notQCorrelated(n, nq)), N))
    p_q = np.zeros_like(p_notq)
    perms = list(permutations(range(1, n + 1)))
    for pm in perms:
        p_q += sv_oracle.probabilities(sv_oracle.run(ops(res.qCorrelated(n, nq, perm=pm)), N))
    return 0.5 * p_notq + 0.5 * p_q / len(perms)


@pytest.mark.parametrize("n,count", [(2, 10_000_000), (3, 16_000_000)])
def test_joint_distribution_chi2_tv(engine, n, count):
    """All w^(n+1) joint outcomes: chi-square over the support, total
    variation, and no sample outside the support (exactness of the zeros)."""
    nq, w = engine.sizes(n)
    prob = _reference_joint(n)                    # index = L0 L1 .. Ln base w (qubit 0 = MSB)
    lists = engine.sample(n, 0xD157 + n, 0, count)
    idx = torch.zeros(count, dtype=torch.int64, device=engine.device)
    for g in range(n + 1):
        idx = idx * w + lists[g, :count].to(torch.int64)
    hist = torch.bincount(idx, minlength=w ** (n + 1)).cpu().numpy()
    assert hist.sum() == count
    supp = prob > 0
    assert hist[~supp].sum() == 0, "sampled an outcome of probability 0"
    K = int(supp.sum())
    chi2 = stats.chisquare(hist[supp], prob[supp] * count)
    assert chi2.pvalue > P_MIN, chi2
    tv = 0.5 * np.abs(hist / count - prob).sum()
    assert tv < TV_SLACK * math.sqrt(K / count), (tv, K)


def test_n7_permutation_uniform_and_independent(engine):
    """n = 7: at Q positions pi(g) = L_g ^ L_0 must be uniform over all 5040
    permutations (Lehmer rank histogram) and independent of r = L_0
    (8 x 5040 contingency table)."""
    n, count = 7, 24_000_000
    lists = engine.sample(n, 0xBEEF, 0, count)[:, :count]
    q = lists[0] != lists[1]
    L = lists[:, q].to(torch.int64)
    r = L[0]
    pi = L[1:] ^ r                                    # (7, m), a permutation of 1..7 per column
    m = pi.shape[1]
    assert m > 11_000_000
    assert bool((torch.sort(pi, dim=0).values == torch.arange(1, n + 1, device=pi.device)[:, None]).all())
    rank = torch.zeros(m, dtype=torch.int64, device=pi.device)
    for i in range(n):                               # Lehmer code, most significant digit first
        smaller = (pi[i + 1:] < pi[i]).sum(0) if i + 1 < n else torch.zeros_like(rank)
        rank = rank * (n - i) + smaller
    nperm = math.factorial(n)
    h = torch.bincount(rank, minlength=nperm).cpu().numpy()
    assert h.shape[0] == nperm and h.min() > 0
    assert stats.chisquare(h).pvalue > P_MIN
    table = torch.bincount(r * nperm + rank, minlength=8 * nperm).reshape(8, nperm).cpu().numpy()
    ind = stats.chi2_contingency(table, correction=False)
    assert ind.pvalue > P_MIN, ind.pvalue
