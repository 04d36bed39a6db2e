"""GPU parity of the HIP kernels against the oracle (C twin + numpy restatement)."""
import json

import numpy as np
import pytest
import torch

import oracle_lib
import statevector as sv_oracle
import tfg_oracle as orc
from conftest import GOLDEN, sub

pytestmark = pytest.mark.gpu

KATS = [
    ([0, 0, 0, 0], 0, [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, 0xFFFFFFFFFFFFFFFF, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], 0x299F31D0A4093822,
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


def test_philox_device_kat(engine):
    for ctr, key, want in KATS:
        assert list(engine.philox(np.array(ctr, np.uint32), key)[0]) == want
    rng = np.random.default_rng(1)
    ctr = rng.integers(0, 2 ** 32, (4096, 4), dtype=np.uint64).astype(np.uint32)
    key = 0x0123456789ABCDEF
    assert np.array_equal(engine.philox(ctr, key), oracle_lib.philox(ctr, key))


def _program_distribution(prog, N):
    """Full outcome distribution of a compiled program (product of its factors)."""
    dist = {0: 1.0}
    for f in range(prog["nfac"]):
        bits, uniform, off = prog["desc"][f][:3]
        K = 1 << bits
        col_p = {}
        for c in range(K):
            thr = int(prog["thr"][off + c])
            keep = 1.0 if uniform else thr / 2 ** 32
            for pat, p in ((int(prog["pat"][off + c]), keep), (int(prog["apat"][off + c]), 1 - keep)):
                if p > 0:
                    col_p[pat] = col_p.get(pat, 0.0) + p / K
        new = {}
        for a, pa in dist.items():
            for b, pb in col_p.items():
                new[a ^ b] = new.get(a ^ b, 0.0) + pa * pb
        dist = new
    return dist


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5])
def test_program_matches_reference_statevector(engine, n):
    """Compiled tables == probabilities of the reference's own gate lists (gates.json)."""
    gates = json.loads((GOLDEN / "gates.json").read_text())[str(n)]
    N = gates["size"]
    info = engine.prepare(n)
    # not-Q circuit
    ops = [(g, t, c) for g, t, c in gates["notq"]]
    probs = sv_oracle.probabilities(sv_oracle.run(ops, N))
    dist = _program_distribution(info["notq"], N)
    idx = np.nonzero(probs > 1e-30)[0]
    assert sorted(dist) == sorted(int(i) for i in idx)
    for i in idx:
        assert abs(dist[int(i)] - probs[i]) < 1e-12
    # Q circuit: every recorded permutation; the program is pi-free, the mask is
    # the permutation layout the sampler draws
    nq = gates["nq"]
    for case in gates["q"]:
        ops = [(g, t, c) for g, t, c in case["ops"]]
        probs = sv_oracle.probabilities(sv_oracle.run(ops, N))
        mask = sum(int(v) << (N - (g + 1) * nq) for g, v in enumerate(case["perm"], start=1))
        dist = _program_distribution(info["q"], N)
        idx = np.nonzero(probs > 1e-30)[0]
        assert sorted(a ^ mask for a in dist) == sorted(int(i) for i in idx)
        for a, p in dist.items():
            assert abs(p - probs[a ^ mask]) < 1e-12


@pytest.mark.parametrize("n", [6, 7, 8, 11, 12, 15])
def test_program_registers_large_n(engine, n):
    """Per-factor check at sizes where the full state does not fit: the program's
    marginal over each group equals the closed form (A1/A2)."""
    info = engine.prepare(n)
    nq, w = engine.sizes(n)
    N = (n + 1) * nq
    for kind in ("notq", "q"):
        prog = info[kind]
        total_bits = sum(int(d[0]) for d in prog["desc"])
        assert all(int(d[1]) == 1 for d in prog["desc"]), "H/X/CX resources are uniform"
        if kind == "q":
            assert total_bits == nq  # the GHZ registers: L_g = r for all g
            pats = set(int(p) for p in prog["pat"])
            want = {sum(r << (N - (g + 1) * nq) for g in range(n + 1)) for r in range(w)}
            assert pats == want
        else:
            assert total_bits == n * nq  # L0 = L1 and L1..Ln free


@pytest.mark.parametrize("n,first,count", [(1, 0, 1001), (2, 7, 999), (3, 0, 4096), (4, 1, 30_001),
                                           (5, 3, 777), (6, 0, 30_000), (7, 1 << 33, 5003), (8, 2, 40_003),
                                           (9, 5, 40_000), (10, 0, 50_001), (11, 0, 100_003),
                                           (11, (1 << 40) + 5, 20_001), (13, 99, 3000), (15, 1, 8191)])
def test_sampler_bit_exact(engine, n, first, count):
    seed = 0x5EED ^ (n << 20)
    info = engine.prepare(n)
    lists = engine.sample(n, seed, first, count)
    torch.cuda.synchronize()
    got = lists[:, :count].cpu().numpy()
    ref = oracle_lib.sample(n, seed, first, count, info["notq"], info["q"], info["closed"])
    assert np.array_equal(got, ref)


def test_shard_invariance(engine):
    """Lists depend only on the global entry index: any split gives the same bytes."""
    n, seed, total = 11, 77, 50_000
    full = engine.sample(n, seed, 0, total)[:, :total].cpu().numpy()
    cuts = [0, 1, 4097, 12_345, 33_333, total]
    parts = [engine.sample(n, seed, a, b - a)[:, : b - a].cpu().numpy() for a, b in zip(cuts, cuts[1:])]
    assert np.array_equal(np.concatenate(parts, axis=1), full)


def test_structure_and_chi2(engine):
    """At Q positions all n+1 values are distinct and L_g XOR L_1 is a permutation
    pattern; elsewhere L0 == L1; marginals uniform (chi-square)."""
    from scipy import stats
    n, count = 11, 2_000_000
    nq, w = engine.sizes(n)
    L = engine.sample(n, 2024, 0, count)[:, :count].cpu().numpy().astype(np.int64)
    q = L[0] != L[1]
    frac = q.mean()
    assert abs(frac - 0.5) < 5 * np.sqrt(0.25 / count)
    Lq = L[:, q]
    srt = np.sort(Lq, axis=0)
    assert (np.diff(srt, axis=0) != 0).all()
    x = Lq[1:] ^ Lq[0]  # pi(g) for g = 1..n
    assert np.array_equal(np.sort(x, axis=0), np.repeat(np.arange(1, n + 1)[:, None], x.shape[1], 1))
    for g in range(n + 1):
        cnt = np.bincount(L[g], minlength=w)
        assert stats.chisquare(cnt).pvalue > 1e-4
    # pi(1) uniform over 1..n at Q positions, pairs (L2, L3) independent at non-Q
    assert stats.chisquare(np.bincount(x[0], minlength=n + 1)[1:]).pvalue > 1e-4
    nonq = L[:, ~q]
    joint = np.bincount(nonq[2] * w + nonq[3], minlength=w * w)
    assert stats.chisquare(joint).pvalue > 1e-4


@pytest.mark.parametrize("n,count", [(3, 10_001), (7, 40_000), (11, 123_457), (15, 5000)])
def test_counts_match_oracle(engine, n, count):
    seed = 99 + n
    info = engine.prepare(n)
    lists, c_fused = engine.sample_check(n, seed, 5, count)
    c_sep = engine.check_counts(lists, n, count)
    torch.cuda.synchronize()
    ref_lists = oracle_lib.sample(n, seed, 5, count, info["notq"], info["q"], info["closed"])
    H, C, P, bad = oracle_lib.counts(ref_lists, n)
    assert bad == 0
    for c in (c_fused, c_sep):
        gH, gC, gP = c.numpy()
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)
    # numpy restatement agrees as well
    H2, C2, P2 = orc.counts(ref_lists, n)
    assert np.array_equal(H2, H) and np.array_equal(C2, C) and np.array_equal(P2, P)


def test_counts_on_fixture_lists(engine):
    """Count mode on the injected fixture lists, incl. tampered / uniform ones with
    collisions (slow path) -- against the numpy restatement."""
    arrays = np.load(GOLDEN / "protocol_lists.npz")
    for name in arrays.files:
        L = arrays[name]
        n = L.shape[0] - 1
        d = torch.zeros((n + 1, (L.shape[1] + 63) // 64 * 64), dtype=torch.uint8, device=engine.device)
        d[:, : L.shape[1]] = torch.from_numpy(L)
        c = engine.check_counts(d, n, L.shape[1])
        gH, gC, gP = c.numpy()
        H, C, P = orc.counts(L, n)
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P), name


def test_counts_accumulate_and_invalid(engine):
    n, count = 7, 10_000
    lists = engine.sample(n, 5, 0, count)
    a = engine.check_counts(lists, n, count)
    b = engine.check_counts(lists, n, count, counts=engine.alloc_counts(n))
    engine.check_counts(lists, n, count, counts=b, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(b.H, 2 * a.H) and torch.equal(b.C, 2 * a.C) and torch.equal(b.P, 2 * a.P)
    bad = lists.clone()
    q = (bad[0, :count] != bad[1, :count]).nonzero()[:3, 0]
    bad[5, q] = 200
    engine.check_counts(bad, n, count)
    assert engine.last_stats()[0] == 3


@pytest.mark.parametrize("n", [3, 11])
def test_counts_out_of_range_values(engine, n):
    """Values >= W (tfg.py:94 Cond2) in Q and in not-Q entries, scattered so
    that some waves see one and others none: the quad-level range test must
    fall back to the per-entry test exactly (stats[0] = bad Q entries, which
    add nothing to H / C / P; not-Q entries are never counted)."""
    count = 50_000
    lists = engine.sample(n, 77, 0, count)
    torch.cuda.synchronize()
    L = lists[:, :count].cpu().numpy().copy()
    rng = np.random.default_rng(n)
    isq = np.nonzero(L[0] != L[1])[0]
    notq = np.nonzero(L[0] == L[1])[0]
    for k in rng.choice(isq, 7, replace=False):  # bad Q entries
        L[rng.integers(2, n + 1), k] = rng.integers(1 << oracle_lib.n_qubits(n), 256)
    for k in rng.choice(notq, 5, replace=False):  # bad not-Q entries: not counted at all
        L[rng.integers(2, n + 1), k] = 255
    k = isq[0]  # a bad Q entry that also collides
    L[2, k], L[3, k] = 250, 250
    d = torch.zeros_like(lists)
    d[:, :count] = torch.from_numpy(L)
    c = engine.check_counts(d, n, count)
    gH, gC, gP = c.numpy()
    H, C, P, bad = oracle_lib.counts(L, n)
    assert bad == engine.last_stats()[0] >= 7
    assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5])
def test_full_statevector_vs_oracle(engine, n):
    gates = json.loads((GOLDEN / "gates.json").read_text())[str(n)]
    N = gates["size"]
    for ops in [gates["notq"]] + [c["ops"] for c in gates["q"]]:
        trip = np.array([(0 if g == "H" else 1, t, c) for g, t, c in ops], np.int32)
        sv = engine.statevector(N, trip)
        torch.cuda.synchronize()
        ref = sv_oracle.run([tuple(o) for o in ops], N)
        assert np.max(np.abs(sv.cpu().numpy() - ref)) < 1e-12
        idx, prob = engine.support(sv, N)
        ridx, rprob = sv_oracle.support(sv_oracle.probabilities(ref), 1e-24)
        assert np.array_equal(idx, ridx) and np.max(np.abs(prob - rprob)) < 1e-12


@pytest.mark.parametrize("q", [1, 2, 3, 5, 10])
def test_statevector_random_circuits_fused_runs(engine, q):
    """Random H / X / CX lists with long runs of X gates and of CX gates that
    share a control (those runs become one XOR-mask pass each, incl. repeated
    targets that cancel, bit 0 in the mask and the control on bit 0) -- vs the
    dense oracle, which applies every gate on its own."""
    rng = np.random.default_rng(1000 + q)
    for trial in range(6):
        ops = []
        while len(ops) < 40:
            kind = rng.integers(3)
            if kind == 0:
                ops.append(("H", int(rng.integers(q)), -1))
            elif kind == 1:
                for _ in range(int(rng.integers(1, 6))):
                    ops.append(("X", int(rng.integers(q)), -1))
            elif q > 1:
                c = int(rng.integers(q))
                for _ in range(int(rng.integers(1, 8))):
                    t = int(rng.integers(q - 1))
                    ops.append(("X", t + (t >= c), c))
        trip = np.array([(0 if g == "H" else 1, t, c) for g, t, c in ops], np.int32)
        sv = engine.statevector(q, trip)
        torch.cuda.synchronize()
        ref = sv_oracle.run(ops, q)
        assert np.max(np.abs(sv.cpu().numpy() - ref)) < 1e-12, (q, trial)


@pytest.mark.parametrize("q", [1, 2, 4, 7, 12])
def test_statevector_fused_h_and_product_prefix(engine, q):
    """Gate fusion of qba_sv_prepare / qba_sv_apply vs the dense oracle, which
    applies every gate on its own: random single-qubit layers (H, X, repeated
    H that cancel, H X H = Z-type sign flips) folded into the init pass,
    interleaved with CX gates after which single-qubit gates on touched
    qubits must stay in order, and long H runs over > QBA_HSET_MAX qubits
    (several Walsh-Hadamard passes, bit 0 in and out of the set)."""
    rng = np.random.default_rng(7000 + q)
    for trial in range(8):
        ops = []
        for _ in range(int(rng.integers(4, 30))):  # single-qubit prefix layer
            ops.append((["H", "X"][int(rng.integers(2))], int(rng.integers(q)), -1))
        while len(ops) < 60:
            r = rng.integers(4)
            if r == 0 and q > 1:
                c = int(rng.integers(q))
                t = int(rng.integers(q - 1))
                ops.append(("X", t + (t >= c), c))
            elif r == 1:  # an H run over a random subset, possibly repeated qubits
                for t in rng.integers(q, size=int(rng.integers(1, 2 * q + 1))):
                    ops.append(("H", int(t), -1))
            else:
                ops.append((["H", "X"][int(rng.integers(2))], int(rng.integers(q)), -1))
        trip = np.array([(0 if g == "H" else 1, t, c) for g, t, c in ops], np.int32)
        ref = sv_oracle.run(ops, q)
        for fn in (engine.statevector, engine.statevector_unfused):
            sv = fn(q, trip)
            torch.cuda.synchronize()
            assert np.max(np.abs(sv.cpu().numpy() - ref)) < 1e-12, (q, trial, fn.__name__)
    # all-H register: one product pass, uniform amplitudes
    trip = np.array([(0, t, -1) for t in range(q)], np.int32)
    sv = engine.statevector(q, trip).cpu().numpy()
    assert np.max(np.abs(sv - 2.0 ** (-q / 2))) < 1e-15


@pytest.mark.parametrize("q", [2, 3, 6, 11])
def test_statevector_commuting_cx_windows(engine, q):
    """Windows of pairwise-commuting X / CX gates with several controls (one
    qba_k_sv_xmulti pass, controls on bit 0 -> scalar path, > 8 controls ->
    window split), broken by a gate whose target is a window control -- vs
    the dense oracle."""
    rng = np.random.default_rng(9100 + q)
    for trial in range(10):
        ops = [(["H", "X"][int(rng.integers(2))], int(rng.integers(q)), -1) for _ in range(2 * q)]
        for _ in range(4):
            perm = rng.permutation(q)
            nc = int(rng.integers(1, max(2, q // 2) + 1))
            ctl, tgt = [int(x) for x in perm[:nc]], [int(x) for x in perm[nc:]]
            if not tgt:
                continue
            for _ in range(int(rng.integers(1, 3 * q))):
                t = tgt[int(rng.integers(len(tgt)))]
                c = -1 if rng.random() < 0.2 else ctl[int(rng.integers(len(ctl)))]
                ops.append(("X", t, c))
            if rng.random() < 0.5:  # breaks the window: a control becomes a target
                ops.append(("X", ctl[0], tgt[0]))
            if rng.random() < 0.3:
                ops.append(("H", int(rng.integers(q)), -1))
        trip = np.array([(0 if g == "H" else 1, t, c) for g, t, c in ops], np.int32)
        ref = sv_oracle.run(ops, q)
        for fn in (engine.statevector, engine.statevector_unfused):
            sv = fn(q, trip)
            torch.cuda.synchronize()
            assert np.max(np.abs(sv.cpu().numpy() - ref)) < 1e-12, (q, trial, fn.__name__)


def test_ghz_register_statevector(engine):
    """One entangled register of the Q resource (n+1 qubits) at n=19: support
    {0...0, 1...1}, each 1/2 (the per-register closed form of A2)."""
    q = 20
    trip = np.array([(0, 0, -1)] + [(1, t, 0) for t in range(1, q)], np.int32)
    sv = engine.statevector(q, trip)
    idx, prob = engine.support(sv, q)
    assert list(idx) == [0, (1 << q) - 1]
    assert np.max(np.abs(prob - 0.5)) < 1e-12


def test_compaction_multiblock_scan(engine):
    """isQCorrList over more than 8192 tiles of 4096 entries: the tile counts
    are scanned by the three-launch path (block sums, their scan, block
    scans); the ascending index list must equal numpy's, including a ragged
    last tile and runs of empty tiles."""
    rng = np.random.default_rng(11)
    count = 8192 * 4096 + 3 * 4096 + 777
    l0 = rng.integers(0, 4, count, dtype=np.uint8)
    l1 = l0.copy()
    flip = rng.random(count) < 0.3
    flip[5_000_000:9_000_000] = False          # empty tiles
    flip[20_000_000:20_100_000] = True         # full tiles
    l1[flip] ^= 1
    want = np.nonzero(l0 != l1)[0]
    got = engine.isq_indices(engine.to_device(l0), engine.to_device(l1))
    assert got.shape == want.shape and np.array_equal(got, want)


def test_exact_mode_kernels(engine):
    rng = np.random.default_rng(3)
    for count in (1, 17, 1000, 70_001):
        l0 = rng.integers(0, 4, count).astype(np.uint8)
        l1 = np.where(rng.random(count) < 0.5, l0, rng.integers(0, 4, count)).astype(np.uint8)
        d0, d1 = engine.to_device(l0), engine.to_device(l1)
        assert np.array_equal(engine.isq_indices(d0, d1), orc.is_qcorr_indices(l0, l1))
        order = rng.permutation(count).astype(np.int64)
        for v in range(4):
            assert engine.select_eq(order, d1, v).tolist() == orc.p_filter(order, l1, v)
        idx = rng.integers(0, count, min(count, 500)).astype(np.int64)
        assert tuple(engine.gather(d0, idx)) == orc.gather(l0, idx)
    with pytest.raises(sub("_lib").QbaError):
        engine.gather(d0, np.array([count], np.int64))


def test_consistent_kernel_kat(engine):
    """qba_consistent + host Cond1 == the reference's consistent() on its KAT table."""
    for case in json.loads((GOLDEN / "consistent.json").read_text()):
        tuples = list({tuple(t) for t in case["L"]})
        if not tuples:
            assert case.get("error") == "StopIteration"
            continue
        lens = {len(t) for t in tuples}
        if len(lens) > 1:
            got = False
        else:
            got = engine.consistent_rows(np.array(tuples, np.int64).reshape(len(tuples), -1),
                                         case["v"], case["w"])
        assert got == case["result"], case


def test_codec_kat(engine):
    for case in json.loads((GOLDEN / "codec.json").read_text()):
        raw = engine.to_device(np.array(case["raw"], np.int64))
        vals = engine.bits_to_values(raw, case["sizeL"], case["nq"]).cpu().numpy()
        assert vals.tolist() == case["ints"]
        back = engine.values_to_bits(engine.to_device(vals), case["sizeL"], case["nq"]).cpu().numpy()
        assert back.tolist() == case["raw"]


def test_log_tuples_exact_order(engine):
    """The reference's own captured runs (logs tests/): every honest lieutenant
    packet's L holds the sender's tuple gathered in the ORDER IN WHICH THAT
    SENDER RECEIVED P (the wire order of the packet that delivered P).

    The logs predate the current tfg.py (they print 'w =' where tfg.py:136
    prints '|W| ='); in that version the tuple follows the received order,
    while the current code iterates the rebuilt set (tfg.py:240, 291).  Either
    way the gather kernel must reproduce a tuple from a given index order."""
    logs = json.loads((GOLDEN / "logs.json").read_text())
    arrays = np.load(GOLDEN / "logs.npz")
    checked = 0
    for info in logs:
        L = arrays[info["file"][:-4]]
        pk = info["packets"]
        for i, p in enumerate(pk):
            if p["src"] < 2 or p["bad"] or not p["P_order"]:
                continue
            li = engine.to_device(L[p["src"]])
            incoming = [q for q in pk[:i] if q["dst"] == p["src"] and set(q["P_order"]) == set(p["P_order"])]
            hits = [[int(x) for x in engine.gather(li, np.array(q["P_order"], np.int64))] in p["L"]
                    for q in incoming]
            assert any(hits), (info["file"], p["src"], p["dst"])
            checked += 1
    assert checked == 205


def test_batched_instances(engine):
    """Batched mode (configs[3] shape, scaled down): instance i == an ordinary
    run with seed base+i, bit for bit, lists and counts."""
    n, n_inst, count, base = 7, 37, 3001, 1000
    info = engine.prepare(n)
    lists, c = engine.sample_check_batched(n, base, n_inst, count)
    torch.cuda.synchronize()
    for i in (0, 1, 17, 36):
        ref = oracle_lib.sample(n, base + i, 0, count, info["notq"], info["q"], info["closed"])
        assert np.array_equal(lists[i, :, :count].cpu().numpy(), ref)
        H, C, P, bad = oracle_lib.counts(ref, n)
        assert np.array_equal(c.H[i].cpu().numpy(), H)
        assert np.array_equal(c.C[i].cpu().numpy(), C)
        assert np.array_equal(c.P[i].cpu().numpy(), P)


def test_closed_form_flags(engine):
    """tfg.py's two circuits compile to the closed-form sampler for n <= 11
    (the programs are proven to be exactly their distributions) and to the
    canonical-table sampler above."""
    for n in (1, 2, 3, 7, 8, 11, 12, 15):
        info = engine.prepare(n)
        assert info["canonical"]
        assert info["closed"] == (n <= 11), n


def test_general_program_path(engine):
    """A circuit pair that is NOT tfg.py's (group 3 = copy of group 2 in the
    not-Q circuit) runs on the general alias-table sampler; bit-exact vs the
    C twin, and the count pass on its lists matches the oracle."""
    resource = sub("resource")
    n = 3
    nq = resource.n_qubits(n)
    notq = resource.Gate((n + 1) * nq)
    for qb in range(nq, 3 * nq):
        notq.add_operation("H", targets=qb)
    for j in range(nq):
        notq.add_operation("X", targets=j, controls=nq + j)
        notq.add_operation("X", targets=3 * nq + j, controls=2 * nq + j)
    q = resource.qCorrelated(n, nq, perm=[1, 2, 3])
    try:
        info = engine.compile(n, notq, q)
        assert not info["closed"] and not info["canonical"]
        seed, count = 4242, 70_001
        lists, counts = engine.sample_check(n, seed, 3, count)
        torch.cuda.synchronize()
        got = lists[:, :count].cpu().numpy()
        ref = oracle_lib.sample(n, seed, 3, count, info["notq"], info["q"], False)
        assert np.array_equal(got, ref)
        assert np.array_equal(got[3][got[0] == got[1]], got[2][got[0] == got[1]])
        H, C, P, bad = oracle_lib.counts(ref, n)
        gH, gC, gP = counts.numpy()
        assert bad == 0 and np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)
    finally:
        engine.prepare(n, perm=list(range(1, n + 1)))


def test_chunked_launches():
    """Launches are split into chunks of QBA_CHUNK entries (2^31; 32-bit
    in-kernel offsets and u32 bins).  With a small chunk forced through the
    test seam (qba_test_set_knobs), lists and counts must not change."""
    eng = sub("engine").Engine(0).set_test_knobs(chunk=40000)
    try:
        n, seed, first, count = 11, 31337, 999, 123_457
        info = eng.prepare(n)
        lists, counts = eng.sample_check(n, seed, first, count)
        torch.cuda.synchronize()
        got = lists[:, :count].cpu().numpy()
        ref = oracle_lib.sample(n, seed, first, count, info["notq"], info["q"], info["closed"])
        assert np.array_equal(got, ref)
        H, C, P, bad = oracle_lib.counts(ref, n)
        gH, gC, gP = counts.numpy()
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)
        c2 = eng.alloc_counts(n)
        eng.check_counts(lists, n, count, c2)
        assert np.array_equal(c2.numpy()[0], H)
    finally:
        eng.close()


@pytest.mark.parametrize("n,first,count", [(11, (1 << 33) - 4000, 12_008), (11, (1 << 34) - 3, 20_001),
                                           (7, (3 << 33) - 8, 16)])
def test_launch_split_at_counter_word(engine, n, first, count):
    """A launch never crosses a multiple of 2^33 entries (the high word of the
    Philox pair counter e >> 1 is uniform inside a launch): a call across one
    is split there, and lists and counts still equal the C twin's."""
    seed = 0xC0FFEE + n
    info = engine.prepare(n)
    lists, counts = engine.sample_check(n, seed, first, count)
    torch.cuda.synchronize()
    got = lists[:, :count].cpu().numpy()
    ref = oracle_lib.sample(n, seed, first, count, info["notq"], info["q"], info["closed"])
    assert np.array_equal(got, ref)
    H, C, P, _ = oracle_lib.counts(ref, n)
    gH, gC, gP = counts.numpy()
    assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)
    assert np.array_equal(engine.sample(n, seed, first, count)[:, :count].cpu().numpy(), ref)


def test_counts_repeated_accumulate_stats():
    """The count reduction (slab rows + qba_k_reduce) against the oracle on a
    fresh context: several n, repeated launches, accumulation, check-only
    launches and the stats of out-of-range values (set, then cleared)."""
    eng = sub("engine").Engine(0)
    try:
        for n, count in [(1, 999), (3, 10_001), (11, 123_457), (11, 5), (15, 4099)]:
            info = eng.prepare(n)
            seed = 4242 + n
            ref = oracle_lib.sample(n, seed, 7, count, info["notq"], info["q"], info["closed"])
            H, C, P, bad = oracle_lib.counts(ref, n)
            for _ in range(3):
                lists, c = eng.sample_check(n, seed, 7, count)
                gH, gC, gP = c.numpy()
                assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P), (n, count)
            eng.sample_check(n, seed, 7, count, lists, c, accumulate=True)
            gH, gC, gP = c.numpy()
            assert np.array_equal(gH, 2 * H) and np.array_equal(gC, 2 * C) and np.array_equal(gP, 2 * P)
            c2 = eng.check_counts(lists, n, count)
            assert np.array_equal(c2.numpy()[0], H)
        n, count = 7, 10_000
        eng.prepare(n)
        lists = eng.sample(n, 5, 0, count)
        bad = lists.clone()
        q = (bad[0, :count] != bad[1, :count]).nonzero()[:3, 0]
        bad[5, q] = 200
        eng.check_counts(bad, n, count)
        assert eng.last_stats()[0] == 3
        eng.check_counts(lists, n, count)
        assert eng.last_stats()[0] == 0
    finally:
        eng.close()


@pytest.mark.parametrize("count", [1, 3, 4, 5, 7, 8, 9, 15, 17, 4099])
def test_tiny_and_ragged_counts(engine, count):
    """Tail handling: fewer entries than one thread-step, ragged remainders
    (lists and counts vs the oracle, fused and check-only)."""
    n, seed, first = 11, 2024, 10
    info = engine.prepare(n)
    lists, c = engine.sample_check(n, seed, first, count)
    c2 = engine.check_counts(lists, n, count)
    torch.cuda.synchronize()
    got = lists[:, :count].cpu().numpy()
    ref = oracle_lib.sample(n, seed, first, count, info["notq"], info["q"], info["closed"])
    assert np.array_equal(got, ref)
    H, C, P, bad = oracle_lib.counts(ref, n)
    for cc in (c, c2):
        gH, gC, gP = cc.numpy()
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)


def test_unaligned_rows_narrow_path(engine):
    """Rows that are only 4-byte aligned (base offset 4, ld = 4 mod 8) run the
    one-quad-per-step kernels; same lists and counts as the oracle."""
    n, seed, count = 7, 77, 50_003
    info = engine.prepare(n)
    ld = (count + 63) // 64 * 64 + 4
    buf = torch.zeros((n + 1, ld), dtype=torch.uint8, device=engine.device)
    view = buf[:, 4:]
    assert view.data_ptr() % 8 == 4 and view.stride(0) % 8 == 4
    lists, c = engine.sample_check(n, seed, 1, count, lists=view)
    c2 = engine.check_counts(view, n, count)
    torch.cuda.synchronize()
    got = view[:, :count].cpu().numpy()
    ref = oracle_lib.sample(n, seed, 1, count, info["notq"], info["q"], info["closed"])
    assert np.array_equal(got, ref)
    assert not buf[:, :4].any() and not buf[:, 4 + count:].any()  # nothing written outside
    H, C, P, bad = oracle_lib.counts(ref, n)
    for cc in (c, c2):
        gH, gC, gP = cc.numpy()
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P)


def test_adversarial_collisions_wide_and_narrow(engine):
    """Check-only mode on lists full of collisions (every Q entry has repeated
    values): the pair slow path, on both row alignments, vs the oracle."""
    n, count = 11, 30_001
    rng = np.random.default_rng(5)
    L = rng.integers(0, 4, (n + 1, count)).astype(np.uint8)  # 4 values for 12 groups
    H, C, P, bad = oracle_lib.counts(L, n)
    assert bad == 0 and C.sum() > P.sum() * (n + 1)
    for off in (0, 4):
        ld = (count + 63) // 64 * 64 + off
        buf = torch.zeros((n + 1, ld), dtype=torch.uint8, device=engine.device)
        view = buf[:, off:]
        assert view.stride(0) % 8 == off
        view[:, :count] = torch.from_numpy(L).to(engine.device)
        c = engine.check_counts(view, n, count)
        gH, gC, gP = c.numpy()
        assert np.array_equal(gH, H) and np.array_equal(gC, C) and np.array_equal(gP, P), off


def test_check_gather_vs_oracle(engine):
    """qba_check_gather: consistent(v, L, w) over tuples gathered
    on the device from several parties' lists, each in its own index order --
    against the oracle's consistent on the same tuples (as a set): honest
    packets, duplicates that collapse, partial collisions, values > w and == v,
    empty tuples, and out-of-range indices / parties."""
    rng = np.random.default_rng(77)
    n, count = 7, 5000
    engine.prepare(n)
    lists = engine.sample(n, 123, 0, count)
    L = lists[:, :count].cpu().numpy().astype(np.int64)
    w = 8
    isq = np.nonzero(L[0] != L[1])[0]
    checked = 0
    for trial in range(60):
        m = int(rng.integers(1, 6))
        ln = int(rng.integers(0, 40))
        base = rng.choice(isq, ln, replace=False) if ln else np.zeros(0, np.int64)
        party = [int(x) for x in rng.choice(np.arange(2, n + 1), m)]
        idx = np.stack([rng.permutation(base) if rng.random() < 0.5 else base for _ in range(m)]) \
            if ln else np.zeros((m, 0), np.int64)
        if trial % 7 == 3 and m > 1:
            party[1] = party[0]
            idx[1] = idx[0]  # identical tuple: collapses in the set
        v = int(rng.integers(0, w + 2))
        lv = L.copy()
        if trial % 5 == 4 and ln:
            lv[party[0], idx[0][0]] = w + 3  # value outside [0, w]
        d = torch.zeros_like(lists)
        d[:, :count] = torch.from_numpy(lv.astype(np.uint8))
        tuples = {tuple(int(lv[party[a]][j]) for j in idx[a]) for a in range(m)}
        want = orc.consistent(v, tuples, w)
        assert engine.check_gather(d, count, idx, party, v, w) == want, trial
        checked += 1
    assert checked == 60
    with pytest.raises(sub("engine").QbaError):
        engine.check_gather(lists, count, np.array([[0, count]]), [2], 0, w)
    with pytest.raises(sub("engine").QbaError):
        engine.check_gather(lists, count, np.array([[0, 1]]), [n + 5], 0, w)
    with pytest.raises(sub("engine").QbaError):
        engine.check_gather(lists, count, np.zeros((0, 3), np.int64), [], 0, w)


def test_invalid_arguments_leave_context_usable(engine):
    """Malformed calls on a live context fail with QbaError (nothing launched
    or read out of bounds), and the context keeps working afterwards: party
    counts outside [1, 15], ld < count, missing outputs, malformed gates, nq
    outside [1, 8], indices outside a list."""
    lm = sub("_lib")
    n, count = 11, 4096
    engine.prepare(n)
    lists = engine.sample(n, 1, 0, count)
    ptr = lists.data_ptr()
    s = engine.stream()
    bad_calls = [
        ("qba_sample", engine.ctx, 0, 1, 0, count, ptr, lists.stride(0), s),
        ("qba_sample", engine.ctx, 16, 1, 0, count, ptr, lists.stride(0), s),
        ("qba_sample", engine.ctx, n, 1, 0, count, ptr, count - 1, s),
        ("qba_sample_check", engine.ctx, n, 1, 0, count, ptr, lists.stride(0), None, None, None, 0, s),
        ("qba_check_counts", engine.ctx, n, ptr, count, count - 1, None, None, None, 0, s),
    ]
    for name, *args in bad_calls:
        with pytest.raises(lm.QbaError):
            lm.call(name, *args)
    sv = torch.empty(1 << 4, dtype=torch.float64, device=engine.device)
    for gates in ([(0, 4, -1)], [(0, 1, 2)], [(1, 2, 2)], [(2, 0, -1)], [(1, 0, -3)]):
        g = np.array(gates, np.int32)
        with pytest.raises(lm.QbaError):
            engine.statevector(4, g, out=sv)
        with pytest.raises(lm.QbaError):
            engine.apply_gates(sv, 4, g)
    raw = torch.zeros(64, dtype=torch.int64, device=engine.device)
    vals = torch.zeros(8, dtype=torch.uint8, device=engine.device)
    for nq in (0, 9):
        with pytest.raises(lm.QbaError):
            lm.call("qba_bits_to_values", engine.ctx, raw.data_ptr(), 8, nq, vals.data_ptr(), s)
    lc = lists[1, :count].contiguous()
    with pytest.raises(lm.QbaError):
        engine.select_eq(np.array([0, count], np.int64), lc, 3)
    # still usable: the same calls with valid arguments match the oracle
    info = engine.prepare(n)
    got, c = engine.sample_check(n, 9, 0, count)
    ref = oracle_lib.sample(n, 9, 0, count, info["notq"], info["q"], info["closed"])
    assert np.array_equal(got[:, :count].cpu().numpy(), ref)
    H, C, P, _ = oracle_lib.counts(ref, n)
    assert np.array_equal(c.numpy()[0], H)
