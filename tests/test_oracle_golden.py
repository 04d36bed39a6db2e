"""CPU suite: pin the oracle (and the host's pure-Python pieces) to the reference.

Golden vectors come from running the reference itself (tests/golden/
gen_golden.py) and from its five captured runs (logs tests/).
"""
import json
import re
from pathlib import Path

import numpy as np
import pytest
from scipy import stats

import oracle_lib
import statevector as sv_oracle
import tfg_oracle as orc
from conftest import GOLDEN, PKG_NAME, ROOT, sub

KATS = [  # Random123 philox4x32-10 known answers
    ([0, 0, 0, 0], 0, [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
    ([0xFFFFFFFF] * 4, 0xFFFFFFFFFFFFFFFF, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
    ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], 0x299F31D0A4093822,
     [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
]


def test_philox_oracle_kat():
    for ctr, key, want in KATS:
        assert list(oracle_lib.philox(np.array(ctr, np.uint32), key)[0]) == want


def test_consistent_kat():
    for case in json.loads((GOLDEN / "consistent.json").read_text()):
        L = {tuple(t) for t in case["L"]}
        if "error" in case:
            with pytest.raises(StopIteration):
                orc.consistent(case["v"], L, case["w"])
        else:
            assert orc.consistent(case["v"], L, case["w"]) == case["result"], case


def test_codec_kat():
    for case in json.loads((GOLDEN / "codec.json").read_text()):
        assert orc.measure_to_ints(case["raw"], case["sizeL"], case["nq"]) == case["ints"]
        raw = orc.lists_to_raw(np.array([case["ints"]]), case["nq"])[0]
        assert raw.tolist() == case["raw"]


def test_resource_gate_lists_match_reference():
    """resource.py emits exactly the reference's gate lists (tfg.py:15-65)."""
    res = sub("resource")
    gates = json.loads((GOLDEN / "gates.json").read_text())
    for n_s, g in gates.items():
        n = int(n_s)
        nq = res.n_qubits(n)
        assert nq == g["nq"] == orc.n_qubits(n)
        assert [list(o) for o in res.notQCorrelated(n, nq).ops] == g["notq"]
        assert [list(o) for o in orc.notq_gates(n)] == g["notq"]
        for case in g["q"]:
            assert [list(o) for o in res.qCorrelated(n, nq, perm=case["perm"]).ops] == case["ops"]
            assert [list(o) for o in orc.q_gates(n, case["perm"])] == case["ops"]
            rs = np.random.RandomState(case["seed"])
            drawn = res.qCorrelated(n, nq, rng=rs)
            assert drawn.perm.tolist() == case["perm"]  # same np.random call order
        circ = res.genNQCorrCircuit(n, nq)
        meas = [[o[0], o[1], o[2]] for o in circ.ops if o[0] == "MEASURE"]
        assert meas == g["measure"]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5])
def test_statevector_oracle_closed_form(n):
    """Dense simulation of the reference's gate lists == the closed form of
    SURVEY.md §8(a) A1/A2 (the probability golden vectors, exact powers of 2)."""
    g = json.loads((GOLDEN / "gates.json").read_text())[str(n)]
    N, nq, w = g["size"], g["nq"], g["w"]
    probs = sv_oracle.probabilities(sv_oracle.run([tuple(o) for o in g["notq"]], N))
    idx, p = sv_oracle.support(probs, 1e-30)
    vals = [[(int(i) >> (N - (k + 1) * nq)) & (w - 1) for k in range(n + 1)] for i in idx]
    assert len(idx) == w ** n and np.allclose(p, w ** -n, atol=1e-15, rtol=0)
    assert all(v[0] == v[1] for v in vals)
    for case in g["q"]:
        probs = sv_oracle.probabilities(sv_oracle.run([tuple(o) for o in case["ops"]], N))
        idx, p = sv_oracle.support(probs, 1e-30)
        assert len(idx) == w and np.allclose(p, 1.0 / w, atol=1e-15, rtol=0)
        for i in idx:
            v = [(int(i) >> (N - (k + 1) * nq)) & (w - 1) for k in range(n + 1)]
            assert [v[k] ^ v[0] for k in range(1, n + 1)] == case["perm"]


LOGS = json.loads((GOLDEN / "logs.json").read_text())
LOG_ARRAYS = np.load(GOLDEN / "logs.npz")


@pytest.mark.parametrize("info", LOGS, ids=[i["file"] for i in LOGS])
def test_log_invariants(info):
    """Real qsimov output (the captured runs): the structure the sampler must
    reproduce.  At Q positions all n+1 values differ and L_g XOR L_0 is a
    permutation of 1..n; elsewhere L0 == L1; marginals are uniform."""
    L = LOG_ARRAYS[info["file"][:-4]].astype(np.int64)
    n = info["n"]
    w = 2 ** orc.n_qubits(n)
    assert info["w"] == w
    q = L[0] != L[1]
    assert 0.4 < q.mean() < 0.6
    Lq = L[:, q]
    assert (np.diff(np.sort(Lq, axis=0), axis=0) != 0).all()
    x = np.sort(Lq[1:] ^ Lq[0], axis=0)
    assert (x == np.arange(1, n + 1)[:, None]).all()
    for g in range(n + 1):
        assert stats.chisquare(np.bincount(L[g], minlength=w)).pvalue > 1e-4


@pytest.mark.parametrize("info", LOGS, ids=[i["file"] for i in LOGS])
def test_log_set_orders(info):
    """The host's set constructions reproduce the reference's printed orders:
    isQCorr (tfg.py:327) and every receiver's set(buff) rebuild (tfg.py:240)."""
    L = LOG_ARRAYS[info["file"][:-4]]
    isq = set(orc.is_qcorr_indices(L[0], L[1]).tolist())  # as protocol.Party.commander_setup
    assert list(isq) == info["isQCorr_order"]
    pk = info["packets"]
    n_checked = 0
    for i, p in enumerate(pk):
        if p["src"] < 2 or p["bad"] or not p["P_order"]:
            continue
        incoming = [q for q in pk[:i] if q["dst"] == p["src"] and set(q["P_order"]) == set(p["P_order"])]
        assert any(list(set(np.array(q["P_order"], np.int64))) == p["P_order"] for q in incoming)
        n_checked += 1
    assert n_checked == {"log_11.txt": 90, "log_3.txt": 2, "log_dC_3.txt": 4,
                         "log_d_11.txt": 108, "log_d_3.txt": 1}[info["file"]]


def test_log_outcomes():
    by = {i["file"]: i for i in LOGS}
    assert by["log_3.txt"]["decisions"] == [3, 3, 3] and by["log_3.txt"]["success"]
    assert by["log_dC_3.txt"]["decisions"] == [2, 0, 0] and by["log_dC_3.txt"]["dishonest"] == [1]
    assert by["log_d_11.txt"]["dishonest"] == [1, 2, 5, 7, 11]
    assert all(i["success"] for i in LOGS)
    for i in LOGS:
        assert orc.success(i["decisions"], i["dishonest"]) == i["success"]


def test_counts_c_twin_matches_numpy():
    arrays = np.load(GOLDEN / "protocol_lists.npz")
    for name in arrays.files[:25]:
        L = arrays[name]
        n = L.shape[0] - 1
        H, C, P, bad = oracle_lib.counts(L, n)
        H2, C2, P2 = orc.counts(L, n)
        assert bad == 0 and np.array_equal(H, H2) and np.array_equal(C, C2) and np.array_equal(P, P2)


def _declared_symbols():
    text = (ROOT / "include" / "qba.h").read_text()
    return sorted(set(re.findall(r"^QBA_API\s+[\w\s\*]+?\b(qba_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol():
    """libqba.so loads (no GPU needed) and exports every entry point of qba.h."""
    lib_mod = sub("_lib")
    lib = lib_mod.lib()
    declared = _declared_symbols()
    assert len(declared) >= 22
    for name in declared:
        assert hasattr(lib, name), name
        assert name in lib_mod.SIGNATURES, name
    assert set(lib_mod.SIGNATURES) == set(declared)
    assert lib.qba_version() >= 100


def test_shipped_library_reads_no_environment_knob():
    """the launch-shape knobs the GPU tests use (chunk size,
    pair-bin threshold, grid cap) reach the library only through
    qba_test_set_knobs; the shipped library reads no environment variable, so
    a stray variable cannot change kernel selection in production."""
    blob = Path(sub("_lib").LIB_PATH).read_bytes()
    for name in (b"QBA_LIST_GRID", b"QBA_PB_MIN_ENTRIES", b"QBA_CHUNK_ENTRIES"):
        assert name not in blob, name
    csrc = ROOT / PKG_NAME / "csrc"
    for f in sorted(csrc.glob("*.hip")) + sorted(csrc.glob("*.cpp")) + sorted(csrc.glob("*.h")):
        assert "getenv" not in f.read_text(), f.name


def test_shipped_library_has_no_experiment_switch():
    """The libqba.so in the tree (the one the GPU tests, smoke and bench load)
    is no experiment build (qba_build_flags() == 0), and the shipped sources
    hold no attribution probe or tuning override: those live in
    tools/exp/probes.patch, applied to a copy by tools/exp/build.sh PROBES=1."""
    import re
    lib = sub("_lib").lib()
    assert lib.qba_build_flags() == 0
    csrc = ROOT / "tfg---quantum-byzantine-agreement_amd" / "csrc"
    for f in sorted(csrc.glob("*.h")) + sorted(csrc.glob("*.hip")):
        text = f.read_text()
        assert not re.search(r"#\s*if(n?def)?\b.*\bQBA_EXP_", text), f.name
        assert not re.search(r"#\s*ifndef\s+QBA_(WIDE_QPT|QUEUE|PAIRWISE|NT_STORE|PAIRBINS|LBLOCK|DBLOCK)\b", text), f.name
    assert (ROOT / "tools" / "exp" / "probes.patch").exists()


def test_library_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    eng = sub("engine")
    with pytest.raises(sub("_lib").QbaError):
        eng.Engine(0)


def test_alias_table_host():
    """Vose alias tables (host build) reproduce the distribution to 2^-32."""
    eng = sub("engine")
    rng = np.random.default_rng(0)
    for k in (1, 2, 3, 7, 16, 256):
        p = rng.random(k)
        p[rng.random(k) < 0.2] = 0.0
        if p.sum() == 0:
            p[0] = 1.0
        thr, alias = eng.alias_build(p)
        q = np.zeros(k)
        for i in range(k):
            keep = int(thr[i]) / 2 ** 32
            q[i] += keep / k
            q[alias[i]] += (1 - keep) / k
        assert np.allclose(q, p / p.sum(), atol=k * 2.0 ** -31)


_NULL_CTX_PROBE = r'''
import ctypes as C, importlib, json, sys
sys.path.insert(0, sys.argv[1])
lm = importlib.import_module("tfg---quantum-byzantine-agreement_amd._lib")
lib = lm.lib()
skip = {"qba_last_error", "qba_version", "qba_build_flags", "qba_destroy", "qba_rccl_unique_id"}
out = {}
for name, argt in sorted(lm.SIGNATURES.items()):
    if name in skip:
        continue
    args = []
    for t in argt:
        if t in (C.c_double, C.c_float):
            args.append(0.0)
        elif t in (C.c_void_p, C.c_char_p) or hasattr(t, "contents") or getattr(t, "_type_", None) is not None and t.__name__.startswith("LP_"):
            args.append(None)
        else:
            args.append(0)
    rc = getattr(lib, name)(*args)
    out[name] = [int(rc), lib.qba_last_error().decode()]
print(json.dumps(out))
'''


def test_entry_points_reject_null_arguments():
    """Every entry point called with a NULL context / NULL buffers / zero
    sizes returns a negative status with a message on qba_last_error(), and
    touches nothing (no GPU needed; run in a child process so that a crash
    would fail this test instead of the suite)."""
    import json as _json
    import subprocess
    import sys as _sys
    r = subprocess.run([_sys.executable, "-c", _NULL_CTX_PROBE, str(ROOT)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = _json.loads(r.stdout.strip().splitlines()[-1])
    assert len(res) >= 28
    for name, (rc, msg) in res.items():
        assert rc < 0, (name, rc)
        assert msg.startswith(name + ":"), (name, msg)
