"""INTEGRATION.md's ctypes stub (tests/integration_stub.py, embedded verbatim
in the document) composes with tfg.py: generacionListas returns the
reference's rawS bit layout (tfg.py:84, 142-156), measure_to_ints decodes it
on the device (tfg.py:128-129) and add_own_and_check reproduces
L.add(own) + consistent() (tfg.py:87-98, 189-192) -- checked against the
oracle.  The CPU test keeps the document and the file identical."""
import importlib.util
import re

import numpy as np
import pytest

import tfg_oracle as orc
from conftest import ROOT

STUB = ROOT / "tests" / "integration_stub.py"


def test_document_embeds_the_tested_stub():
    doc = (ROOT / "INTEGRATION.md").read_text()
    blocks = re.findall(r"```python\n(.*?)```", doc, re.S)
    assert any(b.strip() == STUB.read_text().strip() for b in blocks), "INTEGRATION.md stub != tests/integration_stub.py"


def _stub():
    spec = importlib.util.spec_from_file_location("qba_stub", STUB)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.gpu
def test_stub_against_oracle():
    import oracle_lib
    stub = _stub()
    stub.init(0)
    n, size, seed = 3, 1000, 7
    nq, w = 2, 4
    stub.compile_resource(n, nq)
    raw = stub.generacionListas(n, size, nq, w, seed)
    assert raw.shape == (n + 1, nq * size) and raw.dtype == np.int64 and set(np.unique(raw)) <= {0, 1}
    info = {"nfac": 0, "desc": np.zeros((0, 6), np.int32), "pat": np.zeros(1, np.uint64),
            "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    want = oracle_lib.sample(n, seed, 0, size, info, info, closed=True)
    lists = [stub.measure_to_ints(raw[g], size, nq) for g in range(n + 1)]
    for g in range(n + 1):
        assert lists[g].cpu().numpy().tolist() == orc.measure_to_ints(raw[g], size, nq) == want[g].tolist()
    rng = np.random.default_rng(1)
    li = want[2]
    for trial in range(40):
        P = set(rng.choice(size, int(rng.integers(0, 40)), replace=False).tolist())
        own = tuple(int(li[j]) for j in np.fromiter(P, np.int64, len(P)))
        L = set()
        for _ in range(int(rng.integers(0, 4))):
            kind = rng.integers(4)
            if kind == 0:
                L.add(own)                                   # a duplicate of own (set semantics)
            elif kind == 1:
                L.add(tuple(int(x) for x in rng.integers(0, w + 2, len(P))))  # values up to w+1
            elif kind == 2:
                L.add(tuple(int(x) for x in rng.integers(0, w, max(len(P) - 1, 0))))  # Cond1
            else:
                L.add(tuple((x + 1) % w for x in own))
        v = int(rng.integers(0, w + 1))
        ref = set(L)
        ref.add(own)
        expect = orc.consistent(v, ref, w)
        got_L = set(L)
        assert stub.add_own_and_check(lists[2], P, v, got_L, w) == expect, trial
        assert got_L == ref
