"""Count-mode protocol against the reference run in canonical (sorted-set) order."""
import json

import numpy as np
import pytest

from conftest import GOLDEN, sub
from oracle_engine import OracleEngine

CASES = json.loads((GOLDEN / "protocol.json").read_text())
LISTS = np.load(GOLDEN / "protocol_lists.npz")


def _compare(run, want):
    assert run.error == want["error"]
    assert run.error_ranks == want["error_ranks"]
    assert run.result["decisions"] == want["decisions"]
    assert run.result["dishonest"] == want["dishonest"]
    assert run.result["success"] == want["success"]
    assert {str(k): v for k, v in run.V.items()} == want["V"]
    assert run.accept == want["accept"]
    assert run.reject == want["reject"]
    assert run.sent == want["sent"]


def _run(engine, case):
    protocol, countmode = sub("protocol"), sub("countmode")
    return protocol.run_local(case["n"], case["sizeL"], case["nDishonest"], engine, seed=case["seed"],
                              lists=LISTS[case["name"]], timeout=60, party_cls=countmode.CountParty)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_countmode_canonical_cpu_host(case):
    _compare(_run(OracleEngine(), case), case["canonical"])


@pytest.mark.gpu
def test_countmode_canonical_gpu(engine):
    for case in CASES:
        _compare(_run(engine, case), case["canonical"])


@pytest.mark.gpu
def test_countmode_sampled_honest_run(engine):
    """End to end on device-sampled lists (no host lists at all): with honest
    parties every lieutenant accepts the commander's order."""
    protocol, countmode = sub("protocol"), sub("countmode")
    run = protocol.run_local(11, 2_000_000, 0, engine, seed=4, party_cls=countmode.CountParty)
    assert run.result["success"] and run.error is None
    assert len(set(run.result["decisions"])) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 9, 23])
def test_countmode_config1_matches_c_twin(engine, seed):
    """BASELINE configs[1] as stated: n = 11, 3 dishonest, sizeL = 1e6 of
    device-sampled lists.  The whole count-mode run on the GPU engine equals
    the same run whose count tables come from the C twin (oracle, same
    Philox schedule): decisions, dishonest ids, V_i, accept / reject / sent
    of every rank."""
    protocol, countmode = sub("protocol"), sub("countmode")
    kw = dict(seed=seed, timeout=120, party_cls=countmode.CountParty)
    got = protocol.run_local(11, 1_000_000, 3, engine, **kw)
    want = protocol.run_local(11, 1_000_000, 3, OracleEngine(), **kw)
    assert len(got.result["dishonest"]) == 3
    assert got.result == want.result and got.V == want.V and got.error_ranks == want.error_ranks
    assert got.accept == want.accept and got.reject == want.reject and got.sent == want.sent
