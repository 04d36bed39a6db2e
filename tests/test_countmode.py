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
