"""The mpi4py-free transport (ctypes MPICH binding, mpi.py) under a real
``mpiexec``: the reference's interface ``mpiexec -n <n+1> python tfg.py ...``
(README.md:4).

* the binding's handles equal the installed MPICH mpi.h;
* fixture cases of tests/golden/protocol.json reproduced by n+1 real MPI
  processes (host logic with the numpy OracleEngine): with barrier-epoch
  rounds (comm.EpochComm) every field must match -- decisions, V_i,
  accept/reject/sent per rank, messages and bytes; with the reference's own
  racy rounds an honest run (nDishonest = 0: no round re-broadcasts, so no
  race) must match as well;
* the CLI end to end under mpiexec (in-process GPU-free engine is not
  available to the CLI, so that run is a GPU test in test_mpi_gpu below).
"""
import json
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

from conftest import GOLDEN, ROOT, sub

MPIEXEC = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
HAVE_MPI = os.path.exists(MPIEXEC)
CASES = {c["name"]: c for c in json.loads((GOLDEN / "protocol.json").read_text())}
needs_mpi = pytest.mark.skipif(not HAVE_MPI, reason="no mpiexec in this image")


def _mpiexec(nranks, args, timeout=120):
    env = dict(os.environ)
    env.pop("PMI_RANK", None)
    cmd = [MPIEXEC, "-n", str(nranks), sys.executable, str(ROOT / "tests" / "mpi_driver.py")] + args
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def _compare(got, want, traffic=True):
    for k in ("error", "error_ranks", "decisions", "dishonest", "success", "V", "accept", "reject", "sent"):
        assert got[k] == want[k], (k, got[k], want[k])
    if traffic:
        assert got["messages"] == want["messages"] and got["bytes"] == want["bytes"]


def test_mpich_handles_match_header():
    mpi = sub("mpi")
    hdr = Path("/opt/conda/include/mpi.h")
    if not hdr.exists():
        pytest.skip("no MPICH mpi.h")
    text = hdr.read_text()

    def const(name):
        m = re.search(rf"#define {name}\s+\(\(\w+\)(0x[0-9a-fA-F]+)\)", text)
        return int(m.group(1), 16)

    assert const("MPI_COMM_WORLD") == mpi.COMM_WORLD_HANDLE
    assert const("MPI_INT") == mpi.INT.handle and const("MPI_BYTE") == mpi.BYTE.handle
    assert const("MPI_LONG") == mpi.LONG.handle and const("MPI_INT64_T") == mpi.INT64_T.handle
    assert int(re.search(r"#define MPI_ANY_SOURCE\s+\((-?\d+)\)", text).group(1)) == mpi.ANY_SOURCE
    assert int(re.search(r"#define MPI_ANY_TAG\s+\((-?\d+)\)", text).group(1)) == mpi.ANY_TAG
    body = re.search(r"typedef struct MPI_Status \{(.*?)\}", text, re.S).group(1)
    fields = re.findall(r"int (\w+);", body)
    assert fields == [f for f, _ in mpi._CStatus._fields_]


def test_protocol_constants_follow_the_comm():
    """The protocol takes INT / ANY_SOURCE / ANY_TAG from the communicator's
    own library (advisor finding: LocalWorld's -1 is MPI_PROC_NULL in MPICH)."""
    comm, mpi = sub("comm"), sub("mpi")
    lc = comm.LocalWorld(2).comms[0]
    assert comm.mpi_of(lc).ANY_SOURCE == -1
    assert comm.mpi_of(mpi.Comm(mpi.COMM_WORLD_HANDLE)).ANY_SOURCE == -2
    assert comm.mpi_of(mpi.Comm(mpi.COMM_WORLD_HANDLE)).INT is mpi.INT


@needs_mpi
@pytest.mark.parametrize("name", ["case003", "case004", "case005", "case009", "case011", "case012", "case013",
                                  "case028", "case043", "case044", "case046", "case050", "case056"])
def test_mpiexec_epoch_rounds_match_fixtures(name):
    case = CASES[name]
    got = _mpiexec(case["n"] + 1, [name, "--rounds", "epoch"])
    _compare(got, case["exact"])


@needs_mpi
@pytest.mark.parametrize("name", ["case011", "case013"])
def test_mpiexec_count_mode_matches_canonical(name):
    case = CASES[name]
    got = _mpiexec(case["n"] + 1, [name, "--rounds", "epoch", "--mode", "count"])
    _compare(got, case["canonical"], traffic=False)


@needs_mpi
@pytest.mark.parametrize("name,owners", [("case011", 2), ("case013", 2), ("case011", 3), ("case013", 4)])
def test_mpiexec_count_mode_sharded_owners(name, owners):
    """The mpiexec GPU-owner branch at G > 1 (tfg.count_owners: owner
    selection, the group id sent from rank 0 over MPI, ShardCounter over the
    owners' shards of the injected lists) with the numpy engine and an MPI
    all-reduce in place of RCCL: decisions equal the canonical fixtures."""
    case = CASES[name]
    assert case["n"] + 1 >= owners
    got = _mpiexec(case["n"] + 1, [name, "--rounds", "epoch", "--mode", "count", "--owners", str(owners)])
    _compare(got, case["canonical"], traffic=False)


@needs_mpi
@pytest.mark.parametrize("name", ["case009", "case010"])
def test_mpiexec_reference_rounds_honest(name):
    """nDishonest = 0: the round loop never re-broadcasts, so the reference's
    own (racy) rounds are deterministic and must match too."""
    case = CASES[name]
    assert case["nDishonest"] == 0
    got = _mpiexec(case["n"] + 1, [name, "--rounds", "reference"])
    _compare(got, case["exact"], traffic=False)


# ---------------------------------------------------------------------------
# GPU: the CLI itself under mpiexec (one process per party, GPU engines)
# ---------------------------------------------------------------------------
def _cli(args, nranks=None, timeout=300):
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    base = [sys.executable, "-m", "tfg---quantum-byzantine-agreement_amd.tfg"] + args
    cmd = ([MPIEXEC, "-n", str(nranks)] + base) if nranks else base
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=str(ROOT))
    assert out.returncode == 0, out.stdout[-1500:] + out.stderr[-1500:]
    return [l for l in out.stdout.splitlines() if l.split(":")[0] in ("Decisions", "Dishonests", "Success")], out.stdout


@pytest.mark.gpu
@needs_mpi
@pytest.mark.parametrize("mode", ["exact", "count"])
def test_cli_mpiexec_epoch_equals_inprocess(mode):
    """`mpiexec -n 4 python -m ...tfg 1000 1` (4 GPU processes, ctypes MPICH,
    barrier-epoch rounds) decides exactly like the in-process run with the
    same seeds (LocalWorld, the fixtures' semantics)."""
    args = ["1000", "1", "--seed", "5", "--quiet", "--mode", mode]
    ref, _ = _cli(args + ["--parties", "3"])
    got, _ = _cli(args + ["--rounds", "epoch"], nranks=4)
    assert got == ref and len(ref) == 3


@pytest.mark.gpu
def test_rccl_single_rank_allreduce(engine):
    """The C ABI's RCCL path end to end on one GPU (a 1-rank communicator:
    the all-reduce is the identity)."""
    import torch
    uid = engine.rccl_unique_id()
    assert len(uid) == 128
    engine.rccl_init(uid, 1, 0)
    t = torch.arange(5392, dtype=torch.int64, device=engine.device) * 7
    engine.allreduce_i64(t)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(5392, dtype=torch.int64, device=engine.device) * 7)


@pytest.mark.gpu
def test_cli_count_mode_sizeL_1e9():
    """SURVEY §8(f)1 end to end: `tfg 1e9 3 --parties 11 --mode count` -- 1e9
    entries sampled and checked on the GPU, the protocol decided from the
    count tables; honest lieutenants agree."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "tests"))
    from oracle_engine import OracleEngine
    lines, out = _cli(["1e9", "3", "--parties", "11", "--mode", "count", "--seed", "11", "--timing"])
    print(out)
    # the same run (rank seeds 11*1000 + r, list seed 11) with its count
    # tables from the C twin over all 1e9 entries (oracle, OpenMP): the CLI
    # must print exactly its Decisions / Dishonests / Success lines
    protocol, countmode = sub("protocol"), sub("countmode")
    ref = protocol.run_local(11, 10 ** 9, 3, OracleEngine(), seed=11, list_seed=11, timeout=600,
                             party_cls=countmode.CountParty)
    want = [f"Decisions: {np.array(ref.result['decisions'])}", f"Dishonests: {np.array(ref.result['dishonest'])}",
            f"Success: {ref.result['success']}"]
    assert lines == want, (lines, want)
    assert len(ref.result["dishonest"]) == 3
