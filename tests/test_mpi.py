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
@pytest.mark.parametrize("name", ["case009", "case010"])
def test_mpiexec_reference_rounds_honest(name):
    """nDishonest = 0: the round loop never re-broadcasts, so the reference's
    own (racy) rounds are deterministic and must match too."""
    case = CASES[name]
    assert case["nDishonest"] == 0
    got = _mpiexec(case["n"] + 1, [name, "--rounds", "reference"])
    _compare(got, case["exact"], traffic=False)
