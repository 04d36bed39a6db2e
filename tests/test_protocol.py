"""Protocol parity: the host (exact mode) against the reference's own QBA runs.

tests/golden/protocol.json holds, for 60 injected-list cases, what the
reference tfg.py produced on the same in-process MPI world with the same
per-rank seeds: decisions, dishonest ids, Success, every honest lieutenant's
V_i, per-rank consistent() accept/reject counts, packets sent and the total
message count / bytes on the wire.  The host must reproduce all of it.

The CPU variant drives the host with a numpy oracle engine (host logic only);
the GPU variant runs the product path through libqba's HIP kernels.
"""
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
    assert run.messages == want["messages"]
    assert run.bytes == want["bytes"]


def _run(engine, case, **party_kwargs):
    protocol = sub("protocol")
    return protocol.run_local(case["n"], case["sizeL"], case["nDishonest"], engine,
                              seed=case["seed"], lists=LISTS[case["name"]], timeout=60,
                              party_kwargs=party_kwargs or None)


class _RowEngine(OracleEngine):
    """The numpy oracle engine presenting itself as a device engine (it has
    lists_to_bits), so an in-process run takes the device-row list sends."""

    def lists_to_bits(self, *a):  # pragma: no cover - never called on the device-row path
        raise AssertionError("the device-row path must not encode lists")


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_protocol_exact_cpu_host(case):
    _compare(_run(OracleEngine(), case), case["exact"])


@pytest.mark.parametrize("case", CASES[::6], ids=[c["name"] for c in CASES[::6]])
def test_protocol_exact_device_rows_cpu_host(case):
    """In-process runs hand each rank its list row (comm.DeviceRow) instead of
    the int64-per-bit wire encoding; decisions, V_i, accept/reject, sends and
    the accounted messages / bytes stay the fixtures'."""
    _compare(_run(_RowEngine(), case), case["exact"])


@pytest.mark.gpu
def test_protocol_exact_gpu(engine):
    """The product path in-process: device rows, no wire codec."""
    for case in CASES:
        _compare(_run(engine, case), case["exact"])


@pytest.mark.gpu
def test_protocol_exact_gpu_wire(engine):
    """The same fixtures with the reference's wire layout for the lists
    (tfg.py:142-161, the --wire / mpiexec form)."""
    for case in CASES:
        _compare(_run(engine, case, wire=True), case["exact"])


def test_consistent_host_kat():
    """Host consistent(): Cond1 / StopIteration semantics with the oracle engine."""
    protocol = sub("protocol")
    eng = OracleEngine()
    for case in json.loads((GOLDEN / "consistent.json").read_text()):
        L = {tuple(t) for t in case["L"]}
        if "error" in case:
            with pytest.raises(StopIteration):
                protocol.consistent(case["v"], L, case["w"], eng)
        else:
            assert protocol.consistent(case["v"], L, case["w"], eng) == case["result"]


def test_decide_order_empty_raises():
    protocol = sub("protocol")
    with pytest.raises(ValueError):
        protocol.decide_order(set(), 3, False)
    assert protocol.decide_order({4, 2}, 9, False) == 2
    assert protocol.decide_order(set(), 9, True) == 9


def test_wire_cache_and_packet_roundtrip():
    """protocol.WireCache: one int64 wire array per P set / L tuple object, in
    the object's iteration order; rebuilt after the dishonest P.clear()
    (tfg.py:280); a received tuple's buffer is reused.  recv_pvl rebuilds P
    with Python ints whose set iterates exactly as the numpy-int64 set the
    reference builds (tfg.py:209)."""
    proto = sub("protocol")
    wc = proto.WireCache()
    rng = np.random.default_rng(3)
    P = set(int(x) for x in rng.choice(1 << 20, 3000, replace=False))
    a = wc(P)
    assert a.dtype == np.int64 and list(a) == list(P) and wc(P) is a
    P.clear()
    assert len(wc(P)) == 0
    t = tuple(int(x) for x in rng.integers(0, 16, 500))
    buf = np.asarray(t, dtype=np.int64)
    wc.put(t, buf)
    assert wc(t) is buf
    raw = rng.choice(1 << 30, 5000, replace=False).astype(np.int64)
    assert list(set(raw.tolist())) == [int(x) for x in set(raw)]


# ---------------------------------------------------------------------------
# the native restatement of CPython 3.10's set order and tuple hash
# (qba_host_pyset_order / qba_host_pytuple_hash) against the live interpreter
# ---------------------------------------------------------------------------
def test_native_set_order_matches_cpython():
    import sys
    protocol = sub("protocol")
    if sys.version_info[:2] != (3, 10):
        pytest.skip("the restatement is of CPython 3.10's setobject.c")
    rng = np.random.default_rng(7)
    for trial in range(400):
        n = int(rng.choice([0, 1, 2, 5, 9, 17, 100, 1000, 4999, 31_000, 50_001, 70_000]))
        hi = int(rng.choice([8, 1000, 10 ** 6, 10 ** 9, 2 ** 62]))
        keys = rng.integers(0, hi, size=n, dtype=np.int64)
        if trial % 3 == 0:
            keys.sort()
        if trial % 11 == 0:
            keys = -keys
        if trial % 7 == 0 and n:
            keys[::3] = keys[0]  # duplicates collapse
        want = list(set(keys.tolist()))
        got = protocol.PSet.build(keys)
        assert got.arr.tolist() == want, (trial, n, hi)
        assert repr(got) == repr(set(keys.tolist()))
    # the reference's own hop: a numpy array straight into set() (numpy scalars)
    buf = rng.integers(0, 10 ** 6, size=31_000, dtype=np.int64)
    assert protocol.PSet.build(buf).arr.tolist() == [int(x) for x in set(buf)]


def test_native_tuple_hash_and_set_of_tuples_match_cpython():
    import sys
    protocol = sub("protocol")
    if sys.version_info[:2] != (3, 10):
        pytest.skip("the restatement is of CPython 3.10's tuplehash")
    rng = np.random.default_rng(8)
    for _ in range(300):
        t = rng.integers(-3, 16, size=int(rng.integers(0, 64)), dtype=np.int64)
        assert hash(protocol.PTuple(t)) == hash(tuple(t.tolist()))
        assert protocol.PTuple(t) == tuple(t.tolist())
        assert repr(protocol.PTuple(t)) == repr(tuple(t.tolist()))
    for _ in range(50):  # L: a set of tuples, with repeats that must collapse
        rows = [rng.integers(0, 16, size=40, dtype=np.int64) for _ in range(int(rng.integers(1, 8)))]
        rows += [rows[0].copy()]
        native = {protocol.PTuple(r) for r in rows}
        python = {tuple(r.tolist()) for r in rows}
        assert [tuple(x) for x in native] == list(python)
        assert repr(native) == repr(python)


@pytest.mark.parametrize("name", ["case003", "case013", "case043"])
def test_protocol_python_sets_path(name, monkeypatch):
    """The plain-Python set path (any other interpreter, or QBA_PYTHON_SETS=1)
    gives the same fixture results as the native restatement."""
    protocol = sub("protocol")
    monkeypatch.setattr(protocol, "NATIVE_SETS", False)
    case = next(c for c in CASES if c["name"] == name)
    _compare(_run(OracleEngine(), case), case["exact"])


def test_local_world_device_row_messages():
    """comm.DeviceRow through a LocalWorld: delivered by reference into a
    RowSlot, accounted as its wire message (size items x 8 B), truncation and
    a plain-buffer receive refused."""
    comm = sub("comm")
    w = comm.LocalWorld(2, coop=False)
    row = np.arange(10, dtype=np.uint8)

    def body(c):
        if c.rank == 0:
            c.Send([comm.DeviceRow(row, 30), None], dest=1)
            return None
        slot = comm.RowSlot(30)
        c.Recv([slot, None], source=0)
        return slot.row

    res = w.run(body)
    assert res[1] is row and w.sent_messages == 1 and w.sent_bytes == 240
    w2 = comm.LocalWorld(2, coop=False, timeout=5)

    def bad(c):
        if c.rank == 0:
            c.Send([comm.DeviceRow(row, 31), None], dest=1)
            return None
        c.Recv([comm.RowSlot(30), None], source=0)

    with pytest.raises(Exception):
        w2.run(bad)


@pytest.mark.parametrize("case", [c for c in CASES if c["n"] == 3][:3], ids=lambda c: c["name"])
def test_protocol_out_of_range_injection_rows_equal_wire(case):
    """Injected values >= w: the wire carries nq bits per value (tfg.py:84,
    128-129), so the in-process device-row run must see the values the wire
    run decodes -- both runs agree on every outcome."""
    L = LISTS[case["name"]].astype(np.int64).copy()
    rng = np.random.default_rng(7)
    w = 1 << sub("resource").n_qubits(case["n"])
    pick = rng.choice(L.size, 40, replace=False)
    L.flat[pick] += w * rng.integers(1, 4, 40)  # same low nq bits, out of range
    protocol = sub("protocol")

    def run(engine, **kw):
        return protocol.run_local(case["n"], case["sizeL"], case["nDishonest"], engine, seed=case["seed"],
                                  lists=L, timeout=60, party_kwargs=kw or None)

    rows, wire = run(_RowEngine()), run(OracleEngine(), wire=True)
    assert (rows.error, rows.result, rows.V, rows.accept, rows.reject) == \
        (wire.error, wire.result, wire.V, wire.accept, wire.reject)
    # and both equal the in-range lists' run (the low nq bits are unchanged)
    _compare(rows, case["exact"])
