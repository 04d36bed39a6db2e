"""bench.py's launch contract: `python bench.py --gpus N` starts the N ranks
itself when it is not already under torchrun, and prints exactly one JSON
line (rank 0's) -- so the driver can call --gpus 8 exactly as it calls
--gpus 1."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_bench_self_launch_cpu():
    """The launcher itself (no GPU): two ranks of a stub worker under
    torch.distributed.run over gloo; one JSON line with the world it saw."""
    env = _env(QBA_BENCH_WORKER=str(ROOT / "tests" / "bench_worker_stub.py"), QBA_BENCH_LAUNCH_TIMEOUT="240")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["sum"] == 2
    assert line["argv"][:2] == ["--gpus", "2"] and "--steps" in line["argv"]


def test_bench_self_launch_refuses_single_gpu_configs():
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--config", "1"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "single-GPU" in p.stderr


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_gpu():
    """The real headline with --gpus 2 on a one-GPU box: both ranks share
    device 0 and reduce over gloo (QBA_SHARE_DEVICE / QBA_DIST_BACKEND: a
    rehearsal, not a measurement).  One line, n_gpus 2, sizeL = 2 shards, the
    honest lists verified collision-free."""
    env = _env(QBA_SHARE_DEVICE="1", QBA_DIST_BACKEND="gloo", QBA_BENCH_LAUNCH_TIMEOUT="150")
    p = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["steps"] == 5 and line["warmup"] == 2
    assert line["config"]["sizeL"] == 2 * 125_000_000 and line["value"] > 0
    v = line["verification"]
    assert v["offdiag_collisions"] == 0
    # the reduced counts are the C twin's over entries [0, 2.5e8) (the recorded
    # prefix of configs[2]); at 8 ranks the same check is counts_equal_1e9_golden
    assert v["counts_equal_golden"] is True, v
    assert "counts_equal_1e9_golden" not in v
    # the rows both ranks wrote, checksummed on the device, and the number of
    # ranks the all-reduce itself summed
    assert v["rows_equal_golden"] is True and v["rows_equal_golden_per_rank"] == [True, True], v
    assert v["allreduce_ranks"] == 2 and v["backend"] == "gloo", v
    rl = line["rank_launch_ms"]
    assert len(rl["per_rank"]) == 2 and 0 < rl["min"] <= rl["max"]


def test_bench_golden_verification_cpu():
    """bench.verify_counts on the recorded configs[2] prefixes: equal counts
    pass, one changed count fails, sizes without a fixture report none, and
    world 8 (sizeL = 1e9) names the 1e9 check explicitly."""
    import importlib.util
    import numpy as np
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    for world in (1, 2, 4, 8):
        H, C, P = (x.copy() for x in b.golden_counts(11, 0x5EED, 125_000_000, world))
        assert int(C.sum()) == int(P.sum()) * 12  # honest: every Q entry collision-free
        v = b.verify_counts(11, 0x5EED, 125_000_000, world, H, C, P)
        assert v["counts_equal_golden"] is True and v["offdiag_collisions"] == 0
        assert ("counts_equal_1e9_golden" in v) == (world == 8)
        H[3, 4, 5] += 1
        assert b.verify_counts(11, 0x5EED, 125_000_000, world, H, C, P)["counts_equal_golden"] is False
    assert b.golden_counts(11, 0x5EED, 1e6, 1) is None and b.golden_counts(11, 1, 125_000_000, 1) is None
    assert "counts_equal_golden" not in b.verify_counts(11, 7, 125_000_000, 2, H, C, P)
    # shard 0 is what BENCH_r03's single-GPU line reported as q_entries
    assert int(b.golden_counts(11, 0x5EED, 125_000_000, 1)[2].sum()) == 62_495_452
    assert int(b.golden_counts(11, 0x5EED, 125_000_000, 8)[2].sum()) == 500_010_356  # |P| over sizeL = 1e9


def test_config2_totals_fixture_matches_c_twin_shard0():
    """The fixture's first prefix (entries [0, 1.25e8)) recomputed by the C
    twin's closed-form schedule (a few seconds on the host)."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_lib
    z = np.load(ROOT / "tests" / "golden" / "config2_totals_n11_5eed.npz")
    empty = {"nfac": 0, "desc": np.zeros((16, 6), np.int32), "pat": np.zeros(1, np.uint64),
             "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    H, C, P, bad = oracle_lib.stream_counts(11, 0x5EED, 0, 125_000_000, empty, empty, closed=True)
    assert bad == 0
    assert np.array_equal(H, z["H_1"]) and np.array_equal(C, z["C_1"]) and np.array_equal(P, z["P_1"])


def _bench_mod():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


@pytest.mark.parametrize("count", [1, 2, 4099, 100_003])
def test_row_sums_of_stored_rows_match_c_twin(count):
    """bench.device_row_sums (run here on CPU tensors; on the GPU over the
    rows the timed kernel wrote) from nibble rows and from byte rows equals
    the C twin's streamed checksum of the same entries, odd counts included."""
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_lib
    b = _bench_mod()
    empty = {"nfac": 0, "desc": np.zeros((16, 6), np.int32), "pat": np.zeros(1, np.uint64),
             "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    n, seed, first = 11, 0x5EED, 6 * 125_000_000 + 10
    L = oracle_lib.sample(n, seed, first, count, empty, empty, True)
    want = oracle_lib.stream_row_sums(n, seed, first, count, empty, empty, True)
    assert np.array_equal(oracle_lib.row_sums(L), want)
    nb = (count + 1) // 2
    pk = np.zeros((n + 1, nb + 7), np.uint8)
    pk[:, : count // 2] = L[:, 0:count - count % 2:2] | (L[:, 1::2][:, : count // 2] << 4)
    if count % 2:
        pk[:, nb - 1] = L[:, -1]
    got = b.device_row_sums(torch.from_numpy(pk), n, count, True).numpy()
    assert np.array_equal(got, want.astype(np.int64))
    byte = np.zeros((n + 1, count + 5), np.uint8)
    byte[:, :count] = L
    assert np.array_equal(b.device_row_sums(torch.from_numpy(byte), n, count, False).numpy(), want.astype(np.int64))


def test_row_golden_verification_cpu():
    """bench.verify_rows: the recorded shards pass, one changed sum fails,
    other workloads report nothing."""
    import numpy as np
    b = _bench_mod()
    S = np.load(ROOT / "tests" / "golden" / "config2_rows_n11_5eed.npz")["S"].astype(np.int64)
    for world in (1, 2, 4, 8):
        v = b.verify_rows(11, 0x5EED, 125_000_000, [S[r] for r in range(world)])
        assert v["rows_equal_golden"] is True and v["rows_equal_golden_per_rank"] == [True] * world
    bad = [S[0], S[1].copy()]
    bad[1][7, 1] += 1
    v = b.verify_rows(11, 0x5EED, 125_000_000, bad)
    assert v["rows_equal_golden"] is False and v["rows_equal_golden_per_rank"] == [True, False]
    assert b.verify_rows(11, 1, 125_000_000, [S[0]]) == {}


def test_config2_rows_fixture_matches_c_twin_last_shard():
    """The row fixture's shard 7 (entries [8.75e8, 1e9)) recomputed by the C twin."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_lib
    empty = {"nfac": 0, "desc": np.zeros((16, 6), np.int32), "pat": np.zeros(1, np.uint64),
             "apat": np.zeros(1, np.uint64), "thr": np.zeros(1, np.uint64)}
    S = np.load(ROOT / "tests" / "golden" / "config2_rows_n11_5eed.npz")["S"]
    assert np.array_equal(oracle_lib.stream_row_sums(11, 0x5EED, 7 * 125_000_000, 125_000_000, empty, empty, True),
                          S[7])
