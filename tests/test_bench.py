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
                        "--per-gpu", "2.5e7"], env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["steps"] == 5 and line["warmup"] == 2
    assert line["config"]["sizeL"] == 2 * 25_000_000 and line["value"] > 0
    assert line["verification"]["offdiag_collisions"] == 0
    # the reduced P counts both shards' Q entries: about half of 2 x 2.5e7
    assert abs(line["verification"]["q_entries"] - 25_000_000) < 50_000
