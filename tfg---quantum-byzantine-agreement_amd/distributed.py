"""Multi-GPU plumbing: sizeL is sharded across ranks (one process per GPU).

Entry k of the global list is drawn from Philox keyed by k itself, so a rank
computes exactly the entries it owns and the lists are bit-identical for any
number of GPUs.  The only exchange is one sum all-reduce of
the int64 count histograms H, C and P (≈43 KB at n=11): RCCL over xGMI on
MI355X (torch.distributed backend "nccl"), gloo in the CPU tests.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch


def shard_bounds(total: int, rank: int, world: int) -> Tuple[int, int]:
    """[first, first+count) of rank's contiguous shard of `total` entries."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    per = -(-total // world)
    first = min(rank * per, total)
    return first, min(per, total - first)


def world_from_env() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from torchrun's environment (1-process default).

    QBA_SHARE_DEVICE=1 maps every local rank to device 0: a rehearsal of the
    N-rank path on a one-GPU box (with QBA_DIST_BACKEND=gloo, since RCCL
    refuses two ranks on one device).  Never set for a measurement."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("QBA_SHARE_DEVICE") == "1":
        local = 0
    return int(os.environ.get("RANK", "0")), local, int(os.environ.get("WORLD_SIZE", "1"))


def init(backend: Optional[str] = None) -> Tuple[int, int, int]:
    rank, local, world = world_from_env()
    if world > 1 and not torch.distributed.is_initialized():
        if backend is None:
            backend = os.environ.get("QBA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        torch.distributed.init_process_group(backend=backend)
    return rank, local, world


def group_ranks(device=None) -> int:
    """How many ranks the collective itself sums: a one-element int64 1 from
    every rank, all-reduced over the default group (RCCL under the "nccl"
    backend).  1 without a process group.  A line that reports N ranks
    proves with it that the all-reduce its counts went through saw N."""
    if not (torch.distributed.is_initialized() and torch.distributed.get_world_size() > 1):
        return 1
    one = torch.ones(1, dtype=torch.int64, device=device)
    torch.distributed.all_reduce(one, op=torch.distributed.ReduceOp.SUM)
    return int(one.item())


def allreduce_counts(flat: torch.Tensor) -> torch.Tensor:
    """Sum the flat int64 [H | C | P] buffer over ranks, in place."""
    if torch.distributed.is_initialized() and torch.distributed.get_world_size() > 1:
        torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM)
    return flat


def allreduce_counts_async(flat: torch.Tensor):
    """Start the sum of the flat [H | C | P] buffer over ranks; returns the
    work handle (wait() orders the caller's stream after it) or None when
    there is nothing to reduce (one rank)."""
    if torch.distributed.is_initialized() and torch.distributed.get_world_size() > 1:
        return torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM, async_op=True)
    return None


def count_layout(n: int) -> Tuple[int, int, int, int]:
    """Sizes (H, C, P, total) of the flat count buffer for n parties."""
    w = 1 << int(n).bit_length()
    h, c, p = w * (n + 1) * w, w * (n + 1) * (n + 1), w
    return h, c, p, h + c + p


def split_counts(flat: torch.Tensor, n: int):
    """Views (H, C, P) into a flat [H | C | P] buffer."""
    w = 1 << int(n).bit_length()
    h, c, p, _ = count_layout(n)
    H = flat[:h].view(w, n + 1, w)
    C = flat[h:h + c].view(w, n + 1, n + 1)
    P = flat[h + c:h + c + p]
    return H, C, P
