#!/usr/bin/env python3
"""Headline benchmark: list entries sampled+verified per second at n = 11.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

One step = one pass of the hot path over this rank's shard of sizeL: every
entry is Born-sampled from the compiled resource program (Philox keyed by the
global entry index), its n+1 list bytes are written to HBM, and the count-mode
checks (isQCorr, P_u, every party's tuple histogram and every pairwise
collision, the inputs of consistent()) are accumulated -- then, for N > 1, the
count histograms are summed over ranks with one RCCL all-reduce.

Workload (config.workload): BASELINE.json configs[2] -- n = 11 parties,
3 dishonest, sizeL = 1e9 sharded over 8 GPUs -- i.e. 1.25e8 entries per GPU.
At N GPUs each rank owns 1.25e8 entries (weak scaling; N = 8 is exactly
sizeL = 1e9).  configs[1] (sizeL = 1e6 on one GPU, 12 MB of lists) is
cache-resident and launch-bound and is covered by the parity tests.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
PKG = "tfg---quantum-byzantine-agreement_amd"

METRIC = "list entries sampled+verified/sec (node) at n=11; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.3 TB/s measured copy


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=11)
    ap.add_argument("--dishonest", type=int, default=3)
    ap.add_argument("--per-gpu", type=float, default=1.25e8, help="entries per GPU per step")
    ap.add_argument("--mode", choices=["fused", "split"], default="fused")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=str(ROOT / "profiles" / "traffic_n11.json"),
                    help="PMC-derived HBM bytes per launch (profiles/), if present")
    return ap.parse_args()


def cpu_baseline(n, seed, info, target_s):
    """The oracle's C twin (OpenMP, all host threads) on a bounded sample."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_lib
    sample = 1 << 18
    t0 = time.perf_counter()
    oracle_lib.sample_counts(n, seed, 0, sample, info["notq"], info["q"], info["closed"])
    dt = time.perf_counter() - t0
    sample = int(min(max(sample, sample * target_s / max(dt, 1e-6)), 1 << 27))
    t0 = time.perf_counter()
    oracle_lib.sample_counts(n, seed, 0, sample, info["notq"], info["q"], info["closed"])
    dt = time.perf_counter() - t0
    return {"value": sample / dt, "unit": "entries/s", "cores": oracle_lib.threads(), "kind": "port",
            "sample": f"{sample} entries of the same n={n} workload: C twin (oracle/sampler_ref.c) "
                      f"sample + count, {dt:.2f} s"}


def main():
    args = parse()
    import torch
    dist_mod = importlib.import_module(f"{PKG}.distributed")
    eng_mod = importlib.import_module(f"{PKG}.engine")
    rank, local, world = dist_mod.init()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    eng = eng_mod.Engine(local)
    n = args.n
    per = int(args.per_gpu)
    info = eng.prepare(n)
    first = rank * per  # weak scaling: rank r owns global entries [r*per, (r+1)*per)
    lists = eng.alloc_lists(n, per)
    _, _, _, total = dist_mod.count_layout(n)
    flat = torch.zeros(total, dtype=torch.int64, device=eng.device)
    H, C, P = dist_mod.split_counts(flat, n)
    counts = eng_mod.Counts(H, C, P)
    stream = torch.cuda.current_stream()

    def step():
        if args.mode == "fused":
            eng.sample_check(n, args.seed, first, per, lists, counts)
        else:
            eng.sample(n, args.seed, first, per, lists)
            eng.check_counts(lists, n, per, counts)
        dist_mod.allreduce_counts(flat)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        if args.mode == "fused":
            eng.sample_check(n, args.seed, first, per, lists, counts)
        else:
            eng.sample(n, args.seed, first, per, lists)
            eng.check_counts(lists, n, per, counts)
        ev[i][1].record(stream)
        dist_mod.allreduce_counts(flat)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=eng.device)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    t_max = float(t.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    # verification result of the last step: honest Q positions never collide
    Hn, Cn, Pn = (x.cpu().numpy() for x in (H, C, P))
    offdiag = int(Cn.sum() - sum(Cn[:, g, g].sum() for g in range(n + 1)))
    if rank != 0:
        return
    entries = per * world * args.steps
    value = entries / t_max
    bytes_per_entry = 2 * (n + 1)
    achieved = bytes_per_entry * per / (kern_ms * 1e-3) / 1e9
    traffic = None
    tp = Path(args.traffic)
    if tp.exists():
        tj = json.loads(tp.read_text())
        if tj.get("per_launch_entries") == per and tj.get("n") == n and tj.get("mode") == args.mode:
            traffic = tj.get("hbm_bytes_per_launch")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "entries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: lists Born-sampled on the device (Philox4x32-10 keyed by entry index); no dataset",
        "config": {
            "workload": f"BASELINE configs[2] shard: n={n} parties, {args.dishonest} dishonest, "
                        f"{per:.3g} entries/GPU (sizeL={per * world:.3g} over {world} GPU)",
            "n_parties": n, "n_dishonest": args.dishonest, "entries_per_gpu": per,
            "sizeL": per * world, "mode": args.mode,
            "parallelism": f"sizeL sharded over {world} GPU(s), RCCL all-reduce of counts",
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": "qba_k_lists<11,1> (+qba_k_reduce)" if args.mode == "fused" else "qba_k_lists<11,0>+<11,2>",
            "algorithmic_bytes_per_entry": bytes_per_entry, "kernel_ms": kern_ms,
        },
        "verification": {"q_entries": int(Pn.sum()), "offdiag_collisions": offdiag},
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, args.seed, info, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
