#!/usr/bin/env python3
"""Headline benchmark: list entries sampled+verified per second at n = 11.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

`python bench.py --gpus N` outside torchrun launches the N ranks itself (one
process per GPU under torch.distributed.run, see launch_ranks) and prints rank
0's line, so both forms measure the same thing.

One step (default, --config 2) = one pass of the hot path over this rank's
shard of sizeL: every entry is Born-sampled from the compiled resource program
(Philox keyed by the global entry index), its n+1 list values are written to
HBM, and the count-mode checks run on every Q-correlated entry from registers:
isQCorr (L0 != L1, tfg.py:327), P_u, every party's tuple histogram, and
Cond3's pairwise test (tfg.py:96-98: the union of the entry's one-hot values
must have n+1 bits; an entry that fails it counts every equal pair into C) --
the inputs of consistent(); for N > 1 the count histograms are then summed
over ranks with one RCCL all-reduce.

Workload (config.workload): BASELINE.json configs[2] -- n = 11 parties,
3 dishonest, sizeL = 1e9 sharded over 8 GPUs -- i.e. 1.25e8 entries per GPU.
At N GPUs each rank owns 1.25e8 entries (weak scaling; N = 8 is exactly
sizeL = 1e9).  The metric is a node figure, so the node configuration sets
the per-GPU shard; configs[1] (sizeL = 1e6, 12 MB of lists: cache-resident and
launch-bound) is --config 1.

Other BASELINE.json configs (one JSON line each, one GPU):
  --config 0  configs[0]: n=3, nDis=1, sizeL=1000 protocol run (the
              reference's CPU case) on the exact-mode host; CPU baseline = the
              same host on the numpy oracle.
  --config 1  configs[1]: n=11, sizeL=1e6, K steps captured in one hipGraph,
              the median of 5 timed replays.
  --config 3  configs[3]: 4096 independent n=7 instances x sizeL=1e5.
  --config 4  configs[4]: the largest resource register in fp64 HBM (GHZ
              register of the Q circuit, n+1 qubits); GB/s of its fused CX
              pass and the register's preparation time.

roofline.achieved = the HBM bytes the fused pass must move per launch -- the
lists written once ((n+1)/2 B per entry as nibble rows, (n+1) B as byte rows;
the checks run from registers and never re-read them) -- / the step's device
time, measured with HIP events on the stream the kernels run on; frac is that
over the 8 TB/s peak, a physical fraction (roofline.traffic: the PMC-measured
bytes of this build, within ~3 % of it).  BASELINE's own scoring convention
(2(n+1) B per entry: lists written + read back once) is reported beside it as
roofline.metric_scale.  The step is one deferred sample_check call: the
fused kernel, which also reduces the PREVIOUS step's counts in workgroups
after its own (qba_k_lists_pbdef); the last step's reduction is the flush
inside the timed region (QBA_BENCH_DEFER=0: the synchronous call, list kernel
+ qba_k_reduce per step).  One event pair brackets the K
timed launches (device time / K): an event pair around every launch costs
~10 us of GPU time per step (markers between the kernels; rocprofv3 trace:
10.4 us gaps before each list kernel, none with one pair), which would be
charged to the step.  QBA_BENCH_EVENTS=step restores the per-launch pairs.

verification (outside the timed region): the all-reduced H, C, P against
the C twin's totals of entries [0, N x 1.25e8) (counts_equal_golden; at N = 8
counts_equal_1e9_golden), position-weighted checksums of every row each rank
wrote, computed on the device, against the C twin's checksums of that shard
(rows_equal_golden), and allreduce_ranks: a one-element int64 1 all-reduced
over the counts' process group before the timing (RCCL under the nccl
backend), which must equal N.
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
DATA = "synthetic: lists Born-sampled on the device (Philox4x32-10 keyed by entry index); no dataset"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 200 for configs 1-3, 20 otherwise)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps (default: 50 for configs 1-3, 3 otherwise)")
    ap.add_argument("--config", type=int, default=2, choices=[0, 1, 2, 3, 4])
    ap.add_argument("--n", type=int, default=11)
    ap.add_argument("--dishonest", type=int, default=3)
    ap.add_argument("--per-gpu", type=float, default=1.25e8, help="entries per GPU per step")
    ap.add_argument("--mode", choices=["fused", "split", "sample"], default="fused",
                    help="fused (the headline), split (sample then check), sample (diagnostic: no check)")
    ap.add_argument("--layout", choices=["packed", "bytes"], default="packed",
                    help="list rows as nibbles (qba_*_packed, the shipped hot path) or one byte per value")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sv-qubits", type=int, default=None, help="--config 4 register size")
    ap.add_argument("--traffic", default=str(ROOT / "profiles" / "traffic_n11.json"),
                    help="PMC-derived HBM bytes per launch (profiles/), if present")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# CPU baselines (the only place bench.py touches oracle/)
# ---------------------------------------------------------------------------
def cpu_baseline_counts(n, seed, info, target_s):
    """The oracle's C twin (same schedule, same counts; OpenMP on every host
    thread it is given) over a bounded sample, in 2^25-entry chunks."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_lib
    chunk = 1 << 25
    done, t0 = 0, time.perf_counter()
    while True:
        oracle_lib.sample_counts(n, seed, done, chunk, info["notq"], info["q"], info["closed"])
        done += chunk
        dt = time.perf_counter() - t0
        if dt >= target_s or done >= 1 << 32:
            break
    return {"value": done / dt, "unit": "entries/s", "cores": oracle_lib.threads(), "kind": "port",
            "sample": f"{done} entries (entries [0, {done})) of the same n={n} workload: C twin "
                      f"(oracle/sampler_ref.c) sample + count, {dt:.1f} s"}


def cpu_baseline_mpiexec(runs):
    """BASELINE.md CPU plan item 2: the Python restatement of tfg.py under a
    real `mpiexec -n 4` at configs[0] (tests/mpi_cpu_baseline.py: the
    package's protocol host, one process per party, numpy engine on the host
    cores).  Reports the protocol wall per run (max over ranks) and the whole
    command's wall, start-up included (as `time mpiexec -n 4 python tfg.py
    1000 1` would).  None when no mpiexec is installed."""
    import shutil
    import subprocess
    mpiexec = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
    if not os.path.exists(mpiexec):
        return None
    env = {k: v for k, v in os.environ.items() if not k.startswith(("PMI_", "OMPI_"))}
    t0 = time.perf_counter()
    p = subprocess.run([mpiexec, "-n", "4", sys.executable, str(ROOT / "tests" / "mpi_cpu_baseline.py"),
                        "--runs", str(runs)], capture_output=True, text=True, timeout=300, env=env)
    wall = time.perf_counter() - t0
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode or not lines:
        return {"error": (p.stderr or p.stdout)[-300:]}
    r = json.loads(lines[-1])
    return {"value": r["entries_per_s"], "unit": "entries/s (protocol run, sizeL=1000)", "cores": 4,
            "kind": "port", "ms_per_run": r["ms_per_run_median"], "command_wall_s": wall,
            "sample": f"mpiexec -n 4: {runs} protocol runs of n=3, 1 dishonest, sizeL=1000 (+1 warm-up), the "
                      "package's host with the numpy engine on the host CPU, one process per party "
                      "(tests/mpi_cpu_baseline.py); command_wall_s includes MPI and Python start-up"}


def _lib_sha16():
    """sha256 (16 hex) of the libqba.so this process loads (PMC figures are per build)."""
    import hashlib
    lib = importlib.import_module(f"{PKG}._lib")
    return hashlib.sha256(Path(lib.LIB_PATH).read_bytes()).hexdigest()[:16]


GOLDEN_TOTALS = ROOT / "tests" / "golden" / "config2_totals_n11_5eed.npz"


def golden_counts(n, seed, per, world):
    """The C twin's H, C, P over entries [0, per * world) when that is a
    prefix tests/golden/gen_config2_totals.py recorded (n = 11, seed 0x5EED,
    1.25e8 entries per rank, world 1, 2, 4 or 8 -- world 8 is sizeL = 1e9),
    else None.  A fixture (data), not the oracle: the weak-scaling line checks
    its own all-reduced counts with it."""
    if n != 11 or seed != 0x5EED or per != 125_000_000 or world not in (1, 2, 4, 8) or not GOLDEN_TOTALS.exists():
        return None
    import numpy as np
    z = np.load(GOLDEN_TOTALS)
    return z[f"H_{world}"], z[f"C_{world}"], z[f"P_{world}"]


def verify_counts(n, seed, per, world, H, C, P):
    """bench.py's verification block for one set of all-reduced counts."""
    import numpy as np
    offdiag = int(C.sum() - sum(C[:, g, g].sum() for g in range(n + 1)))
    # offdiag_collisions: equal pairs g != h at Q-correlated entries, found by
    # the kernel's per-entry Cond3 test (tfg.py:96-98); 0 for honest lists
    out = {"q_entries": int(P.sum()), "offdiag_collisions": offdiag}
    ref = golden_counts(n, seed, per, world)
    if ref is not None:
        same = bool(np.array_equal(H, ref[0]) and np.array_equal(C, ref[1]) and np.array_equal(P, ref[2]))
        out["counts_equal_golden"] = same
        out["golden"] = (f"C-twin H/C/P over entries [0, {per * world}) "
                         f"(tests/golden/{GOLDEN_TOTALS.name}, key {world})")
        if per * world == 10 ** 9:
            out["counts_equal_1e9_golden"] = same
    return out


GOLDEN_ROWS = ROOT / "tests" / "golden" / "config2_rows_n11_5eed.npz"


def device_row_sums(lists, n, count, packed):
    """Position-weighted checksums of the rows a step wrote, computed on the
    device from the rows as stored: int64 [n+1, 2] with, per row g,
    (sum_k L_g[k], sum_k L_g[k] * (k+1)) over the step's columns k (nibble
    rows: column 2b = the low nibble of byte b, 2b+1 the high one).  Outside
    the timed region; the same sums as oracle_lib.stream_row_sums."""
    import torch
    g = n + 1
    s0 = torch.zeros(g, dtype=torch.int64, device=lists.device)
    s1 = torch.zeros(g, dtype=torch.int64, device=lists.device)
    nb = (count + 1) // 2 if packed else count
    step = 1 << 22
    for off in range(0, nb, step):
        m = min(step, nb - off)
        x = lists[:g, off:off + m].to(torch.int64)
        k = torch.arange(off, off + m, dtype=torch.int64, device=lists.device)
        if packed:
            lo, hi = x & 15, x >> 4
            s0 += lo.sum(1) + hi.sum(1)
            s1 += (lo * (2 * k + 1)).sum(1) + (hi * (2 * k + 2)).sum(1)
        else:
            s0 += x.sum(1)
            s1 += (x * (k + 1)).sum(1)
    return torch.stack([s0, s1], 1)


def verify_rows(n, seed, per, sums):
    """bench.py's row check: sums[r] (int64 [n+1, 2], rank r's device_row_sums
    of its shard's rows) against the C twin's sums of shard r
    (tests/golden/gen_config2_rows.py), when recorded; else {}."""
    import numpy as np
    if n != 11 or seed != 0x5EED or per != 125_000_000 or len(sums) > 8 or not GOLDEN_ROWS.exists():
        return {}
    S = np.load(GOLDEN_ROWS)["S"].astype(np.int64)
    same = [bool(np.array_equal(np.asarray(s, dtype=np.int64), S[r])) for r, s in enumerate(sums)]
    return {"rows_equal_golden": all(same), "rows_equal_golden_per_rank": same,
            "rows_golden": f"C-twin row sums (sum L_g[k], sum L_g[k]*(k+1)) of every rank's shard rows "
                           f"(tests/golden/{GOLDEN_ROWS.name})"}


# Measured issue cost per wave64 VALU instruction on one SIMD at 8 waves
# (tools/exp/valu_rate.hip, profiles/r4/micro/valu_rate.txt): simple ops
# (v_add_u32 2.31, v_bitop3_b32 2.42) and the 64-bit multiply that
# SQ_INSTS_VALU_INT64 counts (v_mad_u64_u32, 4.56 -- Philox's multiply)
VALU_CYC_SIMPLE, VALU_CYC_INT64 = 2.31, 4.56


def issue_roofline(tj, entries, launch_ms):
    """roofline.issue: the fused kernel's issue-side ceiling from the PMC
    counters of this build (tools/pmc_traffic.py: chip-wide medians per
    launch).  Shader cycles per launch = GRBM_GUI_ACTIVE / 8 (8 XCDs); a
    wave64 VALU instruction issues in 2 cycles on a 32-lane CDNA4 SIMD at
    best (valu_busy_frac), the 64-bit multiplies in ~4.6 (valu_busy_frac_weighted:
    the measured costs above; v_perm_b32 / v_mul_*_u32 at 4.25 are priced as
    simple ops, so it is still a floor); 1,024 SIMDs and 256 LDS units."""
    c = tj.get("issue_counters_per_launch") or {}
    if "GRBM_GUI_ACTIVE" not in c or "SQ_INSTS_VALU" not in c:
        return None
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    valu_ipc = c["SQ_INSTS_VALU"] / (1024 * cyc)
    out = {"cycles_per_launch": cyc,
           "effective_clock_ghz": cyc / (launch_ms * 1e6) if launch_ms else None,
           "valu_lane_ops_per_entry": c["SQ_INSTS_VALU"] * 64 / entries,
           "valu_insts_per_simd_cycle": valu_ipc,
           "valu_busy_frac": 2 * valu_ipc}
    # measured, not priced: SQ_ACTIVE_INST_VALU counts the quad-cycles (4 shader
    # cycles) in which a wave issued a VALU instruction; per SIMD over the
    # launch's quad-cycles it is the VALU's busy fraction as the hardware saw
    # it (every VALU instruction of this kernel occupies one quad-cycle: the
    # count equals SQ_INSTS_VALU)
    if "SQ_ACTIVE_INST_VALU" in c:
        out["valu_active_frac"] = c["SQ_ACTIVE_INST_VALU"] / (1024 * cyc / 4)
    if "SQ_INSTS_VALU_INT64" in c:
        i64 = c["SQ_INSTS_VALU_INT64"]
        out["valu_busy_frac_weighted"] = ((c["SQ_INSTS_VALU"] - i64) * VALU_CYC_SIMPLE
                                          + i64 * VALU_CYC_INT64) / (1024 * cyc)
    if "SQ_LDS_IDX_ACTIVE" in c:
        out["lds_active_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (256 * cyc)
        out["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(c["SQ_LDS_IDX_ACTIVE"], 1.0)
    if "SQ_INSTS_LDS_ATOMIC" in c:
        out["lds_atomics_per_entry"] = c["SQ_INSTS_LDS_ATOMIC"] * 64 / entries
    if "SQ_INSTS_LDS" in c:
        out["lds_insts_per_entry"] = c["SQ_INSTS_LDS"] * 64 / entries
    busy = {"VALU": out.get("valu_active_frac", out.get("valu_busy_frac_weighted", out["valu_busy_frac"])),
            "LDS": out.get("lds_active_frac", 0.0)}
    top = max(busy, key=busy.get)
    out["binds"] = (f"{top} issue ({busy[top]:.0%} busy; "
                    + ", ".join(f"{k} {v:.0%}" for k, v in busy.items() if k != top)
                    + ("): neither unit saturated, the rest is dependency latency the 8 waves per SIMD do not hide"
                       if busy[top] < 0.8 else "): near saturation -- cycles follow the VALU instruction count"))
    return out


# ---------------------------------------------------------------------------
# configs[2]: the headline (default)
# ---------------------------------------------------------------------------
def headline(args):
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
    packed = args.layout == "packed"
    lists = eng.alloc_packed(n, per) if packed else eng.alloc_lists(n, per)
    _, _, _, total = dist_mod.count_layout(n)
    # The fused packed step defers its count reduction into the NEXT step's
    # list kernel (qba_sample_check_packed_deferred: the pair-bin kernel runs
    # the pending reduction in workgroups after its own, dispatched into the
    # CUs its last list workgroups leave idle), so step i's counts are
    # complete once step i+1 is enqueued, and the last step's after the
    # flush -- all inside the timed region, and checked against the golden
    # totals below.  One kernel per step instead of list kernel + reduce
    # launch: steady step 277.9 -> 271.9 us, the driver's window 352.5 ->
    # 344.4 us in rocprofv3 traces of one box (profiles/r5/defer/).
    # QBA_BENCH_DEFER=0 restores the synchronous step.
    # N > 1: a step's all-reduce runs asynchronously (RCCL's own stream) as
    # soon as its counts are complete; a count buffer is written again only
    # after its all-reduce was waited for.
    deferred = packed and args.mode == "fused" and os.environ.get("QBA_BENCH_DEFER", "1") == "1"
    nbuf = 3 if world > 1 else 1
    flats = [torch.zeros(total, dtype=torch.int64, device=eng.device) for _ in range(nbuf)]
    counts = [eng_mod.Counts(*dist_mod.split_counts(f, n)) for f in flats]
    pending = [None] * nbuf
    stream = torch.cuda.current_stream()
    # what the collective itself saw: ones all-reduced over the same group the
    # counts go through (RCCL under the nccl backend); must be the world size
    ranks_seen = dist_mod.group_ranks(eng.device)
    if ranks_seen != world:
        raise SystemExit(f"the all-reduce summed {ranks_seen} ranks, WORLD_SIZE={world}")
    backend = torch.distributed.get_backend() if world > 1 else None

    def wait_buf(b):
        if pending[b] is not None:
            pending[b].wait()
            pending[b] = None

    def step(i):
        b = i % nbuf
        if deferred:
            # this launch completes step i-1's counts (buffer (i-1) % nbuf)
            # and later writes buffer b: both must be free of all-reduces
            wait_buf((i - 1) % nbuf)
            wait_buf(b)
            eng.sample_check_packed(n, args.seed, first, per, lists, counts[b], deferred=True)
            if i > 0 and world > 1:
                pending[(i - 1) % nbuf] = dist_mod.allreduce_counts_async(flats[(i - 1) % nbuf])
            return
        wait_buf(b)
        if packed:
            if args.mode == "fused":
                eng.sample_check_packed(n, args.seed, first, per, lists, counts[b])
            elif args.mode == "sample":
                eng.sample_packed(n, args.seed, first, per, lists)
            else:
                eng.sample_packed(n, args.seed, first, per, lists)
                eng.check_counts_packed(lists, n, per, counts[b])
        elif args.mode == "fused":
            eng.sample_check(n, args.seed, first, per, lists, counts[b])
        elif args.mode == "sample":
            eng.sample(n, args.seed, first, per, lists)
        else:
            eng.sample(n, args.seed, first, per, lists)
            eng.check_counts(lists, n, per, counts[b])
        pending[b] = dist_mod.allreduce_counts_async(flats[b])

    def drain(last):
        if deferred and last >= 0:
            eng.flush_deferred()  # the last step's reduction
            if world > 1:
                wait_buf(last % nbuf)
                pending[last % nbuf] = dist_mod.allreduce_counts_async(flats[last % nbuf])
        for b in range(nbuf):
            wait_buf(b)

    for i in range(args.warmup):
        step(i)
    drain(args.warmup - 1)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    per_step_events = os.environ.get("QBA_BENCH_EVENTS", "loop") == "step"
    t0 = time.perf_counter()
    if not per_step_events:
        ev[0][0].record(stream)
    for i in range(args.steps):
        if per_step_events:
            ev[i][0].record(stream)
        step(i)
        if per_step_events:
            ev[i][1].record(stream)
    drain(args.steps - 1)
    if not per_step_events:
        ev[0][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=eng.device)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    t_max = float(t.item())
    if per_step_events:
        kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    else:
        kern_ms = ev[0][0].elapsed_time(ev[0][1]) / args.steps
    H, C, P = counts[(args.steps - 1) % nbuf].H, counts[(args.steps - 1) % nbuf].C, counts[(args.steps - 1) % nbuf].P
    # every rank's own launch time (HIP events on its stream), for diagnosing a flat scaling curve
    kt = torch.tensor([kern_ms], dtype=torch.float64, device=eng.device)
    if world > 1:
        ks = [torch.zeros_like(kt) for _ in range(world)]
        torch.distributed.all_gather(ks, kt)
        rank_ms = [float(k.item()) for k in ks]
    else:
        rank_ms = [kern_ms]

    # verification result of the last step (the all-reduced counts): honest Q
    # positions never collide, and against the C twin's totals when recorded
    Hn, Cn, Pn = (x.cpu().numpy() for x in (H, C, P))
    # ... and the rows it wrote (every step writes the same rows): checksums on
    # the device, gathered from every rank
    rs = device_row_sums(lists, n, per, packed)
    if world > 1:
        gathered = [torch.zeros_like(rs) for _ in range(world)]
        torch.distributed.all_gather(gathered, rs)
        row_sums = [x.cpu().numpy() for x in gathered]
    else:
        row_sums = [rs.cpu().numpy()]
    if rank != 0:
        eng.close()
        return
    entries = per * world * args.steps
    value = entries / t_max
    bytes_per_entry = 2 * (n + 1)  # BASELINE's scoring convention (metric_scale)
    row_bytes = (n + 1) / 2 if packed else n + 1  # list bytes per entry as stored
    # the HBM bytes the pass must move: fused / sample write the lists once,
    # split writes them and reads them back
    moved_per_entry = row_bytes * (2 if args.mode == "split" else 1)
    achieved = moved_per_entry * per / (kern_ms * 1e-3) / 1e9
    metric_gbs = bytes_per_entry * per / (kern_ms * 1e-3) / 1e9
    traffic, traffic_note, issue = None, "no PMC traffic file for this workload", None
    tp = Path(args.traffic)
    if tp.exists():
        tj = json.loads(tp.read_text())
        sha = _lib_sha16()
        if tj.get("per_launch_entries") == per and tj.get("n") == n and tj.get("mode") == args.mode and \
                tj.get("layout", "bytes") == args.layout:
            if tj.get("libqba_sha16") == sha:
                traffic, traffic_note = tj.get("hbm_bytes_per_launch"), f"PMC FETCH+WRITE of this build ({sha})"
                issue = issue_roofline(tj, per, kern_ms)
                if issue is not None:
                    issue["source"] = f"PMC passes of this build ({sha}), tools/pmc_traffic.py"
            else:
                traffic_note = f"stale: {tp.name} was measured on build {tj.get('libqba_sha16')}, running {sha}"
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
        "dtype": _dtype(packed),
        "data": DATA,
        "config": {
            "workload": f"BASELINE configs[2] shard: n={n} parties, {args.dishonest} dishonest, "
                        f"{per:.3g} entries/GPU (sizeL={per * world:.3g} over {world} GPU)",
            "n_parties": n, "n_dishonest": args.dishonest, "entries_per_gpu": per,
            "sizeL": per * world, "mode": args.mode, "sampler": "closed" if info["closed"] else "tables",
            "list_layout": "nibble rows: 4 bits per value, (n+1) x sizeL/2 bytes (qba_sample_check_packed)"
                           if packed else "byte rows: (n+1) x sizeL bytes (qba_sample_check)",
            "parallelism": f"sizeL sharded over {world} GPU(s)" + (
                ", one all-reduce of counts per step ("
                + ("RCCL" if torch.distributed.get_backend() == "nccl" else torch.distributed.get_backend())
                + ", asynchronous: overlaps the next step, double-buffered counts)" if world > 1
                else ", no collective at N=1"),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            # frac is physical since round 5; BENCH_r01-r04 scored
            # BASELINE's 2(n+1) B/entry here, now roofline.metric_scale.frac
            "frac_convention": "physical: the bytes the pass must move (lists written once as stored) / time; "
                               "rounds 1-4 reported BASELINE's 2(n+1) B/entry here (see metric_scale.frac)",
            "kernel": (f"qba_k_lists_pbdef<{n},*> (list kernel; the previous step's count reduction runs in "
                       "its tail)" if deferred else f"qba_k_lists<{n},1,*> + qba_k_reduce") if args.mode == "fused"
                      else f"qba_k_lists<{n},0,*> + qba_k_lists<{n},2,*> + reduce",
            "algorithmic_bytes_per_entry": moved_per_entry, "launch_ms": kern_ms,
            "algorithmic_bytes_note": ("the lists written once as " + ("nibble rows" if packed else "byte rows")
                                       + (" and read back once (split: sample, then check)" if args.mode == "split"
                                          else "; the checks run from registers")),
            # the bytes the launch really moves (PMC) over the same time
            "traffic_gbs": traffic / (kern_ms * 1e-3) / 1e9 if traffic else None,
            "traffic_frac": traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
            "traffic_source": traffic_note,
            "metric_scale": {"bytes_per_entry": bytes_per_entry, "achieved_gbs": metric_gbs,
                             "frac": metric_gbs / HBM_PEAK_GBS,
                             "note": "BASELINE.md's convention: 2(n+1) B per entry (byte lists written once + "
                                     "read back once), charged even though the fused pass never re-reads them; "
                                     "not a physical fraction (can pass 1)"},
            "issue": issue,
        },
        "verification": {**verify_counts(n, args.seed, per, world, Hn, Cn, Pn),
                         **verify_rows(n, args.seed, per, row_sums),
                         "allreduce_ranks": ranks_seen, "backend": backend},
        "rank_launch_ms": {"min": min(rank_ms), "max": max(rank_ms), "per_rank": rank_ms},
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_counts(n, args.seed, info, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    eng.close()


# ---------------------------------------------------------------------------
# the other configs (one GPU)
# ---------------------------------------------------------------------------
def _dtype(packed):
    return "u4 lists (nibble rows), i64 counts" if packed else "u8 lists (byte rows), i64 counts"


def _line(args, value, unit, workload, roofline, extra=None, higher=True, dtype="u8"):
    out = {"metric": METRIC, "value": value, "unit": unit, "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "higher_is_better": higher, "scaling": "weak", "vs_baseline": None,
           "dtype": dtype, "data": DATA, "config": {"workload": workload, "parallelism": "1 GPU"},
           "roofline": roofline}
    out.update(extra or {})
    return out


def config0(args, eng):
    """configs[0]: mpiexec -n 4 python tfg.py 1000 1 -> the tfg.py-compatible
    host's in-process world, exact-order checks on the GPU engine."""
    protocol = importlib.import_module(f"{PKG}.protocol")
    runs = []
    for s in range(max(1, args.warmup)):  # warm: compiles n=3, grows the staging buffers
        protocol.run_local(3, 1000, 1, eng, seed=1000 + s)
    t0 = time.perf_counter()
    for s in range(args.steps):
        runs.append(protocol.run_local(3, 1000, 1, eng, seed=1 + s))
    dt = (time.perf_counter() - t0) / args.steps
    extra = {"ms_per_step": dt * 1e3,
             "protocol": {"success": [r.result["success"] for r in runs[:5]],
                          "messages": runs[0].messages, "bytes": runs[0].bytes}}
    if not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "oracle"))
        sys.path.insert(0, str(ROOT / "tests"))
        from oracle_engine import OracleEngine  # numpy restatement (test infrastructure)
        import numpy as np
        import tfg_oracle as orc
        oe = OracleEngine()
        lists = [orc.closed_form_lists(3, 1000, np.random.default_rng(s)) for s in range(args.steps)]
        t0 = time.perf_counter()
        for s in range(args.steps):
            protocol.run_local(3, 1000, 1, oe, seed=1 + s, lists=lists[s])
        cdt = (time.perf_counter() - t0) / args.steps
        extra["cpu_baseline"] = {"value": 1000 / cdt, "unit": "entries/s", "cores": 1, "kind": "port",
                                 "sample": f"{args.steps} protocol runs, numpy oracle engine in place of "
                                           f"the GPU engine (lists drawn on the host)"}
        mpi_leg = cpu_baseline_mpiexec(max(args.steps, 10))
        if mpi_leg is not None:
            extra["cpu_baseline_mpiexec"] = mpi_leg
    return _line(args, 1000 / dt, "entries/s (whole protocol run, sizeL=1000)",
                 "BASELINE configs[0]: n=3 parties, 1 dishonest, sizeL=1000, protocol rounds "
                 "(in-process mpiexec world)",
                 {"bound": "latency", "achieved": None, "peak": None, "unit": None, "frac": None,
                  "traffic": None, "note": "host protocol rounds; per-packet device calls"}, extra)


C1_REPLAYS = 5


def config1(args, eng):
    """configs[1]: n=11, sizeL=1e6 on one GPU; K steps in one hipGraph.

    The steps use the deferred reduction (qba_sample_check_packed_deferred,
    include/qba.h): step k's count reduction runs in W workgroups of step
    k+1's list kernel -- on CUs the 163 list workgroups leave idle -- instead
    of a separate launch, and the graph ends with the flush of the last step,
    so every step's counts are complete inside the timed replay.  The
    synchronous form (list kernel + reduce launch per step) is timed beside it
    (sync_us_per_step)."""
    import torch
    n, count = 11, 1_000_000
    info = eng.prepare(n)
    packed = args.layout == "packed"
    lists = eng.alloc_packed(n, count) if packed else eng.alloc_lists(n, count)
    counts = eng.alloc_counts(n)
    fused = eng.sample_check_packed if packed else eng.sample_check

    def timed(deferred):
        fused(n, args.seed, 0, count, lists, counts, deferred=deferred)  # allocates scratch before capture
        fused(n, args.seed, 0, count, lists, counts, deferred=deferred)
        eng.flush_deferred()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(args.steps):
                    fused(n, args.seed, 0, count, lists, counts, deferred=deferred)
                if deferred:
                    eng.flush_deferred()
        torch.cuda.synchronize()
        for _ in range(max(1, args.warmup)):
            g.replay()
        torch.cuda.synchronize()
        # C1_REPLAYS timed replays of K passes each (configs[1]
        # is launch-bound, so repeat >= 1000 passes and report the median): the
        # median replay, so that one replay hit by a host or power-state hiccup
        # (+50 % on a 1.8-ms replay, tools/exp/c1_modes.py) does not set the line
        walls, devs = [], []
        for _ in range(C1_REPLAYS):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            t0 = time.perf_counter()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) / args.steps)
            devs.append(a.elapsed_time(b) * 1e-3 / args.steps)
        i = sorted(range(C1_REPLAYS), key=lambda k: walls[k])[C1_REPLAYS // 2]
        return walls[i], devs[i], walls

    sync_wall, sync_dev, _ = timed(False)
    wall, dev, walls = timed(True)
    # the verification result of the last step, checked against a synchronous pass
    ref = eng.alloc_counts(n)
    fused(n, args.seed, 0, count, lists, ref)
    torch.cuda.synchronize()
    same = all(torch.equal(x, y) for x, y in zip((counts.H, counts.C, counts.P), (ref.H, ref.C, ref.P)))
    ach = (6 if packed else 12) * count / dev / 1e9  # lists written once (the checks run from registers)
    extra = {"ms_per_step": wall * 1e3, "sync_us_per_step": sync_wall * 1e6,
             "device_us_per_step": dev * 1e6, "sync_device_us_per_step": sync_dev * 1e6,
             "replays": {"count": C1_REPLAYS, "passes_each": args.steps, "statistic": "median replay",
                         "us_per_pass": [round(w * 1e6, 3) for w in walls]},
             "reduction": "deferred: step k's counts reduced inside step k+1's list kernel, the last by "
                          "the flush at the end of the graph (qba_sample_check_packed_deferred)",
             "verification": {"deferred_counts_equal_sync": bool(same)}}
    if not args.no_cpu_baseline:
        extra["cpu_baseline"] = cpu_baseline_counts(n, args.seed, info, args.cpu_seconds / 2)
    return _line(args, count / wall, "entries/s",
                 "BASELINE configs[1]: n=11 parties, 3 dishonest, sizeL=1e6 on one GPU "
                 f"({args.steps} steps in one hipGraph; median of {C1_REPLAYS} timed replays)",
                 {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": ach / HBM_PEAK_GBS, "traffic": None,
                  "algorithmic_bytes_per_entry": 6 if packed else 12,
                  "metric_scale": {"bytes_per_entry": 24, "achieved_gbs": 24 * count / dev / 1e9,
                                   "frac": 24 * count / dev / 1e9 / HBM_PEAK_GBS},
                  "note": ("6 MB of nibble-row" if packed else "12 MB of byte-row")
                          + " lists stay in the 256 MB Infinity Cache; launch-bound"}, extra,
                 dtype=_dtype(packed))


def config3(args, eng, n_inst=4096, count=100_000):
    """configs[3]: 4096 independent 7-party instances x sizeL=1e5 per GPU."""
    import torch
    n = 7
    packed = args.layout == "packed"
    lists, c = eng.sample_check_batched(n, args.seed, n_inst, count, packed=packed)
    for _ in range(args.warmup):
        eng.sample_check_batched(n, args.seed, n_inst, count, lists, packed=packed)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for _ in range(args.steps):
        lists, c = eng.sample_check_batched(n, args.seed, n_inst, count, lists, packed=packed)
    b.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    dev = a.elapsed_time(b) * 1e-3 / args.steps
    ent = n_inst * count
    row = (n + 1) / 2 if packed else n + 1  # list bytes per entry, written once
    ach = row * ent / dev / 1e9
    # every instance's equal-pair counts (found by the per-entry Cond3 test):
    # C[u][g][g] = |P_u| on the diagonal, 0 off it for honest lists
    honest = bool((c.C.sum((1, 2, 3)) == c.P.sum(1) * (n + 1)).all().item())
    extra = {"ms_per_step": wall * 1e3, "verification": {"all_instances_collision_free": honest}}
    if not args.no_cpu_baseline:
        extra["cpu_baseline"] = cpu_baseline_batched(n, args.seed, count, eng.prepare(n), args.cpu_seconds)
    return _line(args, ent / wall, "entries/s",
                 f"BASELINE configs[3]: {n_inst} independent n=7 instances x sizeL={count} per GPU",
                 {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": ach / HBM_PEAK_GBS, "traffic": None, "algorithmic_bytes_per_entry": row,
                  "metric_scale": {"bytes_per_entry": 16, "achieved_gbs": 16 * ent / dev / 1e9,
                                   "frac": 16 * ent / dev / 1e9 / HBM_PEAK_GBS,
                                   "note": "BASELINE's 2(n+1) B per entry (lists written + read back); "
                                           "the batched kernel writes them once and never re-reads them"},
                  "list_layout": "nibble rows (4 B/entry at n=7)" if packed else "byte rows (8 B/entry)"},
                 extra, dtype=_dtype(packed))


def cpu_baseline_batched(n, seed, count, info, target_s):
    """BASELINE.md CPU plan item 3 for configs[3]: the C twin's batched counts
    (oracle_batched_counts: one instance per OpenMP thread at a time, the same
    keys and count semantics) over a bounded slice of the 4096 instances."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle_lib
    step = max(oracle_lib.threads(), 1)
    done, t0 = 0, time.perf_counter()
    while done < 4096:
        oracle_lib.batched_counts(n, seed + done, step, count, info["notq"], info["q"], info["closed"])
        done += step
        if time.perf_counter() - t0 >= target_s:
            break
    dt = time.perf_counter() - t0
    return {"value": done * count / dt, "unit": "entries/s", "cores": oracle_lib.threads(), "kind": "port",
            "sample": f"{done} of the 4096 instances (keys seed + [0, {done})) x sizeL={count}, n={n}: C twin "
                      f"(oracle/sampler_ref.c oracle_batched_counts) sample + count, {dt:.1f} s"}


def config4(args, eng):
    """configs[4]: the largest resource register whose fp64 statevector fits HBM.

    The register is the Q resource's GHZ register (tfg.py:38-39 restricted to
    one bit of every group): H on its first qubit, then q-1 CX gates from it.
    The CX gates share their control, so the engine applies them as ONE
    XOR-mask pass over the control = 1 half (gate fusion); the line reports
    that pass's bandwidth and the whole preparation's time."""
    import numpy as np
    import torch
    free, _ = torch.cuda.mem_get_info()
    q = args.sv_qubits
    if q is None:
        q = 1
        while (8 << (q + 1)) < free * 0.95:
            q += 1
    sv = torch.empty(1 << q, dtype=torch.float64, device=eng.device)
    gates = np.array([(0, 0, -1)] + [(1, t, 0) for t in range(1, q)], np.int32)  # GHZ register
    eng.statevector(q, gates[:1], out=sv)
    torch.cuda.synchronize()
    idx0, _ = eng.support(sv, q, cap=16)  # the register after H: |0...0> + |10...0>
    assert list(idx0) == [0, 1 << (q - 1)], idx0
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    eng.apply_gates(sv, q, gates[1:])
    b.record()
    torch.cuda.synchronize()
    t = a.elapsed_time(b) * 1e-3
    a2, b2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a2.record()
    eng.statevector(q, gates, out=sv)  # the whole register: init + H pass + fused CX pass
    b2.record()
    torch.cuda.synchronize()
    prep = a2.elapsed_time(b2) * 1e-3
    a2.record()
    eng.statevector_unfused(q, gates, out=sv)  # init pass + H pass + CX pass
    b2.record()
    torch.cuda.synchronize()
    prep_unfused = a2.elapsed_time(b2) * 1e-3
    idx, prob = eng.support(sv, q, cap=16)
    # the fused CX pass reads and writes the control = 1 half once: 8 B per amplitude of the state
    gbs = 8 * (1 << q) / t / 1e9
    ok = len(idx) == 2 and abs(prob[0] - 0.5) < 1e-12 and abs(prob[1] - 0.5) < 1e-12
    del sv
    torch.cuda.empty_cache()
    full = full_circuit_n7(eng)
    return _line(args, gbs, "GB/s (gate passes)",
                 f"BASELINE configs[4]: GHZ register of the Q resource, {q} qubits fp64 "
                 f"(n={q - 1} parties), {(8 << q) / 2 ** 30:.0f} GiB",
                 {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": gbs / HBM_PEAK_GBS, "traffic": None,
                  "algorithmic_bytes_per_amplitude_pass": 8,
                  "note": f"the {q - 1} CX gates share their control: one XOR-mask pass over the "
                          "control = 1 half (read + written once)"},
                 {"ms_per_step": t * 1e3,
                  "register_prep_ms": prep * 1e3, "register_prep_unfused_ms": prep_unfused * 1e3,
                  "register_prep_note": "prep = qba_sv_prepare: H folded into the init pass (write-only), "
                                        "then the CX pass; unfused = init pass + H pass + CX pass",
                  "cx_gates_fused_per_pass": q - 1,
                  "verification": {"support": [int(i) for i in idx], "probs": [float(p) for p in prob],
                                   "ghz_exact": bool(ok)},
                  "full_circuit_n7": full}, dtype="f64")


def full_circuit_n7(eng, n=7):
    """configs[4]'s other reading: the largest n whose WHOLE
    resource circuit fits as one dense state -- n = 7, 24 qubits, 128 MiB
    real fp64.  Both of tfg.py's circuits (tfg.py:15-22, 25-40; pi fixed)
    are prepared gate by gate on the device and their support is checked
    exactly against the closed form: not-Q = W^n equiprobable words with
    L0 = L1, Q = the W words {r ^ pi(g)} at 1/W each (qubit 0 = MSB)."""
    import numpy as np
    import torch
    res = importlib.import_module(f"{PKG}.resource")
    nq = res.n_qubits(n)
    N, W = (n + 1) * nq, 1 << nq
    perm = np.roll(np.arange(1, n + 1), 3)
    out = {"qubits": N, "n_parties": n, "state_MiB": (8 << N) >> 20}
    sv = torch.empty(1 << N, dtype=torch.float64, device=eng.device)
    for kind, gate in (("notq", res.notQCorrelated(n, nq)), ("q", res.qCorrelated(n, nq, perm=perm))):
        tri = gate.triples()
        eng.statevector(N, tri, out=sv)  # warm
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.statevector(N, tri, out=sv)
        b.record()
        torch.cuda.synchronize()
        idx, prob = eng.support(sv, N, cap=1 << 22)
        shift = [N - (g + 1) * nq for g in range(n + 1)]
        if kind == "notq":
            fields = np.stack([(idx >> s) & (W - 1) for s in shift])
            exact = (len(idx) == W ** n and bool((fields[0] == fields[1]).all())
                     and bool(np.all(np.abs(prob - float(W) ** -n) < 1e-12)))
        else:
            pi = np.concatenate([[0], perm])
            want = np.sort([sum(int(r ^ pi[g]) << shift[g] for g in range(n + 1)) for r in range(W)])
            exact = np.array_equal(np.sort(idx), want) and bool(np.all(np.abs(prob - 1.0 / W) < 1e-12))
        out[kind] = {"gates": int(len(tri)), "prep_ms": a.elapsed_time(b), "support": int(len(idx)),
                     "exact": bool(exact)}
    return out


def launch_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` with no WORLD_SIZE in the environment: start
    the N ranks ourselves, exactly as the driver's torchrun line would (one
    process per GPU, rendezvous on 127.0.0.1), and relay rank 0's JSON line.

    This process never touches the GPU (no torch import): the ranks are
    children started with subprocess, not an exec of this process.
    QBA_BENCH_WORKER names another script to launch in place of this one (the
    CPU test of the launcher); QBA_BENCH_LAUNCH_TIMEOUT bounds the whole run."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = os.environ.get("QBA_BENCH_WORKER") or str(Path(__file__).resolve())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", script, *argv]
    timeout = float(os.environ.get("QBA_BENCH_LAUNCH_TIMEOUT", "1500"))
    # stdout is relayed line by line (the driver reads the one JSON line),
    # stderr passes straight through
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, _ = proc.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        import signal
        os.killpg(proc.pid, signal.SIGKILL)  # the launcher's own process group only
        proc.communicate()
        print(f"bench.py: {n}-rank launch exceeded {timeout:.0f} s", file=sys.stderr)
        return 124
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    for ln in out.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if proc.returncode == 0 and len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    for ln in lines:
        print(ln, flush=True)
    return proc.returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.config != 2:
            raise SystemExit("--config 0/1/3/4 are single-GPU measurements")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    # After the GPU idles the headline's launches dip to ~450 us (the clock
    # drops to ~1.9 GHz at launches 6-12) and settle at ~316 us after ~100
    # launches (per-launch trace: profiles/r2/drift_fused_final.txt), so its
    # default window is 50 untimed + 200 timed launches (~0.1 s in total);
    # the driver's own --steps 20 --warmup 5 window is reported as given.
    # configs[1] and [3] run the same kernels, so they get the same window
    long_window = args.config in (1, 2, 3)
    if args.steps is None:
        args.steps = 200 if long_window else 20
    if args.warmup is None:
        args.warmup = 50 if long_window else 3
    if args.config == 2:
        headline(args)
        return
    if args.gpus != 1 or int(os.environ.get("WORLD_SIZE", "1")) != 1:
        raise SystemExit("--config 0/1/3/4 are single-GPU measurements")
    import torch
    torch.cuda.set_device(0)
    eng = importlib.import_module(f"{PKG}.engine").Engine(0)
    fn = {0: config0, 1: config1, 3: config3, 4: config4}[args.config]
    print(json.dumps(fn(args, eng)), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
