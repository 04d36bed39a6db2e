"""Stand-in for one bench.py rank in the CPU test of bench.py's self-launch
(QBA_BENCH_WORKER): joins the torch.distributed world the launcher started
(gloo), does bench.py's barrier / max-over-ranks timing, and rank 0 prints
one JSON line naming the world it saw and the arguments it was given."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dist.barrier()
    t0 = time.perf_counter()
    x = torch.ones(4, dtype=torch.int64)
    dist.all_reduce(x)
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "stub", "n_gpus": world, "sum": int(x[0]),
                          "local_ranks_seen": world, "argv": sys.argv[1:], "t_max": float(t)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
