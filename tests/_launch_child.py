"""A rank of tests/test_bench_launcher.py: joins the gloo group bench.py's
launcher set up through the environment, checks the world size it was told,
and rank 0 prints one JSON line (as bench.py's rank 0 does)."""
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    want = int(sys.argv[1])
    fail_rank = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    rank = int(os.environ["RANK"])
    if rank == fail_rank:
        sys.exit(3)
    dist.init_process_group("gloo", init_method="env://")
    assert dist.get_world_size() == want == int(os.environ["WORLD_SIZE"])
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    ranks = [None] * want
    dist.all_gather_object(ranks, {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]), "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"world_size": dist.get_world_size(), "sum": int(t.item()), "ranks": ranks}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
