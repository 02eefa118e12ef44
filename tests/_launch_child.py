"""A rank of tests/test_bench_launcher.py: joins the gloo group bench.py's
launcher set up through the environment, checks the world size it was told,
and rank 0 prints one JSON line (as bench.py's rank 0 does).

With a third argument "line" the rank also runs bench.py's post-timing path
as the GPU ranks do: rank_timing (max wall, every rank's
kernel time all-gathered), per_rank_roofline, and rank0_legs with bench.py's
real cpu_baseline (a short sample of the c1 shape) on rank 0 while the other
ranks wait -- and rank 0 puts those fields on its line."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    want = int(sys.argv[1])
    fail_rank = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    line = len(sys.argv) > 3 and sys.argv[3] == "line"
    rank = int(os.environ["RANK"])
    if rank == fail_rank:
        sys.exit(3)
    dist.init_process_group("gloo", init_method="env://")
    assert dist.get_world_size() == want == int(os.environ["WORLD_SIZE"])
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    ranks = [None] * want
    dist.all_gather_object(ranks, {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]), "pid": os.getpid()})
    out = {"world_size": dist.get_world_size(), "sum": int(t.item()), "ranks": ranks}
    if line:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import numpy as np
        import bench
        import mbedtls_amd as M
        # a rank-dependent fake step: rank r's kernels take 10 + r ms
        wall, kern = bench.rank_timing(dist, 0.1 * (rank + 1), [10.0 + rank] * 3, "cpu")
        pr = bench.per_rank_roofline(kern, 32793 * (1 << 20))
        km = np.zeros(1, dtype=M.KEY_MATERIAL)
        km["cipher"] = M.CIPHER_AES_128_GCM
        km["key"][0, :16] = np.arange(16, dtype=np.uint8)
        ran = []

        def cpu():
            ran.append(time.time())
            return bench.cpu_baseline("AES-128-GCM", M.VERSION_TLS1_2, 1400, 1400, 1424, 1536, km, 0.05, "encrypt")
        cpu_line, e2e = bench.rank0_legs(dist, rank, cpu, lambda: {"value": 1.0, "what": "stub"})
        left = torch.tensor([time.time()], dtype=torch.float64)
        allleft = [torch.empty_like(left) for _ in range(want)]
        dist.all_gather(allleft, left)
        out.update(wall=wall, kernel_ms=kern, roofline=pr, cpu_baseline=cpu_line, e2e=e2e,
                   cpu_ran_on_this_rank=bool(ran), cpu_started=ran[0] if ran else None,
                   left_barrier=[float(x.item()) for x in allleft])
        if rank != 0:
            assert not ran and cpu_line is None and e2e is None
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
