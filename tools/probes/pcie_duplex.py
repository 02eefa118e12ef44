"""PCIe ceiling for the host-buffer pipeline: pinned H2D alone,
D2H alone, both at once on two streams (copy engines), and H2D beside a
kernel that writes its output straight into pinned host memory (the
pipeline's D2H direction).  Prints one JSON line."""
import json
import time

import torch

N = 1 << 31
dev = torch.device("cuda")
h_in = torch.empty(N, dtype=torch.uint8).pin_memory()
h_out = torch.empty(N, dtype=torch.uint8).pin_memory()
d_a = torch.empty(N, dtype=torch.uint8, device=dev)
d_b = torch.randint(0, 255, (N,), dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=3):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return best


def h2d():
    d_a.copy_(h_in, non_blocking=True)


def d2h():
    h_out.copy_(d_b, non_blocking=True)


def both():
    with torch.cuda.stream(s1):
        d_a.copy_(h_in, non_blocking=True)
    with torch.cuda.stream(s2):
        h_out.copy_(d_b, non_blocking=True)


out = {"bytes": N, "h2d_GBps": N / timed(h2d) / 1e9, "d2h_GBps": N / timed(d2h) / 1e9}
t = timed(both)
out["duplex_each_GBps"] = N / t / 1e9
out["duplex_total_GBps"] = 2 * N / t / 1e9
print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)
