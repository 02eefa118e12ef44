#!/usr/bin/env python3
"""Where the GPU pays off at the reference's call sites.

The reference protects one record per call (ssl_msg.c:2697 send, :3835
receive) on the CPU.  This measures, on one box, records per second of:

* cpu_evp   -- the ssl_msg.c framing around OpenSSL 3 EVP (oracle/evp_bench.c,
               the CPU baseline leg of bench.py) on the box's CPU share, a
               steady stream of records (the CPU needs no batching);
* gpu_host  -- tlsrec_host_batch_encrypt: a batch of n records in pinned host
               memory (socket buffers) -> device -> host, one synchronous call,
               for n = 1 .. 256 K (what a terminator gets per event-loop turn);
* gpu_dev   -- tlsrec_batch_encrypt on device-resident records, launch + sync
               per batch.

and prints one JSON line per (record size, n) plus a summary line with the
smallest n at which each GPU form beats the CPU leg.

    python tools/bench_crossover.py [--sizes 1400,16383] [--max-n 262144]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1400,16383")
    ap.add_argument("--max-n", type=int, default=1 << 18)
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    a = ap.parse_args()
    import torch
    import mbedtls_amd as M
    import oracle as O
    import bench
    dev = torch.device("cuda")
    threads, how = bench.host_cores()
    key, iv = bytes(range(32)), bytes(range(100, 112))
    km = M.key_material(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, key, iv)
    kt = M.KeyTable(1)
    kt.load(km)
    summary = {}
    for content in [int(x) for x in a.sizes.split(",")]:
        inner = content + 1 + (16 - (content + 1) % 16) % 16
        wire = inner + 16
        stride = (wire + 127) // 128 * 128
        # ---- CPU: steady-state EVP rate on the box's CPU share -------------
        n_cpu = max(1024, int(2e9 // stride) // 8)
        arena = np.zeros(n_cpu * stride, dtype=np.uint8)
        st = np.zeros(n_cpu, dtype=np.int32)
        el, reps = 0.0, 0
        while el < a.cpu_seconds:
            el += O.evp_bench(O.AES_256_GCM, O.TLS1_3, key, iv, 1, arena, stride, content, n_cpu, 0, threads, st)
            reps += 1
        assert (st == 0).all()
        cpu_rps = n_cpu * reps / el
        del arena
        print(json.dumps({"content": content, "leg": "cpu_evp", "threads": threads, "records_per_s": round(cpu_rps),
                          "GiBps": round(cpu_rps * inner / 2**30, 2), "cores_how": how}), flush=True)
        # ---- GPU: batches of n --------------------------------------------
        N = a.max_n
        span = N * stride
        h_in = torch.empty(span, dtype=torch.uint8).pin_memory()
        h_out = torch.empty(span, dtype=torch.uint8).pin_memory()
        h_in.copy_(torch.randint(0, 256, (span,), dtype=torch.uint8))
        d_in = h_in.to(dev)
        d_out = torch.empty_like(d_in)
        recs = M.records(N)
        recs["buf_off"] = np.arange(N, dtype=np.uint64) * stride
        recs["buf_len"] = stride
        recs["data_len"] = content
        recs["ctr"] = M.seq_bytes(np.arange(N, dtype=np.uint64))
        recs["type"] = 23
        recs["ver"] = (3, 3)
        res = M.results(N)
        d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(N * 16, dtype=torch.uint8, device=dev)
        best = {"gpu_host": None, "gpu_dev": None}
        n = 1
        while n <= N:
            reps = max(3, min(200, int(2e8 // (n * stride))))
            M.host_batch(False, kt, recs, res, n, h_in, h_out)         # warm-up
            t0 = time.perf_counter()
            for _ in range(reps):
                M.host_batch(False, kt, recs, res, n, h_in, h_out)
            host_s = (time.perf_counter() - t0) / reps
            assert (res["status"][:n] == 0).all()
            M.batch_encrypt(kt, d_recs, d_res, n, d_in, d_out, mean_bytes=wire)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                M.batch_encrypt(kt, d_recs, d_res, n, d_in, d_out, mean_bytes=wire)
                torch.cuda.synchronize()
            dev_s = (time.perf_counter() - t0) / reps
            row = {"content": content, "n": n, "gpu_host_us": round(host_s * 1e6, 1),
                   "gpu_host_records_per_s": round(n / host_s), "gpu_dev_us": round(dev_s * 1e6, 1),
                   "gpu_dev_records_per_s": round(n / dev_s), "cpu_evp_records_per_s": round(cpu_rps),
                   "gpu_host_vs_cpu": round(n / host_s / cpu_rps, 3), "gpu_dev_vs_cpu": round(n / dev_s / cpu_rps, 3)}
            print(json.dumps(row), flush=True)
            for leg, rps in (("gpu_host", n / host_s), ("gpu_dev", n / dev_s)):
                if best[leg] is None and rps > cpu_rps:
                    best[leg] = n
            n *= 4
        summary[content] = {"cpu_evp_records_per_s": round(cpu_rps), "cpu_threads": threads,
                            "crossover_n_host_batch": best["gpu_host"], "crossover_n_device_batch": best["gpu_dev"]}
        del h_in, h_out, d_in, d_out
    print(json.dumps({"summary": summary}), flush=True)
    kt.close()


if __name__ == "__main__":
    main()
