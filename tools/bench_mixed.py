#!/usr/bin/env python3
"""Batch throughput with single-record calls alongside.

The record server (server.hip) holds 64 CUs while it lives.  This runs the c2
batch (AES-256-GCM decrypt, TLS 1.3, 16 KiB records, one key; --records of
them per step) alone, then with T threads issuing single-record
tlsrec_encrypt_buf / _decrypt_buf calls (1 400-B AES-256-GCM records on their
own connection) as fast as they can, and prints one JSON line:

  batch GiB/s solo and mixed, the single-record round trips per second and
  their p50 / p99 latency during the batch and alone, how many the record
  server served, and the hipDeviceSynchronize latency right after a
  single-record call (the server grid's remaining life).

    TLSREC_SERVER_YIELD=0 TLSREC_SERVER_IDLE_MS=20 python tools/bench_mixed.py   # r03 behaviour
    python tools/bench_mixed.py                                                 # r04: yield + idle exit
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    import torch
    import mbedtls_amd as M
    from mbedtls_amd import _abi
    from tests.prng import prng_bytes
    dev = torch.device("cuda")
    n, content, inner, wire, stride = a.records, 16383, 16384, 16400, 16512
    key, iv = prng_bytes(1, 32), prng_bytes(2, 16)
    km = M.key_material(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, key, iv)
    kt = M.KeyTable(1)
    kt.load(km)
    d = M.records(n)
    d["buf_off"] = np.arange(n, dtype=np.uint64) * stride
    d["buf_len"] = stride
    d["data_len"] = content
    d["ctr"] = M.seq_bytes(np.arange(n, dtype=np.uint64))
    d["type"] = 23
    d["ver"] = (3, 3)
    A = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev)
    B = torch.empty_like(A)
    res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    M.batch_encrypt(kt, torch.from_numpy(d.view(np.uint8).copy()).to(dev), res, n, A, B)
    dd = d.copy()
    dd["data_len"] = wire
    drecs = torch.from_numpy(dd.view(np.uint8).copy()).to(dev)
    C = torch.empty_like(A)
    torch.cuda.synchronize()

    def steps(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            M.batch_decrypt(kt, drecs, res, n, B, C)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        assert int((res.view(torch.int32)[0::4] != 0).sum()) == 0
        return n * inner * k / el / 2**30

    L = _abi.load()
    stats = L.tlsrec__server_stats
    stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3

    def served():
        s, f, ln = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        stats(ctypes.byref(s), ctypes.byref(f), ctypes.byref(ln))
        return s.value, f.value, ln.value

    steps(2)
    solo = steps(a.steps)

    stop = threading.Event()
    lat = [[] for _ in range(a.threads)]
    errs = []

    def single(k):
        kk, ii = prng_bytes(10 + k, 32), prng_bytes(20 + k, 16)
        t = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_256_GCM, kk, kk, ii, ii)
        pt = prng_bytes(30 + k, 1400)
        i = 0
        try:
            while not stop.is_set():
                rec = M.Record(ctr=i.to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=bytearray(pt) + bytearray(64),
                               data_offset=0, data_len=1400)
                t0 = time.perf_counter()
                r1 = t.encrypt_buf(rec)
                r2 = t.decrypt_buf(rec)
                lat[k].append(time.perf_counter() - t0)
                if r1 or r2 or rec.data() != pt:
                    errs.append((k, i, r1, r2))
                    return
                i += 1
        finally:
            t.close()

    def single_phase(run_batch):
        for x in lat:
            x.clear()
        s0 = served()
        th = [threading.Thread(target=single, args=(k,)) for k in range(a.threads)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        time.sleep(0.05)
        rate = steps(a.steps) if run_batch else (time.sleep(0.5) or None)
        stop.set()
        for x in th:
            x.join()
        el = time.perf_counter() - t0
        stop.clear()
        s1 = served()
        all_l = np.array([v for x in lat for v in x]) * 1e6
        return rate, {"round_trips_per_s": round(len(all_l) / el, 1),
                      "p50_us": round(float(np.percentile(all_l, 50)), 1) if len(all_l) else None,
                      "p99_us": round(float(np.percentile(all_l, 99)), 1) if len(all_l) else None,
                      "served": s1[0] - s0[0], "fallback": s1[1] - s0[1], "grid_launches": s1[2] - s0[2]}

    mixed, single_during = single_phase(True)
    _, single_alone = single_phase(False)
    # hipDeviceSynchronize right after a single-record call
    t = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_256_GCM, key, key, iv, iv)
    syncs = []
    for i in range(20):
        rec = M.Record(ctr=(1000 + i).to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=bytearray(1464),
                       data_offset=0, data_len=1400)
        assert t.encrypt_buf(rec) == 0
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        syncs.append((time.perf_counter() - t0) * 1e3)
        time.sleep(0.03)
    t.close()
    yields = L.tlsrec__server_yields
    yields.restype = ctypes.c_uint64
    out = {"label": a.label, "env": {k: os.environ[k] for k in os.environ if k.startswith("TLSREC_SERVER")},
           "batch": f"c2 shape: {n} x 16 KiB AES-256-GCM TLS 1.3 decrypt per step, {a.steps} steps",
           "batch_GiBps_solo": round(solo, 1), "batch_GiBps_mixed": round(mixed, 1),
           "batch_mixed_vs_solo": round(mixed / solo, 4), "single_threads": a.threads,
           "single_during_batch": single_during, "single_alone": single_alone,
           "device_sync_after_single_ms": {"p50": round(float(np.median(syncs)), 3), "max": round(max(syncs), 3)},
           "server_yields": int(yields()), "errors": errs[:3]}
    print(json.dumps(out), flush=True)
    kt.close()


if __name__ == "__main__":
    main()
