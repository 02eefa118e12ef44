#!/usr/bin/env python3
"""Probe the host-buffer pipeline (tlsrec_host_batch_decrypt): rate vs chunk
size, against device-only kernels on chunk-sized batches and bare copies."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mbedtls_amd as M
    dev = torch.device("cuda", 0)
    content, inner, wire = 16383, 16384, 16400
    stride = 16512
    E = int(sys.argv[1]) if len(sys.argv) > 1 else 130048
    km = np.zeros(1, dtype=M.KEY_MATERIAL)
    km["cipher"] = M.CIPHER_AES_256_GCM
    km["tls_minor"] = 4
    km["fixed_ivlen"] = 12
    km["taglen"] = 16
    km["key"] = 7
    km["iv"][0, :12] = 9
    kt = M.KeyTable(1)
    kt.load(km)
    d = M.records(E)
    d["buf_off"] = np.arange(E, dtype=np.uint64) * stride
    d["buf_len"] = stride
    d["data_len"] = content
    d["ctr"] = M.seq_bytes(np.arange(E, dtype=np.uint64))
    d["type"] = 23
    d["ver"] = (3, 3)
    a = torch.randint(0, 256, (E * stride,), dtype=torch.uint8, device=dev)
    dd = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    res = torch.zeros(E * 16, dtype=torch.uint8, device=dev)
    M.batch_encrypt(kt, dd, res, E, a, a)
    torch.cuda.synchronize()
    host_in = torch.empty(E * stride, dtype=torch.uint8).pin_memory()
    host_out = torch.empty(E * stride, dtype=torch.uint8).pin_memory()
    host_in.copy_(a)
    d["data_len"] = wire
    hres = M.results(E)
    out = {}
    for chunk_mb in (16, 64, 256, 1024):
        M.host_batch(True, kt, d, hres, E, host_in, host_out, chunk_bytes=chunk_mb << 20)
        t0 = time.perf_counter()
        M.host_batch(True, kt, d, hres, E, host_in, host_out, chunk_bytes=chunk_mb << 20)
        el = time.perf_counter() - t0
        ok = bool((hres["status"] == 0).all())
        out[f"pipe_{chunk_mb}MiB_GiBps"] = round(E * inner / el / 2**30, 2)
        out[f"pipe_{chunk_mb}MiB_ok"] = ok
    # kernel-only on chunk-sized device batches
    dd2 = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    outd = torch.empty_like(a)
    for chunk_mb in (16, 64, 256):
        c = (chunk_mb << 20) // stride
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for lo in range(0, E - c + 1, c):
            M.batch_decrypt(kt, dd2[lo * 40:(lo + c) * 40], res, c, a, outd)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[f"kern_{chunk_mb}MiB_GiBps"] = round((E // c) * c * inner / el / 2**30, 2)
    # raw pinned copies
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a.copy_(host_in, non_blocking=True)
    torch.cuda.synchronize()
    out["h2d_GBps"] = round(E * stride / (time.perf_counter() - t0) / 1e9, 2)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    half = (E // 2) * stride
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        a[:half].copy_(host_in[:half], non_blocking=True)
    with torch.cuda.stream(s2):
        host_out[half:2 * half].copy_(outd[half:2 * half], non_blocking=True)
    torch.cuda.synchronize()
    out["bidir_each_GBps"] = round(half / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
