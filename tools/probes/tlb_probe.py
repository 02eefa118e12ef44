#!/usr/bin/env python3
"""Does the arena's allocation change the c4s GCM kernel's L1 TLB misses?

c4s (64 K keys x 64 records x 1 400 B, AES-256-GCM / ChaCha20-Poly1305
alternating per key, round-robin) with its two record arenas allocated by
hipMalloc (what torch does) or hipExtMallocWithFlags(hipDeviceMallocContiguous),
physically contiguous memory the driver can map with large fragments.  Prints
one JSON line per allocation: decrypt GiB/s over --steps steps.

    python tools/probes/tlb_probe.py [--alloc default|contiguous] [--steps 10]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alloc", choices=["default", "contiguous"], default="default")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    import mbedtls_amd as M
    from tests.prng import prng_array
    hip = ctypes.CDLL("libamdhip64.so")
    nkeys, rpk, content, wire, inner, stride = 1 << 16, 64, 1400, 1424, 1408, 1536
    n = nkeys * rpk
    size = n * stride

    def alloc():
        p = ctypes.c_void_p()
        flags = 0x4 if a.alloc == "contiguous" else 0x0
        r = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(size), ctypes.c_uint(flags))
        if r != 0:
            raise RuntimeError(f"hipExtMallocWithFlags({a.alloc}) failed: {r}")
        return p.value
    A, B = alloc(), alloc()
    # fill A with random bytes from a device tensor, in chunks
    chunk = 1 << 30
    for off in range(0, size, chunk):
        c = min(chunk, size - off)
        t = torch.randint(0, 256, (c,), dtype=torch.uint8, device="cuda")
        hip.hipMemcpy(ctypes.c_void_p(A + off), ctypes.c_void_p(t.data_ptr()), ctypes.c_size_t(c), 3)
        del t
    raw = prng_array(0x7115EC0DE, nkeys * 48).reshape(nkeys, 48)
    km = np.zeros(nkeys, dtype=M.KEY_MATERIAL)
    km["cipher"] = np.where(np.arange(nkeys) % 2 == 0, M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305)
    km["tls_minor"], km["fixed_ivlen"], km["taglen"] = 4, 12, 16
    km["key"] = raw[:, :32]
    km["iv"][:, :12] = raw[:, 32:44]
    kt = M.KeyTable(nkeys)
    kt.load(km)
    d = M.records(n)
    d["buf_off"] = np.arange(n, dtype=np.uint64) * stride
    d["buf_len"] = stride
    d["data_len"] = content
    d["slot"] = (np.arange(n) % nkeys).astype(np.uint32)
    d["ctr"] = M.seq_bytes(np.arange(n, dtype=np.uint64))
    d["type"] = 23
    d["ver"] = (3, 3)
    res = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    M.batch_encrypt(kt, torch.from_numpy(d.view(np.uint8).copy()).cuda(), res, n, A, A, mean_bytes=wire)
    torch.cuda.synchronize()
    assert int((res.view(torch.int32)[0::4] != 0).sum()) == 0
    dd = d.copy()
    dd["data_len"] = wire
    drecs = torch.from_numpy(dd.view(np.uint8).copy()).cuda()
    for _ in range(2):
        M.batch_decrypt(kt, drecs, res, n, A, B, mean_bytes=wire)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        M.batch_decrypt(kt, drecs, res, n, A, B, mean_bytes=wire)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    ok = int((res.view(torch.int32)[0::4] != 0).sum()) == 0
    print(json.dumps({"alloc": a.alloc, "GiBps": round(n * inner / el / 2**30, 2), "ms_per_step": round(el * 1e3, 3),
                      "all_ok": ok}), flush=True)
    kt.close()
    hip.hipFree(ctypes.c_void_p(A))
    hip.hipFree(ctypes.c_void_p(B))


if __name__ == "__main__":
    main()
