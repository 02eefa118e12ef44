#!/usr/bin/env python3
"""Can the record kernels write their output straight into pinned host
memory (zero-copy D2H over PCIe) at link rate?  Device batch decrypt with the
output arena = a pinned host tensor, vs device output + SDMA copy."""
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
    content, inner, wire, stride = 16383, 16384, 16400, 16512
    E = 16256
    km = np.zeros(1, dtype=M.KEY_MATERIAL)
    km["cipher"] = M.CIPHER_AES_256_GCM
    km["tls_minor"] = 4
    km["fixed_ivlen"] = 12
    km["taglen"] = 16
    km["key"] = 7
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
    plain = a.clone()
    dd = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    res = torch.zeros(E * 16, dtype=torch.uint8, device=dev)
    M.batch_encrypt(kt, dd, res, E, a, a)
    d["data_len"] = wire
    dd = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    host_out = torch.zeros(E * stride, dtype=torch.uint8).pin_memory()
    out = {}
    for lanes in (8, 16, 64):
        for tgt in ("device", "host"):
            o = torch.empty_like(a) if tgt == "device" else host_out
            M.batch_decrypt(kt, dd, res, E, a, o, lanes=lanes)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                M.batch_decrypt(kt, dd, res, E, a, o, lanes=lanes)
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / 3
            ok = int((res.view(torch.int32)[0::4] != 0).sum()) == 0
            if tgt == "host":
                ok &= bool(torch.equal(host_out.view(E, stride)[:64, :content], plain.view(E, stride)[:64, :content].cpu()))
            out[f"L{lanes}_{tgt}_GiBps"] = round(E * inner / el / 2**30, 2)
            out[f"L{lanes}_{tgt}_ok"] = ok
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
