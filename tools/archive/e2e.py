#!/usr/bin/env python3
"""End-to-end record decrypt rate with the records starting and ending in
host memory ("records start and end in host socket buffers").

Pipeline, per chunk of C records (config c2 shape: TLS 1.3 AES-256-GCM,
16 KiB records, 128-B record slots):
    H2D stream:     pinned host ciphertext chunk -> device slot k
    compute stream: tlsrec_batch_decrypt on slot k (out of place)
    D2H stream:     device plaintext slot k -> pinned host output chunk
with NSLOT device slots in rotation and events between the streams, so the
two copy directions and the kernels overlap.  Prints one JSON line with the
end-to-end payload GiB/s plus the copy-only rates for context.

    python tools/e2e.py [--records N] [--chunk C] [--slots S]
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
    ap.add_argument("--records", type=int, default=1 << 18)
    ap.add_argument("--chunk", type=int, default=1 << 14)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import mbedtls_amd as M
    from tests.prng import prng_array

    dev = torch.device("cuda", 0)
    n, C = args.records, args.chunk
    assert n % C == 0
    content, inner, wire = 16383, 16384, 16400
    stride = (wire + 127) // 128 * 128
    km = np.zeros(1, dtype=M.KEY_MATERIAL)
    raw = prng_array(0x7115EC0DE, 48)
    km["cipher"] = M.CIPHER_AES_256_GCM
    km["tls_minor"] = 4
    km["fixed_ivlen"] = 12
    km["taglen"] = 16
    km["key"] = raw[:32]
    km["iv"][0, :12] = raw[32:44]
    kt = M.KeyTable(1)
    kt.load(km)

    # descriptors: chunk-relative buf_off (identical for every chunk), global seq
    def descs(seq0, count, data_len, dtype_type):
        d = M.records(count)
        d["buf_off"] = np.arange(count, dtype=np.uint64) * stride
        d["buf_len"] = stride
        d["data_offset"] = 0
        d["data_len"] = data_len
        d["slot"] = 0
        d["ctr"] = M.seq_bytes(np.arange(seq0, seq0 + count, dtype=np.uint64))
        d["type"] = dtype_type
        d["ver"] = (3, 3)
        return d

    enc_desc = torch.from_numpy(descs(0, n, content, 23).view(np.uint8).copy()).to(dev)
    dec_desc = torch.from_numpy(descs(0, n, wire, 23).view(np.uint8).copy()).to(dev)
    # the chunk-relative offsets need per-chunk descriptor slices (same layout)
    dec_chunks = []
    for c in range(n // C):
        d = descs(c * C, C, wire, 23)
        dec_chunks.append(torch.from_numpy(d.view(np.uint8).copy()).to(dev))
    res = torch.zeros(C * 16, dtype=torch.uint8, device=dev)

    # ---- host "socket buffers": ciphertexts made on the GPU (verified encrypt path)
    host_in = torch.empty(n * stride, dtype=torch.uint8).pin_memory()
    host_out = torch.empty(n * stride, dtype=torch.uint8).pin_memory()
    plain_sample = {}
    for c in range(n // C):
        a = torch.randint(0, 256, (C * stride,), dtype=torch.uint8, device=dev)
        for i in (0, C - 1):
            plain_sample[c * C + i] = a[i * stride:i * stride + content].cpu().numpy().copy()
        d = descs(c * C, C, content, 23)
        dd = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        M.batch_encrypt(kt, dd, res, C, a, a)
        host_in[c * C * stride:(c + 1) * C * stride].copy_(a)
    torch.cuda.synchronize()
    del enc_desc, dec_desc

    slots_in = [torch.empty(C * stride, dtype=torch.uint8, device=dev) for _ in range(args.slots)]
    slots_out = [torch.empty(C * stride, dtype=torch.uint8, device=dev) for _ in range(args.slots)]
    s_h2d, s_cmp, s_d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()

    def run_pipeline():
        h2d_done = [torch.cuda.Event() for _ in range(n // C)]
        cmp_done = [torch.cuda.Event() for _ in range(n // C)]
        d2h_done = [torch.cuda.Event() for _ in range(n // C)]
        for c in range(n // C):
            k = c % args.slots
            lo, hi = c * C * stride, (c + 1) * C * stride
            with torch.cuda.stream(s_h2d):
                if c >= args.slots:
                    s_h2d.wait_event(cmp_done[c - args.slots])   # slot's previous kernel has read it
                slots_in[k].copy_(host_in[lo:hi], non_blocking=True)
                h2d_done[c].record(s_h2d)
            with torch.cuda.stream(s_cmp):
                s_cmp.wait_event(h2d_done[c])
                if c >= args.slots:
                    s_cmp.wait_event(d2h_done[c - args.slots])   # slot's previous output drained
                M.batch_decrypt(kt, dec_chunks[c], res, C, slots_in[k], slots_out[k], stream=s_cmp)
                cmp_done[c].record(s_cmp)
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(cmp_done[c])
                host_out[lo:hi].copy_(slots_out[k], non_blocking=True)
                d2h_done[c].record(s_d2h)
        torch.cuda.synchronize()

    run_pipeline()   # warm-up
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        run_pipeline()
        times.append(time.perf_counter() - t0)
    t = min(times)

    ok = True
    for i, pt in plain_sample.items():
        got = host_out[i * stride:i * stride + content].numpy()
        ok &= bool(np.array_equal(got, pt))

    # copy-only and kernel-only rates over the same bytes
    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def h2d_only():
        for c in range(n // C):
            slots_in[c % args.slots].copy_(host_in[c * C * stride:(c + 1) * C * stride], non_blocking=True)

    def d2h_only():
        for c in range(n // C):
            host_out[c * C * stride:(c + 1) * C * stride].copy_(slots_out[c % args.slots], non_blocking=True)

    def kern_only():
        for c in range(n // C):
            M.batch_decrypt(kt, dec_chunks[c], res, C, slots_in[c % args.slots], slots_out[c % args.slots])

    th, td, tk = min(timed(h2d_only) for _ in range(2)), min(timed(d2h_only) for _ in range(2)), \
        min(timed(kern_only) for _ in range(2))
    gib = n * inner / 2**30
    out = {"what": "end-to-end TLS 1.3 AES-256-GCM decrypt, pinned host in -> device -> pinned host out",
           "records": n, "chunk_records": C, "device_slots": args.slots, "record_slot_bytes": stride,
           "payload_GiB_per_s": round(gib / t, 2), "records_per_s": round(n / t, 1),
           "h2d_only_GB_per_s": round(n * stride / th / 1e9, 2),
           "d2h_only_GB_per_s": round(n * stride / td / 1e9, 2),
           "kernels_only_payload_GiB_per_s": round(gib / tk, 2),
           "plaintext_spot_check_ok": ok}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
