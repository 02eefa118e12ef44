#!/usr/bin/env python3
"""Throughput of the stream record layer (tlsrec_stream_decrypt /
tlsrec_stream_encrypt): C connections x R records of `content` bytes of
application data each, TLS 1.3, one key per connection.  The receive side
gets the record streams the send side produced (checked against the oracle
on a sample of connections).  Prints one JSON line per direction.

    python tools/bench_stream.py [--conns 65536] [--recs 16] [--content 16384] [--cipher 2]
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
    ap.add_argument("--conns", type=int, default=65536)
    ap.add_argument("--recs", type=int, default=16)
    ap.add_argument("--content", type=int, default=16384)
    ap.add_argument("--cipher", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall-time target of each CPU leg's sample")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    from tools import rowlib
    import torch
    import mbedtls_amd as M
    from mbedtls_amd import stream as S
    from tests.prng import prng_array
    dev = torch.device("cuda")
    C, R, L = a.conns, a.recs, a.content
    nkeys = C
    km = np.zeros(nkeys, dtype=M.KEY_MATERIAL)
    raw = prng_array(0x57AE, nkeys * 48).reshape(nkeys, 48)
    km["cipher"], km["tls_minor"], km["fixed_ivlen"], km["taglen"] = a.cipher, 4, 12, 16
    km["key"] = raw[:, :32]
    km["iv"][:, :12] = raw[:, 32:44]
    kt = M.KeyTable(nkeys)
    kt.load(km)
    per_in = R * L
    per_out = S.out_size(M.VERSION_TLS1_3, a.cipher, 16, per_in, L)
    stride_in = (per_in + 127) // 128 * 128
    stride_out = (per_out + 127) // 128 * 128
    tin = torch.randint(0, 256, (C * stride_in,), dtype=torch.uint8, device=dev)
    tout = torch.zeros(C * stride_out, dtype=torch.uint8, device=dev)
    d = np.zeros(C, dtype=S.STREAM_OUT)
    d["in_off"] = np.arange(C, dtype=np.uint64) * stride_in
    d["in_len"] = per_in
    d["slot"] = np.arange(C) % nkeys
    d["out_off"] = np.arange(C, dtype=np.uint64) * stride_out
    d["type"] = 23
    d["max_frag"] = L
    dout = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    n = C * R
    recs = torch.zeros(n * 40, dtype=torch.uint8, device=dev)
    res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    sres = torch.zeros(C * 32, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    t_enc = timed(lambda: S.encrypt(kt, dout, C, tin, tout, recs, res, n, sres))
    ms_enc, _ = rowlib.event_timed(lambda: S.encrypt(kt, dout, C, tin, tout, recs, res, n, sres), a.steps)
    so = sres.cpu().numpy().view(S.STREAM_OUT_RES)
    assert (so["status"] == 0).all() and (so["out_len"] == per_out).all()
    # oracle check of a few connections' record streams
    import oracle as O
    ok = True
    for i in (0, C // 2, C - 1):
        k = km[i]
        t = O.Transform(O.TLS1_3, {1: O.AES_128_GCM, 2: O.AES_256_GCM, 3: O.CHACHA20_POLY1305}[a.cipher],
                        bytes(k["key"][:16 if a.cipher == 1 else 32]), bytes(k["key"][:16 if a.cipher == 1 else 32]),
                        bytes(k["iv"]), bytes(k["iv"]))
        pt = tin[i * stride_in:i * stride_in + per_in].cpu().numpy().tobytes()
        r, want, _, _ = O.stream_encrypt(t, pt, 23, bytes(8), L)
        ok &= r == 0 and tout[i * stride_out:i * stride_out + per_out].cpu().numpy().tobytes() == want
    # receive side: decrypt the produced streams in place (fresh copy each step)
    di = np.zeros(C, dtype=S.STREAM_IN)
    di["off"] = np.arange(C, dtype=np.uint64) * stride_out
    di["len"] = per_out
    di["slot"] = np.arange(C) % nkeys
    din = torch.from_numpy(di.view(np.uint8).copy()).to(dev)
    work = torch.empty_like(tout)
    work.copy_(tout)
    S.decrypt(kt, din, C, work, recs, res, n, sres)
    torch.cuda.synchronize()
    si = sres.cpu().numpy().view(S.STREAM_IN_RES)
    assert (si["status"] == 0).all() and (si["nrec"] == R).all()
    # time: decrypt of already-decrypted bytes would fail the tag, so time on copies
    times = []
    for _ in range(a.steps):
        work.copy_(tout)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        S.decrypt(kt, din, C, work, recs, res, n, sres)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t_dec = float(np.mean(times))
    ms_dec, _ = rowlib.event_timed(lambda: S.decrypt(kt, din, C, work, recs, res, n, sres), a.steps,
                                   prep=lambda: work.copy_(tout))
    si = sres.cpu().numpy().view(S.STREAM_IN_RES)
    assert (si["status"] == 0).all()
    payload = float(C) * per_in
    # SURVEY 8(d)'s rule with the 5-B headers: send reads the application data
    # and writes the records (headers, ciphertext, tags); receive reads the
    # records and writes each record's inner plaintext (content + type byte)
    # and a 4-B status
    inner = L + 1
    alg = {"stream_encrypt": C * (per_in + per_out), "stream_decrypt": C * (per_out + R * (inner + 4))}
    rules = {"stream_encrypt": "application data read + records (5-B headers, ciphertext, tags) written",
             "stream_decrypt": "records (5-B headers, ciphertext, tags) read + inner plaintext and a 4-B status "
                               "per record written"}
    kernels = {"stream_encrypt": "stream frame + tlsrec_gcm_kernel / tlsrec_chachapoly_kernel",
               "stream_decrypt": "stream header walk / descriptors + AEAD kernel + in-order finish"}
    for name, t, ms in (("stream_encrypt", t_enc, ms_enc), ("stream_decrypt", t_dec, ms_dec)):
        cpu = None if a.no_cpu else rowlib.cpu_stream_legs(False, a.cipher, L, R,
                                                           "send" if name == "stream_encrypt" else "receive",
                                                           a.cpu_seconds)
        print(json.dumps({"metric": f"TLS record-stream {name} throughput (device-resident, framing included)",
                          "value": round(payload / t / 2**30, 3), "unit": "GiB/s",
                          "records_per_s": round(n / t), "ms_per_call": round(t * 1e3, 3),
                          "config": {"connections": C, "records_per_connection": R, "content_bytes": L,
                                     "cipher": a.cipher, "tls": "1.3"},
                          "roofline": rowlib.roofline(alg[name], ms, rules[name], kernels[name]),
                          "cpu_baseline": cpu,
                          "check": {"oracle_sample_ok": bool(ok)}}), flush=True)


if __name__ == "__main__":
    main()
