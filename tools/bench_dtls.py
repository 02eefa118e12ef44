#!/usr/bin/env python3
"""Throughput of the DTLS 1.2 datagram record layer (tlsrec_dtls_encrypt /
tlsrec_dtls_decrypt): C connections x R datagrams (one record of `content`
bytes each), TLS 1.2 keys, one key per connection, anti-replay on.  The
receive side gets the datagrams the send side produced (checked against the
oracle on a sample of connections).  Prints one JSON line per direction.

    python tools/bench_dtls.py [--conns 65536] [--recs 16] [--content 1400] [--cipher 1]
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
    ap.add_argument("--content", type=int, default=1400)
    ap.add_argument("--cipher", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall-time target of each CPU leg's sample")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    from tools import rowlib
    import torch
    import mbedtls_amd as M
    from mbedtls_amd import dtls as D
    from mbedtls_amd import stream as S
    from tests.prng import prng_array
    dev = torch.device("cuda")
    C, R, L = a.conns, a.recs, a.content
    kl = M.KEYLEN[a.cipher]
    km = np.zeros(C, dtype=M.KEY_MATERIAL)
    raw = prng_array(0xD715, C * 48).reshape(C, 48)
    km["cipher"], km["tls_minor"], km["taglen"] = a.cipher, 3, M.TAGLEN[a.cipher]
    km["fixed_ivlen"] = 12 if a.cipher == M.CIPHER_CHACHA20_POLY1305 else 4
    km["key"][:, :kl] = raw[:, :kl]
    km["iv"][:, :12] = raw[:, 32:44]
    kt = M.KeyTable(C)
    kt.load(km)
    per_in = R * L
    per_out = D.out_size(a.cipher, 16, 0, per_in, L)
    wire = per_out // R
    stride_in = (per_in + 127) // 128 * 128
    stride_out = (per_out + 127) // 128 * 128
    tin = torch.randint(0, 256, (C * stride_in,), dtype=torch.uint8, device=dev)
    tout = torch.zeros(C * stride_out, dtype=torch.uint8, device=dev)
    d = np.zeros(C, dtype=S.STREAM_OUT)
    d["in_off"] = np.arange(C, dtype=np.uint64) * stride_in
    d["in_len"] = per_in
    d["slot"] = np.arange(C)
    d["out_off"] = np.arange(C, dtype=np.uint64) * stride_out
    d["type"] = 23
    d["max_frag"] = L
    d["out_ctr"][:, 1] = 1                                    # epoch 1, sequence 0
    dout = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    n = C * R
    recs = torch.zeros(n * 40, dtype=torch.uint8, device=dev)
    res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    disp = torch.zeros(n, dtype=torch.int32, device=dev)
    sres = torch.zeros(C * 32, dtype=torch.uint8, device=dev)
    cres = torch.zeros(C * 48, dtype=torch.uint8, device=dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    t_enc = timed(lambda: D.encrypt(kt, dout, C, tin, tout, recs, res, n, sres))
    ms_enc, _ = rowlib.event_timed(lambda: D.encrypt(kt, dout, C, tin, tout, recs, res, n, sres), a.steps)
    so = sres.cpu().numpy().view(S.STREAM_OUT_RES)
    assert (so["status"] == 0).all() and (so["out_len"] == per_out).all()
    import oracle as O
    ok = True
    for i in (0, C // 2, C - 1):
        k = km[i]
        t = O.Transform(O.TLS1_2, a.cipher, bytes(k["key"][:kl]), bytes(k["key"][:kl]), bytes(k["iv"]),
                        bytes(k["iv"]))
        pt = tin[i * stride_in:i * stride_in + per_in].cpu().numpy().tobytes()
        r, want, _, _ = O.dtls_encrypt(t, pt, 23, bytes([0, 1]) + bytes(6), L)
        ok &= r == 0 and tout[i * stride_out:i * stride_out + per_out].cpu().numpy().tobytes() == want
    # receive side: every record its own datagram, decrypted in place (fresh copy each step)
    dg = np.zeros(n, dtype=D.DGRAM)
    dg["off"] = (np.arange(C, dtype=np.uint64)[:, None] * stride_out
                 + np.arange(R, dtype=np.uint64)[None, :] * wire).reshape(-1)
    dg["len"] = wire
    di = np.zeros(C, dtype=D.DTLS_IN)
    di["first_dgram"] = np.arange(C) * R
    di["ndgram"] = R
    di["slot"] = np.arange(C)
    di["in_epoch"] = 1
    di["flags"] = M.DTLS_ANTI_REPLAY
    din = torch.from_numpy(di.view(np.uint8).copy()).to(dev)
    tdg = torch.from_numpy(dg.view(np.uint8).copy()).to(dev)
    work = torch.empty_like(tout)
    times = []
    for _ in range(a.steps + 1):
        work.copy_(tout)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.decrypt(kt, din, C, tdg, n, work, recs, res, disp, n, cres)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t_dec = float(np.mean(times[1:]))
    ms_dec, _ = rowlib.event_timed(lambda: D.decrypt(kt, din, C, tdg, n, work, recs, res, disp, n, cres), a.steps,
                                   prep=lambda: work.copy_(tout))
    ci = cres.cpu().numpy().view(D.DTLS_IN_RES)
    assert (ci["status"] == 0).all() and (ci["naccepted"] == R).all() and (ci["window_top"] == R - 1).all()
    payload = float(C) * per_in
    # SURVEY 8(d)'s rule with the 13-B headers: send reads the application data
    # and writes the datagrams; receive reads the datagrams and writes each
    # record's plaintext and a 4-B status
    alg = {"dtls_encrypt": C * (per_in + per_out), "dtls_decrypt": C * (per_out + R * (L + 4))}
    rules = {"dtls_encrypt": "application data read + datagrams (13-B headers, explicit nonces, ciphertext, tags) "
                             "written",
             "dtls_decrypt": "datagrams (13-B headers, explicit nonces, ciphertext, tags) read + plaintext and a "
                             "4-B status per record written"}
    kernels = {"dtls_encrypt": "DTLS frame + tlsrec_gcm_kernel / tlsrec_chachapoly_kernel",
               "dtls_decrypt": "datagram header walk / anti-replay + AEAD kernel + in-order finish"}
    for name, t, ms in (("dtls_encrypt", t_enc, ms_enc), ("dtls_decrypt", t_dec, ms_dec)):
        cpu = None if a.no_cpu else rowlib.cpu_stream_legs(True, a.cipher, L, R,
                                                           "send" if name == "dtls_encrypt" else "receive",
                                                           a.cpu_seconds)
        print(json.dumps({"metric": f"DTLS 1.2 {name} throughput (device-resident, datagram framing and "
                                    "anti-replay included)",
                          "value": round(payload / t / 2**30, 3), "unit": "GiB/s",
                          "records_per_s": round(n / t), "ms_per_call": round(t * 1e3, 3),
                          "config": {"connections": C, "datagrams_per_connection": R, "content_bytes": L,
                                     "cipher": a.cipher, "protocol": "DTLS 1.2"},
                          "roofline": rowlib.roofline(alg[name], ms, rules[name], kernels[name]),
                          "cpu_baseline": cpu,
                          "check": {"oracle_sample_ok": bool(ok)}}), flush=True)


if __name__ == "__main__":
    main()
