"""Shared measurement pieces of the SURVEY §8(f) row benches
(tools/bench_stream.py, bench_dtls.py, bench_keysched.py), so that their
lines carry what bench.py's does:

  roofline      the call's algorithmic bytes (SURVEY §8(d)'s rule, headers
                included) over its GPU time, timed with HIP events on the
                stream the call's kernels run on, as a fraction of the 8 TB/s
                HBM peak;
  cpu_baseline  the same row on the host's cores: the oracle's restatement
                ("port": oracle/rows_bench.c over oracle/stream.c, dtls.c,
                keysched.c) and, for the AEADs OpenSSL has, the same framing
                around OpenSSL EVP ("evp": oracle/evp_bench.c
                evp_mixed_stream), one key context per connection, connection
                c on thread c % threads; the faster leg is the value.

The oracle is imported only here, after the GPU part of a tool has run (it
is the checker and the CPU baseline, never the measured path)."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def roofline(alg_bytes_per_call, kernel_ms, rule, kernels):
    """The call's algorithmic bytes over its GPU time (HIP events around the
    call on its launch stream)."""
    ach = alg_bytes_per_call / (kernel_ms / 1e3) / 1e9 if kernel_ms > 0 else 0.0
    return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "algorithmic_bytes_per_call": int(alg_bytes_per_call), "algorithmic_bytes_rule": rule,
            "kernel_ms_avg": round(kernel_ms, 4), "kernels": kernels,
            "timing": "HIP events on the call's stream around each timed call (every kernel of the call)"}


def event_timed(fn, steps, prep=None):
    """Mean GPU ms (HIP events on the current stream) and wall seconds of
    `steps` calls of fn; prep() runs untimed before each call."""
    import time
    import torch
    st = torch.cuda.current_stream()
    ms, wall = [], []
    for _ in range(steps):
        if prep:
            prep()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
        ms.append(a.elapsed_time(b))
    return float(np.mean(ms)), float(np.mean(wall))


def _grow(target_s, n0, cap_n, run):
    """run(n) -> seconds of one pass over n connections; grow n until a pass
    takes about target_s (or the memory cap), then repeat passes to target_s."""
    n = n0
    while True:
        el = run(n)
        if el >= target_s or n >= cap_n:
            break
        n = min(cap_n, int(n * max(2.0, min(8.0, target_s / max(el, 1e-3)))))
    reps, tot = 1, el
    while tot < target_s:
        tot += run(n)
        reps += 1
    return n, reps, tot


def cpu_stream_legs(dtls, cipher, content, recs, direction, target_s, seed=0xC9B0):
    """CPU baseline of a stream / DTLS row: `recs` records of `content` bytes
    per connection, direction 'send' or 'receive', TLS 1.3 (stream) or DTLS
    1.2.  Returns bench.py's cpu_baseline shape (legs + the faster one)."""
    import oracle as O
    from bench import host_cores
    from tests.prng import prng_array
    threads, how = host_cores()
    tls = O.TLS1_2 if dtls else O.TLS1_3
    kl = O.KEYLEN[cipher]
    per_in = recs * content
    cap_bytes = 512 << 20

    state = {}

    def conns(n):
        if state.get("n") == n:
            return state
        raw = prng_array(seed, n * 48).reshape(n, 48)
        keys = np.zeros((n, 32), dtype=np.uint8)
        keys[:, :kl] = raw[:, :kl]
        ivs = np.ascontiguousarray(raw[:, 32:44])
        ts = [O.Transform(tls, cipher, bytes(k[:kl]), bytes(k[:kl]), bytes(v) + bytes(4), bytes(v) + bytes(4))
              for k, v in zip(keys, ivs)]
        wire = O.dtls_record_wire(ts[0], content) if dtls else O.stream_record_wire(ts[0], content)
        per_out = recs * wire
        in_stride, out_stride = (per_in + 127) // 128 * 128, (per_out + 127) // 128 * 128
        pt = prng_array(seed ^ 1, n * in_stride).reshape(n, in_stride)
        sealed = np.zeros((n, out_stride), dtype=np.uint8)
        stt = np.zeros(n, dtype=np.int32)
        O.bench_stream_rows(ts, dtls, 1, pt, in_stride, per_in, sealed, out_stride, content, threads, stt)
        assert (stt == 0).all(), "CPU leg: sealing the sample failed"
        em = None
        if cipher in O.EVP_CIPHERS:
            if state.get("em"):
                state["em"].close()
            em = O.EvpMixed(np.full(n, cipher, dtype=np.uint8), keys, ivs, tls, threads)
        state.clear()
        state.update(n=n, ts=ts, em=em, wire=wire, per_out=per_out, in_stride=in_stride, out_stride=out_stride,
                     pt=pt, sealed=sealed, work=np.empty_like(sealed), st=stt)
        return state

    cap_n = max(16, cap_bytes // max(1, 2 * ((per_in + 127) // 128 * 128 + recs * (content + 64))))

    def leg(kind):
        def run(n):
            s = conns(n)
            st = s["st"]
            st[:] = 1
            if direction == "send":
                if kind == "evp":
                    el = s["em"].stream(dtls, 1, s["pt"], s["in_stride"], per_in, s["work"], s["out_stride"], content, st)
                else:
                    el = O.bench_stream_rows(s["ts"], dtls, 1, s["pt"], s["in_stride"], per_in, s["work"],
                                             s["out_stride"], content, threads, st)
            else:
                np.copyto(s["work"], s["sealed"])          # untimed: receive decrypts in place
                step = s["wire"] if dtls else 0
                if kind == "evp":
                    el = s["em"].stream(dtls, 0, s["work"], s["out_stride"], s["per_out"], None, 0, step, st)
                else:
                    el = O.bench_stream_rows(s["ts"], dtls, 0, s["work"], s["out_stride"], s["per_out"], None, 0,
                                             step, threads, st)
            assert (st == 0).all(), f"CPU leg {kind}: record errors {np.unique(st)}"
            return el
        n, reps, el = _grow(target_s, 64, cap_n, run)
        what = ("ssl_msg.c record framing around OpenSSL 3 EVP AEADs (oracle/evp_bench.c evp_mixed_stream)"
                if kind == "evp" else
                "the oracle's restatement (oracle/rows_bench.c over oracle/" + ("dtls.c" if dtls else "stream.c") + ")")
        return {"value": round(n * reps * per_in / el / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
                "leg": kind, "records_per_s": round(n * reps * recs / el, 1),
                "sample": f"{n} connections x {recs} records x {content} B ({reps} passes), {direction}, "
                          f"{'DTLS 1.2' if dtls else 'TLS 1.3 stream'}, one key per connection: {what}, "
                          f"{el:.2f} s wall on {threads} threads"}

    legs = []
    if cipher in O.EVP_CIPHERS:
        legs.append(leg("evp"))
    legs.append(leg("port"))
    if state.get("em"):
        state["em"].close()
    out = dict(max(legs, key=lambda x: x["value"]))
    out["cores_how"] = how
    out["headline"] = "the faster of the legs"
    out["legs"] = legs
    return out


def cpu_keysched_leg(alg, keylen, update, target_s, seed=0x5EC):
    """CPU baseline of the key-schedule row: KeyUpdate + HKDF-Expand-Label
    key / iv per connection (oracle/keysched.c through oracle/rows_bench.c) on
    the host's cores.  The GPU row also builds the key-table slot (AES
    expansion, H, GHASH tables), which this leg does not: a lower bound on
    the CPU's work."""
    import oracle as O
    from bench import host_cores
    from tests.prng import prng_array
    threads, how = host_cores()
    cache = {}

    def run(n):
        if n not in cache:
            cache.clear()
            cache[n] = prng_array(seed, n * 48)
        el, _, st = O.bench_keysched(alg, cache[n], n, update, keylen, threads)
        assert (st == 0).all()
        return el
    n, reps, el = _grow(target_s, 1024, 1 << 22, run)
    return {"value": round(n * reps / el), "unit": "connections/s", "cores": threads, "kind": "port", "leg": "port",
            "cores_how": how,
            "sample": f"{n} connections ({reps} passes): {'KeyUpdate + ' if update else ''}HKDF-Expand-Label key / iv "
                      f"(oracle/keysched.c via oracle/rows_bench.c), {el:.2f} s wall on {threads} threads; the "
                      f"key-table slot build (AES expansion, H, GHASH tables) is not in this leg"}
