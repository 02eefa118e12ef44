#!/usr/bin/env python3
"""Throughput of the batched TLS 1.3 key schedule (tlsrec_tls13_keytab_derive):
64 K connection-direction traffic secrets in HBM -> KeyUpdate -> write_key /
write_iv -> key-table slots (AES expansion, H, GHASH tables).  Prints one JSON
line; the derive kernel and the key-setup kernel are timed separately with
HIP events on the call's stream.

    python tools/bench_keysched.py [--count 65536] [--cipher 2] [--steps 5]
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
    ap.add_argument("--count", type=int, default=65536)
    ap.add_argument("--cipher", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--update", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall-time target of the CPU sample")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    from tools import rowlib
    import torch
    import mbedtls_amd as M
    from mbedtls_amd import keysched as K
    from tests.prng import prng_array
    dev = torch.device("cuda")
    secrets = torch.from_numpy(prng_array(0x5EC, a.count * 48)).to(dev)
    kt = M.KeyTable(a.count)
    st = torch.cuda.current_stream()
    K.keytab_derive(kt, 0, a.count, a.cipher, secrets, key_update=bool(a.update))
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(st)
        K.keytab_derive(kt, 0, a.count, a.cipher, secrets, key_update=bool(a.update))
        e.record(st)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    import oracle as O
    alg = O.SHA384 if a.cipher == 2 else O.SHA256
    keylen = 16 if a.cipher == 1 else 32
    cpu = None if a.no_cpu else rowlib.cpu_keysched_leg(alg, keylen, bool(a.update), a.cpu_seconds)
    # algorithmic bytes per connection: the 48-B secret read (and written back
    # after a KeyUpdate), the key-table slot written -- its 1 KiB state (round
    # keys, H, H powers) and the 70 KiB of GHASH tables the GCM kernels read
    slot = 1024 + (7 * 512 + 26 * 32 + 64) * 16
    per = 48 * (2 if a.update else 1) + slot
    print(json.dumps({"metric": "TLS 1.3 traffic-key derivations into the key table per second",
                      "value": round(a.count / (ms / 1e3)), "unit": "connections/s", "count": a.count,
                      "cipher": a.cipher, "key_update": a.update, "ms_per_batch_events": round(ms, 4),
                      "ms_per_batch_wall": round(wall * 1e3, 4),
                      "roofline": rowlib.roofline(per * a.count, ms, "per connection: secret read (and written after "
                                                  "a KeyUpdate) + the key-table slot written (1 KiB state + 70 KiB "
                                                  "GHASH tables)", "tls13 derive + key setup"),
                      "cpu_baseline": cpu}))


if __name__ == "__main__":
    main()
