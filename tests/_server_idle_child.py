"""Child process of tests/test_server_gpu.py::test_idle_boundary_submits_are_never_withdrawn:
single-record calls spaced around the record server's idle limit (the parent
sets TLSREC_SERVER_IDLE_MS), each checked against the oracle; prints one JSON
line with the server's counters."""
import ctypes
import json
import sys
import time

import numpy as np

import mbedtls_amd as M
import oracle as O
from mbedtls_amd import _abi
from tests.prng import prng_bytes


def main(calls, test_lib=False):
    if test_lib:
        # the test-hooks build (TLSREC_TEST_SERVER_POST_DELAY_US): every binding
        # of this process goes to it
        with _abi.use_library():
            return _main(calls)
    return _main(calls)


def _main(calls):
    L = _abi.load()
    L.tlsrec__server_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3
    L.tlsrec__server_closing.restype = ctypes.c_uint64
    rng = np.random.default_rng(5)
    ts = {}
    for c in (M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305):
        kl = M.KEYLEN[c]
        key, iv = prng_bytes(70 + c, kl), prng_bytes(80 + c, 16)
        ts[c] = (M.Transform(M.VERSION_TLS1_3, c, key, key, iv, iv), O.Transform(M.VERSION_TLS1_3, c, key, key, iv, iv))
    # warm the path (first grid launch, code objects) before counting
    for c, (t, _) in ts.items():
        rec = M.Record(ctr=bytes(8), type=23, ver=b"\x03\x03", buf=bytearray(200), data_offset=0, data_len=10)
        assert t.encrypt_buf(rec) == 0
    s0 = [ctypes.c_uint64() for _ in range(3)]
    L.tlsrec__server_stats(*[ctypes.byref(x) for x in s0])
    why0 = (ctypes.c_uint64 * 4)()
    L.tlsrec__server_why(why0)
    errors = []
    for i in range(calls):
        gap = float(rng.uniform(0, 400e-6))
        t_end = time.perf_counter() + gap
        while time.perf_counter() < t_end:
            pass
        c = (M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305)[i % 2]
        ln = 16383 if i % 7 == 3 else 1400
        t, ot = ts[c]
        pt = prng_bytes(1000 + i, ln)
        ctr = (i + 1).to_bytes(8, "big")
        buf = bytearray(pt) + bytearray(32)
        rec = M.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=bytearray(buf), data_offset=0, data_len=ln)
        orec = O.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=bytearray(buf), data_offset=0, data_len=ln)
        st, ost = t.encrypt_buf(rec), ot.encrypt_buf(orec)
        if (st, rec.data_len) != (ost, orec.data_len) or bytes(rec.buf) != bytes(orec.buf):
            errors.append(("encrypt", i, st, ost))
    s1 = [ctypes.c_uint64() for _ in range(3)]
    L.tlsrec__server_stats(*[ctypes.byref(x) for x in s1])
    why = (ctypes.c_uint64 * 4)()
    L.tlsrec__server_why(why)
    for t, _ in ts.values():
        t.close()
    print(json.dumps({"calls": calls, "served": s1[0].value - s0[0].value, "fallback": s1[1].value - s0[1].value,
                      "launches": s1[2].value - s0[2].value, "why": [why[k] - why0[k] for k in range(4)],
                      "closing": int(L.tlsrec__server_closing()), "errors": errors}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 600, test_lib="--test-lib" in sys.argv)
