"""Batch calls through libtlsrec.so on the SYSTEM HIP runtime (/opt/rocm, no
torch in the process -- the runtime a C host links): a sequence of encrypt
('e') and decrypt ('d') calls over a many-key table, each call's results
array pre-filled with 0x55 (or 0x00, which reads as success), reporting how
many results each call wrote and how many carry a kernel's verdict (encrypt:
status 0 with the protected length 1456; decrypt of the static descriptors:
INVALID_MAC) -- with a zero pre-fill only the verdict count tells an unwritten
result from a real one.

    python tests/sysrt_seq.py <records> <keys> <sequence> [pageable|memset|pinned] [prefill byte]

Run as a subprocess by tests/test_c_host.py (not collected by pytest).
Regression: with the stream-ordered allocator (hipMallocAsync) for the
bucket scratch, the first call after a direction change silently wrote no
results under this runtime.  Prints one JSON line.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
from mbedtls_amd import _abi  # noqa: E402
import mbedtls_amd as M  # noqa: E402

L = _abi.load()
n, NK, seq = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
MODE = sys.argv[4] if len(sys.argv) > 4 else "pageable"
FILL = int(sys.argv[5], 0) if len(sys.argv) > 5 else 0x55


def dmalloc(nb):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nb)) == 0
    return p


def h2d(d, a):
    if MODE == "pinned":   # stage through page-locked memory
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(a.nbytes), 0) == 0
        ctypes.memmove(p, a.ctypes.data, a.nbytes)
        assert hip.hipMemcpy(d, p, ctypes.c_size_t(a.nbytes), 1) == 0
        hip.hipHostFree(p)
    else:
        assert hip.hipMemcpy(d, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1) == 0


def d2h(a, d):
    assert hip.hipMemcpy(a.ctypes.data_as(ctypes.c_void_p), d, ctypes.c_size_t(a.nbytes), 2) == 0


km = np.zeros(NK, dtype=M.KEY_MATERIAL)
rng = np.random.default_rng(1)
km["cipher"] = [M.CIPHER_CHACHA20_POLY1305 if i & 1 else M.CIPHER_AES_256_GCM for i in range(NK)]
km["tls_minor"] = 4
km["fixed_ivlen"] = 12
km["taglen"] = 16
km["key"] = rng.integers(0, 256, (NK, 32))
km["iv"][:, :12] = rng.integers(0, 256, (NK, 12))
kt = ctypes.c_void_p()
assert L.tlsrec_keytab_create(ctypes.byref(kt), NK) == 0
assert L.tlsrec_keytab_load(kt, 0, NK, km.ctypes.data, 0, None) == 0
stride = 1536
recs = M.records(n)
recs["buf_off"] = np.arange(n) * stride
recs["buf_len"] = stride
recs["data_len"] = 1424
recs["slot"] = np.arange(n) % NK
recs["ctr"] = M.seq_bytes(np.arange(n) // NK)
recs["type"] = 23
recs["ver"] = (3, 3)
arena = rng.integers(0, 256, n * stride).astype(np.uint8)
da, dr, ds = dmalloc(arena.nbytes), dmalloc(recs.nbytes), dmalloc(n * 16)
h2d(da, arena)
h2d(dr, recs)
written, verdicts = [], []
fillword = int.from_bytes(bytes([FILL]) * 4, "little")
fillword = fillword - (1 << 32) if fillword >= 1 << 31 else fillword
for c in seq:
    r = np.full(n * 16, FILL, dtype=np.uint8).view(M.BATCH_RES)
    if MODE == "memset":
        assert hip.hipMemset(ds, FILL, ctypes.c_size_t(n * 16)) == 0
        hip.hipDeviceSynchronize()
    else:
        h2d(ds, r)
    fn = L.tlsrec_batch_decrypt if c == "d" else L.tlsrec_batch_encrypt
    assert fn(kt, dr, ds, n, da, da, 0, None) == 0
    hip.hipDeviceSynchronize()
    d2h(r, ds)
    raw = r.view(np.uint8).reshape(n, 16)
    written.append(int((raw != FILL).any(axis=1).sum()))
    if c == "e":
        ok = (r["status"] == 0) & (r["data_len"] == 1456)
    else:
        ok = r["status"] == M.ERR_SSL_INVALID_MAC
    verdicts.append(int(ok.sum()))
L.tlsrec_keytab_free(kt)
print(json.dumps({"records": n, "keys": NK, "sequence": seq, "mode": MODE, "fill": FILL, "written": written,
                  "verdicts": verdicts}))
