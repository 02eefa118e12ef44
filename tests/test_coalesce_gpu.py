"""Coalesced single-record calls (engine.hip: flat combining per key-table
page).  Concurrent tlsrec_encrypt_buf / tlsrec_decrypt_buf calls of many
threads -- every AEAD family, both TLS versions, both directions in flight at
once -- are carried by shared launches; every call's result must be exactly
the reference's for its own record (ciphertext against the oracle, round trip
back to the plaintext), as the reference call sites ssl_msg.c:2697 / :3835
expect from one call per record."""
import ctypes
import threading

import pytest

import mbedtls_amd as M
import oracle as O
from mbedtls_amd import _abi
from tests.prng import prng_bytes

pytestmark = pytest.mark.gpu

SUITES = [(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3), (M.CIPHER_CHACHA20_POLY1305, M.VERSION_TLS1_3),
          (M.CIPHER_AES_128_GCM, M.VERSION_TLS1_2), (M.CIPHER_AES_128_CCM, M.VERSION_TLS1_2),
          (M.CIPHER_AES_192_GCM, M.VERSION_TLS1_3), (M.CIPHER_CHACHA20_POLY1305, M.VERSION_TLS1_2),
          (M.CIPHER_ARIA_128_GCM, M.VERSION_TLS1_2), (M.CIPHER_AES_256_CCM_8, M.VERSION_TLS1_2)]


def _stats():
    f = _abi.load().tlsrec__engine_stats
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    b, r = ctypes.c_uint64(), ctypes.c_uint64()
    f(ctypes.byref(b), ctypes.byref(r))
    return b.value, r.value


def _server_stats():
    f = _abi.load().tlsrec__server_stats
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3
    s, fb, ln = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    f(ctypes.byref(s), ctypes.byref(fb), ctypes.byref(ln))
    return s.value


@pytest.mark.parametrize("server", [True, False], ids=["server", "launch_path"])
def test_concurrent_calls_are_coalesced_and_exact(server):
    """AES-GCM / ChaCha20-Poly1305 calls go to the record server (server.hip)
    when it is on; the coalescing launch path carries the rest, and all of
    them when it is off"""
    _abi.load().tlsrec__server_enable(1 if server else 0)
    nthreads, per = 16, 40
    b0, r0 = _stats()
    s0 = _server_stats()
    errors = []

    def worker(tid):
        cipher, ver = SUITES[tid % len(SUITES)]
        kl = M.KEYLEN[cipher]
        key, iv = prng_bytes(3000 + tid, kl), prng_bytes(4000 + tid, 16)
        t = M.Transform(ver, cipher, key, key, iv, iv)
        ot = O.Transform(ver, cipher, key, key, iv, iv)
        head = 8 if ver == M.VERSION_TLS1_2 and cipher != M.CIPHER_CHACHA20_POLY1305 else 0
        try:
            for n in range(per):
                ln = (n * 389 + tid * 71) % 3000 + (n % 3)
                pt = prng_bytes(tid * 1000 + n, ln)
                buf = bytearray(head + ln + 64)
                buf[head:head + ln] = pt
                ctr = (n + 7 * tid).to_bytes(8, "big")
                rec = M.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=buf, data_offset=head, data_len=ln)
                orec = O.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=bytearray(buf), data_offset=head, data_len=ln)
                st, ost = t.encrypt_buf(rec), ot.encrypt_buf(orec)
                if (st, rec.data_offset, rec.data_len, rec.type) != (ost, orec.data_offset, orec.data_len, orec.type):
                    errors.append((tid, n, "encrypt fields", st, ost))
                    continue
                if st == 0 and rec.data() != orec.data():
                    errors.append((tid, n, "ciphertext differs from the oracle"))
                    continue
                if st != 0:
                    continue
                if t.decrypt_buf(rec) != 0 or rec.data() != pt or rec.type != 23:
                    errors.append((tid, n, "round trip"))
        except Exception as e:          # noqa: BLE001 (reported below)
            errors.append((tid, "exception", repr(e)))
        finally:
            t.close()

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=300)
    _abi.load().tlsrec__server_enable(1)
    assert not errors, errors[:5]
    b1, r1 = _stats()
    batches, records = b1 - b0, r1 - r0
    served = _server_stats() - s0
    assert records + served == 2 * nthreads * per
    assert batches < records, "no call was coalesced with another"
    assert (served > 0) == server
