"""Single-record engine hygiene (ADVICE / VERDICT r03), through the test-hooks
build libtlsrec_test.so where a hook is needed:

* a coalesced batch whose staging allocation fails reports ALLOC_FAILED to
  every caller it carried and leaves their records untouched -- never the
  unfilled result (the reference's fail-closed `auth_done` check,
  /root/reference/library/ssl_msg.c:1260 / :1804);
* freeing a transform zeroizes every key-derived byte of its device slots,
  including the record server's H^1..H^64 (mbedtls_ssl_transform_free
  zeroizes the whole context, ssl_msg.c:6084-6099);
* the record server serves correctly when the key state it reads sits at
  addresses whose low 32 bits have bit 31 set (the readfirstlane
  sign-extension fault of r03, pinned deterministically);
* hipStreamPerThread scratch of a thread is freed when the thread exits.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import pytest

import mbedtls_amd as M
import oracle as O
from mbedtls_amd import _abi
from tests import batchlib as B
from tests.prng import prng_bytes

pytestmark = pytest.mark.gpu


def _server_stats(lib):
    f = lib.tlsrec__server_stats
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3
    s, fb, ln = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    f(ctypes.byref(s), ctypes.byref(fb), ctypes.byref(ln))
    return s.value, fb.value


def _record(ln, seed, head=0):
    pt = prng_bytes(seed, ln)
    buf = bytearray(head) + bytearray(pt) + bytearray(64)
    return pt, buf


def test_staging_allocation_failure_fails_closed():
    with _abi.use_library() as lib:
        lib.tlsrec__server_enable(0)                 # the coalescing launch path stages the record
        fail = lib.tlsrec__test_fail_staging
        fail.argtypes = [ctypes.c_int]
        key, iv = prng_bytes(11, 32), prng_bytes(12, 16)
        t = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_256_GCM, key, key, iv, iv)
        ot = O.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_256_GCM, key, key, iv, iv)
        try:
            pt, buf = _record(1400, 5)
            rec = M.Record(ctr=bytes(8), type=23, ver=b"\x03\x03", buf=bytearray(buf), data_offset=0, data_len=1400)
            assert t.encrypt_buf(rec) == 0          # the staging set exists now
            fail(1)
            rec2 = M.Record(ctr=(1).to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=bytearray(buf),
                            data_offset=0, data_len=1400)
            assert t.encrypt_buf(rec2) == M.ERR_SSL_ALLOC_FAILED
            assert (rec2.data_offset, rec2.data_len, rec2.type) == (0, 1400, 23)
            # the content is untouched (the host may already have written the
            # TLS 1.3 inner type and padding behind it, as ssl_msg.c:853-868 does)
            assert bytes(rec2.buf[:1400]) == pt, "a record no kernel ran was changed"
            # several callers coalesced into one failing batch: every one gets the error
            fail(1000)
            errs = []
            start = threading.Barrier(6)

            def one(k):
                r = M.Record(ctr=(100 + k).to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=bytearray(buf),
                             data_offset=0, data_len=1400)
                start.wait()
                st = t.encrypt_buf(r)
                if st != M.ERR_SSL_ALLOC_FAILED or bytes(r.buf[:1400]) != pt:
                    errs.append((k, st))
            th = [threading.Thread(target=one, args=(k,)) for k in range(6)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            fail(0)
            assert not errs, errs
            # and the engine recovers: the next call is served and matches the oracle
            orec = O.Record(ctr=(1).to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=bytearray(buf),
                            data_offset=0, data_len=1400)
            assert t.encrypt_buf(rec2) == 0 and ot.encrypt_buf(orec) == 0
            assert bytes(rec2.buf) == bytes(orec.buf)
            assert t.decrypt_buf(rec2) == 0 and rec2.data() == pt
        finally:
            fail(0)
            t.close()
            lib.tlsrec__server_enable(1)


@pytest.mark.parametrize("cipher", [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305])
def test_transform_free_zeroizes_device_slots(cipher):
    with _abi.use_library() as lib:
        dump = lib.tlsrec__test_engine_slot_dump
        dump.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        key, iv = prng_bytes(21, 32), prng_bytes(22, 16)
        t = M.Transform(M.VERSION_TLS1_3, cipher, key, key, iv, iv)
        slots = (int(t._t.slot_enc), int(t._t.slot_dec))
        bufs = [np.zeros(1024, np.uint8) for _ in range(3)]

        def snap(s):
            assert dump(s, *(b.ctypes.data for b in bufs)) == 0
            return [b.copy() for b in bufs]

        before = [snap(s) for s in slots]
        for st, gh, hp in before:
            assert st.any()                           # key material is there
            if cipher != M.CIPHER_CHACHA20_POLY1305:
                assert gh.any() and hp.any()          # GHASH tables, the server's H powers
        t.close()
        for s in slots:
            st, gh, hp = snap(s)
            assert not st.any() and not gh.any() and not hp.any(), f"slot {s} keeps key-derived bytes"


def test_server_reads_key_state_at_bit31_addresses():
    """The server's poll loop widens the 48-bit pointers it reads with
    readfirstlane; placing the slot state, GHASH tables and H powers where
    bit 31 of the low word is set pins the r03 sign-extension fix."""
    import torch
    with _abi.use_library() as lib:
        lib.tlsrec__server_enable(1)
        shadow = lib.tlsrec__test_server_shadow
        shadow.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        region = torch.empty((2 << 30) + (1 << 20), dtype=torch.uint8, device="cuda")
        s0, _ = _server_stats(lib)
        shadow(region.data_ptr(), region.numel())
        errs, n = [], 0
        try:
            for cipher in (M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305):
                for ver in (M.VERSION_TLS1_2, M.VERSION_TLS1_3):
                    kl = M.KEYLEN[cipher]
                    key, iv = prng_bytes(31 + cipher, kl), prng_bytes(41 + cipher, 16)
                    t = M.Transform(ver, cipher, key, key, iv, iv)
                    ot = O.Transform(ver, cipher, key, key, iv, iv)
                    head = 8 if ver == M.VERSION_TLS1_2 and cipher != M.CIPHER_CHACHA20_POLY1305 else 0
                    try:
                        for ln in (1, 100, 1400, 16383):
                            n += 1
                            pt, buf = _record(ln, 1000 + ln + cipher, head)
                            ctr = (n * 7).to_bytes(8, "big")
                            rec = M.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=bytearray(buf), data_offset=head,
                                           data_len=ln)
                            orec = O.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=bytearray(buf),
                                            data_offset=head, data_len=ln)
                            if t.encrypt_buf(rec) != 0 or ot.encrypt_buf(orec) != 0 or bytes(rec.buf) != bytes(orec.buf):
                                errs.append(("encrypt", cipher, ver, ln))
                                continue
                            if t.decrypt_buf(rec) != 0 or rec.data() != pt:
                                errs.append(("decrypt", cipher, ver, ln))
                    finally:
                        t.close()
        finally:
            shadow(None, 0)
        s1, _ = _server_stats(lib)
        del region
    assert not errs, errs
    assert s1 - s0 >= n, f"only {s1 - s0} of {2 * n} calls were served by the record server"


def test_per_thread_stream_scratch_freed_at_thread_exit():
    """Batches on hipStreamPerThread get scratch per thread; a thread's entry
    goes away with the thread (a server with short-lived threads must not
    accumulate device memory)."""
    lib = _abi.load()
    cnt = lib.tlsrec__scratch_entries
    cnt.restype = ctypes.c_uint32
    cnt.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    slots = B.random_slots(77, [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305], [M.VERSION_TLS1_3], 6)
    recs = B.plaintext_records(slots, [1400] * 48, seed=78)
    b = B.Batch(slots, recs)
    PER_THREAD = 2                                   # (hipStream_t) 2 = hipStreamPerThread
    errs = []

    def work():
        try:
            out, res = b.run_gpu(False, stream=PER_THREAD)
            bad = b.compare(False, out, res)
            if bad:
                errs.append(bad[:2])
        except Exception as e:                       # noqa: BLE001 -- reported below
            errs.append(repr(e))

    work()                                           # the main thread's entry (kept: it stays alive)
    n0 = cnt(None)
    for _ in range(3):
        th = [threading.Thread(target=work) for _ in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    assert not errs, errs
    work()             # a later acquire (any thread) frees the exited threads' entries
    assert cnt(None) == n0, f"{cnt(None) - n0} scratch entries of exited threads remain"
