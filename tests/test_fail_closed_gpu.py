"""Fail-closed batch results: the reference refuses to report success unless
authentication ran (`if (auth_done != 1) return MBEDTLS_ERR_SSL_INTERNAL_ERROR`,
/root/reference/library/ssl_msg.c:1260 encrypt, :1804 decrypt).

The engine's equivalent: before any AEAD kernel of a batch runs, every result
reads INTERNAL_ERROR (the guard kernel in identity order, the bucket count
kernel otherwise, the staged result of the single-record engine), and only the
kernel that handles the record overwrites it.  These tests pre-fill the
results with ZERO (= success) and use the test hook tlsrec__test_skip_record to
leave one record unreached by every AEAD kernel: that record must read
INTERNAL_ERROR, every other record must match the oracle."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import mbedtls_amd as M
from mbedtls_amd import _abi
from tests import batchlib as B

pytestmark = pytest.mark.gpu


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def skip_hook():
    """the test-hooks build (libtlsrec_test.so) serves every binding for the
    test: the release library has no hook to leave a record unreached"""
    with _abi.use_library() as lib:
        f = lib.tlsrec__test_skip_record
        f.argtypes = [ctypes.c_uint32]
        f.restype = None
        yield f
        f(0xFFFFFFFF)


def _check(batch, decrypt, out, res, skipped, inplace=True):
    """every record but `skipped` bit-exact against the oracle; `skipped`
    reads INTERNAL_ERROR and its buffer is untouched"""
    assert int(res[skipped]["status"]) == M.ERR_SSL_INTERNAL_ERROR, res[skipped]
    o = batch.offs[skipped]
    r = batch.recs[skipped]
    assert bytes(out[o:o + len(r.buf)]) == bytes(r.buf), "an unreached record's bytes changed"
    bad = batch.compare(decrypt, out, res)
    bad = [b for b in bad if not b.startswith(f"rec {skipped}:")]
    assert not bad, bad[:5]


ONE_KEY = [
    ("AES-256-GCM", "TLS1.3", True),
    ("AES-128-GCM", "TLS1.2", False),
    ("CHACHA20-POLY1305", "TLS1.3", False),
    ("CHACHA20-POLY1305", "TLS1.2", True),
    ("AES-128-CCM", "TLS1.2", True),
    ("ARIA-128-GCM", "TLS1.2", False),
    ("CAMELLIA-256-CCM", "TLS1.2", True),
]


@pytest.mark.parametrize("cipher,ver,decrypt", ONE_KEY)
@pytest.mark.parametrize("skipped", [0, 5, 15])
def test_identity_order_unreached_record_fails_closed(skip_hook, cipher, ver, decrypt, skipped):
    """single key table (identity order, the c2 path): the guard kernel"""
    assert _gpu()
    slots = B.random_slots(31, [B.CIPHERS[cipher]], [B.VERSIONS[ver]], 1)
    lengths = [1400, 0, 1, 16383, 17, 1024, 333, 4096, 15, 16, 2000, 64, 100, 7, 1500, 9000]
    if decrypt:
        recs, _ = B.sealed_records(slots, lengths, seed=901)
    else:
        recs = B.plaintext_records(slots, lengths, seed=901)
    b = B.Batch(slots, recs)
    skip_hook(skipped)
    out, res = b.run_gpu(decrypt)        # results pre-filled with zero (= success)
    skip_hook(0xFFFFFFFF)
    _check(b, decrypt, out, res, skipped)


@pytest.mark.parametrize("decrypt", [True, False])
@pytest.mark.parametrize("skipped", [0, 1, 2, 3, 37, 63])
def test_bucket_order_unreached_record_fails_closed(skip_hook, decrypt, skipped):
    """many keys (bucket order): the count kernel writes the sentinel; records
    0..3 belong to AES-256-GCM, ChaCha20-Poly1305, AES-128-CCM, Camellia-128-GCM"""
    assert _gpu()
    ciphers = [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305, M.CIPHER_AES_128_CCM, M.CIPHER_CAMELLIA_128_GCM]
    slots = B.random_slots(32, ciphers, [M.VERSION_TLS1_2, M.VERSION_TLS1_3], 8)
    lengths = [(i * 337) % 2000 + (i % 3) for i in range(64)]
    if decrypt:
        recs, _ = B.sealed_records(slots, lengths, seed=902)
    else:
        recs = B.plaintext_records(slots, lengths, seed=902)
    b = B.Batch(slots, recs)
    skip_hook(skipped)
    out, res = b.run_gpu(decrypt)
    skip_hook(0xFFFFFFFF)
    _check(b, decrypt, out, res, skipped)


def test_without_hook_every_record_gets_a_verdict(skip_hook):
    """the same batches with the hook off: no INTERNAL_ERROR anywhere"""
    assert _gpu()
    slots = B.random_slots(33, [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305], [M.VERSION_TLS1_3], 4)
    recs, _ = B.sealed_records(slots, [1400] * 32, seed=903)
    b = B.Batch(slots, recs)
    out, res = b.run_gpu(True)
    assert (res["status"] == 0).all()
    assert not b.compare(True, out, res)


def test_single_record_api_unreached_returns_internal_error(skip_hook):
    """tlsrec_encrypt_buf / _decrypt_buf: the result slot is staged as
    INTERNAL_ERROR with the record; an unreached record returns it and leaves
    rec untouched (the previous call's verdict must not leak into it)"""
    assert _gpu()
    key, iv = bytes(range(32)), bytes(range(100, 116))
    t = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_256_GCM, key, key, iv, iv)
    try:
        payload = bytes(range(200))
        rec = M.Record(ctr=bytes(8), type=23, ver=b"\x03\x03", buf=bytearray(payload + bytes(64)),
                       data_offset=0, data_len=len(payload))
        assert t.encrypt_buf(rec) == 0          # a good call first: its verdict is 0
        skip_hook(0)
        rec2 = M.Record(ctr=(1).to_bytes(8, "big"), type=23, ver=b"\x03\x03",
                        buf=bytearray(payload + bytes(64)), data_offset=0, data_len=len(payload))
        assert t.encrypt_buf(rec2) == M.ERR_SSL_INTERNAL_ERROR
        assert rec2.data_len == len(payload) and rec2.data_offset == 0 and rec2.type == 23
        assert bytes(rec2.buf[:len(payload)]) == payload
        assert t.decrypt_buf(rec) == M.ERR_SSL_INTERNAL_ERROR
        skip_hook(0xFFFFFFFF)
        assert t.decrypt_buf(rec) == 0 and rec.data() == payload
    finally:
        t.close()


def test_host_pipeline_unreached_record_fails_closed(skip_hook):
    """tlsrec_host_batch_decrypt: records in host memory, results pre-filled 0"""
    assert _gpu()
    slots = B.random_slots(34, [M.CIPHER_AES_128_GCM], [M.VERSION_TLS1_2], 1)
    recs, _ = B.sealed_records(slots, [1400] * 24, seed=904)
    b = B.Batch(slots, recs)
    kt = M.KeyTable(1)
    kt.load(b.key_materials())
    arena = b.arena.copy()
    res = np.zeros(len(recs), dtype=M.BATCH_RES)
    skip_hook(7)
    try:
        M.host_batch(True, kt, b.desc, res, len(recs), arena, arena)
    finally:
        skip_hook(0xFFFFFFFF)
        kt.close()
    _check(b, True, arena, res, 7)
