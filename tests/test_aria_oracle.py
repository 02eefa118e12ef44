"""ARIA-GCM and ARIA-CCM in the CPU restatement (the ARIA entries of
mbedtls_ssl_cipher_to_psa, library/ssl_tls.c:2248-2289).

ARIA itself lives in the absent TF-PSA-Crypto; oracle/aria.c restates RFC 5794.
Pinned here by
  1. the RFC 5794 Appendix A block vectors (128/192/256-bit keys);
  2. OpenSSL 3.0.2 EVP ARIA-GCM: raw AEAD outputs and whole TLS 1.2 records
     (ciphertext bytes; the reference ships no ARIA record KAT -- its 96
     ssl_crypt_record ARIA cases, test_suite_ssl.data, pin behaviour only);
  3. the ssl_crypt_record / ssl_crypt_record_small semantics for ARIA-GCM
     (test_suite_ssl.function:1567-1856), with and without connection IDs.
"""
import pytest

import oracle as O
from tests import _openssl as S
from tests.prng import prng_bytes
from tests.test_cid_oracle import build_cid_transforms

ARIA = {"aria128gcm": O.ARIA_128_GCM, "aria192gcm": O.ARIA_192_GCM, "aria256gcm": O.ARIA_256_GCM,
        "aria128ccm": O.ARIA_128_CCM, "aria192ccm": O.ARIA_192_CCM, "aria256ccm": O.ARIA_256_CCM}
h = bytes.fromhex


@pytest.mark.parametrize("key,ct", [
    ("000102030405060708090a0b0c0d0e0f", "d718fbd6ab644c739da95f3be6451778"),
    ("000102030405060708090a0b0c0d0e0f1011121314151617", "26449c1805dbe7aa25a468ce263a9e79"),
    ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f", "f92bd7c79fb72e2f2b8f80c1972d24fc"),
])
def test_rfc5794_vectors(key, ct):
    assert O.aria_encrypt_block(h(key), h("00112233445566778899aabbccddeeff")).hex() == ct


def test_sboxes_are_permutations():
    import ctypes
    f = O.lib().orc_aria_sbox
    f.restype = ctypes.POINTER(ctypes.c_uint8)
    sb = [bytes(f(i)[:256]) for i in range(4)]
    for t in sb:
        assert len(set(t)) == 256
    for x in range(256):                     # SB3 = SB1^-1, SB4 = SB2^-1
        assert sb[2][sb[0][x]] == x and sb[3][sb[1][x]] == x
    assert sb[1][0] == 0xE2 and sb[0][0] == 0x63


@pytest.mark.skipif(S.lib() is None, reason="libcrypto not present")
def test_aria_gcm_vs_openssl():
    for i in range(60):
        rnd = prng_bytes(0xA51A + i, 96)
        kl = (16, 24, 32)[i % 3]
        L = [0, 1, 15, 16, 17, 64, 255, 1400, 4097, 16384][i % 10]
        pt, aad, iv = prng_bytes(i, L), rnd[64:64 + (i % 30)], rnd[32:44]
        assert O.aria_gcm_encrypt(rnd[:kl], iv, aad, pt) == S.seal("aria-gcm", rnd[:kl], iv, aad, pt), (kl, L)


@pytest.mark.skipif(S.lib() is None, reason="libcrypto not present")
@pytest.mark.parametrize("cipher", list(ARIA.values()), ids=list(ARIA))
def test_aria_records_vs_openssl(cipher):
    """TLS 1.2 ARIA-GCM records: explicit nonce = seq, AAD = seq|type|ver|len16."""
    kl = O.KEYLEN[cipher]
    for n in (0, 1, 16, 100, 1400, 16384):
        rnd = prng_bytes(0xAB + n + cipher, 64)
        key, iv, ctr = rnd[:kl], rnd[32:48], rnd[48:56]
        t = O.Transform(O.TLS1_2, cipher, key, key, iv, iv)
        content = prng_bytes(n, n)
        buf = bytearray(8 + n + 16)
        buf[8:8 + n] = content
        rec = O.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=buf, data_offset=8, data_len=n)
        assert t.encrypt_buf(rec) == 0
        aad = ctr + b"\x17\x03\x03" + n.to_bytes(2, "big")
        if cipher >= O.ARIA_128_CCM:
            ct, tag = S.ccm_seal(key, iv[:4] + ctr, aad, content, 16, name="aria-ccm")
        else:
            ct, tag = S.seal("aria-gcm", key, iv[:4] + ctr, aad, content)
        assert rec.data() == ctr + ct + tag


def _pair(cipher, ver):
    kl = O.KEYLEN[cipher]
    key0, key1 = bytes([1]) * kl, bytes([2]) * kl
    ive, ivd = bytes([3]) * 16, bytes([4]) * 16
    return O.Transform(ver, cipher, key0, key1, ive, ivd), O.Transform(ver, cipher, key1, key0, ivd, ive)


@pytest.mark.parametrize("cipher", list(ARIA.values()), ids=list(ARIA))
@pytest.mark.parametrize("ver", [O.TLS1_2, O.TLS1_3], ids=["tls12", "tls13"])
def test_crypt_record_aria(cipher, ver):
    """ssl_crypt_record (test_suite_ssl.function:1567-1695) for ARIA-GCM."""
    t0, t1 = _pair(cipher, ver)
    for n in range(15, -1, -1):
        t_dec, t_enc = (t0, t1) if n % 3 == 0 else (t1, t0)
        buf = bytearray(512)
        rec = O.Record(ctr=bytes([n]) * 8, type=42, ver=bytes([n, n]), buf=buf, data_offset=16, data_len=1 + n)
        buf[16:17 + n] = bytes([42]) * (1 + n)
        assert t_enc.encrypt_buf(rec) == 0
        assert t_dec.decrypt_buf(rec) == 0
        assert (rec.type, rec.data_offset, rec.data_len) == (42, 16, 1 + n)
        assert rec.data() == bytes([42]) * (1 + n)


@pytest.mark.parametrize("cipher", list(ARIA.values()), ids=list(ARIA))
def test_crypt_record_aria_cid(cipher):
    """The reference's ARIA ssl_crypt_record cases with cids 4:4 / 4:0."""
    for cids in ((4, 4), (4, 0)):
        t0, t1 = build_cid_transforms(cipher, *cids)
        for n in range(15, -1, -1):
            t_dec, t_enc = (t0, t1) if n % 3 == 0 else (t1, t0)
            buf = bytearray(512)
            rec = O.Record(ctr=bytes([n]) * 8, type=42, ver=bytes([n, n]), buf=buf, data_offset=16, data_len=1 + n)
            buf[16:17 + n] = bytes([42]) * (1 + n)
            assert t_enc.encrypt_buf(rec) == 0
            assert t_dec.decrypt_buf(rec) == 0
            assert rec.data() == bytes([42]) * (1 + n)
