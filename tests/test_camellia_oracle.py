"""Camellia-GCM and Camellia-CCM in the CPU restatement (the
Camellia entries of mbedtls_ssl_cipher_to_psa, library/ssl_tls.c:2297-2345).

Camellia lives in the absent TF-PSA-Crypto; oracle/camellia.c restates RFC 3713.
Pinned here by
  1. the RFC 3713 Appendix A block vectors (128/192/256-bit keys);
  2. OpenSSL 3.0.2 Camellia-ECB on random keys and blocks;
  3. whole TLS 1.2 records against GCM (SP 800-38D) and CCM (SP 800-38C)
     assembled in this file around OpenSSL's Camellia-ECB / -CBC -- OpenSSL has
     no Camellia AEAD, and the reference ships no Camellia record KAT (its
     ssl_crypt_record Camellia cases, test_suite_ssl.data, pin behaviour only);
  4. the ssl_crypt_record semantics (test_suite_ssl.function:1567-1695), with
     and without connection IDs.
"""
import pytest

import oracle as O
from tests import _openssl as S
from tests.prng import prng_bytes
from tests.test_cid_oracle import build_cid_transforms

CAM = {"camellia128gcm": O.CAMELLIA_128_GCM, "camellia192gcm": O.CAMELLIA_192_GCM,
       "camellia256gcm": O.CAMELLIA_256_GCM, "camellia128ccm": O.CAMELLIA_128_CCM,
       "camellia192ccm": O.CAMELLIA_192_CCM, "camellia256ccm": O.CAMELLIA_256_CCM}
h = bytes.fromhex
needs_ssl = pytest.mark.skipif(S.lib() is None, reason="libcrypto not present")


@pytest.mark.parametrize("key,ct", [
    ("0123456789abcdeffedcba9876543210", "67673138549669730857065648eabe43"),
    ("0123456789abcdeffedcba98765432100011223344556677", "b4993401b3e996f84ee5cee7d79b09b9"),
    ("0123456789abcdeffedcba987654321000112233445566778899aabbccddeeff", "9acc237dff16d76c20ef7c919e3a7509"),
])
def test_rfc3713_vectors(key, ct):
    assert O.camellia_encrypt_block(h(key), h("0123456789abcdeffedcba9876543210")).hex() == ct


@needs_ssl
def test_camellia_vs_openssl_ecb():
    for i in range(48):
        r = prng_bytes(0xCA + i, 48)
        key, blk = r[:(16, 24, 32)[i % 3]], r[32:48]
        assert O.camellia_encrypt_block(key, blk) == S.camellia(key, blk)


def _gmul(x, y):
    r, v = 0, y
    for i in range(127, -1, -1):
        if (x >> i) & 1:
            r ^= v
        v = (v >> 1) ^ (0xE1 << 120) if v & 1 else v >> 1
    return r


def _ghash(hk, aad, ct):
    def blocks(b):
        b = b + bytes(-len(b) % 16)
        return [int.from_bytes(b[i:i + 16], "big") for i in range(0, len(b), 16)]
    y = 0
    for blk in blocks(aad) + blocks(ct) + [(len(aad) * 8 << 64) | (len(ct) * 8)]:
        y = _gmul(y ^ blk, hk)
    return y


def gcm_ref(key, nonce, aad, pt):
    """SP 800-38D over OpenSSL Camellia-ECB (96-bit IV)."""
    hk = int.from_bytes(S.camellia(key, bytes(16)), "big")
    nb = (len(pt) + 15) // 16
    ctrs = b"".join(nonce + (i + 2).to_bytes(4, "big") for i in range(nb))
    ks = S.camellia(key, ctrs) if nb else b""
    ct = bytes(a ^ b for a, b in zip(pt, ks))
    ej0 = int.from_bytes(S.camellia(key, nonce + b"\0\0\0\1"), "big")
    return ct, (ej0 ^ _ghash(hk, aad, ct)).to_bytes(16, "big")


def ccm_ref(key, nonce, aad, pt, tag_len=16):
    """SP 800-38C over OpenSSL Camellia-ECB / -CBC (13-byte nonce would be L=2;
    TLS uses 12 bytes -> L = 3)."""
    q = 15 - len(nonce)
    b0 = bytes([(0x40 if aad else 0) | ((tag_len - 2) // 2) << 3 | (q - 1)]) + nonce + len(pt).to_bytes(q, "big")
    a = len(aad).to_bytes(2, "big") + aad if aad else b""
    mac_in = b0 + a + bytes(-len(a) % 16) + pt + bytes(-len(pt) % 16)
    mac = S.camellia(key, mac_in, "cbc", bytes(16))[-16:]
    nb = (len(pt) + 15) // 16
    ctr = lambda i: bytes([q - 1]) + nonce + i.to_bytes(q, "big")
    ks = S.camellia(key, b"".join(ctr(i + 1) for i in range(nb))) if nb else b""
    ct = bytes(x ^ y for x, y in zip(pt, ks))
    s0 = S.camellia(key, ctr(0))
    return ct, bytes(x ^ y for x, y in zip(mac, s0))[:tag_len]


@needs_ssl
def test_camellia_gcm_raw():
    for n in (0, 1, 15, 16, 17, 64, 1000):
        r = prng_bytes(0xC6 + n, 64)
        key, nonce, aad, pt = r[:32], r[32:44], r[44:57], prng_bytes(n + 5, n)
        assert O.aria_gcm_encrypt(key, nonce, aad, pt, bc=2) == gcm_ref(key, nonce, aad, pt)


@needs_ssl
@pytest.mark.parametrize("cipher", list(CAM.values()), ids=list(CAM))
def test_camellia_records_vs_openssl(cipher):
    """TLS 1.2 Camellia-GCM / -CCM records: explicit nonce = seq, AAD = seq|type|ver|len16."""
    kl = O.KEYLEN[cipher]
    for n in (0, 1, 16, 100, 1400, 16384):
        rnd = prng_bytes(0xCB + n + cipher, 64)
        key, iv, ctr = rnd[:kl], rnd[32:48], rnd[48:56]
        t = O.Transform(O.TLS1_2, cipher, key, key, iv, iv)
        content = prng_bytes(n, n)
        buf = bytearray(8 + n + 16)
        buf[8:8 + n] = content
        rec = O.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=buf, data_offset=8, data_len=n)
        assert t.encrypt_buf(rec) == 0
        aad = ctr + b"\x17\x03\x03" + n.to_bytes(2, "big")
        ref = ccm_ref if cipher >= O.CAMELLIA_128_CCM else gcm_ref
        ct, tag = ref(key, iv[:4] + ctr, aad, content)
        assert rec.data() == ctr + ct + tag


def _pair(cipher, ver):
    kl = O.KEYLEN[cipher]
    key0, key1 = bytes([1]) * kl, bytes([2]) * kl
    ive, ivd = bytes([3]) * 16, bytes([4]) * 16
    return O.Transform(ver, cipher, key0, key1, ive, ivd), O.Transform(ver, cipher, key1, key0, ivd, ive)


@pytest.mark.parametrize("cipher", list(CAM.values()), ids=list(CAM))
@pytest.mark.parametrize("ver", [O.TLS1_2, O.TLS1_3], ids=["tls12", "tls13"])
def test_crypt_record_camellia(cipher, ver):
    """ssl_crypt_record (test_suite_ssl.function:1567-1695) for Camellia AEADs."""
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


@pytest.mark.parametrize("cipher", list(CAM.values()), ids=list(CAM))
def test_crypt_record_camellia_cid(cipher):
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
