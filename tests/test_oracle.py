"""Pin the CPU restatement (oracle/) before trusting it as the GPU checker.

1. the reference's own TLS 1.3 record KATs (test_suite_ssl.data:2776-2834),
   run at padding granularity 1 exactly as ssl_tls13_record_protection does
   when padding_used == granularity (test_suite_ssl.function:2201-2299);
2. published standards vectors (FIPS-197, GCM spec, RFC 8439);
3. the committed record fixtures (oracle output cross-checked against
   OpenSSL at generation time), re-derived here;
4. the round-trip semantics of ssl_crypt_record / ssl_crypt_record_small
   (test_suite_ssl.function:1567-1856) with the mbedtls_test_ssl_build_
   transforms fixtures (tests/src/test_helpers/ssl_helpers.c:1361-1651);
5. AEAD negative cases the reference does not test.
"""
import hashlib
import json
import os

import pytest

import oracle as O
from tests import _openssl as S
from tests.prng import prng_bytes

G = os.path.join(os.path.dirname(__file__), "golden")
h = bytes.fromhex


def _load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)


@pytest.mark.parametrize("kat", _load("reference_kats.json"), ids=lambda k: k["name"])
def test_reference_record_kats(kat):
    sk, si, ck, ci = (h(kat[x]) for x in ("server_key", "server_iv", "client_key", "client_iv"))
    # mbedtls_ssl_tls13_populate_transform: the sender writes with its own keys
    if kat["endpoint"] == "client":
        send = O.Transform(O.TLS1_3, O.AES_128_GCM, ck, sk, ci, si, granularity=1)
        recv = O.Transform(O.TLS1_3, O.AES_128_GCM, sk, ck, si, ci, granularity=1)
    else:
        send = O.Transform(O.TLS1_3, O.AES_128_GCM, sk, ck, si, ci, granularity=1)
        recv = O.Transform(O.TLS1_3, O.AES_128_GCM, ck, sk, ci, si, granularity=1)
    pt, ct = h(kat["plaintext"]), h(kat["ciphertext"])
    buf = bytearray(len(ct) + 16)
    buf[:len(pt)] = pt
    rec = O.Record(ctr=bytes(7) + bytes([kat["ctr"]]), type=23, ver=b"\x03\x03",
                   buf=buf, data_offset=0, data_len=len(pt))
    assert send.encrypt_buf(rec) == 0
    assert rec.data() == ct
    assert rec.type == 23
    assert recv.decrypt_buf(rec) == 0
    assert rec.data() == pt and rec.type == 23


def test_standard_vectors():
    s = _load("standard_vectors.json")
    for v in s["aes_block"]:
        assert O.aes_encrypt_block(h(v["key"]), h(v["pt"])).hex() == v["ct"]
    for v in s["gcm"]:
        ct, tag = O.gcm_encrypt(h(v["key"]), h(v["iv"]), h(v["aad"]), h(v["pt"]))
        assert (ct.hex(), tag.hex()) == (v["ct"], v["tag"])
        r, pt = O.gcm_decrypt(h(v["key"]), h(v["iv"]), h(v["aad"]), ct, tag)
        assert r == 0 and pt.hex() == v["pt"]
    for v in s["ccm"]:
        ct, tag = O.ccm_encrypt(h(v["key"]), h(v["nonce"]), h(v["aad"]), h(v["pt"]), len(h(v["tag"])))
        assert (ct.hex(), tag.hex()) == (v["ct"], v["tag"])
    for v in s["chacha20_block"]:
        assert O.chacha20_block(h(v["key"]), v["counter"], h(v["nonce"]))[:16].hex() == v["out16"]
    for v in s["poly1305"]:
        assert O.poly1305(h(v["key"]), h(v["msg"])).hex() == v["tag"]
    for v in s["chachapoly"]:
        ct, tag = O.chachapoly_encrypt(h(v["key"]), h(v["nonce"]), h(v["aad"]), h(v["pt"]))
        assert ct[:16].hex() == v["ct16"] and tag.hex() == v["tag"]


CIPHERS = {"AES-128-GCM": O.AES_128_GCM, "AES-256-GCM": O.AES_256_GCM,
           "CHACHA20-POLY1305": O.CHACHA20_POLY1305, "AES-192-GCM": O.AES_192_GCM,
           "AES-128-CCM": O.AES_128_CCM, "AES-192-CCM": O.AES_192_CCM, "AES-256-CCM": O.AES_256_CCM,
           "AES-128-CCM-8": O.AES_128_CCM_8, "AES-192-CCM-8": O.AES_192_CCM_8, "AES-256-CCM-8": O.AES_256_CCM_8,
           "ARIA-128-GCM": O.ARIA_128_GCM, "ARIA-192-GCM": O.ARIA_192_GCM, "ARIA-256-GCM": O.ARIA_256_GCM,
           "ARIA-128-CCM": O.ARIA_128_CCM, "ARIA-192-CCM": O.ARIA_192_CCM, "ARIA-256-CCM": O.ARIA_256_CCM,
           "CAMELLIA-128-GCM": O.CAMELLIA_128_GCM, "CAMELLIA-192-GCM": O.CAMELLIA_192_GCM,
           "CAMELLIA-256-GCM": O.CAMELLIA_256_GCM, "CAMELLIA-128-CCM": O.CAMELLIA_128_CCM,
           "CAMELLIA-192-CCM": O.CAMELLIA_192_CCM, "CAMELLIA-256-CCM": O.CAMELLIA_256_CCM}
VERSIONS = {"TLS1.2": O.TLS1_2, "TLS1.3": O.TLS1_3}


def test_record_fixtures():
    fx = _load("records.json")
    for c in fx["cases"]:
        cipher, ver = CIPHERS[c["cipher"]], VERSIONS[c["version"]]
        t = O.Transform(ver, cipher, h(c["key_enc"]), h(c["key_dec"]), h(c["iv_enc"]), h(c["iv_dec"]))
        L = c["len"]
        payload = prng_bytes(c["seed"] ^ 0xA5A5, L)
        head = 8 if (ver == O.TLS1_2 and cipher != O.CHACHA20_POLY1305) else 0
        buf = bytearray(head + L + 64)
        buf[head:head + L] = payload
        rec = O.Record(ctr=h(c["ctr"]), type=c["type"], ver=b"\x03\x03", buf=buf,
                       data_offset=head, data_len=L)
        assert t.encrypt_buf(rec) == 0
        assert (rec.data_offset, rec.data_len, rec.type) == (c["out_offset"], c["out_len"], c["out_type"])
        assert hashlib.sha256(rec.data()).hexdigest() == c["wire_sha256"]
        # decrypt with the peer transform (keys swapped) restores the record
        peer = O.Transform(ver, cipher, h(c["key_dec"]), h(c["key_enc"]), h(c["iv_dec"]), h(c["iv_enc"]))
        assert peer.decrypt_buf(rec) == 0
        assert rec.data() == payload and rec.type == c["type"] and rec.data_offset == head


def _build_transforms(cipher, ver):
    """mbedtls_test_ssl_build_transforms (ssl_helpers.c:1361-1651): key0 =
    0x01.., key1 = 0x02.., iv_enc = 0x03.., iv_dec = 0x04.."""
    kl = O.KEYLEN[cipher]
    key0, key1 = bytes([1]) * kl, bytes([2]) * kl
    ive, ivd = bytes([3]) * 16, bytes([4]) * 16
    t_in = O.Transform(ver, cipher, key0, key1, ive, ivd)
    t_out = O.Transform(ver, cipher, key1, key0, ivd, ive)
    return t_in, t_out


@pytest.mark.parametrize("cipher", list(CIPHERS.values()), ids=list(CIPHERS))
@pytest.mark.parametrize("ver", list(VERSIONS.values()), ids=list(VERSIONS))
def test_crypt_record_semantics(cipher, ver):
    """ssl_crypt_record (test_suite_ssl.function:1567-1695)."""
    t0, t1 = _build_transforms(cipher, ver)
    for n in range(15, -1, -1):
        t_dec, t_enc = (t0, t1) if n % 3 == 0 else (t1, t0)
        buf = bytearray(512)
        rec = O.Record(ctr=bytes([n]) * 8, type=42, ver=bytes([n, n]), buf=buf,
                       data_offset=16, data_len=1 + n)
        buf[16:17 + n] = bytes([42]) * (1 + n)
        r = t_enc.encrypt_buf(rec)
        assert r == 0
        if ver == O.TLS1_3:
            assert rec.type == 23
        assert t_dec.decrypt_buf(rec) == 0
        assert (rec.type, rec.ver, rec.data_offset, rec.data_len) == (42, bytes([n, n]), 16, 1 + n)
        assert rec.data() == bytes([42]) * (1 + n)


@pytest.mark.parametrize("cipher", list(CIPHERS.values()), ids=list(CIPHERS))
@pytest.mark.parametrize("ver", list(VERSIONS.values()), ids=list(VERSIONS))
def test_crypt_record_small_semantics(cipher, ver):
    """ssl_crypt_record_small (test_suite_ssl.function:1697-1856): every mode
    must see at least one success; failures must be BUFFER_TOO_SMALL."""
    t0, t1 = _build_transforms(cipher, ver)
    buflen = 256
    for mode in (1, 2, 3):
        seen = False
        for off in range(0, 97):
            if mode == 1:
                do, dl = off, buflen - off - 128
            elif mode == 2:
                do, dl = 64, buflen - 64 - off
            else:
                do, dl = off, buflen - 2 * off
            buf = bytearray(buflen)
            buf[do:do + dl] = bytes([42]) * dl
            rec = O.Record(ctr=bytes([off]) * 8, type=42, ver=bytes([off, off]), buf=buf,
                           data_offset=do, data_len=dl)
            r = t1.encrypt_buf(rec)
            if r == O.ERR_BUFFER_TOO_SMALL:
                continue
            assert r == 0
            seen = True
            assert t0.decrypt_buf(rec) == 0
            assert (rec.type, rec.data_offset, rec.data_len) == (42, do, dl)
            assert rec.data() == bytes([42]) * dl
        assert seen


@pytest.mark.parametrize("cipher", list(CIPHERS.values()), ids=list(CIPHERS))
@pytest.mark.parametrize("ver", list(VERSIONS.values()), ids=list(VERSIONS))
def test_negative(cipher, ver):
    t0, t1 = _build_transforms(cipher, ver)
    head = 8 if (ver == O.TLS1_2 and cipher != O.CHACHA20_POLY1305) else 0

    def sealed(n=40):
        buf = bytearray(256)
        rec = O.Record(ctr=bytes(8), type=23, ver=b"\x03\x03", buf=buf, data_offset=head, data_len=n)
        buf[head:head + n] = bytes(range(n))
        assert t1.encrypt_buf(rec) == 0
        return rec

    # bit flips in ciphertext, tag, AAD fields, and nonce (ctr) -> INVALID_MAC
    for where in ("ct", "tag", "type", "ver", "ctr"):
        rec = sealed()
        if where == "ct":
            rec.buf[rec.data_offset + head + 1] ^= 1
        elif where == "tag":
            rec.buf[rec.data_offset + rec.data_len - 1] ^= 0x80
        elif where == "type":
            rec.type ^= 1
        elif where == "ver":
            rec.ver = bytes([rec.ver[0], rec.ver[1] ^ 1])
        else:
            rec.ctr = bytes(7) + b"\x01"
        if where == "ctr" and ver == O.TLS1_2 and cipher != O.CHACHA20_POLY1305:
            # explicit nonce travels in the record; ctr only enters the AAD
            pass
        assert t0.decrypt_buf(rec) == O.ERR_INVALID_MAC
        # PSA wipes the output buffer on authentication failure
        assert all(b == 0 for b in rec.buf[rec.data_offset:])
    # shorter than the tag -> INVALID_MAC (ssl_msg.c:1371-1377)
    buf = bytearray(64)
    rec = O.Record(ctr=bytes(8), type=23, ver=b"\x03\x03", buf=buf, data_offset=0, data_len=head + 15)
    assert t0.decrypt_buf(rec) == O.ERR_INVALID_MAC
    # oversize content -> BAD_INPUT_DATA (ssl_msg.c:831-839)
    buf = bytearray(16384 + 64)
    rec = O.Record(ctr=bytes(8), type=23, ver=b"\x03\x03", buf=buf, data_offset=head, data_len=16385)
    assert t1.encrypt_buf(rec) == O.ERR_BAD_INPUT_DATA


def test_all_zero_inner_plaintext_is_invalid_record():
    """TLS 1.3 inner plaintext with no non-zero byte (ssl_msg.c:1812-1817)."""
    key, iv = bytes([7]) * 32, bytes([9]) * 16
    for cipher, name in ((O.AES_256_GCM, "gcm"), (O.CHACHA20_POLY1305, "chacha")):
        inner = bytes(32)
        ctr = bytes(8)
        aad = bytes([23, 3, 3]) + (len(inner) + 16).to_bytes(2, "big")
        nonce = iv[:12]
        if S.lib() is not None:
            ct, tag = S.seal(name, key, nonce, aad, inner)
        else:
            ct, tag = (O.gcm_encrypt(key, nonce, aad, inner) if name == "gcm"
                       else O.chachapoly_encrypt(key, nonce, aad, inner))
        t = O.Transform(O.TLS1_3, cipher, key, key, iv, iv)
        buf = bytearray(ct + tag)
        rec = O.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=buf, data_offset=0, data_len=len(buf))
        assert t.decrypt_buf(rec) == O.ERR_INVALID_RECORD


@pytest.mark.skipif(S.lib() is None, reason="libcrypto not present")
def test_differential_openssl():
    for i in range(300):
        rnd = prng_bytes(0x1234 + i, 64)
        L = [0, 1, 15, 16, 17, 255, 1400, 4097][i % 8]
        pt = prng_bytes(i, L)
        aad = rnd[44:44 + (i % 14)]
        nonce = rnd[32:44]
        for kl in (16, 32):
            assert O.gcm_encrypt(rnd[:kl], nonce, aad, pt) == S.seal("gcm", rnd[:kl], nonce, aad, pt)
        assert O.chachapoly_encrypt(rnd[:32], nonce, aad, pt) == S.seal("chacha", rnd[:32], nonce, aad, pt)
