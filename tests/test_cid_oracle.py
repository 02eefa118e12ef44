"""DTLS 1.2 connection-ID records in the CPU restatement.

The reference's CID path of mbedtls_ssl_encrypt_buf / _decrypt_buf:
  - encrypt: rec->cid = transform->out_cid (ssl_msg.c:874-875); with a CID the
    content is wrapped as DTLSInnerPlaintext (content || real type || zeros to
    the padding granularity, :878-897, :466-491) and the outer type becomes
    MBEDTLS_SSL_MSG_CID = 25;
  - AAD (RFC 9146, ssl_msg.c:683-724): 0xff x 8 || 25 || cid_len || 25 ||
    version || epoch+seq || cid || len(DTLSInnerPlaintext);
  - decrypt: the record's CID must equal transform->in_cid, else
    MBEDTLS_ERR_SSL_UNEXPECTED_CID (:1313-1320); after the AEAD the inner
    plaintext is parsed, all-zero -> INVALID_RECORD (:1821-1829).
Pinned by the reference's ssl_crypt_record / ssl_crypt_record_small cases with
cid lengths 4:4 and 4:0 (test_suite_ssl.data, e.g. :1465, :2337-2341; CIDs
are random, ssl_helpers.c:1384-1388, 1569-1576) and by OpenSSL sealing the
inner plaintext under an AAD assembled here from RFC 9146 (the reference ships
no CID ciphertext KAT: parity for the ciphertext bytes is pinned by OpenSSL +
the RFC 9146 AAD layout, not by a reference vector).
"""
import pytest

import oracle as O
from tests import _openssl as S
from tests.prng import prng_bytes

CID_TYPE = 25
ERR_UNEXPECTED_CID = -0x6000
CIPHERS = {"aes128gcm": O.AES_128_GCM, "aes192gcm": O.AES_192_GCM, "aes256gcm": O.AES_256_GCM,
           "chachapoly": O.CHACHA20_POLY1305, "aes128ccm": O.AES_128_CCM, "aes256ccm": O.AES_256_CCM,
           "aes128ccm8": O.AES_128_CCM_8, "aes256ccm8": O.AES_256_CCM_8}


def build_cid_transforms(cipher, cid0_len, cid1_len, seed=7):
    """mbedtls_test_ssl_build_transforms with CIDs (ssl_helpers.c:1361-1651):
    t_in: in = cid0, out = cid1; t_out: in = cid1, out = cid0."""
    kl = O.KEYLEN[cipher]
    key0, key1 = bytes([1]) * kl, bytes([2]) * kl
    ive, ivd = bytes([3]) * 16, bytes([4]) * 16
    cid0, cid1 = prng_bytes(seed, 4)[:cid0_len], prng_bytes(seed + 1, 4)[:cid1_len]
    t_in = O.Transform(O.TLS1_2, cipher, key0, key1, ive, ivd)
    t_out = O.Transform(O.TLS1_2, cipher, key1, key0, ivd, ive)
    t_in.set_cid(cid0, cid1)
    t_out.set_cid(cid1, cid0)
    return t_in, t_out


def rfc9146_aad(rec_type, ver, ctr, cid, inner_len):
    return (b"\xff" * 8 + bytes([rec_type, len(cid), rec_type]) + bytes(ver) + bytes(ctr) + bytes(cid)
            + inner_len.to_bytes(2, "big"))


@pytest.mark.parametrize("cipher", list(CIPHERS.values()), ids=list(CIPHERS))
@pytest.mark.parametrize("cids", [(4, 4), (4, 0), (0, 4)], ids=["4:4", "4:0", "0:4"])
def test_crypt_record_cid(cipher, cids):
    """ssl_crypt_record (test_suite_ssl.function:1567-1695) with CIDs."""
    t0, t1 = build_cid_transforms(cipher, *cids)
    for n in range(15, -1, -1):
        t_dec, t_enc = (t0, t1) if n % 3 == 0 else (t1, t0)
        buf = bytearray(512)
        rec = O.Record(ctr=bytes([n]) * 8, type=42, ver=bytes([n, n]), buf=buf, data_offset=16, data_len=1 + n)
        buf[16:17 + n] = bytes([42]) * (1 + n)
        assert t_enc.encrypt_buf(rec) == 0
        if rec.cid:
            assert rec.type == CID_TYPE                      # test_suite_ssl.function:1651-1657
        assert t_dec.decrypt_buf(rec) == 0
        assert (rec.type, rec.ver, rec.data_offset, rec.data_len) == (42, bytes([n, n]), 16, 1 + n)
        assert rec.data() == bytes([42]) * (1 + n)


@pytest.mark.parametrize("cipher", list(CIPHERS.values()), ids=list(CIPHERS))
def test_crypt_record_small_cid(cipher):
    """ssl_crypt_record_small (test_suite_ssl.function:1697-1856), cids 4:4."""
    t0, t1 = build_cid_transforms(cipher, 4, 4)
    buflen = 256
    for mode in (1, 2, 3):
        seen = False
        for off in range(0, 97):
            do, dl = {1: (off, buflen - off - 128), 2: (64, buflen - 64 - off), 3: (off, buflen - 2 * off)}[mode]
            buf = bytearray(buflen)
            buf[do:do + dl] = bytes([42]) * dl
            rec = O.Record(ctr=bytes([off]) * 8, type=42, ver=bytes([off, off]), buf=buf, data_offset=do, data_len=dl)
            r = t1.encrypt_buf(rec)
            if r == O.ERR_BUFFER_TOO_SMALL:
                continue
            assert r == 0
            seen = True
            assert t0.decrypt_buf(rec) == 0
            assert (rec.type, rec.data_offset, rec.data_len) == (42, do, dl)
        assert seen


@pytest.mark.skipif(S.lib() is None, reason="libcrypto not present")
@pytest.mark.parametrize("cipher", list(CIPHERS.values()), ids=list(CIPHERS))
def test_cid_records_vs_openssl(cipher):
    """Ciphertext bytes: OpenSSL seals the DTLSInnerPlaintext under the RFC 9146
    AAD and the nonce of ssl_build_record_nonce (ssl_msg.c:768-781)."""
    for i, (n, cid_len) in enumerate([(0, 1), (1, 4), (14, 4), (15, 8), (31, 16), (200, 32), (1400, 5)]):
        kl = O.KEYLEN[cipher]
        rnd = prng_bytes(0x51D + 97 * i + cipher, 96)
        key, iv, ctr, cid = rnd[:kl], rnd[32:48], rnd[48:56], rnd[56:56 + cid_len]
        t = O.Transform(O.TLS1_2, cipher, key, key, iv, iv)
        t.set_cid(cid, cid)
        head = 8 if cipher != O.CHACHA20_POLY1305 else 0
        content = prng_bytes(i, n)
        buf = bytearray(head + n + 64)
        buf[head:head + n] = content
        rec = O.Record(ctr=ctr, type=23, ver=b"\xfe\xfd", buf=buf, data_offset=head, data_len=n)
        assert t.encrypt_buf(rec) == 0
        assert rec.type == CID_TYPE and rec.cid == cid
        pad = (16 - (n + 1) % 16) % 16
        inner = content + b"\x17" + bytes(pad)
        aad = rfc9146_aad(CID_TYPE, b"\xfe\xfd", ctr, cid, len(inner))
        if cipher == O.CHACHA20_POLY1305:
            nonce = bytes(a ^ b for a, b in zip(iv[:12], bytes(4) + ctr))
            ct, tag = S.seal("chacha", key, nonce, aad, inner)
        else:
            nonce = iv[:4] + ctr
            if cipher in (O.AES_128_GCM, O.AES_192_GCM, O.AES_256_GCM):
                ct, tag = S.seal("gcm", key, nonce, aad, inner)
            else:
                ct, tag = S.ccm_seal(key, nonce, aad, inner, O.TAGLEN[cipher])
        want = (ctr if head else b"") + ct + tag
        assert rec.data() == want, (cipher, n, cid_len)


@pytest.mark.parametrize("cipher", [O.AES_128_GCM, O.CHACHA20_POLY1305, O.AES_128_CCM_8])
def test_cid_negative(cipher):
    t0, t1 = build_cid_transforms(cipher, 4, 4)
    # a record whose CID differs from in_cid (length or bytes): UNEXPECTED_CID, untouched
    for bad in (b"", b"\x00\x01\x02", None):
        buf = bytearray(128)
        rec = O.Record(ctr=bytes(8), type=23, ver=b"\xfe\xfd", buf=buf, data_offset=8, data_len=20)
        assert t1.encrypt_buf(rec) == 0
        rec.cid = bytes([rec.cid[0] ^ 1]) + rec.cid[1:] if bad is None else bad
        snap = bytes(buf)
        assert t0.decrypt_buf(rec) == ERR_UNEXPECTED_CID
        assert bytes(buf) == snap
    # an all-zero DTLSInnerPlaintext authenticates but is INVALID_RECORD
    kl = O.KEYLEN[cipher]
    key, iv, ctr, cid = bytes([9]) * kl, bytes([5]) * 16, bytes([0, 1, 0, 0, 0, 0, 0, 7]), b"\xc1\xd0"
    t = O.Transform(O.TLS1_2, cipher, key, key, iv, iv)
    t.set_cid(cid, cid)
    inner = bytes(16)
    aad = rfc9146_aad(CID_TYPE, b"\xfe\xfd", ctr, cid, len(inner))
    if cipher == O.CHACHA20_POLY1305:
        ct, tag = O.chachapoly_encrypt(key, bytes(a ^ b for a, b in zip(iv[:12], bytes(4) + ctr)), aad, inner)
        wire = ct + tag
    elif cipher == O.AES_128_GCM:
        ct, tag = O.gcm_encrypt(key, iv[:4] + ctr, aad, inner)
        wire = ctr + ct + tag
    else:
        ct, tag = O.ccm_encrypt(key, iv[:4] + ctr, aad, inner, 8)
        wire = ctr + ct + tag
    buf = bytearray(wire)
    rec = O.Record(ctr=ctr, type=CID_TYPE, ver=b"\xfe\xfd", buf=buf, data_offset=0, data_len=len(buf), cid=cid)
    assert t.decrypt_buf(rec) == O.ERR_INVALID_RECORD
