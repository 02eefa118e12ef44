"""DTLS 1.2 datagram record loops in the CPU restatement (oracle/dtls.c).

Pinned by
  - the reference's 19 anti-replay vectors (test_suite_ssl.data:763-818,
    ssl_dtls_replay, test_suite_ssl.function:1510-1541), transcribed into
    tests/golden/dtls_replay.json by tests/golden/make_dtls_replay.py;
  - OpenSSL EVP opening every DTLS record the write loop produces under the
    TLS 1.2 AEAD rules with the DTLS header fields (nonce = fixed IV ||
    epoch+seq for GCM/CCM, fixed IV ^ epoch+seq for ChaCha20-Poly1305, AAD =
    epoch+seq || type || FE FD || length, ssl_msg.c:568-781) -- the reference
    ships no DTLS record ciphertext KAT, so the record bytes are pinned by
    OpenSSL + the RFC 6347 header layout, not by a reference vector;
  - the read loop's dispositions, stated here case by case from
    ssl_get_next_record / ssl_parse_record_header / ssl_prepare_record_content.
"""
import json
import os

import pytest

import oracle as O
from tests import _openssl as S
from tests.prng import prng_bytes

REPLAY = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dtls_replay.json")))["cases"]
X = bytes.fromhex
INV_REC, INV_MAC = -0x7200, -0x7180
ERR_INTERNAL = -0x6C00
ERR_UNEXPECTED_CID = -0x6000


def state(**kw):
    st = O.DtlsState()
    st.anti_replay = 1
    for k, v in kw.items():
        setattr(st, k, v)
    return st


@pytest.mark.parametrize("case", REPLAY, ids=lambda c: c["name"])
def test_reference_replay_vectors(case):
    st = state()
    for p in case["prevs"]:
        O.dtls_replay_update(st, bytes(2) + X(p))
    assert O.dtls_replay_check(st, bytes(2) + X(case["new"])) == case["ret"]


def pair(cipher, seed=1, cid=b""):
    kl = O.KEYLEN[cipher]
    key, iv = prng_bytes(seed, kl), prng_bytes(seed + 1, 16)
    t_out = O.Transform(O.TLS1_2, cipher, key, key, iv, iv)
    t_in = O.Transform(O.TLS1_2, cipher, key, key, iv, iv)
    if cid:
        t_out.set_cid(b"", cid)
        t_in.set_cid(cid, b"")
    return t_out, t_in


def ctr(epoch, seq):
    return epoch.to_bytes(2, "big") + seq.to_bytes(6, "big")


def records(t_out, n, epoch=1, seq0=0, size=300, typ=23, seed=5):
    """n single-record datagrams (one mbedtls_ssl_write each)."""
    out = []
    for k in range(n):
        st, w, nrec, _ = O.dtls_encrypt(t_out, prng_bytes(seed + k, size), typ, ctr(epoch, seq0 + k), 16384)
        assert st == 0 and nrec == 1
        out.append(w)
    return out


OSSL = {O.AES_128_GCM: "gcm", O.AES_256_GCM: "gcm", O.CHACHA20_POLY1305: "chacha20-poly1305",
        O.AES_128_CCM: "ccm", O.AES_128_CCM_8: "ccm"}


@pytest.mark.parametrize("cipher", list(OSSL), ids=["aes128gcm", "aes256gcm", "chachapoly", "aes128ccm", "ccm8"])
def test_dtls_records_vs_openssl(cipher):
    kl = O.KEYLEN[cipher]
    key, iv = prng_bytes(11, kl), prng_bytes(12, 16)
    t = O.Transform(O.TLS1_2, cipher, key, key, iv, iv)
    pt = prng_bytes(13, 1000)
    c = ctr(3, 0x123456789A)
    st, w, nrec, after = O.dtls_encrypt(t, pt, 23, c, 400)
    assert st == 0 and nrec == 3
    assert after == ctr(3, 0x123456789A + 3)
    pos = 0
    for k in range(3):
        h = w[pos:pos + 13]
        n = min(400, 1000 - 400 * k)
        ck = ctr(3, 0x123456789A + k)
        assert h[0] == 23 and h[1:3] == b"\xfe\xfd" and h[3:11] == ck
        body = int.from_bytes(h[11:13], "big")
        rec = w[pos + 13:pos + 13 + body]
        aad = ck + bytes([23, 0xfe, 0xfd]) + n.to_bytes(2, "big")
        taglen = 8 if cipher == O.AES_128_CCM_8 else 16
        if cipher == O.CHACHA20_POLY1305:
            nonce = bytes(a ^ b for a, b in zip(iv[:12], bytes(4) + ck))
            ct, tag = rec[:-16], rec[-16:]
            assert S.open_("chacha20-poly1305", key, nonce, aad, ct, tag) == pt[400 * k:400 * k + n]
        else:
            assert rec[:8] == ck                     # explicit IV = record sequence number
            nonce = iv[:4] + rec[:8]
            ct, tag = rec[8:-taglen], rec[-taglen:]
            if cipher in (O.AES_128_CCM, O.AES_128_CCM_8):
                want_ct, want_tag = S.ccm_seal(key, nonce, aad, pt[400 * k:400 * k + n], taglen)
                assert (ct, tag) == (want_ct, want_tag)
            else:
                assert S.open_(OSSL[cipher], key, nonce, aad, ct, tag) == pt[400 * k:400 * k + n]
        pos += 13 + body
    assert pos == len(w)


@pytest.mark.parametrize("cipher", [O.AES_128_GCM, O.AES_256_GCM, O.CHACHA20_POLY1305, O.AES_256_CCM_8,
                                    O.ARIA_128_GCM, O.CAMELLIA_256_CCM])
@pytest.mark.parametrize("cid", [b"", b"\x01\x02\x03\x04"], ids=["nocid", "cid4"])
def test_round_trip(cipher, cid):
    t_out, t_in = pair(cipher, cid=cid)
    dgs = records(t_out, 5)
    # two records packed in one datagram as well
    dgs = dgs[:3] + [dgs[3] + dgs[4]]
    st = state(in_epoch=1, cid_len=len(cid))
    res, recs, after = O.dtls_decrypt(t_in, st, dgs)
    assert res["status"] == 0 and res["naccepted"] == 5 and res["nrec"] == 5 and res["dgrams_done"] == 4
    assert [r[4] for r in recs] == [0] * 5
    assert (st.window_top, st.window) == (4, 0b11111)
    for k, (dg, off, doff, dlen, disp, typ) in enumerate(recs):
        assert typ == 23 and dlen == 300
        assert after[dg][off + doff:off + doff + dlen] == prng_bytes(5 + k, 300)
    if cid:
        assert dgs[0][0] == 25 and dgs[0][11:15] == cid


def test_dispositions():
    t_out, t_in = pair(O.AES_128_GCM)
    good = records(t_out, 8, epoch=1)
    old = records(t_out, 1, epoch=0, seq0=50)[0]
    nxt = records(t_out, 1, epoch=2, seq0=60)[0]
    bad = bytearray(good[2])
    bad[40] ^= 1
    dgs = [good[0], good[0],                       # replay: second copy skipped
           old, nxt,                               # other epochs: skipped
           bytes(bad) + good[3],                   # MAC failure drops the rest of the datagram
           good[3],                                # ... so the same record in a later datagram is new
           b"\x17\xfe\xfd" + bytes(8),             # 11 bytes: INVALID_RECORD, datagram dropped
           good[4] + b"\x40" + good[5][1:],        # bad type after a good record: rest dropped
           good[5], good[2]]
    st = state(in_epoch=1)
    res, recs, _ = O.dtls_decrypt(t_in, st, dgs)
    disp = [r[4] for r in recs]
    assert disp == [0, O.ERR_UNEXPECTED_RECORD, O.ERR_UNEXPECTED_RECORD, O.ERR_EARLY_MESSAGE, INV_MAC,
                    O.DTLS_DROPPED, 0, 0, 0, 0], disp
    assert res == {"status": 0, "nrec": 10, "naccepted": 5, "dgrams_done": len(dgs), "invalid_dgrams": 2}
    assert st.badmac_seen == 0                     # counted only with a limit (ssl_msg.c:4857-4858)


def test_badmac_limit_and_fatal_errors():
    t_out, t_in = pair(O.AES_256_GCM)
    good = records(t_out, 6)
    bad = [bytearray(g) for g in good]
    for b in bad:
        b[30] ^= 4
    st = state(in_epoch=1, badmac_limit=2)
    res, recs, _ = O.dtls_decrypt(t_in, st, [good[0], bytes(bad[1]), good[2], bytes(bad[3]), good[4], good[5]])
    assert res["status"] == INV_MAC and res["naccepted"] == 2 and res["dgrams_done"] == 3
    assert [r[4] for r in recs] == [0, INV_MAC, 0, INV_MAC, O.DTLS_NOT_REACHED, O.DTLS_NOT_REACHED]
    assert st.badmac_seen == 2
    # trailing 1..12 bytes after a record: fetch_input's INTERNAL_ERROR (ssl_msg.c:1921-1926)
    st = state(in_epoch=1)
    res, recs, _ = O.dtls_decrypt(t_in, st, [good[0] + b"\x17\xfe\xfd", good[1]])
    assert res["status"] == ERR_INTERNAL and [r[4] for r in recs] == [0, O.DTLS_NOT_REACHED]
    # an empty datagram is CONN_EOF
    res, _, _ = O.dtls_decrypt(t_in, state(in_epoch=1), [b""])
    assert res["status"] == O.ERR_CONN_EOF


def test_cid_rules():
    cid = b"\xaa\xbb\xcc"
    t_out, t_in = pair(O.CHACHA20_POLY1305, cid=cid)
    plain_out, _ = pair(O.CHACHA20_POLY1305)
    with_cid = records(t_out, 2)
    no_cid = records(plain_out, 1, seq0=7)[0]
    # the endpoint expects CIDs: a record without one is UNEXPECTED_CID, fatal unless ignored
    for ignore, want in ((1, 0), (0, ERR_UNEXPECTED_CID)):
        st = state(in_epoch=1, cid_len=3, ignore_unexpected_cid=ignore)
        res, recs, _ = O.dtls_decrypt(t_in, st, [with_cid[0], no_cid, with_cid[1]])
        assert res["status"] == want
        assert recs[1][4] == ERR_UNEXPECTED_CID
        assert [r[4] for r in recs][2] == (0 if ignore else O.DTLS_NOT_REACHED)
    # an endpoint without CIDs cannot parse a tls12_cid header: the datagram is dropped
    st = state(in_epoch=1, cid_len=0)
    res, recs, _ = O.dtls_decrypt(t_in, st, [with_cid[0]])
    assert res["status"] == 0 and res["nrec"] == 0 and res["invalid_dgrams"] == 1


def test_anti_replay_disabled_and_window_shift():
    t_out, t_in = pair(O.AES_128_GCM)
    a = records(t_out, 1, seq0=100)[0]
    b = records(t_out, 1, seq0=30)[0]
    res, recs, _ = O.dtls_decrypt(t_in, state(in_epoch=1), [a, b, a])
    assert [r[4] for r in recs] == [0, O.ERR_UNEXPECTED_RECORD, O.ERR_UNEXPECTED_RECORD]
    res, recs, _ = O.dtls_decrypt(t_in, state(in_epoch=1, anti_replay=0), [a, b, a])
    assert [r[4] for r in recs] == [0, 0, 0]


def test_version_check_quirk():
    """mbedtls_ssl_read_version's DTLS mapping wraps: FE FD -> TLS 1.2 passes,
    03 03 maps above TLS 1.2 and fails, 00 00 maps to 0x0200 and passes."""
    t_out, t_in = pair(O.AES_128_GCM)
    g = records(t_out, 1)[0]
    for v, ok in ((b"\xfe\xfd", True), (b"\xfe\xff", True), (b"\x03\x03", False), (b"\x00\x00", True)):
        res, recs, _ = O.dtls_decrypt(t_in, state(in_epoch=1), [g[:1] + v + g[3:]])
        if ok:   # parsed; the AAD carries the received version, so only FE FD authenticates
            assert res["nrec"] == 1 and recs[0][4] == (0 if v == b"\xfe\xfd" else INV_MAC)
        else:
            assert res["nrec"] == 0 and res["invalid_dgrams"] == 1
