"""The CPU legs of the SURVEY §8(f) rows: the oracle's
stream / DTLS record layers and key schedule timed over many connections
(oracle/rows_bench.c, the "port" leg) and the same framing around OpenSSL
EVP (oracle/evp_bench.c evp_mixed_stream, the "evp" leg).  Pinned here on
CPU: both legs send byte-identical record streams, each receives the
other's, and the threaded key schedule equals the one-call restatement."""
import numpy as np
import pytest

import oracle as O
from tests.prng import prng_array


def _conns(cipher, tls, C, seed):
    kl = O.KEYLEN[cipher]
    raw = prng_array(seed, C * 48).reshape(C, 48)
    keys = np.zeros((C, 32), dtype=np.uint8)
    keys[:, :kl] = raw[:, :kl]
    ivs = np.ascontiguousarray(raw[:, 32:44])
    ts = [O.Transform(tls, cipher, bytes(k[:kl]), bytes(k[:kl]), bytes(v) + bytes(4), bytes(v) + bytes(4))
          for k, v in zip(keys, ivs)]
    return keys, ivs, ts


@pytest.mark.parametrize("dtls,cipher,content,recs", [(False, O.AES_256_GCM, 1400, 16), (False, O.CHACHA20_POLY1305, 1400, 4),
                                                       (False, O.AES_128_GCM, 16384, 2), (True, O.AES_128_GCM, 1400, 16),
                                                       (True, O.CHACHA20_POLY1305, 1400, 8)])
def test_port_and_evp_legs_agree(dtls, cipher, content, recs):
    C = 37
    tls = O.TLS1_2 if dtls else O.TLS1_3
    keys, ivs, ts = _conns(cipher, tls, C, 0x5EED + cipher)
    per_in = recs * content
    wire = O.dtls_record_wire(ts[0], content) if dtls else O.stream_record_wire(ts[0], content)
    per_out = recs * wire
    in_stride = (per_in + 127) // 128 * 128
    out_stride = (per_out + 127) // 128 * 128
    pt = prng_array(7, C * in_stride).reshape(C, in_stride)
    out_port = np.zeros((C, out_stride), dtype=np.uint8)
    out_evp = np.zeros((C, out_stride), dtype=np.uint8)
    st = np.ones(C, dtype=np.int32)
    assert O.bench_stream_rows(ts, dtls, 1, pt, in_stride, per_in, out_port, out_stride, content, 3, st) >= 0
    assert (st == 0).all(), st
    em = O.EvpMixed(np.full(C, cipher, dtype=np.uint8), keys, ivs, tls, 3)
    st[:] = 1
    em.stream(dtls, 1, pt, in_stride, per_in, out_evp, out_stride, content, st)
    assert (st == 0).all(), st
    assert np.array_equal(out_port[:, :per_out], out_evp[:, :per_out])
    # each leg receives (in place) what the other sent
    a, b = out_port.copy(), out_evp.copy()
    step = wire if dtls else 0
    st[:] = 1
    O.bench_stream_rows(ts, dtls, 0, b, out_stride, per_out, None, 0, step, 3, st)
    assert (st == 0).all(), st
    st[:] = 1
    em.stream(dtls, 0, a, out_stride, per_out, None, 0, step, st)
    assert (st == 0).all(), st
    em.close()
    # the plaintext is back in both (TLS 1.3: each record's content before its type byte)
    hdr, head = (13, 8 if cipher != O.CHACHA20_POLY1305 else 0) if dtls else (5, 0)
    for c in (0, C // 2, C - 1):
        for r in range(recs):
            lo = r * wire + hdr + head
            want = pt[c, r * content:(r + 1) * content]
            assert np.array_equal(a[c, lo:lo + content], want)
            assert np.array_equal(b[c, lo:lo + content], want)


def test_tampered_stream_fails_in_both_legs():
    C, content, recs = 5, 1400, 4
    keys, ivs, ts = _conns(O.AES_256_GCM, O.TLS1_3, C, 99)
    per_in = recs * content
    wire = O.stream_record_wire(ts[0], content)
    per_out = recs * wire
    pt = prng_array(8, C * per_in).reshape(C, per_in)
    out = np.zeros((C, per_out), dtype=np.uint8)
    st = np.zeros(C, dtype=np.int32)
    O.bench_stream_rows(ts, False, 1, pt, per_in, per_in, out, per_out, content, 2, st)
    out[2, wire + 100] ^= 1
    a, b = out.copy(), out.copy()
    O.bench_stream_rows(ts, False, 0, a, per_out, per_out, None, 0, 0, 2, st)
    assert st[2] == O.ERR_INVALID_MAC and (np.delete(st, 2) == 0).all()
    em = O.EvpMixed(np.full(C, O.AES_256_GCM, dtype=np.uint8), keys, ivs, O.TLS1_3, 2)
    em.stream(False, 0, b, per_out, per_out, None, 0, 0, st)
    em.close()
    assert st[2] == O.ERR_INVALID_MAC and (np.delete(st, 2) == 0).all()


@pytest.mark.parametrize("alg,keylen,update", [(O.SHA384, 32, True), (O.SHA256, 16, False), (O.SHA256, 32, True)])
def test_threaded_keysched_matches_restatement(alg, keylen, update):
    n = 50
    sec = prng_array(0x5EC, n * 48)
    _, out, st = O.bench_keysched(alg, sec, n, update, keylen, 4)
    assert (st == 0).all()
    H = O.hash_len(alg)
    for i in (0, 17, n - 1):
        s = bytes(sec[48 * i:48 * i + H])
        if update:
            s = O.tls13_update_traffic_secret(alg, s)
        assert bytes(out[i, :keylen]) == O.tls13_hkdf_expand_label(alg, s, b"key", b"", keylen)
        assert bytes(out[i, keylen:]) == O.tls13_hkdf_expand_label(alg, s, b"iv", b"", 12)
