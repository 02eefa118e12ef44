"""The OpenSSL-EVP CPU-baseline leg (oracle/evp_bench.c) computes exactly what
the oracle restatement computes: same ciphertext bytes for encrypt, same
plaintext / status for decrypt (incl. a tampered record), TLS 1.2 and 1.3.
CPU only; it pins the bench's cpu_baseline to the reference semantics."""
import numpy as np
import pytest

import oracle as O
from tests.prng import prng_bytes


@pytest.mark.parametrize("cipher", O.EVP_CIPHERS)
@pytest.mark.parametrize("ver", [O.TLS1_2, O.TLS1_3])
@pytest.mark.parametrize("content", [0, 1, 100, 1400, 16383])
def test_evp_leg_matches_oracle(cipher, ver, content):
    kl = O.KEYLEN[cipher]
    key, iv = prng_bytes(cipher * 3 + ver, kl), prng_bytes(cipher * 5 + ver, 16)
    head = 8 if ver == O.TLS1_2 and cipher != O.CHACHA20_POLY1305 else 0
    inner = content + 1 + (16 - (content + 1) % 16) % 16 if ver == O.TLS1_3 else content
    wire = head + inner + 16
    stride = (wire + 127) // 128 * 128
    n, seq0 = 9, 1000
    arena = np.zeros(n * stride, dtype=np.uint8)
    for i in range(n):
        arena[i * stride + head:i * stride + head + content] = np.frombuffer(prng_bytes(i + content, content), np.uint8)
    plain = arena.copy()
    st = np.zeros(n, dtype=np.int32)
    O.evp_bench(cipher, ver, key, iv, 1, arena, stride, content, n, seq0, 3, st)
    assert (st == 0).all()
    t = O.Transform(ver, cipher, key, key, iv, iv)
    for i in range(n):
        buf = bytearray(plain[i * stride:(i + 1) * stride].tobytes())
        seq = (seq0 + i).to_bytes(8, "big")
        rec = O.Record(ctr=seq, type=23, ver=b"\x03\x03", buf=buf, data_offset=head, data_len=content)
        assert t.encrypt_buf(rec) == 0
        assert rec.data_offset == 0 and rec.data_len == wire
        assert arena[i * stride:i * stride + wire].tobytes() == rec.data(), i
    arena[2 * stride + wire - 3] ^= 1                  # tamper record 2's tag
    O.evp_bench(cipher, ver, key, iv, 0, arena, stride, wire, n, seq0, 2, st)
    assert st[2] == O.ERR_INVALID_MAC
    assert all(st[i] == 0 for i in range(n) if i != 2)
    for i in range(n):
        if i != 2:
            got = arena[i * stride + head:i * stride + head + content]
            assert got.tobytes() == plain[i * stride + head:i * stride + head + content].tobytes()


@pytest.mark.parametrize("ver", [O.TLS1_2, O.TLS1_3])
@pytest.mark.parametrize("content", [1400, 16383])
def test_mixed_connection_legs_match_oracle(ver, content):
    """The c4 / c4s CPU legs: one context per connection (EVP) / one transform
    per connection (port), record i under connection i % nconn with sequence
    number i // nconn, AES-256-GCM and ChaCha20-Poly1305 alternating.  Both
    legs' ciphertexts equal the oracle's record by record; a tampered record
    fails its MAC in both decrypt legs."""
    nconn, n = 6, 20
    ciphers = np.array([O.AES_256_GCM if c % 2 == 0 else O.CHACHA20_POLY1305 for c in range(nconn)], np.uint8)
    keys = np.frombuffer(prng_bytes(501 + ver, nconn * 32), np.uint8).reshape(nconn, 32)
    ivs = np.frombuffer(prng_bytes(502 + ver, nconn * 12), np.uint8).reshape(nconn, 12)
    heads = [8 if ver == O.TLS1_2 and c != O.CHACHA20_POLY1305 else 0 for c in ciphers]
    inner = content + 1 + (16 - (content + 1) % 16) % 16 if ver == O.TLS1_3 else content
    stride = (8 + inner + 16 + 127) // 128 * 128
    plain = np.zeros(n * stride, dtype=np.uint8)
    for i in range(n):
        h = heads[i % nconn]
        plain[i * stride + h:i * stride + h + content] = np.frombuffer(prng_bytes(900 + i, content), np.uint8)
    ts = [O.Transform(ver, int(c), bytes(k), bytes(k), bytes(v) + bytes(4), bytes(v) + bytes(4))
          for c, k, v in zip(ciphers, keys, ivs)]
    evp = O.EvpMixed(ciphers, keys, ivs, ver, 3)
    try:
        a_evp, a_port = plain.copy(), plain.copy()
        st = np.zeros(n, dtype=np.int32)
        evp.run(1, a_evp, stride, content, n, st)
        assert (st == 0).all()
        O.bench_multi(ts, 1, a_port, stride, content, n, 3, st)
        assert (st == 0).all()
        for i in range(n):
            c = i % nconn
            h = heads[c]
            buf = bytearray(plain[i * stride:(i + 1) * stride].tobytes())
            rec = O.Record(ctr=(i // nconn).to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=buf,
                           data_offset=h, data_len=content)
            assert ts[c].encrypt_buf(rec) == 0
            wire = rec.data_len
            assert a_evp[i * stride:i * stride + wire].tobytes() == rec.data(), i
            assert a_port[i * stride:i * stride + wire].tobytes() == rec.data(), i
        wires = [heads[i % nconn] + inner + 16 for i in range(n)]
        assert len(set(wires)) <= 2
        for arena, run in ((a_evp, lambda a, w: evp.run(0, a, stride, w, n, st)),
                           (a_port, lambda a, w: O.bench_multi(ts, 0, a, stride, w, n, 2, st))):
            if len(set(wires)) == 1:
                arena[3 * stride + wires[3] - 2] ^= 1
                run(arena, wires[0])
                assert st[3] == O.ERR_INVALID_MAC and all(st[i] == 0 for i in range(n) if i != 3)
    finally:
        evp.close()


@pytest.mark.parametrize("cipher", O.EVP_CIPHERS)
@pytest.mark.parametrize("ver", [O.TLS1_2, O.TLS1_3])
def test_bulk_checker_matches_oracle(cipher, ver):
    """evp_check_records (the bulk GPU-vs-OpenSSL checker of
    tests/test_evp_parity_gpu.py): its seal equals the oracle's records at
    variable lengths under several keys, its compare mode accepts exactly the
    oracle's bytes and flags a one-bit change."""
    nkeys, n = 3, 24
    kl = O.KEYLEN[cipher]
    keys = np.frombuffer(prng_bytes(700 + cipher + ver, nkeys * 32), np.uint8).reshape(nkeys, 32).copy()
    keys[:, kl:] = 0
    ivs = np.frombuffer(prng_bytes(701 + cipher + ver, nkeys * 12), np.uint8).reshape(nkeys, 12)
    head = 8 if ver == O.TLS1_2 and cipher != O.CHACHA20_POLY1305 else 0
    lens = np.array([0, 1, 15, 16, 17, 1400, 16383, 255] * 3, dtype=np.uint32)
    keyidx = np.arange(n, dtype=np.uint32) % nkeys
    seq = np.frombuffer(prng_bytes(702, 8 * n), np.uint64).copy()
    size = head + lens + 32 + 16
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum((size + 127) // 128 * 128)[:-1]
    plain = np.zeros(int(off[-1] + size[-1]), dtype=np.uint8)
    for i in range(n):
        plain[int(off[i]) + head:int(off[i]) + head + int(lens[i])] = np.frombuffer(prng_bytes(800 + i, int(lens[i])),
                                                                                   np.uint8)
    sealed = plain.copy()
    assert (O.evp_check_records(0, cipher, ver, keys, ivs, keyidx, seq, off, lens, sealed, threads=3) == 0).all()
    ts = [O.Transform(ver, cipher, bytes(k[:kl]), bytes(k[:kl]), bytes(v) + bytes(4), bytes(v) + bytes(4))
          for k, v in zip(keys, ivs)]
    for i in range(n):
        o = int(off[i])
        buf = bytearray(plain[o:o + int(size[i])].tobytes())
        rec = O.Record(ctr=int(seq[i]).to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=buf, data_offset=head,
                       data_len=int(lens[i]))
        assert ts[keyidx[i]].encrypt_buf(rec) == 0
        assert sealed[o:o + rec.data_len].tobytes() == rec.data(), i
    assert (O.evp_check_records(1, cipher, ver, keys, ivs, keyidx, seq, off, lens, plain, sealed) == 0).all()
    bad = sealed.copy()
    bad[int(off[5]) + head + 3] ^= 4
    r = O.evp_check_records(1, cipher, ver, keys, ivs, keyidx, seq, off, lens, plain, bad)
    assert r[5] == 1 and (np.delete(r, 5) == 0).all()
    assert (O.evp_check_records(2, cipher, ver, keys, ivs, keyidx, seq, off, lens, plain, plain.copy()) == 0).all()
