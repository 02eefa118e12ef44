"""GPU parity: the HIP path (through the C ABI of libtlsrec.so) against the
oracle restatement and the committed golden fixtures.  Bit-exact: every
output byte of every record buffer and every record field / status.
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import mbedtls_amd as M  # noqa: E402
import oracle as O  # noqa: E402
from tests import batchlib as B  # noqa: E402
from tests.prng import prng_bytes  # noqa: E402

G = os.path.join(os.path.dirname(__file__), "golden")
h = bytes.fromhex
ALL_C = list(B.CIPHERS.values())
ALL_V = list(B.VERSIONS.values())


def _load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)


def test_device_and_library():
    assert M.device_ok(), "libtlsrec did not find a gfx950 device"
    assert "gfx950" in M.version()


@pytest.mark.parametrize("kat", _load("reference_kats.json"), ids=lambda k: k["name"])
def test_reference_kats_gpu(kat):
    """test_suite_ssl.data:2776-2834 through tlsrec_encrypt_buf/decrypt_buf at
    padding granularity 1 (the KATs' configuration)."""
    sk, si, ck, ci = (h(kat[x]) for x in ("server_key", "server_iv", "client_key", "client_iv"))
    if kat["endpoint"] == "client":
        send = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_128_GCM, ck, sk, ci, si, granularity=1)
        recv = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_128_GCM, sk, ck, si, ci, granularity=1)
    else:
        send = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_128_GCM, sk, ck, si, ci, granularity=1)
        recv = M.Transform(M.VERSION_TLS1_3, M.CIPHER_AES_128_GCM, ck, sk, ci, si, granularity=1)
    pt, ct = h(kat["plaintext"]), h(kat["ciphertext"])
    buf = bytearray(len(ct) + 16)
    buf[:len(pt)] = pt
    rec = M.Record(ctr=bytes(7) + bytes([kat["ctr"]]), type=23, ver=b"\x03\x03", buf=buf,
                   data_offset=0, data_len=len(pt))
    assert send.encrypt_buf(rec) == 0
    assert rec.data() == ct and rec.type == 23
    assert recv.decrypt_buf(rec) == 0
    assert rec.data() == pt and rec.type == 23


def test_record_fixtures_gpu():
    fx = _load("records.json")
    for c in fx["cases"]:
        cipher, ver = B.CIPHERS[c["cipher"]], B.VERSIONS[c["version"]]
        t = M.Transform(ver, cipher, h(c["key_enc"]), h(c["key_dec"]), h(c["iv_enc"]), h(c["iv_dec"]))
        peer = M.Transform(ver, cipher, h(c["key_dec"]), h(c["key_enc"]), h(c["iv_dec"]), h(c["iv_enc"]))
        L = c["len"]
        payload = prng_bytes(c["seed"] ^ 0xA5A5, L)
        head = 8 if B.explicit(cipher, ver) else 0
        buf = bytearray(head + L + 64)
        buf[head:head + L] = payload
        rec = M.Record(ctr=h(c["ctr"]), type=c["type"], ver=b"\x03\x03", buf=buf, data_offset=head, data_len=L)
        assert t.encrypt_buf(rec) == 0, c
        assert (rec.data_offset, rec.data_len, rec.type) == (c["out_offset"], c["out_len"], c["out_type"])
        assert hashlib.sha256(rec.data()).hexdigest() == c["wire_sha256"], (c["cipher"], c["version"], L)
        assert peer.decrypt_buf(rec) == 0
        assert rec.data() == payload and rec.type == c["type"]
        t.close()
        peer.close()


EDGE_LENGTHS = [0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 255, 256, 1000, 1400, 4095, 4096, 16383]


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
@pytest.mark.parametrize("ver", ALL_V, ids=list(B.VERSIONS))
@pytest.mark.parametrize("decrypt", [False, True], ids=["enc", "dec"])
def test_batch_vs_oracle(cipher, ver, decrypt):
    slots = B.random_slots(cipher * 10 + ver, [cipher], [ver], 3)
    lengths = EDGE_LENGTHS + [int(x) for x in np.frombuffer(prng_bytes(cipher + ver, 80), np.uint16) % 2000]
    if decrypt:
        recs, _ = B.sealed_records(slots, lengths, seed=cipher * 7 + ver)
    else:
        recs = B.plaintext_records(slots, lengths, seed=cipher * 7 + ver)
    b = B.Batch(slots, recs)
    if cipher == M.CIPHER_CHACHA20_POLY1305:
        lane_opts = [0, 1, 4, 8]
    elif cipher in (M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_AES_192_GCM):
        lane_opts = [0, 4, 16, 64]
    else:
        lane_opts = [0]              # CCM: one lane per record, no lane option
    for lanes in lane_opts:
        out, res = b.run_gpu(decrypt, lanes=lanes)
        bad = b.compare(decrypt, out, res)
        assert not bad, f"lanes={lanes}: " + "; ".join(bad[:5])
    out, res = b.run_gpu(decrypt, inplace=False)
    assert not b.compare(decrypt, out, res, inplace=False)


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
@pytest.mark.parametrize("ver", ALL_V, ids=list(B.VERSIONS))
def test_batch_tamper(cipher, ver):
    """1 bit flipped in every 7th record -> INVALID_MAC there (buffer wiped as
    PSA does), every other record decrypts."""
    slots = B.random_slots(99 + cipher, [cipher], [ver], 2)
    lengths = [17 + 61 * i for i in range(60)]
    recs, pre = B.sealed_records(slots, lengths, seed=1234)
    bad_idx = set(range(0, len(recs), 7))
    for i in bad_idx:
        r = recs[i]
        pos = r.data_offset + (i * 13) % r.data_len
        r.buf[pos] ^= 1 << (i % 8)
    b = B.Batch(slots, recs)
    out, res = b.run_gpu(True)
    assert not b.compare(True, out, res)
    st = res["status"]
    assert set(np.nonzero(st)[0].tolist()) == bad_idx
    assert all(int(st[i]) == M.ERR_SSL_INVALID_MAC for i in bad_idx)


def test_mixed_keys_interleaved():
    """Config-4 shape at test scale: many keys, AES-256-GCM and
    ChaCha20-Poly1305 interleaved by key, records round-robin over keys."""
    nkeys, per = 96, 6
    slots = B.random_slots(4242, [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305],
                           [M.VERSION_TLS1_3], nkeys)
    lengths = [1400 if (i // nkeys) % 2 else 3000 for i in range(nkeys * per)]
    for decrypt in (False, True):
        if decrypt:
            recs, _ = B.sealed_records(slots, lengths, seed=77)
        else:
            recs = B.plaintext_records(slots, lengths, seed=77)
        b = B.Batch(slots, recs)
        out, res = b.run_gpu(decrypt)
        bad = b.compare(decrypt, out, res)
        assert not bad, "; ".join(bad[:5])


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
@pytest.mark.parametrize("ver", ALL_V, ids=list(B.VERSIONS))
def test_crypt_record_small_gpu(cipher, ver):
    """ssl_crypt_record_small (test_suite_ssl.function:1697-1856) through the
    single-record API, checked byte for byte against the oracle."""
    kl = B.keylen(cipher)
    k0, k1, ive, ivd = bytes([1]) * kl, bytes([2]) * kl, bytes([3]) * 16, bytes([4]) * 16
    t_enc = M.Transform(ver, cipher, k1, k0, ivd, ive)
    t_dec = M.Transform(ver, cipher, k0, k1, ive, ivd)
    o_enc = O.Transform(ver, cipher, k1, k0, ivd, ive)
    buflen = 256
    for mode in (1, 2, 3):
        seen = False
        for off in range(0, 97, 3):
            if mode == 1:
                do, dl = off, buflen - off - 128
            elif mode == 2:
                do, dl = 64, buflen - 64 - off
            else:
                do, dl = off, buflen - 2 * off
            buf = bytearray(buflen)
            buf[do:do + dl] = bytes([42]) * dl
            rec = M.Record(ctr=bytes([off]) * 8, type=42, ver=bytes([off, off]), buf=buf, data_offset=do, data_len=dl)
            orec = O.Record(ctr=bytes([off]) * 8, type=42, ver=bytes([off, off]), buf=bytearray(buf),
                            data_offset=do, data_len=dl)
            r = t_enc.encrypt_buf(rec)
            assert r == o_enc.encrypt_buf(orec)
            assert bytes(rec.buf) == bytes(orec.buf)
            assert (rec.data_offset, rec.data_len, rec.type) == (orec.data_offset, orec.data_len, orec.type)
            if r == M.ERR_SSL_BUFFER_TOO_SMALL:
                continue
            assert r == 0
            seen = True
            assert t_dec.decrypt_buf(rec) == 0
            assert (rec.type, rec.data_offset, rec.data_len) == (42, do, dl)
            assert rec.data() == bytes([42]) * dl
        assert seen


def test_large_roundtrip_16k():
    """Size-independent property at full record size: 16 KiB TLS 1.3 records,
    encrypt then decrypt restores every payload; a sample is bit-exact vs the
    oracle."""
    n = 512
    for cipher in (M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305, M.CIPHER_AES_128_CCM_8):
        slots = B.random_slots(5 + cipher, [cipher], [M.VERSION_TLS1_3], 1)
        recs = B.plaintext_records(slots, [16383] * n, seed=9, head=0, tail=17)
        b = B.Batch(slots, recs)
        out, res = b.run_gpu(False)
        wire = 16384 + M.TAGLEN[cipher]
        assert (res["status"] == 0).all() and (res["data_len"] == wire).all()
        sample = B.Batch(slots, recs[:8])
        o_recs, _ = sample.run_oracle(False)
        for i in range(8):
            o = b.offs[i]
            assert bytes(out[o:o + wire]) == o_recs[i].data()
        # decrypt the GPU ciphertext
        b.arena[:] = out
        d = b.desc.copy()
        d["data_offset"] = 0
        d["data_len"] = wire
        d["type"] = 23
        b.desc = d
        out2, res2 = b.run_gpu(True)
        assert (res2["status"] == 0).all() and (res2["data_len"] == 16383).all()
        for i, r in enumerate(recs):
            o = b.offs[i]
            assert bytes(out2[o:o + 16383]) == bytes(r.buf[:16383])


@pytest.mark.parametrize("cipher", [M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM], ids=["AES-128-GCM", "AES-256-GCM"])
def test_gcm_counter_boundary(cipher):
    """Decrypt of records whose GCM counter passes 2^16 (> 1 MiB of
    ciphertext) takes the kernel's uncached-round path; lengths straddle the
    last cached counter.  ssl_decrypt_buf has no size cap of its own (the
    encrypt side stops at OUT_CONTENT_LEN, ssl_msg.c:831, also checked)."""
    slots = B.random_slots(77 + cipher, [cipher], [M.VERSION_TLS1_2, M.VERSION_TLS1_3], 2)
    lengths = [65533 * 16 - 20, 65533 * 16 - 1, 65534 * 16 + 3, 70000 * 16 + 5, 100, 0]
    recs = B.gcm_sealed_records(slots, lengths, seed=31)
    b = B.Batch(slots, recs)
    _, o_stats = b.run_oracle(True)
    assert o_stats == [0] * len(recs)
    for lanes in (0, 64):
        out, res = b.run_gpu(True, lanes=lanes)
        bad = b.compare(True, out, res)
        assert not bad, f"lanes={lanes}: " + "; ".join(bad[:5])
    # encrypt of the same plaintext sizes: BAD_INPUT_DATA above 16384, like the reference
    pb = B.Batch(slots, B.plaintext_records(slots, lengths, seed=31))
    out, res = pb.run_gpu(False)
    assert not pb.compare(False, out, res)
    assert res["status"].tolist()[:4] == [M.ERR_SSL_BAD_INPUT_DATA] * 4


@pytest.mark.parametrize("lanes", [0, 8, 16])
def test_many_keys_all_ciphers_round_robin(lanes):
    """Bucket pass: all 10 AEADs x 2 TLS versions over 150 keys, records
    round-robin over keys (every neighbour has another key), ragged lengths;
    bit-exact vs the oracle for both directions and several lane counts."""
    nkeys = 150
    slots = B.random_slots(9001, ALL_C, [M.VERSION_TLS1_2, M.VERSION_TLS1_3], nkeys)
    lengths = [int(x) for x in np.frombuffer(prng_bytes(31337, 2 * nkeys * 5), np.uint16) % 3000]
    for decrypt in (False, True):
        recs = (B.sealed_records(slots, lengths, seed=5)[0] if decrypt
                else B.plaintext_records(slots, lengths, seed=5))
        b = B.Batch(slots, recs)
        out, res = b.run_gpu(decrypt, lanes=lanes)
        bad = b.compare(decrypt, out, res)
        assert not bad, "; ".join(bad[:5])


@pytest.mark.parametrize("lanes", [2, 4, 16, 64])
def test_gcm_wave_pass(lanes, monkeypatch):
    """Wave-pass GCM variant (TLSREC_GCM_WP=1: per-wave key passes, H^L per
    wave in LDS, per-record tables from HBM): 200 keys of GCM-128/192/256 and
    ChaCha, both TLS versions, ragged lengths incl. the edge list, tampered
    records -- bit-exact vs the oracle in both directions."""
    monkeypatch.setenv("TLSREC_GCM_WP", "1")
    _wave_pass_case(lanes)


@pytest.mark.parametrize("lanes,tm", [(16, "0"), (4, "3"), (2, "3")])
def test_gcm_wave_pass_lane_tree(lanes, tm, monkeypatch):
    """The wave passes' lane tree both ways: from the key's HBM tables at 16
    lanes (TLSREC_GCM_TREEMUL=0; table-free is the default there) and by
    table-free multiplies at 4 and 2 lanes (=3; tables are the default)."""
    monkeypatch.setenv("TLSREC_GCM_WP", "1")
    monkeypatch.setenv("TLSREC_GCM_TREEMUL", tm)
    _wave_pass_case(lanes)


def _wave_pass_case(lanes):
    nkeys = 200
    slots = B.random_slots(777 + lanes, [M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_AES_192_GCM,
                                         M.CIPHER_CHACHA20_POLY1305],
                           [M.VERSION_TLS1_2, M.VERSION_TLS1_3], nkeys)
    lengths = EDGE_LENGTHS + [int(x) for x in np.frombuffer(prng_bytes(4711, 2 * 3 * nkeys), np.uint16) % 5000]
    for decrypt in (False, True):
        recs = (B.sealed_records(slots, lengths, seed=8)[0] if decrypt
                else B.plaintext_records(slots, lengths, seed=8))
        if decrypt:
            for i in range(0, len(recs), 11):
                r = recs[i]
                r.buf[r.data_offset + (i * 7) % r.data_len] ^= 4
        b = B.Batch(slots, recs)
        out, res = b.run_gpu(decrypt, lanes=lanes)
        bad = b.compare(decrypt, out, res)
        assert not bad, "; ".join(bad[:5])


@pytest.mark.parametrize("per_key", [16, 64])
def test_gcm_sized_small_records(per_key):
    """tlsrec_batch_*_sized with a small mean record size: many keys of
    12..127 small records each send the GCM kernels into wave passes at 4
    lanes (16 per key, 36 K records: engine.hip `small4`) or 2 lanes (64 per
    key, 64 K records, the chip-fill bound of `small2`); AES-128/256-GCM and
    ChaCha20-Poly1305 keys, records round-robin over keys, lengths around
    1.4 KiB incl. ragged ones and tampered records -- bit-exact vs the oracle
    in both directions."""
    nkeys = (36864 if per_key < 48 else 65536) // per_key
    slots = B.random_slots(4242 + per_key, [M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305],
                           [M.VERSION_TLS1_3, M.VERSION_TLS1_2], nkeys)
    n = nkeys * per_key
    lengths = [1400 - int(x) for x in np.frombuffer(prng_bytes(4343 + per_key, 2 * n), np.uint16) % 200]
    for decrypt in (False, True):
        recs = (B.sealed_records(slots, lengths, seed=9)[0] if decrypt
                else B.plaintext_records(slots, lengths, seed=9))
        if decrypt:
            for i in range(0, len(recs), 97):
                r = recs[i]
                r.buf[r.data_offset + (i * 13) % r.data_len] ^= 0x10
        b = B.Batch(slots, recs)
        out, res = b.run_gpu(decrypt, mean_bytes=1400)
        bad = b.compare(decrypt, out, res)
        assert not bad, "; ".join(bad[:5])


@pytest.mark.parametrize("nslots,ciphers", [(1, [M.CIPHER_AES_256_GCM]), (1, [M.CIPHER_AES_128_CCM]),
                                            (1, [M.CIPHER_CHACHA20_POLY1305]),
                                            (4, [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305]),
                                            (4, [M.CIPHER_AES_128_CCM_8, M.CIPHER_AES_192_GCM])],
                         ids=["identity-gcm", "identity-ccm", "identity-chacha", "bucket", "bucket-ccm"])
def test_unusable_slot_gets_bad_input(nslots, ciphers):
    """Records naming a slot past the table or never loaded are reported
    BAD_INPUT_DATA with their buffer untouched; the other records are
    processed normally -- with a single-key table (kernels walk the
    descriptors in order) and a multi-key one (bucket pass)."""
    import torch
    slots = B.random_slots(123, ciphers, [M.VERSION_TLS1_3], nslots)
    recs = B.plaintext_records(slots, [100, 2000, 17, 500, 64, 1400], seed=3)
    b = B.Batch(slots, recs)
    d = b.desc.copy()
    cap = nslots + 2                        # slot nslots .. cap-1 never loaded
    d["slot"][1] = cap + 5                  # past the table
    d["slot"][4] = nslots + 1               # inside the table, never loaded
    dev = torch.device("cuda")
    kt = M.KeyTable(cap)
    kt.load(b.key_materials())
    arena = torch.from_numpy(b.arena.copy()).to(dev)
    res = torch.zeros(len(recs) * 16, dtype=torch.uint8, device=dev)
    recs_d = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    M.batch_encrypt(kt, recs_d, res, len(recs), arena, arena)
    torch.cuda.synchronize()
    out = arena.cpu().numpy()
    r = res.cpu().numpy().view(M.BATCH_RES)
    kt.close()
    for i in (1, 4):
        assert int(r["status"][i]) == M.ERR_SSL_BAD_INPUT_DATA
        o = b.offs[i]
        assert bytes(out[o:o + len(recs[i].buf)]) == bytes(recs[i].buf)
    good = B.Batch(slots, [recs[i] for i in (0, 2, 3, 5)])
    o_recs, o_stats = good.run_oracle(False)
    for k, i in enumerate((0, 2, 3, 5)):
        assert int(r["status"][i]) == o_stats[k] == 0
        o = b.offs[i]
        assert bytes(out[o:o + len(recs[i].buf)]) == bytes(o_recs[k].buf)
