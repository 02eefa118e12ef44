"""GPU parity for the record paths a plain round trip never reaches (VERDICT
r01 "next" 1): each case runs the HIP kernels through the C ABI and compares
every status, record field and buffer byte with the oracle.

  (a) authenticated all-zero inner plaintexts -> INVALID_RECORD, the kernel
      exit of ssl_msg.c:1809-1817 (TLS 1.3) and :1821-1826 (DTLS 1.2 + CID),
      for every AEAD and every lane configuration;
  (b) tampered AAD / nonce inputs the kernels rebuild from the descriptor
      (type, ver, ctr, length) -> INVALID_MAC with the output wiped;
  (c) ssl_crypt_record (test_suite_ssl.function:1567-1695: 16 records,
      alternating transforms, ctr = ver = n, type 42, 1 + n bytes of 42) for
      all 22 ids and both TLS versions, without CID, through the single-record
      API and as one batch, ciphertext bytes equal to the oracle's;
  (d) BASELINE config 4 at its stated key count: a 65 536-slot table,
      AES-256-GCM and ChaCha20-Poly1305 alternating per key, records
      round-robin over keys at 16 KiB -- status and length of every record,
      payload restored after encrypt -> decrypt, a sample bit-exact vs the
      oracle; 64 records per key (auto L = 16, workgroup key passes) and 2 per
      key (the wave-pass kernel);
  plus records naming unusable slots in the ARIA / Camellia kernels
  (identity tables and bucket classes).
"""
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

ALL_C = list(B.CIPHERS.values())
ALL_V = list(B.VERSIONS.values())
GCM_AES = (M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_AES_192_GCM)


def _lane_opts(cipher):
    if cipher == M.CIPHER_CHACHA20_POLY1305:
        return [0, 1, 2, 4, 8]
    if cipher in GCM_AES:
        return [0, 4, 8, 16, 64]
    return [0]


def _seal(slots, recs, cids=None):
    """oracle-encrypt `recs`; returns the sealed records ready for decrypt"""
    o_recs, o_stats = B.Batch(slots, recs, cids=cids).run_oracle(False)
    out = []
    for r, o, st in zip(recs, o_recs, o_stats):
        assert st == 0
        out.append(B.Rec(slot=r.slot, buf=bytearray(o.buf), data_offset=o.data_offset, data_len=o.data_len,
                         ctr=r.ctr, type=o.type, ver=r.ver, cid=o.cid))
    return out


def _zero_inner_records(slots, lengths, seed, head):
    """TLS 1.3 / DTLS-CID inner plaintexts: record k%3==0 is all zero
    (content of zeros, type byte 0: INVALID_RECORD after a good tag), k%3==1
    has zero content and a real type, k%3==2 has type 0 after non-zero bytes
    (the reference then takes the last non-zero byte as the type)."""
    recs = []
    for i, L in enumerate(lengths):
        s = i % len(slots)
        payload = bytearray(L)
        kind = i % 3
        if kind == 2 and L:
            payload[:] = prng_bytes(seed + i, L)
            payload[L - 1] = 0
            if L > 1:
                payload[L // 2] |= 1
        buf = bytearray(head + L + 48)
        buf[head:head + L] = payload
        ctr = (seed * 1000 + i).to_bytes(8, "big")
        recs.append(B.Rec(slot=s, buf=buf, data_offset=head, data_len=L, ctr=ctr, type=0 if kind != 1 else 23))
    return recs


ZLEN = [0, 1, 2, 14, 15, 16, 17, 31, 32, 47, 63, 64, 65, 100, 255, 1400, 4096, 16383]


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
def test_invalid_record_tls13(cipher):
    slots = B.random_slots(0x2E80 + cipher, [cipher], [M.VERSION_TLS1_3], 2)
    recs = _seal(slots, _zero_inner_records(slots, ZLEN * 2, 0x51 + cipher, head=0))
    b = B.Batch(slots, recs)
    _, o_stats = b.run_oracle(True)
    assert o_stats.count(M.ERR_SSL_INVALID_RECORD) == len([i for i in range(len(recs)) if i % 3 == 0])
    for lanes in _lane_opts(cipher):
        out, res = b.run_gpu(True, lanes=lanes)
        bad = b.compare(True, out, res)
        assert not bad, f"lanes={lanes}: " + "; ".join(bad[:5])
        st = [int(x) for x in res["status"]]
        assert st == o_stats


@pytest.mark.parametrize("cipher", [M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305])
def test_invalid_record_wave_pass(cipher, monkeypatch):
    """the same exit in the wave-pass GCM variant and a bucketed table"""
    monkeypatch.setenv("TLSREC_GCM_WP", "1")
    slots = B.random_slots(0x2E90 + cipher, [cipher, M.CIPHER_AES_256_GCM], [M.VERSION_TLS1_3], 40)
    recs = _seal(slots, _zero_inner_records(slots, ZLEN * 5, 0x61 + cipher, head=0))
    b = B.Batch(slots, recs)
    _, o_stats = b.run_oracle(True)
    for lanes in (16, 64):
        out, res = b.run_gpu(True, lanes=lanes)
        bad = b.compare(True, out, res)
        assert not bad, f"lanes={lanes}: " + "; ".join(bad[:5])
        assert [int(x) for x in res["status"]] == o_stats


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
def test_invalid_record_dtls_cid(cipher):
    """DTLS 1.2 + CID: DTLSInnerPlaintext of all zeros -> INVALID_RECORD
    (ssl_msg.c:1821-1826); the CID kernel variants"""
    slots = [(cipher, M.VERSION_TLS1_2, prng_bytes(0xC1D + s, 32)[:M.KEYLEN[cipher]], prng_bytes(0xC2D + s, 16), 0)
             for s in range(2)]
    cids = {0: prng_bytes(0xC3D, 4), 1: prng_bytes(0xC4D, 21)}
    head = 0 if cipher == M.CIPHER_CHACHA20_POLY1305 else 8
    pre = _zero_inner_records(slots, ZLEN, 0x71 + cipher, head=head)
    for r in pre:
        r.ver = b"\xfe\xfd"
    recs = _seal(slots, pre, cids=cids)
    assert all(r.cid for r in recs)
    b = B.Batch(slots, recs, cids=cids)
    _, o_stats = b.run_oracle(True)
    assert M.ERR_SSL_INVALID_RECORD in o_stats
    out, res = b.run_gpu(True)
    bad = b.compare(True, out, res)
    assert not bad, "; ".join(bad[:5])
    assert [int(x) for x in res["status"]] == o_stats


def test_invalid_record_single_record_api():
    """tlsrec_decrypt_buf returns INVALID_RECORD with the reference's fields"""
    for cipher in (M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305, M.CIPHER_AES_128_CCM_8,
                   M.CIPHER_CAMELLIA_256_GCM, M.CIPHER_ARIA_128_CCM):
        kl = M.KEYLEN[cipher]
        k, iv = prng_bytes(cipher, kl), prng_bytes(cipher + 1, 16)
        t = M.Transform(M.VERSION_TLS1_3, cipher, k, k, iv, iv)
        ot = O.Transform(M.VERSION_TLS1_3, cipher, k, k, iv, iv)
        for L in (0, 5, 16, 300):
            recs = []
            for R in (M.Record, O.Record):
                recs.append(R(ctr=L.to_bytes(8, "big"), type=0, ver=b"\x03\x03", buf=bytearray(L + 64),
                              data_offset=0, data_len=L))
            g, o = recs
            assert t.encrypt_buf(g) == 0 == ot.encrypt_buf(o)
            assert bytes(g.buf) == bytes(o.buf)
            rg, ro = t.decrypt_buf(g), ot.decrypt_buf(o)
            assert rg == ro == M.ERR_SSL_INVALID_RECORD
            assert (g.type, g.data_offset, g.data_len) == (o.type, o.data_offset, o.data_len)
            assert bytes(g.buf) == bytes(o.buf)
        t.close()


# ---- (b) AAD / nonce inputs ---------------------------------------------------

@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
@pytest.mark.parametrize("ver", ALL_V, ids=list(B.VERSIONS))
def test_tamper_descriptor_fields(cipher, ver):
    """Flip one bit of the record's type, version, sequence number or length
    in the descriptor (the GPU rebuilds AAD and nonce from them) ->
    INVALID_MAC at exactly those records, output wiped as PSA wipes it."""
    slots = B.random_slots(0xAAD + cipher, [cipher], [ver], 2)
    lengths = [33 + 97 * i for i in range(40)]
    recs, _ = B.sealed_records(slots, lengths, seed=0xAAD + ver)
    kinds = {}
    for i, r in enumerate(recs):
        k = i % 5
        if k == 0:
            r.type ^= 1 << (i % 3)
        elif k == 1:
            r.ver = bytes([r.ver[0], r.ver[1] ^ 0x10])
        elif k == 2:
            c = bytearray(r.ctr)
            c[7 - (i % 8)] ^= 0x80
            r.ctr = bytes(c)
        elif k == 3:
            r.data_len -= 1          # one byte short: the length field of the AAD / the tag moves
        else:
            continue
        kinds[i] = k
    b = B.Batch(slots, recs)
    _, o_stats = b.run_oracle(True)
    for lanes in _lane_opts(cipher)[:3]:
        out, res = b.run_gpu(True, lanes=lanes)
        bad = b.compare(True, out, res)
        assert not bad, f"lanes={lanes}: " + "; ".join(bad[:5])
        st = [int(x) for x in res["status"]]
        assert st == o_stats
    for i, k in kinds.items():
        # every field is in the AAD (rec->type, ver, ctr, len: ssl_msg.c:568-735)
        # or the nonce (ctr: :768-781)
        assert o_stats[i] == M.ERR_SSL_INVALID_MAC, (i, k, o_stats[i])
    assert all(o_stats[i] == 0 for i in range(len(recs)) if i not in kinds)


# ---- (c) ssl_crypt_record, no CID ------------------------------------------

def _transforms(cipher, ver, gpu):
    """mbedtls_test_ssl_build_transforms (ssl_helpers.c:1361-1651): keys
    0x01.. / 0x02.., IVs 0x03.. / 0x04.."""
    T = M.Transform if gpu else O.Transform
    kl = M.KEYLEN[cipher]
    key0, key1 = bytes([1]) * kl, bytes([2]) * kl
    ive, ivd = bytes([3]) * 16, bytes([4]) * 16
    t0 = T(ver, cipher, key0, key1, ive, ivd)
    t1 = T(ver, cipher, key1, key0, ivd, ive)
    return t0, t1


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
@pytest.mark.parametrize("ver", ALL_V, ids=list(B.VERSIONS))
def test_crypt_record_gpu(cipher, ver):
    g0, g1 = _transforms(cipher, ver, True)
    o0, o1 = _transforms(cipher, ver, False)
    sealed = []
    for n in range(15, -1, -1):
        (gd, ge), (od, oe) = ((g0, g1), (o0, o1)) if n % 3 == 0 else ((g1, g0), (o1, o0))
        recs = []
        for R in (M.Record, O.Record):
            buf = bytearray(512)
            buf[16:17 + n] = bytes([42]) * (1 + n)
            recs.append(R(ctr=bytes([n]) * 8, type=42, ver=bytes([n, n]), buf=buf, data_offset=16, data_len=1 + n))
        gr, orr = recs
        assert ge.encrypt_buf(gr) == 0 == oe.encrypt_buf(orr)
        assert (gr.type, gr.data_offset, gr.data_len) == (orr.type, orr.data_offset, orr.data_len)
        assert bytes(gr.buf) == bytes(orr.buf), n
        if ver == M.VERSION_TLS1_3:
            assert gr.type == M.MSG_APPLICATION_DATA
        sealed.append((n, bytes(gr.buf), gr.data_offset, gr.data_len, gr.type))
        assert gd.decrypt_buf(gr) == 0
        assert (gr.type, gr.ver, gr.data_offset, gr.data_len) == (42, bytes([n, n]), 16, 1 + n)
        assert gr.data() == bytes([42]) * (1 + n)
    for t in (g0, g1):
        t.close()
    # the same 16 records as one batch: slot 0 = t0's encrypt key, slot 1 = t1's
    kl = M.KEYLEN[cipher]
    slots = [(cipher, ver, bytes([1]) * kl, bytes([3]) * 16, 0), (cipher, ver, bytes([2]) * kl, bytes([4]) * 16, 0)]
    pre = []
    for n in range(15, -1, -1):
        buf = bytearray(512)
        buf[16:17 + n] = bytes([42]) * (1 + n)
        pre.append(B.Rec(slot=1 if n % 3 == 0 else 0, buf=buf, data_offset=16, data_len=1 + n,
                         ctr=bytes([n]) * 8, type=42, ver=bytes([n, n])))
    b = B.Batch(slots, pre)
    out, res = b.run_gpu(False)
    assert not b.compare(False, out, res)
    for i, (n, wire, off, ln, typ) in enumerate(sealed):
        o = b.offs[i]
        assert bytes(out[o:o + 512]) == wire, n
        assert (int(res["data_offset"][i]), int(res["data_len"][i]), int(res["type"][i])) == (off, ln, typ)
    dec = [B.Rec(slot=r.slot, buf=bytearray(w), data_offset=off, data_len=ln, ctr=r.ctr, type=typ, ver=r.ver)
           for r, (n, w, off, ln, typ) in zip(pre, sealed)]
    b = B.Batch(slots, dec)
    out, res = b.run_gpu(True)
    assert not b.compare(True, out, res)
    assert (res["status"] == 0).all()


# ---- (d) config 4 at its key count ----------------------------------------

def _c4_roundtrip(nkeys, per_key, content=16383):
    """nkeys slots (even: AES-256-GCM, odd: ChaCha20-Poly1305), per_key
    records each, records round-robin over keys, 128-byte record slots;
    everything generated and checked on the device except an oracle sample."""
    dev = torch.device("cuda")
    n = nkeys * per_key
    wire = content + 1 + 16
    stride = (wire + 127) // 128 * 128
    raw = np.frombuffer(prng_bytes(0xC4C4 + nkeys + per_key, nkeys * 48), dtype=np.uint8).reshape(nkeys, 48)
    km = np.zeros(nkeys, dtype=M.KEY_MATERIAL)
    km["cipher"] = np.where(np.arange(nkeys) % 2 == 0, M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305)
    km["tls_minor"] = 4
    km["fixed_ivlen"] = 12
    km["taglen"] = 16
    km["key"] = raw[:, :32]
    km["iv"][:, :12] = raw[:, 32:44]
    kt = M.KeyTable(nkeys)
    kt.load(km)
    g = torch.Generator(device=dev)
    g.manual_seed(nkeys * 131 + per_key)
    arena = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev, generator=g)
    plain = arena.clone()
    recs = M.records(n)
    idx = np.arange(n, dtype=np.uint64)
    recs["buf_off"] = idx * stride
    recs["buf_len"] = stride
    recs["data_offset"] = 0
    recs["data_len"] = content
    recs["slot"] = (idx % nkeys).astype(np.uint32)
    recs["ctr"] = M.seq_bytes(idx // nkeys)
    recs["type"] = 23
    recs["ver"] = (3, 3)
    recs_d = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    M.batch_encrypt(kt, recs_d, res, n, arena, arena)
    torch.cuda.synchronize()
    r32 = res.view(torch.int32)
    assert int((r32[0::4] != 0).sum()) == 0
    assert int((r32[2::4] != wire).sum()) == 0
    # oracle sample: records of both ciphers, first and last keys
    sample = sorted({0, 1, 2, 3, nkeys - 2, nkeys - 1, n - 1, n - 2, n // 2, n // 2 + 1})
    for i in sample:
        s = int(recs["slot"][i])
        k = km[s]
        c = int(k["cipher"])
        ot = O.Transform(O.TLS1_3, c, bytes(k["key"][:32]), bytes(k["key"][:32]), bytes(k["iv"]), bytes(k["iv"]))
        buf = bytearray(stride)
        buf[:content] = plain[i * stride:i * stride + content].cpu().numpy().tobytes()
        orec = O.Record(ctr=bytes(recs["ctr"][i]), type=23, ver=b"\x03\x03", buf=buf, data_offset=0,
                        data_len=content)
        assert ot.encrypt_buf(orec) == 0
        assert arena[i * stride:i * stride + wire].cpu().numpy().tobytes() == orec.data(), i
    # decrypt in place with the auto configuration, every record restored
    dec = recs.copy()
    dec["data_len"] = wire
    dec_d = torch.from_numpy(dec.view(np.uint8).copy()).to(dev)
    res.zero_()
    M.batch_decrypt(kt, dec_d, res, n, arena, arena)
    torch.cuda.synchronize()
    assert int((r32[0::4] != 0).sum()) == 0
    assert int((r32[2::4] != content).sum()) == 0
    assert int((res.view(torch.uint8).view(-1, 16)[:, 12] != 23).sum()) == 0
    a2 = arena.view(n, stride)[:, :content]
    p2 = plain.view(n, stride)[:, :content]
    assert torch.equal(a2, p2)
    kt.close()
    del arena, plain


def test_config4_full_key_count():
    """c4 as BASELINE states it: 65 536 keys x 64 records x 16 KiB"""
    _c4_roundtrip(65536, 64)


def test_config4_keys_two_records_each():
    """65 536 keys x 2 records: the many-keys / few-records dispatch"""
    _c4_roundtrip(65536, 2)


# ---- unusable slots in the ARIA / Camellia kernels --------------

@pytest.mark.parametrize("nslots,ciphers", [(1, [M.CIPHER_CAMELLIA_128_GCM]), (1, [M.CIPHER_CAMELLIA_256_CCM]),
                                            (1, [M.CIPHER_ARIA_256_GCM]), (1, [M.CIPHER_ARIA_192_CCM]),
                                            (4, [M.CIPHER_ARIA_128_CCM, M.CIPHER_CAMELLIA_192_CCM]),
                                            (4, [M.CIPHER_CAMELLIA_256_GCM, M.CIPHER_ARIA_128_GCM]),
                                            (4, [M.CIPHER_CHACHA20_POLY1305]),
                                            (4, [M.CIPHER_CHACHA20_POLY1305, M.CIPHER_AES_128_GCM])],
                         ids=["identity-cam-gcm", "identity-cam256-ccm", "identity-aria-gcm", "identity-aria-ccm",
                              "bucket-alt-ccm", "bucket-alt-gcm", "chacha-only-multikey", "bucket-chacha-gcm"])
def test_unusable_slot_alt_ciphers(nslots, ciphers):
    """records naming an out-of-range slot and a never-loaded one: BAD_INPUT_DATA
    and the buffer untouched, in identity order and through the bucket pass
    alike -- including a several-key ChaCha20-Poly1305-only table, which the
    engine walks in identity order, against the bucket path of a
    mixed table"""
    dev = torch.device("cuda")
    slots = B.random_slots(321, ciphers, [M.VERSION_TLS1_2], nslots)
    recs = B.plaintext_records(slots, [100, 2000, 17, 500, 64, 1400], seed=4)
    b = B.Batch(slots, recs)
    d = b.desc.copy()
    cap = nslots + 2
    d["slot"][1] = cap + 5
    d["slot"][4] = nslots + 1
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
