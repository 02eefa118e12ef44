"""GPU parity for DTLS 1.2 connection-ID records: the HIP
kernels through the C ABI against the oracle (tests/test_cid_oracle.py pins
the oracle with the reference's ssl_crypt_record CID cases and OpenSSL).

  - single-record API: ssl_crypt_record with CIDs 4:4 / 4:0 / 0:4
    (test_suite_ssl.function:1567-1695) for every AEAD, ciphertext bytes equal
    to the oracle's;
  - batch API: CIDs of 1..32 bytes (AAD of 2..4 blocks), content lengths
    across block and chunk edges, both directions, bit-exact buffers and
    fields; a record whose CID differs from the slot's -> UNEXPECTED_CID and
    untouched; a tampered record -> INVALID_MAC; mixed CID / non-CID slots.
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
CID_TYPE = 25


def _pair(cipher, cid0_len, cid1_len, gpu=True):
    """mbedtls_test_ssl_build_transforms with CIDs (ssl_helpers.c:1569-1576)."""
    T = M.Transform if gpu else O.Transform
    kl = M.KEYLEN[cipher]
    key0, key1 = bytes([1]) * kl, bytes([2]) * kl
    ive, ivd = bytes([3]) * 16, bytes([4]) * 16
    cid0, cid1 = prng_bytes(7, 4)[:cid0_len], prng_bytes(8, 4)[:cid1_len]
    t_in = T(M.VERSION_TLS1_2, cipher, key0, key1, ive, ivd)
    t_out = T(M.VERSION_TLS1_2, cipher, key1, key0, ivd, ive)
    t_in.set_cid(cid0, cid1)
    t_out.set_cid(cid1, cid0)
    return t_in, t_out


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
@pytest.mark.parametrize("cids", [(4, 4), (4, 0), (0, 4)], ids=["4:4", "4:0", "0:4"])
def test_crypt_record_cid_gpu(cipher, cids):
    g0, g1 = _pair(cipher, *cids)
    o0, o1 = _pair(cipher, *cids, gpu=False)
    for n in range(15, -1, -1):
        (gd, ge), (od, oe) = ((g0, g1), (o0, o1)) if n % 3 == 0 else ((g1, g0), (o1, o0))
        recs = []
        for R in (M.Record, O.Record):
            buf = bytearray(512)
            buf[16:17 + n] = bytes([42]) * (1 + n)
            recs.append(R(ctr=bytes([n]) * 8, type=42, ver=bytes([n, n]), buf=buf, data_offset=16,
                          data_len=1 + n))
        gr, orr = recs
        assert ge.encrypt_buf(gr) == 0 and oe.encrypt_buf(orr) == 0
        assert (gr.type, gr.data_offset, gr.data_len, gr.cid) == (orr.type, orr.data_offset, orr.data_len, orr.cid)
        assert bytes(gr.buf) == bytes(orr.buf), n
        if gr.cid:
            assert gr.type == CID_TYPE
        assert gd.decrypt_buf(gr) == 0
        assert (gr.type, gr.ver, gr.data_offset, gr.data_len) == (42, bytes([n, n]), 16, 1 + n)
        assert gr.data() == bytes([42]) * (1 + n)


def _cid_batch(cipher, lengths, seed, cid_lens):
    slots = [(cipher, M.VERSION_TLS1_2, prng_bytes(seed + s, 32)[:M.KEYLEN[cipher]], prng_bytes(seed + 50 + s, 16), 0)
             for s in range(len(cid_lens))]
    cids = {s: prng_bytes(seed + 100 + s, max(1, n))[:n] for s, n in enumerate(cid_lens) if n}
    head = 0 if cipher == M.CIPHER_CHACHA20_POLY1305 else 8
    recs = B.plaintext_records(slots, lengths, seed, head=head, tail=48)
    for r in recs:
        r.ver = b"\xfe\xfd"
    return slots, cids, recs


@pytest.mark.parametrize("cipher", ALL_C, ids=list(B.CIPHERS))
def test_cid_batch_encrypt_decrypt(cipher):
    lengths = [0, 1, 14, 15, 16, 17, 31, 47, 63, 64, 65, 127, 128, 200, 1400, 4095, 16383, 16384, 3, 9]
    cid_lens = [1, 4, 5, 9, 16, 21, 25, 32, 0]     # AAD 24..55 bytes = 2..4 blocks, and no CID
    slots, cids, recs = _cid_batch(cipher, lengths * 2, 0xC1D0 + cipher, cid_lens)
    for lanes in (0,):
        b = B.Batch(slots, recs, cids=cids)
        out, res = b.run_gpu(False, lanes=lanes)
        bad = b.compare(False, out, res)
        assert not bad, bad[:5]
    # decrypt what the oracle sealed; each record carries its slot's CID
    o_recs, o_stats = B.Batch(slots, recs, cids=cids).run_oracle(False)
    sealed = []
    for r, o, st in zip(recs, o_recs, o_stats):
        assert st == 0
        sealed.append(B.Rec(slot=r.slot, buf=bytearray(o.buf), data_offset=o.data_offset, data_len=o.data_len,
                            ctr=r.ctr, type=o.type, ver=r.ver, cid=o.cid))
    b = B.Batch(slots, sealed, cids=cids)
    out, res = b.run_gpu(True)
    bad = b.compare(True, out, res)
    assert not bad, bad[:5]
    assert all(int(x) == 0 for x in res["status"])


@pytest.mark.parametrize("cipher", [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305, M.CIPHER_AES_128_CCM_8])
def test_cid_batch_negative(cipher):
    lengths = [5, 100, 1000, 33]
    slots, cids, recs = _cid_batch(cipher, lengths, 0xBAD + cipher, [8])
    o_recs, _ = B.Batch(slots, recs, cids=cids).run_oracle(False)
    sealed = []
    for i, (r, o) in enumerate(zip(recs, o_recs)):
        buf, cid = bytearray(o.buf), o.cid
        if i == 0:
            cid = cid[:-1]                                  # wrong length
        elif i == 1:
            cid = bytes([cid[0] ^ 0x80]) + cid[1:]          # wrong bytes
        elif i == 2:
            buf[o.data_offset + o.data_len - 1] ^= 1        # tampered tag
        sealed.append(B.Rec(slot=r.slot, buf=buf, data_offset=o.data_offset, data_len=o.data_len,
                            ctr=r.ctr, type=o.type, ver=r.ver, cid=cid))
    b = B.Batch(slots, sealed, cids=cids)
    out, res = b.run_gpu(True)
    bad = b.compare(True, out, res)
    assert not bad, bad
    st = [int(x) for x in res["status"]]
    assert st == [M.ERR_SSL_UNEXPECTED_CID, M.ERR_SSL_UNEXPECTED_CID, M.ERR_SSL_INVALID_MAC, 0]
    # the CID-mismatch records are left untouched
    for i in (0, 1):
        o = b.offs[i]
        assert bytes(out[o:o + len(sealed[i].buf)]) == bytes(sealed[i].buf)


@pytest.mark.parametrize("cipher", [M.CIPHER_AES_128_GCM, M.CIPHER_CHACHA20_POLY1305, M.CIPHER_AES_256_CCM])
def test_cid_record_in_table_without_cids(cipher):
    """A key table without connection IDs runs the default (CID-free) kernel
    instantiation: a record that carries a CID does not match the slot's empty
    in_cid -> UNEXPECTED_CID, untouched; its neighbours decrypt normally."""
    slots = [(cipher, M.VERSION_TLS1_2, prng_bytes(0xE0 + cipher, 32)[:M.KEYLEN[cipher]], prng_bytes(0xE1, 16), 0)]
    head = 0 if cipher == M.CIPHER_CHACHA20_POLY1305 else 8
    recs = B.plaintext_records(slots, [40, 300, 17], 0xE2 + cipher, head=head, tail=48)
    o_recs, _ = B.Batch(slots, recs).run_oracle(False)
    sealed = [B.Rec(slot=r.slot, buf=bytearray(o.buf), data_offset=o.data_offset, data_len=o.data_len, ctr=r.ctr,
                    type=o.type, ver=r.ver, cid=(b"\x01\x02\x03" if i == 1 else b"")) for i, (r, o) in enumerate(zip(recs, o_recs))]
    b = B.Batch(slots, sealed)
    out, res = b.run_gpu(True)
    assert not b.compare(True, out, res)
    assert [int(x) for x in res["status"]] == [0, M.ERR_SSL_UNEXPECTED_CID, 0]
    o = b.offs[1]
    assert bytes(out[o:o + len(sealed[1].buf)]) == bytes(sealed[1].buf)
    # the single-record API decides the same on the host
    t = M.Transform(M.VERSION_TLS1_2, cipher, slots[0][2], slots[0][2], slots[0][3], slots[0][3])
    r = sealed[1]
    rec = M.Record(ctr=r.ctr, type=r.type, ver=r.ver, buf=bytearray(r.buf), data_offset=r.data_offset,
                   data_len=r.data_len, cid=r.cid)
    assert t.decrypt_buf(rec) == M.ERR_SSL_UNEXPECTED_CID
