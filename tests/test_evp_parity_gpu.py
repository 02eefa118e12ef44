"""Bulk, independent parity of the GPU record path against OpenSSL EVP.

The reference's own tests hold ciphertext KATs only for TLS 1.3 AES-128-GCM
(/root/reference/tests/suites/test_suite_ssl.data:2776-2834).  For the headline
ciphers these tests compare the GPU's own output with OpenSSL 3 libcrypto
(EVP_aes_128_gcm / _256_gcm / EVP_chacha20_poly1305) wrapped in the ssl_msg.c
record framing (oracle/evp_bench.c evp_check_records; pinned on the CPU against
the oracle by tests/test_evp_baseline.py) -- no record passes through this
repository's oracle:

* >= 10^5 records per (cipher, TLS version) and direction,
  at the edge lengths {0, 1, 15, 16, 17, 1400, 16383} plus random lengths,
  16 keys round-robin (bucket order) and one key (identity order);
* config 2 at its stated size (2^20 x 16 KiB TLS 1.3 AES-256-GCM decrypt, the
  8-lane G5 kernel) with 1 record in 1024 bit-flipped, INVALID_MAC expected at
  exactly those indices (ssl_msg.c:1412-1424), every other
  record's plaintext checked on the device, and a strided sample of 4096
  records' ciphertexts checked against EVP.
"""
from __future__ import annotations

import numpy as np
import pytest

import mbedtls_amd as M
import oracle as O

pytestmark = pytest.mark.gpu

EDGE = np.array([0, 1, 15, 16, 17, 1400, 16383], dtype=np.uint32)


def _torch():
    import torch
    assert torch.cuda.is_available(), "needs a GPU"
    return torch


def _threads():
    import bench
    return bench.host_cores()[0]


def _layout(n, head, rng, span=None, misalign=False):
    """lengths (25 % edge values, 75 % uniform 0..2048, every edge value at
    least 100 times; or uniform in span), 128-B aligned record buffers with
    tag / padding room (misalign: each buffer starts 0..127 bytes into its
    128-B slot)"""
    if span:
        lens = rng.integers(span[0], span[1] + 1, n).astype(np.uint32)
    else:
        lens = rng.integers(0, 2049, n).astype(np.uint32)
        pick = rng.random(n) < 0.25
        lens[pick] = EDGE[rng.integers(0, len(EDGE), int(pick.sum()))]
        lens[:len(EDGE) * 100] = np.tile(EDGE, 100)
    size = head + lens.astype(np.uint64) + 48
    al = (size + 127) // 128 * 128 + (128 if misalign else 0)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(al)[:-1]
    if misalign:
        off += rng.integers(0, 128, n).astype(np.uint64)
    return lens, size, off, int(off[-1] + al[-1])


def _keys(cipher, nkeys, rng):
    kl = M.KEYLEN[cipher]
    keys = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    keys[:, kl:] = 0
    ivs = rng.integers(0, 256, (nkeys, 12), dtype=np.uint8)
    return keys, ivs


CASES = [(c, v) for c in (M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305)
         for v in (M.VERSION_TLS1_2, M.VERSION_TLS1_3)]


@pytest.mark.parametrize("nkeys,n", [(16, 100_000), (1, 30_000)], ids=["16keys", "1key"])
@pytest.mark.parametrize("cipher,ver", CASES, ids=lambda x: str(x))
def test_bulk_records_vs_openssl_evp(cipher, ver, nkeys, n):
    _evp_case(cipher, ver, nkeys, n)


@pytest.mark.parametrize("cipher,ver", CASES[:4], ids=lambda x: str(x))
def test_single_key_small_records_four_lanes_vs_openssl_evp(cipher, ver):
    """One key, 70 000 records of 0..2 048 B (every edge length) with a size
    hint under 4 KiB: the single-key key pass at 4 lanes per record (engine.hip,
    r04; it needs >= 16 records per wave of a full grid), both directions
    against OpenSSL EVP"""
    _evp_case(cipher, ver, 1, 70_000, mean_bytes=1100)


@pytest.mark.parametrize("nkeys,rpk,span,mean", [(2048, 64, (1000, 1500), 1300), (2048, 32, (1000, 1500), 1300),
                                                  (4096, 16, (1000, 1500), 1300), (4096, 8, (12000, 16383), 14000),
                                                  (8192, 4, (12000, 16383), 14000)],
                         ids=["L2", "L4", "L8", "L16", "L32"])
@pytest.mark.parametrize("cipher,ver", [(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3), (M.CIPHER_AES_128_GCM, M.VERSION_TLS1_2)],
                         ids=lambda x: str(x))
def test_paired_wave_passes_vs_openssl_evp(cipher, ver, nkeys, rpk, span, mean):
    """many keys x 4..64 records, round-robin over keys, with the record-size
    hint: the paired wave passes (16 waves, two per key table) at 2, 4 and 8
    lanes for ~1.4 KiB records and 16, 32 lanes for ~14 KiB records"""
    _evp_case(cipher, ver, nkeys, nkeys * rpk, lens=span, mean_bytes=mean)


def _evp_case(cipher, ver, nkeys, n, lens=None, mean_bytes=0, misalign=False):
    torch = _torch()
    dev = torch.device("cuda")
    rng = np.random.default_rng(cipher * 100 + ver + nkeys + n)
    head = 8 if ver == M.VERSION_TLS1_2 and cipher != M.CIPHER_CHACHA20_POLY1305 else 0
    lens_, size, off, total = _layout(n, head, rng, lens, misalign)
    lens = lens_
    keys, ivs = _keys(cipher, nkeys, rng)
    kl = M.KEYLEN[cipher]
    km = np.concatenate([M.key_material(cipher, ver, bytes(k[:kl]), bytes(v)) for k, v in zip(keys, ivs)])
    keyidx = (np.arange(n) % nkeys).astype(np.uint32)
    seq = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    plain = rng.integers(0, 256, total, dtype=np.uint8)
    kt = M.KeyTable(nkeys)
    kt.load(km)
    threads = _threads()
    try:
        # ---- encrypt on the GPU, check every byte against EVP -------------
        d = M.records(n)
        d["buf_off"] = off
        d["buf_len"] = size
        d["data_offset"] = head
        d["data_len"] = lens
        d["slot"] = keyidx
        d["ctr"] = M.seq_bytes(seq)
        d["type"] = 23
        d["ver"] = (3, 3)
        arena = torch.from_numpy(plain).to(dev)
        out = torch.zeros_like(arena)
        res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        recs = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        M.batch_encrypt(kt, recs, res, n, arena, out, mean_bytes=mean_bytes)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(M.BATCH_RES)
        inner = lens + 1 + (16 - (lens + 1) % 16) % 16 if ver == M.VERSION_TLS1_3 else lens
        wire = head + inner + 16
        assert (r["status"] == 0).all()
        assert (r["data_offset"] == 0).all() and (r["data_len"] == wire).all()
        got = out.cpu().numpy()
        bad = O.evp_check_records(1, cipher, ver, keys, ivs, keyidx, seq, off, lens, plain, got, threads)
        assert int((bad != 0).sum()) == 0, f"{int((bad != 0).sum())} of {n} records differ from OpenSSL, " \
                                           f"first {np.flatnonzero(bad)[:5]}"
        # ---- decrypt EVP-sealed records on the GPU -------------------------
        sealed = plain.copy()
        st = O.evp_check_records(0, cipher, ver, keys, ivs, keyidx, seq, off, lens, sealed, None, threads)
        assert (st == 0).all()
        dd = d.copy()
        dd["data_offset"] = 0
        dd["data_len"] = wire
        arena = torch.from_numpy(sealed).to(dev)
        res.zero_()
        recs = torch.from_numpy(dd.view(np.uint8).copy()).to(dev)
        M.batch_decrypt(kt, recs, res, n, arena, arena, mean_bytes=mean_bytes)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(M.BATCH_RES)
        assert (r["status"] == 0).all(), np.unique(r["status"])
        assert (r["data_offset"] == head).all() and (r["data_len"] == lens).all() and (r["type"] == 23).all()
        bad = O.evp_check_records(2, cipher, ver, keys, ivs, keyidx, seq, off, lens, plain, arena.cpu().numpy(),
                                  threads)
        assert int((bad != 0).sum()) == 0, f"{int((bad != 0).sum())} plaintexts differ"
    finally:
        kt.close()


def test_c2_full_size_tamper_1_in_1024_and_evp_sample():
    """2^20 x 16 KiB TLS 1.3 AES-256-GCM decrypt (BASELINE configs[1]) through
    the kernel the bench times (single key: identity order, 8 lanes, G5)."""
    torch = _torch()
    dev = torch.device("cuda")
    n, content, inner, wire, stride = 1 << 20, 16383, 16384, 16400, 16512
    rng = np.random.default_rng(0xC2)
    keys, ivs = _keys(M.CIPHER_AES_256_GCM, 1, rng)
    km = M.key_material(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, bytes(keys[0]), bytes(ivs[0]))
    kt = M.KeyTable(1)
    kt.load(km)
    try:
        d = M.records(n)
        d["buf_off"] = np.arange(n, dtype=np.uint64) * stride
        d["buf_len"] = stride
        d["data_len"] = content
        d["ctr"] = M.seq_bytes(np.arange(n, dtype=np.uint64))
        d["type"] = 23
        d["ver"] = (3, 3)
        g = torch.Generator(device=dev)
        g.manual_seed(12345)
        A = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev, generator=g)
        B = torch.empty_like(A)
        res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        M.batch_encrypt(kt, torch.from_numpy(d.view(np.uint8).copy()).to(dev), res, n, A, B)
        torch.cuda.synchronize()
        st = res.view(torch.int32)[0::4]
        assert int((st != 0).sum()) == 0 and bool((res.view(torch.int32)[2::4] == wire).all())

        # EVP: a strided sample of 4096 ciphertexts, sealed independently
        sample = np.arange(0, n, 256, dtype=np.int64)
        rows_a = A.view(n, stride)[torch.from_numpy(sample).to(dev)].cpu().numpy()
        rows_b = B.view(n, stride)[torch.from_numpy(sample).to(dev)].cpu().numpy()
        off = np.arange(len(sample), dtype=np.uint64) * stride
        plain_h, got_h = rows_a.reshape(-1).copy(), rows_b.reshape(-1).copy()
        bad = O.evp_check_records(1, M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, keys, ivs,
                                  np.zeros(len(sample), np.uint32), sample.astype(np.uint64), off,
                                  np.full(len(sample), content, np.uint32), plain_h, got_h, _threads())
        assert int((bad != 0).sum()) == 0, f"{int((bad != 0).sum())} of 4096 sampled ciphertexts differ from OpenSSL"

        # 1 record in 1024 bit-flipped: odd ones in the tag, even ones in the ciphertext
        tam = np.arange(17, n, 1024, dtype=np.int64)
        pos = np.where(np.arange(len(tam)) % 2 == 1, inner + (tam % 16), (tam * 37) % inner)
        flat = torch.from_numpy(tam * stride + pos).to(dev)
        bit = torch.from_numpy((1 << (tam % 8)).astype(np.uint8)).to(dev)
        B[flat] = B[flat] ^ bit
        dd = d.copy()
        dd["data_len"] = wire
        C = torch.empty_like(A)
        res.zero_()
        M.batch_decrypt(kt, torch.from_numpy(dd.view(np.uint8).copy()).to(dev), res, n, B, C)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(M.BATCH_RES)
        want = np.zeros(n, dtype=np.int32)
        want[tam] = M.ERR_SSL_INVALID_MAC
        assert np.array_equal(r["status"], want), np.flatnonzero(r["status"] != want)[:10]
        ok = np.ones(n, bool)
        ok[tam] = False
        assert (r["data_len"][ok] == content).all() and (r["type"][ok] == 23).all()
        # every other record's plaintext, on the device; the tampered ones wiped
        Av, Cv = A.view(n, stride), C.view(n, stride)
        okd = torch.from_numpy(ok).to(dev)
        for lo in range(0, n, 1 << 15):
            hi = lo + (1 << 15)
            same = (Av[lo:hi, :content] == Cv[lo:hi, :content]).all(dim=1)
            assert bool((same | ~okd[lo:hi]).all()), f"plaintext mismatch in rows {lo}..{hi}"
        wiped = Cv[torch.from_numpy(tam).to(dev)]
        assert int(wiped.count_nonzero()) == 0, "a record that failed its tag kept output bytes"
        del A, B, C
    finally:
        kt.close()


@pytest.mark.parametrize("tm", ["15", "7", "0"])
@pytest.mark.parametrize("nkeys,rpk,span,mean", [(2048, 64, (1000, 1500), 1300), (4096, 16, (1000, 1500), 1300),
                                                  (8192, 4, (12000, 16383), 14000)], ids=["L2", "L8", "L32"])
def test_paired_wave_passes_tree_modes_vs_openssl_evp(monkeypatch, tm, nkeys, rpk, span, mean):
    """the wave passes' once-per-record multiplies (AAD fold, lane tree, the
    two final multiplies) from the key's tables in global memory (TREEMUL=0),
    all of them table-free by H as a value (TREEMUL=7), and the r04 default,
    lane powers (TREEMUL=15: AAD and length block in the lane layout, one
    multiply by H^(L-q) per lane)"""
    monkeypatch.setenv("TLSREC_GCM_TREEMUL", tm)
    _evp_case(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, nkeys, nkeys * rpk, lens=span, mean_bytes=mean)


def _evp_sample(torch, dev, A, B, stride, sample, km_keys, km_ivs, slots, cipher, ver, content, threads):
    """EVP check of the sampled records' ciphertexts (B) sealed from A, with a
    compact key table holding only the sample's keys"""
    uk, kidx = np.unique(slots[sample], return_inverse=True)
    n = len(sample)
    rows_a = A.view(-1, stride)[torch.from_numpy(sample).to(dev)].cpu().numpy()
    rows_b = B.view(-1, stride)[torch.from_numpy(sample).to(dev)].cpu().numpy()
    off = np.arange(n, dtype=np.uint64) * stride
    return O.evp_check_records(1, cipher, ver, km_keys[uk], km_ivs[uk], kidx.astype(np.uint32),
                               sample.astype(np.uint64) // len(km_keys), off, np.full(n, content, np.uint32),
                               rows_a.reshape(-1).copy(), rows_b.reshape(-1).copy(), threads)


def _full_size_row(nkeys, rpk, content, key_ciphers, seed, in_place=False):
    """A BASELINE row at its stated size, as bench.py launches it: nkeys keys
    (cipher of key k = key_ciphers[k % len]), nkeys x rpk TLS 1.3 records of
    `content` bytes in 128-B slots, record i under key i % nkeys with sequence
    number i // nkeys, the record-size hint (tlsrec_batch_*_sized).  Encrypt:
    every status and length, a >= 4096-record EVP sample over every cipher
    and the first and last keys.  Decrypt: 1 record in 1024 bit-flipped,
    INVALID_MAC at exactly those indices, every other plaintext checked on the
    device, the failed ones wiped (ssl_msg.c:1043, :1412-1424)."""
    torch = _torch()
    dev = torch.device("cuda")
    n = nkeys * rpk
    inner = content + 1 + (16 - (content + 1) % 16) % 16
    wire = inner + 16
    stride = (wire + 127) // 128 * 128
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    ivs = rng.integers(0, 256, (nkeys, 12), dtype=np.uint8)
    cip = np.array(key_ciphers, dtype=np.uint8)[np.arange(nkeys) % len(key_ciphers)]
    km = np.zeros(nkeys, dtype=M.KEY_MATERIAL)
    km["cipher"] = cip
    km["tls_minor"] = 4
    km["fixed_ivlen"] = 12
    km["taglen"] = 16
    km["key"] = keys
    km["iv"][:, :12] = ivs
    kt = M.KeyTable(nkeys)
    kt.load(km)
    slots = (np.arange(n) % nkeys).astype(np.uint32)
    try:
        d = M.records(n)
        d["buf_off"] = np.arange(n, dtype=np.uint64) * stride
        d["buf_len"] = stride
        d["data_len"] = content
        d["slot"] = slots
        d["ctr"] = M.seq_bytes(np.arange(n, dtype=np.uint64) // nkeys)
        d["type"] = 23
        d["ver"] = (3, 3)
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        A = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev, generator=g)
        B = torch.empty_like(A)
        res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        M.batch_encrypt(kt, torch.from_numpy(d.view(np.uint8).copy()).to(dev), res, n, A, B, mean_bytes=wire)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(M.BATCH_RES)
        assert (r["status"] == 0).all(), np.unique(r["status"], return_counts=True)
        assert (r["data_offset"] == 0).all() and (r["data_len"] == wire).all()
        assert (r["type"] == 23).all()

        # EVP: >= 4096 records over every cipher, with every record of the
        # first and of the last key
        sample = np.unique(np.concatenate([np.arange(0, n, max(1, n // 4100), dtype=np.int64)[:4100],
                                           np.arange(0, n, nkeys, dtype=np.int64)[:4096],
                                           np.arange(nkeys - 1, n, nkeys, dtype=np.int64)[:4096]]))
        assert len(sample) >= 4096
        for c in sorted(set(int(x) for x in key_ciphers)):
            s = sample[cip[slots[sample]] == c]
            assert len(s) >= 4096 // len(set(key_ciphers)) - 8
            bad = _evp_sample(torch, dev, A, B, stride, s, keys, ivs, slots, c, M.VERSION_TLS1_3, content, _threads())
            assert int((bad != 0).sum()) == 0, f"cipher {c}: {int((bad != 0).sum())} of {len(s)} differ from OpenSSL"

        # decrypt with 1 record in 1024 bit-flipped (odd: tag, even: ciphertext)
        tam = np.arange(29, n, 1024, dtype=np.int64)
        pos = np.where(np.arange(len(tam)) % 2 == 1, inner + (tam % 16), (tam * 37) % inner)
        flat = torch.from_numpy(tam * stride + pos).to(dev)
        bit = torch.from_numpy((1 << (tam % 8)).astype(np.uint8)).to(dev)
        B[flat] = B[flat] ^ bit
        dd = d.copy()
        dd["data_len"] = wire
        C = B if in_place else torch.empty_like(A)
        res.zero_()
        M.batch_decrypt(kt, torch.from_numpy(dd.view(np.uint8).copy()).to(dev), res, n, B, C, mean_bytes=wire)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(M.BATCH_RES)
        want = np.zeros(n, dtype=np.int32)
        want[tam] = M.ERR_SSL_INVALID_MAC
        assert np.array_equal(r["status"], want), np.flatnonzero(r["status"] != want)[:10]
        ok = np.ones(n, bool)
        ok[tam] = False
        assert (r["data_len"][ok] == content).all() and (r["type"][ok] == 23).all()
        assert (r["data_offset"][ok] == 0).all()
        Av, Cv = A.view(n, stride), C.view(n, stride)
        okd = torch.from_numpy(ok).to(dev)
        step = max(1, (1 << 28) // stride)
        for lo in range(0, n, step):
            hi = lo + step
            same = (Av[lo:hi, :content] == Cv[lo:hi, :content]).all(dim=1)
            assert bool((same | ~okd[lo:hi]).all()), f"plaintext mismatch in rows {lo}..{hi}"
        wiped = Cv[torch.from_numpy(tam).to(dev), :inner]
        assert int(wiped.count_nonzero()) == 0, "a record that failed its tag kept output bytes"
        del A, B, C
    finally:
        kt.close()
        torch.cuda.empty_cache()


def test_c4s_full_size_mixed_keys_tamper_and_evp_sample():
    """SURVEY 8(d)-4's 1400-B variant at its stated size, as bench.py times it:
    65 536 keys x 64 records x 1 400 B TLS 1.3, AES-256-GCM (even keys) and
    ChaCha20-Poly1305 (odd keys), the line-grouped paired 2-lane GCM passes
    and 2-lane ChaCha20-Poly1305."""
    _full_size_row(1 << 16, 64, 1400, [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305], 0xC45)


def test_c3_c3d_full_size_tamper_and_evp_sample():
    """BASELINE configs[2] (c3) at its stated size, as bench.py times it: one
    key, 2^20 x 1 400 B TLS 1.3 ChaCha20-Poly1305, identity order, 2 lanes per
    record (engine.hip: n / (cu x 8) >= 32).  Encrypt is c3, the tampered
    decrypt of its output is c3d (the same launch)."""
    _full_size_row(1, 1 << 20, 1400, [M.CIPHER_CHACHA20_POLY1305], 0xC3)


def test_c4_full_size_mixed_keys_tamper_and_evp_sample():
    """BASELINE configs[3] (c4) at its stated size, as bench.py times it:
    65 536 keys x 64 records x 16 KiB TLS 1.3, AES-256-GCM (even keys) and
    ChaCha20-Poly1305 (odd keys), the 16-lane GCM key passes and 2-lane
    ChaCha20-Poly1305; decrypted in place (two 69 GB arenas)."""
    _full_size_row(1 << 16, 64, 16383, [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305], 0xC4, in_place=True)


@pytest.mark.parametrize("nkeys,rpk", [(2048, 64), (4096, 32), (4096, 16)], ids=["L2", "L4", "L8"])
@pytest.mark.parametrize("cipher,ver", [(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3), (M.CIPHER_AES_128_GCM, M.VERSION_TLS1_2),
                                        (M.CIPHER_CHACHA20_POLY1305, M.VERSION_TLS1_3)], ids=lambda x: str(x))
def test_line_groups_unaligned_records_vs_openssl_evp(cipher, ver, nkeys, rpk):
    """the line-grouped body of the small-record passes with record buffers at
    arbitrary byte offsets (not 128-B lines) and ragged lengths, so group
    boundaries fall anywhere in a record (the stream / DTLS layers' case)"""
    _evp_case(cipher, ver, nkeys, nkeys * rpk, lens=(900, 1500), mean_bytes=1300, misalign=True)


@pytest.mark.parametrize("nkeys,rpk,span,mean", [(2048, 64, (1000, 1500), 1300), (8192, 4, (12000, 16383), 14000),
                                                  (64, 1024, (0, 4000), 0)], ids=["pairL2", "pairL32", "keypassL8"])
def test_key_ordered_descriptors_vs_openssl_evp(monkeypatch, nkeys, rpk, span, mean):
    """TLSREC_GCM_SRECS=1: the bucket pass also writes the GCM records'
    descriptors in key order and the GCM kernels read them there (paired
    passes and the 16-wave key passes)"""
    monkeypatch.setenv("TLSREC_GCM_SRECS", "1")
    _evp_case(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, nkeys, nkeys * rpk, lens=span, mean_bytes=mean)
    _evp_case(M.CIPHER_AES_128_GCM, M.VERSION_TLS1_2, nkeys, nkeys * rpk, lens=span, mean_bytes=mean)


@pytest.mark.parametrize("nkeys,n", [(1, 30_000), (64, 65_536)], ids=["1key_G5", "64keys_keypass"])
@pytest.mark.parametrize("cipher,ver", CASES[:4], ids=lambda x: str(x))
def test_key_pass_tree_modes_vs_openssl_evp(monkeypatch, cipher, ver, nkeys, n):
    """TLSREC_GCM_TREEMUL=9 on the 16-wave key-pass kernels, single key (the G5
    kernel, 4 lanes per record) and many keys: lane powers are compiled into
    the wave-pass kernels only, so the key passes must ignore bit 3 and still
    match OpenSSL byte for byte"""
    monkeypatch.setenv("TLSREC_GCM_TREEMUL", "9")
    _evp_case(cipher, ver, nkeys, n)


_SMALL16 = (2048, 16, (1000, 1500), 1300)     # DTLS / stream shape: paired passes, 8 lanes
_SMALL40 = (1024, 40, (1000, 1500), 1300)     # paired passes, lane model
_SMALL64 = (512, 64, (1000, 1500), 1300)      # c4s's records per key
_BIG4 = (2048, 4, (12000, 16383), 14000)      # k4's shape: paired passes, 32 lanes
_BIG16 = (512, 16, (12000, 16383), 14000)     # paired passes, 16 lanes


@pytest.mark.parametrize("var,val,shape", [
    ("TLSREC_GCM_G5", "0", (1, 1, None, 0)),
    ("TLSREC_GCM_HBUILD", "0", _SMALL16), ("TLSREC_GCM_HBUILD", "0", _BIG4),
    ("TLSREC_GCM_PAIR", "0", _SMALL16), ("TLSREC_GCM_PAIR", "0", _BIG4),
    ("TLSREC_GCM_PAIR_L", "2", _SMALL40), ("TLSREC_GCM_PAIR_L", "4", _SMALL40), ("TLSREC_GCM_PAIR_L", "8", _SMALL40),
    ("TLSREC_GCM_PAIR_BIG_MAX", "12", _BIG16),
    ("TLSREC_GCM_PAIR_SMALL_MIN", "200", _SMALL64), ("TLSREC_GCM_PAIR_SMALL_MAX", "13", _SMALL16),
], ids=lambda x: x if isinstance(x, str) else (f"{x[0]}x{x[1]}" if isinstance(x, tuple) else str(x)))
def test_engine_overrides_vs_openssl_evp(monkeypatch, var, val, shape):
    """The measurement overrides of the engine's kernel choice (INTEGRATION
    §5) select kernels the default rules use elsewhere or not at all (the
    4-bit Horner table for a single key, the Horner table staged from HBM,
    the 8-wave wave passes instead of the pairs, forced pair lanes, the
    16-wave key passes at the pairs' records per key): every record of both
    directions against OpenSSL under each."""
    nkeys, rpk, lens, mean = shape
    n = 30_000 if nkeys == 1 else nkeys * rpk
    monkeypatch.setenv(var, val)
    _evp_case(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, nkeys, n, lens=lens, mean_bytes=mean)
    _evp_case(M.CIPHER_AES_128_GCM, M.VERSION_TLS1_2, nkeys, n, lens=lens, mean_bytes=mean)
