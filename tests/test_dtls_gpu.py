"""GPU parity of the DTLS 1.2 datagram record layer (tlsrec_dtls_decrypt /
tlsrec_dtls_encrypt through the C ABI) against the oracle's restatement of the
datagram branch of ssl_get_next_record / mbedtls_ssl_write_record
(oracle/dtls.c): byte-exact datagrams, every record's disposition, the
connection state afterwards (anti-replay window, badmac_seen, nb_zero), and
the reference's 19 anti-replay vectors run through whole records."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import mbedtls_amd as M  # noqa: E402
from mbedtls_amd import dtls as D  # noqa: E402
from mbedtls_amd import stream as S  # noqa: E402
import oracle as O  # noqa: E402
from tests.prng import prng_bytes  # noqa: E402

REPLAY = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dtls_replay.json")))["cases"]
X = bytes.fromhex
TLS12_CIPHERS = [c for c in sorted(M.KEYLEN)]
DEV = torch.device("cuda")


def _al(x, a=128):
    return (x + a - 1) // a * a


def ctr(epoch, seq):
    return epoch.to_bytes(2, "big") + (seq % (1 << 48)).to_bytes(6, "big")


class Table:
    """slots: list of (cipher, key, iv, cid) -- TLS 1.2 keys; a slot with a CID
    is one direction (its out_cid when sending, in_cid when receiving)."""

    def __init__(self, slots, tls=M.VERSION_TLS1_2):
        self.slots = slots
        self.kt = M.KeyTable(len(slots))
        self.kt.load(np.concatenate([M.key_material(c, tls, k, iv) for c, k, iv, _ in slots]))
        self.ot = []
        for s, (c, k, iv, cid) in enumerate(slots):
            if cid:
                self.kt.set_cid(s, cid)
            t = O.Transform(O.TLS1_2 if tls == M.VERSION_TLS1_2 else O.TLS1_3, c, k, k, iv, iv)
            t.set_cid(cid, cid)
            self.ot.append(t)
        torch.cuda.synchronize()

    def encrypt(self, jobs):
        """jobs: (slot, plaintext, out_ctr bytes, max_frag, type) -> [(res, datagram bytes back to back, recs, res)]"""
        d = np.zeros(len(jobs), dtype=S.STREAM_OUT)
        pos_in, pos_out, outs, ins = 0, 0, [], []
        for i, (slot, pt, c8, frag, typ) in enumerate(jobs):
            c, _, _, cid = self.slots[slot]
            size = D.out_size(c, 0, len(cid), len(pt), frag)
            d[i]["in_off"], d[i]["in_len"], d[i]["slot"] = pos_in, len(pt), slot
            d[i]["out_off"], d[i]["max_frag"], d[i]["type"] = pos_out, frag, typ
            d[i]["out_ctr"] = np.frombuffer(c8, dtype=np.uint8)
            ins.append(pos_in)
            outs.append((pos_out, size))
            pos_in += _al(len(pt) + 1)
            pos_out += _al(size + 1)
        ina = np.zeros(max(pos_in, 16), dtype=np.uint8)
        for (slot, pt, *_), o in zip(jobs, ins):
            ina[o:o + len(pt)] = np.frombuffer(pt, dtype=np.uint8)
        tin = torch.from_numpy(ina).to(DEV)
        tout = torch.zeros(max(pos_out, 16), dtype=torch.uint8, device=DEV)
        nmax = sum((len(j[1]) + (j[3] or 16384) - 1) // (j[3] or 16384) for j in jobs) + 1
        recs = torch.zeros(nmax * 40, dtype=torch.uint8, device=DEV)
        res = torch.zeros(nmax * 16, dtype=torch.uint8, device=DEV)
        sres = torch.zeros(len(jobs) * 32, dtype=torch.uint8, device=DEV)
        D.encrypt(self.kt, d, len(jobs), tin, tout, recs, res, nmax, sres)
        torch.cuda.synchronize()
        o = tout.cpu().numpy()
        sr = sres.cpu().numpy().view(S.STREAM_OUT_RES)
        rc = recs.cpu().numpy().view(M.BATCH_REC)
        rs = res.cpu().numpy().view(M.BATCH_RES)
        self.last_regions = [o[p:p + size].tobytes() for p, size in outs]   # each job's whole output region
        return [(sr[i], o[p:p + int(sr[i]["out_len"])].tobytes(), rc, rs) for i, (p, _) in enumerate(outs)]

    def decrypt(self, conns):
        """conns: (slot, dict of DtlsState fields, [datagram bytes])"""
        d = np.zeros(len(conns), dtype=D.DTLS_IN)
        dgl, pos, offs = [], 0, []
        for i, (slot, stt, dgs) in enumerate(conns):
            d[i]["first_dgram"], d[i]["ndgram"], d[i]["slot"] = len(dgl), len(dgs), slot
            d[i]["window_top"], d[i]["window"] = stt.get("window_top", 0), stt.get("window", 0)
            d[i]["badmac_seen"], d[i]["badmac_limit"] = stt.get("badmac_seen", 0), stt.get("badmac_limit", 0)
            d[i]["in_epoch"], d[i]["cid_len"], d[i]["nb_zero"] = stt.get("in_epoch", 0), stt.get("cid_len", 0), \
                stt.get("nb_zero", 0)
            d[i]["flags"] = (M.DTLS_ANTI_REPLAY if stt.get("anti_replay", 1) else 0) | \
                (M.DTLS_IGNORE_UNEXPECTED_CID if stt.get("ignore_unexpected_cid", 0) else 0)
            o = []
            for g in dgs:
                dgl.append((pos, len(g)))
                o.append(pos)
                pos += _al(len(g) + 3) + 16 * (len(dgl) % 3)     # assorted alignments
            offs.append(o)
        a = np.zeros(max(pos, 16), dtype=np.uint8)
        for (slot, stt, dgs), o in zip(conns, offs):
            for g, p in zip(dgs, o):
                a[p:p + len(g)] = np.frombuffer(g, dtype=np.uint8)
        dg = np.zeros(max(1, len(dgl)), dtype=D.DGRAM)
        for k, (p, L) in enumerate(dgl):
            dg[k]["off"], dg[k]["len"] = p, L
        ta = torch.from_numpy(a).to(DEV)
        nmax = sum(len(g) // 13 + 1 for c in conns for g in c[2]) + 1
        recs = torch.zeros(nmax * 40, dtype=torch.uint8, device=DEV)
        res = torch.zeros(nmax * 16, dtype=torch.uint8, device=DEV)
        disp = torch.zeros(nmax, dtype=torch.int32, device=DEV)
        cres = torch.zeros(len(conns) * 48, dtype=torch.uint8, device=DEV)
        D.decrypt(self.kt, d, len(conns), dg, len(dgl), ta, recs, res, disp, nmax, cres)
        torch.cuda.synchronize()
        return (ta.cpu().numpy(), recs.cpu().numpy().view(M.BATCH_REC), res.cpu().numpy().view(M.BATCH_RES),
                disp.cpu().numpy(), cres.cpu().numpy().view(D.DTLS_IN_RES), offs)

    def close(self):
        self.kt.close()


def check_vs_oracle(tab, conns, got):
    a, recs, res, disp, cres, offs = got
    for i, (slot, stt, dgs) in enumerate(conns):
        st = O.DtlsState()
        st.anti_replay = stt.get("anti_replay", 1)
        for f in ("window_top", "window", "badmac_seen", "badmac_limit", "in_epoch", "cid_len",
                  "ignore_unexpected_cid", "nb_zero"):
            if f in stt:
                setattr(st, f, stt[f])
        want, wrecs, after = O.dtls_decrypt(tab.ot[slot], st, dgs)
        g = cres[i]
        assert (int(g["status"]), int(g["nrec"]), int(g["naccepted"]), int(g["dgrams_done"]),
                int(g["invalid_dgrams"])) == (want["status"], want["nrec"], want["naccepted"],
                                              want["dgrams_done"], want["invalid_dgrams"]), (i, want)
        assert (int(g["window_top"]), int(g["window"]), int(g["badmac_seen"]), int(g["nb_zero"])) == \
            (st.window_top, st.window, st.badmac_seen, st.nb_zero), i
        f = int(g["first"])
        for k, (dgi, off, doff, dlen, dsp, typ) in enumerate(wrecs):
            assert int(disp[f + k]) == dsp, (i, k, dsp, int(disp[f + k]))
            assert int(recs[f + k]["buf_off"]) == offs[i][dgi] + off, (i, k)
            if dsp in (M.DTLS_DROPPED, M.DTLS_NOT_REACHED, M.ERR_SSL_UNEXPECTED_RECORD):
                # never decrypted by the reference: no plaintext may be left
                # (each byte is the received one, or wiped to zero)
                s0 = offs[i][dgi] + off
                got_b = a[s0:s0 + doff + dlen]
                rx = np.frombuffer(after[dgi][off:off + doff + dlen], dtype=np.uint8)
                assert ((got_b == rx) | (got_b == 0)).all(), (i, k, dsp)
            if dsp == 0:
                r = res[f + k]
                assert (int(r["data_offset"]), int(r["data_len"]), int(r["type"])) == (doff, dlen, typ), (i, k)
                s0 = offs[i][dgi] + off + doff
                assert a[s0:s0 + dlen].tobytes() == after[dgi][off + doff:off + doff + dlen], (i, k)


def _slots(seed, cid_every=0):
    out = []
    for i, c in enumerate(TLS12_CIPHERS):
        b = prng_bytes(seed * 1000 + i, 48)
        cid = prng_bytes(seed + 77 * i, 1 + i % 6) if cid_every and i % cid_every == 0 else b""
        out.append((c, b[:M.KEYLEN[c]], b[32:48], cid))
    return out


@pytest.mark.parametrize("with_cid", [False, True], ids=["nocid", "cid"])
def test_send_then_receive_every_cipher(with_cid):
    slots = _slots(5, cid_every=2 if with_cid else 0)
    tab = Table(slots)
    rng = np.random.default_rng(11)
    jobs = []
    for i in range(3 * len(slots)):
        n = int(rng.choice([0, 1, 15, 16, 300, 1400, 16384, 20000]))
        frag = int(rng.choice([0, 1200, 4096]))
        jobs.append((i % len(slots), prng_bytes(500 + i, n), ctr(1 + i % 3, int(rng.integers(0, 1 << 40))), frag,
                     23 if i % 5 else 22))
    got = tab.encrypt(jobs)
    conns = []
    for (slot, pt, c8, frag, typ), (r, out, rc, rs) in zip(jobs, got):
        st, want, nrec, c2 = O.dtls_encrypt(tab.ot[slot], pt, typ, c8, frag or 16384)
        assert (int(r["status"]), int(r["nrec"]), out, bytes(r["out_ctr"])) == (st, nrec, want, c2)
        # split the datagrams back out (record k: header at buf_off - 13 - cid_len)
        cid = len(slots[slot][3])
        f = int(r["first"])
        dgs = []
        for k in range(nrec):
            start = int(rc[f + k]["buf_off"]) - 13 - cid - int(r["first"]) * 0
            dgs.append((start, 13 + cid + int(rs[f + k]["data_len"])))
        base = dgs[0][0] if dgs else 0
        grams = [out[s - base:s - base + L] for s, L in dgs]
        if len(grams) >= 3:                       # two records packed into one datagram
            grams = [grams[0] + grams[1]] + grams[2:]
        conns.append((slot, {"in_epoch": int.from_bytes(c8[:2], "big"), "cid_len": cid}, grams))
    check_vs_oracle(tab, conns, tab.decrypt(conns))
    tab.close()


def test_reference_replay_vectors_through_records():
    """ssl_dtls_replay (test_suite_ssl.data:763-818) as whole records: the
    `prevs` arrive first (all accepted), then `new` is accepted iff the
    reference's mbedtls_ssl_dtls_replay_check returns 0."""
    key, iv = prng_bytes(1, 16), prng_bytes(2, 16)
    tab = Table([(M.CIPHER_AES_128_GCM, key, iv, b"")])
    t = tab.ot[0]
    conns = []
    for case in REPLAY:
        seqs = [int(p, 16) for p in case["prevs"]] + [int(case["new"], 16)]
        grams = []
        for s in seqs:
            st, w, _, _ = O.dtls_encrypt(t, prng_bytes(s & 0xFFFF, 40), 23, ctr(7, s), 16384)
            assert st == 0
            grams.append(w)
        conns.append((0, {"in_epoch": 7}, grams))
    got = tab.decrypt(conns)
    check_vs_oracle(tab, conns, got)
    _, _, _, disp, cres, _ = got
    for i, case in enumerate(REPLAY):
        last = int(cres[i]["first"]) + int(cres[i]["nrec"]) - 1
        assert int(disp[last]) == (0 if case["ret"] == 0 else M.ERR_SSL_UNEXPECTED_RECORD), case["name"]
        assert int(cres[i]["naccepted"]) == len(case["prevs"]) + (case["ret"] == 0)
    tab.close()


FRAMINGS = [("1", "1"), ("1", "0"), ("0", "0")]
FRAMING_IDS = ["one-pass", "grouped-3-kernels", "bucket-pass-3-kernels"]


def _framing(monkeypatch, fr):
    grouped, fused = fr
    monkeypatch.setenv("TLSREC_GROUPED", grouped)       # the batch without (r06) and with (r05) the bucket pass,
    monkeypatch.setenv("TLSREC_RX_FUSED", fused)        # count / scan / emit as one pass (look-back) or three kernels


@pytest.mark.parametrize("fr", FRAMINGS, ids=FRAMING_IDS)
def test_dispositions_match_oracle(fr, monkeypatch):
    _framing(monkeypatch, fr)
    cid = b"\xaa\xbb\xcc"
    slots = [(M.CIPHER_AES_128_GCM, prng_bytes(3, 16), prng_bytes(4, 16), b""),
             (M.CIPHER_CHACHA20_POLY1305, prng_bytes(5, 32), prng_bytes(6, 16), cid),
             (M.CIPHER_AES_256_CCM_8, prng_bytes(7, 32), prng_bytes(8, 16), b""),
             (M.CIPHER_CHACHA20_POLY1305, prng_bytes(5, 32), prng_bytes(6, 16), b"")]
    tab = Table(slots)

    def rec(slot, seq, epoch=1, n=200, typ=23):
        st, w, _, _ = O.dtls_encrypt(tab.ot[slot], prng_bytes(seq + 31 * slot, n), typ, ctr(epoch, seq), 16384)
        assert st == 0
        return w

    def flip(w, at):
        b = bytearray(w)
        b[at] ^= 0x10
        return bytes(b)

    g = [rec(0, k) for k in range(12)]
    empty = [rec(0, 40 + k, n=0) for k in range(5)]
    conns = [
        (0, {"in_epoch": 1}, [g[0], g[0], rec(0, 50, epoch=0), rec(0, 60, epoch=2), flip(g[2], 40) + g[3], g[3],
                              b"\x17\xfe\xfd" + bytes(8), g[4] + b"\x40" + g[5][1:], g[5], g[2]]),
        # a replayed copy of a record whose first copy fails its MAC is accepted
        (0, {"in_epoch": 1}, [flip(g[6], 50), g[6], g[6]]),
        # badmac_limit reached: fatal, the rest not reached
        (0, {"in_epoch": 1, "badmac_limit": 2}, [g[0], flip(g[1], 30), g[2], flip(g[3], 30), g[4], g[5]]),
        (0, {"in_epoch": 1, "badmac_limit": 3, "badmac_seen": 1}, [flip(g[1], 30), g[2]]),
        # trailing bytes, empty datagram, truncated header
        (0, {"in_epoch": 1}, [g[0] + b"\x17\xfe\xfd", g[1]]),
        (0, {"in_epoch": 1}, [g[0], b"", g[1]]),
        (0, {"in_epoch": 1}, [g[0][:20], g[1][:-1], g[2]]),
        # window state carried in; shift beyond 64; anti-replay off
        (0, {"in_epoch": 1, "window_top": 9, "window": 0b1011}, [g[9], g[8], g[7], g[6], g[10]]),
        (0, {"in_epoch": 1}, [rec(0, 100), rec(0, 30), rec(0, 100), rec(0, 37)]),
        (0, {"in_epoch": 1, "anti_replay": 0}, [g[3], g[3], g[1]]),
        # empty records: nb_zero, then a MAC failure counts as dropped datagram
        (0, {"in_epoch": 1}, [empty[0] + empty[1] + empty[2] + empty[3] + g[11], empty[4]]),
        (0, {"in_epoch": 1, "nb_zero": 2}, [empty[0], g[1]]),
        # non-application zero-length record in TLS 1.2: fatal INVALID_RECORD
        (0, {"in_epoch": 1}, [rec(0, 70, n=0, typ=22), g[1]]),
        # version quirk of mbedtls_ssl_read_version (FE FF / 00 00 parse, 03 03 does not)
        (0, {"in_epoch": 1}, [g[1][:1] + b"\xfe\xff" + g[1][3:], g[1][:1] + b"\x03\x03" + g[1][3:],
                              g[1][:1] + b"\x00\x00" + g[1][3:], g[1]]),
        # CID endpoint: a record without a CID is UNEXPECTED_CID (ignored / fatal)
        (1, {"in_epoch": 1, "cid_len": 3, "ignore_unexpected_cid": 1}, [rec(1, 1), rec(3, 2), rec(1, 3)]),
        (1, {"in_epoch": 1, "cid_len": 3}, [rec(1, 1), rec(3, 2), rec(1, 3)]),
        # a CID the endpoint does not expect: header error
        (1, {"in_epoch": 1, "cid_len": 0}, [rec(1, 1)]),
        # CCM_8 records with a short body (below tag length): INVALID_MAC before the AEAD
        (2, {"in_epoch": 1}, [rec(2, 1), rec(2, 2)[:11] + b"\x00\x05" + bytes(5), rec(2, 3)]),
        # an oversized datagram (read truncated to the in buffer)
        (0, {"in_epoch": 1}, [g[0] + bytes(M.DTLS_MAX_DATAGRAM)]),
    ]
    check_vs_oracle(tab, conns, tab.decrypt(conns))
    tab.close()


@pytest.mark.parametrize("fr", FRAMINGS, ids=FRAMING_IDS)
def test_many_datagrams_per_connection(fr, monkeypatch):
    """Many datagrams per connection: 37 and 50 datagrams of one to three records, a bad MAC
    and a replay among them, and a connection with none -- record order and
    dispositions against the oracle, under every framing path"""
    _framing(monkeypatch, fr)
    slots = [(M.CIPHER_AES_128_GCM, prng_bytes(13, 16), prng_bytes(14, 16), b""),
             (M.CIPHER_CHACHA20_POLY1305, prng_bytes(15, 32), prng_bytes(16, 16), b"")]
    tab = Table(slots)

    def rec(slot, seq, n):
        st, w, _, _ = O.dtls_encrypt(tab.ot[slot], prng_bytes(seq + 97 * slot, n), 23, ctr(1, seq), 16384)
        assert st == 0
        return w

    grams0, seq = [], 0
    for k in range(37):
        g = b""
        for _ in range(1 + k % 3):
            g += rec(0, seq, 40 + 13 * (seq % 7))
            seq += 1
        grams0.append(g)
    bad = bytearray(grams0[20])
    bad[30] ^= 0x04
    grams0[20] = bytes(bad)
    grams0.append(grams0[5])                       # a replayed datagram
    grams1 = [rec(1, k, 100 + k) for k in range(50)]
    conns = [(0, {"in_epoch": 1}, grams0), (1, {"in_epoch": 1}, []), (1, {"in_epoch": 1}, grams1)]
    check_vs_oracle(tab, conns, tab.decrypt(conns))
    tab.close()


@pytest.mark.parametrize("fr", FRAMINGS[:2], ids=FRAMING_IDS[:2])
def test_many_connections_match_oracle(fr, monkeypatch):
    """17 000 connections (67 tiles of the one-pass framing kernel's look-back)
    of 0..3 datagrams, each of one or two records (the register fast path and
    the walk from memory), with replays, other epochs, a bad MAC and a
    trailing byte among them: against the oracle, connection by connection."""
    _framing(monkeypatch, fr)
    slots = [(M.CIPHER_AES_128_GCM, prng_bytes(21, 16), prng_bytes(22, 16), b""),
             (M.CIPHER_CHACHA20_POLY1305, prng_bytes(23, 32), prng_bytes(24, 16), b""),
             (M.CIPHER_AES_256_GCM, prng_bytes(25, 32), prng_bytes(26, 16), b"")]
    tab = Table(slots)
    rng = np.random.default_rng(41)

    def rec(slot, seq, n, epoch=1):
        st, w, _, _ = O.dtls_encrypt(tab.ot[slot], prng_bytes(seq * 7 + slot, n), 23, ctr(epoch, seq), 16384)
        assert st == 0
        return w

    conns = []
    for i in range(17000):
        slot = i % 3
        seq = int(rng.integers(1, 1000))
        grams = []
        for _ in range(int(rng.integers(0, 4))):
            g = rec(slot, seq, int(rng.integers(1, 90)))
            seq += 1
            u = rng.random()
            if u < 0.15:
                g += rec(slot, seq, int(rng.integers(1, 40)))             # two records in one datagram
                seq += 1
            elif u < 0.18:
                g = g[:20] + bytes([g[20] ^ 1]) + g[21:]                   # bad MAC
            elif u < 0.20:
                g += b"\x17"                                             # one trailing byte
            elif u < 0.23:
                g = rec(slot, seq - 1, 30, epoch=2)                        # the next epoch
            grams.append(g)
        if grams and rng.random() < 0.05:
            grams.append(grams[0])                                         # a replay
        conns.append((slot, {"in_epoch": 1}, grams))
    check_vs_oracle(tab, conns, tab.decrypt(conns))
    tab.close()


def test_tls13_slot_is_bad_input():
    tab = Table([(M.CIPHER_AES_128_GCM, bytes(16), bytes(16), b"")], tls=M.VERSION_TLS1_3)
    t12 = O.Transform(O.TLS1_2, O.AES_128_GCM, bytes(16), bytes(16), bytes(16), bytes(16))
    _, w, _, _ = O.dtls_encrypt(t12, b"x" * 50, 23, ctr(1, 1), 16384)
    a, recs, res, disp, cres, offs = tab.decrypt([(0, {"in_epoch": 1}, [w])])
    assert int(cres[0]["status"]) == M.ERR_SSL_BAD_INPUT_DATA and int(cres[0]["nrec"]) == 0
    [(r, out, _, _)] = tab.encrypt([(0, b"y" * 40, ctr(1, 0), 0, 23)])
    assert int(r["status"]) == M.ERR_SSL_BAD_INPUT_DATA and int(r["nrec"]) == 0
    tab.close()


def test_send_counter_wrap():
    tab = Table([(M.CIPHER_AES_256_GCM, prng_bytes(9, 32), prng_bytes(10, 16), b"")])
    c8 = ctr(4, (1 << 48) - 2)
    [(r, out, _, _)] = tab.encrypt([(0, prng_bytes(12, 3000), c8, 1000, 23)])
    st, want, nrec, c2 = O.dtls_encrypt(tab.ot[0], prng_bytes(12, 3000), 23, c8, 1000)
    assert st == M.ERR_SSL_COUNTER_WRAPPING and nrec == 2 and c2 == ctr(4, 0)
    assert (int(r["status"]), int(r["nrec"]), bytes(r["out_ctr"])) == (st, nrec, c2)
    assert out == want
    # the third record would reuse sequence number (4, 0) -- a reused nonce:
    # it is never sealed, and its bytes of the output stay zero (ssl_msg.c:2741-2756)
    region = tab.last_regions[0]
    assert len(region) > len(out) and region[len(out):] == bytes(len(region) - len(out))
    tab.close()
