"""GPU parity of the TLS stream record layer (stream.hip through the C ABI)
against the oracle's restatement of the ssl_get_next_record /
mbedtls_ssl_write_record loops: byte-exact record streams, per-connection
status / consumed / sequence numbers, and every stop condition."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import mbedtls_amd as M  # noqa: E402
from mbedtls_amd import stream as S  # noqa: E402
import oracle as O  # noqa: E402
from tests import batchlib as B  # noqa: E402
from tests.prng import prng_bytes  # noqa: E402

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
X = bytes.fromhex
OC = {c: c for c in M.KEYLEN}      # the oracle uses the same cipher ids as include/tlsrec.h
assert O.AES_256_CCM_8 == M.CIPHER_AES_256_CCM_8 and O.CHACHA20_POLY1305 == M.CIPHER_CHACHA20_POLY1305


def _al(x, a=128):
    return (x + a - 1) // a * a


class Conns:
    """slots: list of (cipher, version, key, iv, granularity); one key table."""

    def __init__(self, slots):
        self.slots = slots
        self.kt = M.KeyTable(len(slots))
        self.kt.load(np.concatenate([M.key_material(c, v, k, iv, g) for c, v, k, iv, g in slots]))
        self.ot = [O.Transform(v, OC[c], k, k, iv, iv, granularity=g or 16) for c, v, k, iv, g in slots]

    def encrypt(self, jobs):
        """jobs: list of (slot, plaintext, out_ctr(int), max_frag, type)"""
        ins, outs, pos_in, pos_out = [], [], 0, 0
        d = np.zeros(len(jobs), dtype=S.STREAM_OUT)
        for i, (slot, pt, ctr, frag, typ) in enumerate(jobs):
            c, v, _, _, g = self.slots[slot]
            size = S.out_size(v, c, g, len(pt), frag)
            d[i]["in_off"], d[i]["in_len"], d[i]["slot"] = pos_in, len(pt), slot
            d[i]["out_off"], d[i]["max_frag"], d[i]["type"] = pos_out, frag, typ
            d[i]["out_ctr"] = np.frombuffer(ctr.to_bytes(8, "big"), dtype=np.uint8)
            ins.append(pos_in)
            outs.append((pos_out, size))
            pos_in += _al(len(pt) + 1)
            pos_out += _al(size + 1)
        ina = np.zeros(max(pos_in, 16), dtype=np.uint8)
        for (slot, pt, *_), o in zip(jobs, ins):
            ina[o:o + len(pt)] = np.frombuffer(pt, dtype=np.uint8)
        dev = torch.device("cuda")
        tin = torch.from_numpy(ina).to(dev)
        tout = torch.zeros(max(pos_out, 16), dtype=torch.uint8, device=dev)
        nmax = sum((len(j[1]) + (j[3] or 16384) - 1) // (j[3] or 16384) for j in jobs) + 1
        recs = torch.zeros(nmax * 40, dtype=torch.uint8, device=dev)
        res = torch.zeros(nmax * 16, dtype=torch.uint8, device=dev)
        sres = torch.zeros(len(jobs) * 32, dtype=torch.uint8, device=dev)
        S.encrypt(self.kt, d, len(jobs), tin, tout, recs, res, nmax, sres)
        torch.cuda.synchronize()
        o = tout.cpu().numpy()
        sr = sres.cpu().numpy().view(S.STREAM_OUT_RES)
        self.last_regions = [o[p:p + size].tobytes() for p, size in outs]   # each job's whole output region
        return [(sr[i], o[p:p + int(sr[i]["out_len"])].tobytes()) for i, (p, _) in enumerate(outs)]

    def decrypt(self, conns):
        """conns: list of (slot, bytes, in_ctr(int), nb_zero)"""
        d = np.zeros(len(conns), dtype=S.STREAM_IN)
        pos, offs = 0, []
        for i, (slot, data, ctr, nbz) in enumerate(conns):
            d[i]["off"], d[i]["len"], d[i]["slot"], d[i]["nb_zero"] = pos, len(data), slot, nbz
            d[i]["in_ctr"] = np.frombuffer(ctr.to_bytes(8, "big"), dtype=np.uint8)
            offs.append(pos)
            pos += _al(len(data) + 1)
        a = np.zeros(max(pos, 16), dtype=np.uint8)
        for (slot, data, *_), o in zip(conns, offs):
            a[o:o + len(data)] = np.frombuffer(data, dtype=np.uint8)
        dev = torch.device("cuda")
        ta = torch.from_numpy(a).to(dev)
        nmax = sum(len(c[1]) // 6 + 1 for c in conns)
        recs = torch.zeros(nmax * 40, dtype=torch.uint8, device=dev)
        res = torch.zeros(nmax * 16, dtype=torch.uint8, device=dev)
        sres = torch.zeros(len(conns) * 32, dtype=torch.uint8, device=dev)
        S.decrypt(self.kt, d, len(conns), ta, recs, res, nmax, sres)
        torch.cuda.synchronize()
        return (ta.cpu().numpy(), recs.cpu().numpy().view(M.BATCH_REC), res.cpu().numpy().view(M.BATCH_RES),
                sres.cpu().numpy().view(S.STREAM_IN_RES), offs)

    def close(self):
        self.kt.close()


@pytest.mark.parametrize("kat", KATS, ids=lambda k: k["name"])
def test_reference_complete_records(kat):
    sk, si, ck, ci = (X(kat[x]) for x in ("server_key", "server_iv", "client_key", "client_iv"))
    wk, wi, rk, ri = (ck, ci, sk, si) if kat["endpoint"] == "client" else (sk, si, ck, ci)
    c = Conns([(M.CIPHER_AES_128_GCM, M.VERSION_TLS1_3, wk, wi, 1), (M.CIPHER_AES_128_GCM, M.VERSION_TLS1_3, rk, ri, 1)])
    ct = X(kat["ciphertext"])
    wire = bytes([23, 3, 3]) + len(ct).to_bytes(2, "big") + ct
    [(r, out)] = c.encrypt([(0, X(kat["plaintext"]), kat["ctr"], 0, 23)])
    assert r["status"] == 0 and r["nrec"] == 1 and out == wire
    # the receiver side of the same connection decrypts with the peer's keys
    c2 = Conns([(M.CIPHER_AES_128_GCM, M.VERSION_TLS1_3, wk, wi, 1)])
    a, recs, res, sres, offs = c2.decrypt([(0, wire, kat["ctr"], 0)])
    assert sres[0]["status"] == 0 and sres[0]["nrec"] == 1 and sres[0]["consumed"] == len(wire)
    o = int(recs[0]["buf_off"]) + int(res[0]["data_offset"])
    assert a[o:o + int(res[0]["data_len"])].tobytes() == X(kat["plaintext"]) and res[0]["type"] == 23
    c.close()
    c2.close()


def _slots(seed):
    return B.random_slots(seed, list(B.CIPHERS.values()), list(B.VERSIONS.values()), 20)


def test_encrypt_then_decrypt_many_connections():
    slots = _slots(41)
    c = Conns(slots)
    rng = np.random.default_rng(7)
    jobs = []
    for i in range(60):
        n = int(rng.choice([0, 1, 15, 300, 16383, 16384, 16385, 40000]))
        frag = int(rng.choice([0, 0, 1000, 4096]))
        jobs.append((i % 20, prng_bytes(1000 + i, n), int(rng.integers(0, 1 << 40)), frag, 23 if i % 7 else 22))
    got = c.encrypt(jobs)
    for (slot, pt, ctr, frag, typ), (r, out) in zip(jobs, got):
        st, want, nrec, ctr2 = O.stream_encrypt(c.ot[slot], pt, typ, ctr.to_bytes(8, "big"), frag or 16384)
        assert (int(r["status"]), int(r["nrec"]), out, bytes(r["out_ctr"])) == (st, nrec, want, ctr2)
    # receive the same streams, some with a partial trailing record
    conns = []
    for i, ((slot, pt, ctr, frag, typ), (r, out)) in enumerate(zip(jobs, got)):
        extra = out[:7] if (i % 3 == 0 and len(out) > 7) else b""
        conns.append((slot, out + extra, ctr, i % 2))
    a, recs, res, sres, offs = c.decrypt(conns)
    for i, (slot, data, ctr, nbz) in enumerate(conns):
        want, wrecs, wbuf = O.stream_decrypt(c.ot[slot], data, ctr.to_bytes(8, "big"), nbz)
        g = sres[i]
        assert (int(g["status"]), int(g["nrec"]), int(g["consumed"]), bytes(g["in_ctr"]), int(g["nb_zero"])) == \
            (want["status"], want["nrec"], want["consumed"], want["in_ctr"], want["nb_zero"]), i
        f = int(g["first"])
        for k, (off, doff, dlen, typ) in enumerate(wrecs):
            rr = res[f + k]
            assert (int(rr["data_offset"]), int(rr["data_len"]), int(rr["type"])) == (doff, dlen, typ)
            assert int(recs[f + k]["buf_off"]) == offs[i] + off
            s0 = offs[i] + off + doff
            assert a[s0:s0 + dlen].tobytes() == wbuf[off + doff:off + doff + dlen]
    c.close()


FRAMINGS = [("1", "1", "1", "16"), ("1", "1", "0", "16"), ("1", "1", "0", "8"), ("1", "1", "0", "4"),
            ("0", "0", "0", "16")]
FRAMING_IDS = ["one-pass", "groupwalk-16", "groupwalk-8", "groupwalk-4", "r05-framing"]


def _framing(monkeypatch, fr):
    gw, grouped, fused, rg = fr
    monkeypatch.setenv("TLSREC_RX_GROUPWALK", gw)       # the r06 lane-group walks or the r05 one-lane walks,
    monkeypatch.setenv("TLSREC_GROUPED", grouped)       # with and without the bucket pass,
    monkeypatch.setenv("TLSREC_RX_FUSED_STREAM", fused) # count / scan / emit as one pass (look-back) or three kernels,
    monkeypatch.setenv("TLSREC_RX_RG", rg)              # 16, 8 or 4 lanes per connection in the walk


@pytest.mark.parametrize("fr", FRAMINGS, ids=FRAMING_IDS)
def test_irregular_record_lengths_match_oracle(fr, monkeypatch):
    """Streams whose records change length mid-stream (runs of one length,
    single odd records, CCS records between, 1..40 records, a trailing
    partial record or a bad header after a run): the lane-group walk (a
    run of equal lengths checked 16 headers at a time)
    must frame exactly what the serial walk does -- records, sequence
    numbers, stop status and position -- under every framing path (1 200
    connections: 75 tiles of the one-pass kernel's look-back)."""
    _framing(monkeypatch, fr)
    slots = _slots(53)
    c = Conns(slots)
    rng = np.random.default_rng(29)
    conns = []
    for i in range(1200):
        slot = i % 20
        t = c.ot[slot]
        ctr0 = int(rng.integers(0, 1 << 40))
        ctr, data = ctr0, b""
        for seg in range(int(rng.integers(1, 6))):
            if t.tls_version == O.TLS1_3 and rng.random() < 0.2:
                data += bytes([20, 3, 3, 0, 1, 1])                       # CCS: passes, no counter step
            frag = int(rng.choice([1, 16, 100, 1400, 4096]))
            n = int(rng.integers(1, 18)) * frag - int(rng.integers(0, frag))
            st, w, nrec, c2 = O.stream_encrypt(t, prng_bytes(7000 + 10 * i + seg, max(n, 1)), 23,
                                               ctr.to_bytes(8, "big"), frag)
            assert st == 0
            data += w
            ctr = int.from_bytes(c2, "big")
        tail = int(rng.integers(0, 4))
        if tail == 1:
            data += data[:3]                                             # partial header
        elif tail == 2:
            data += bytes([23, 3, 3, 0, 40]) + bytes(10)                 # partial record
        elif tail == 3:
            data += bytes([25, 3, 3, 0, 40]) + bytes(45)                 # bad type
        conns.append((slot, data, ctr0, 0))
    a, recs, res, sres, offs = c.decrypt(conns)
    for i, (slot, data, ctr, nbz) in enumerate(conns):
        want, wrecs, wbuf = O.stream_decrypt(c.ot[slot], data, ctr.to_bytes(8, "big"), nbz)
        g = sres[i]
        assert (int(g["status"]), int(g["nrec"]), int(g["consumed"]), bytes(g["in_ctr"]), int(g["nb_zero"])) == \
            (want["status"], want["nrec"], want["consumed"], want["in_ctr"], want["nb_zero"]), (i, want)
        f = int(g["first"])
        for k, (off, doff, dlen, typ) in enumerate(wrecs):
            rr = res[f + k]
            assert (int(rr["data_offset"]), int(rr["data_len"]), int(rr["type"])) == (doff, dlen, typ), (i, k)
            assert int(recs[f + k]["buf_off"]) == offs[i] + off
            s0 = offs[i] + off + doff
            assert a[s0:s0 + dlen].tobytes() == wbuf[off + doff:off + doff + dlen], (i, k)
    c.close()


def _empty_record(t, ctr):
    buf = bytearray(64)
    head = 8 if (t.tls_version == O.TLS1_2 and t.cipher != O.CHACHA20_POLY1305) else 0
    rec = O.Record(ctr=ctr.to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=buf, data_offset=head, data_len=0)
    assert t.encrypt_buf(rec) == 0 and rec.data_offset == 0
    return bytes([23, 3, 3]) + rec.data_len.to_bytes(2, "big") + rec.data()


def _typed_record(t, ctr, typ):
    """a record whose (TLS 1.3: inner) content type is `typ`; after
    decryption ssl_prepare_record_content re-checks it (ssl_msg.c:3914-3917)"""
    buf = bytearray(128)
    head = 8 if (t.tls_version == O.TLS1_2 and t.cipher != O.CHACHA20_POLY1305) else 0
    buf[head:head + 5] = b"hello"
    rec = O.Record(ctr=ctr.to_bytes(8, "big"), type=typ, ver=b"\x03\x03", buf=buf, data_offset=head, data_len=5)
    assert t.encrypt_buf(rec) == 0 and rec.data_offset == 0
    return bytes([rec.type, 3, 3]) + rec.data_len.to_bytes(2, "big") + rec.data()


def test_stop_conditions_match_oracle():
    slots = [(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, prng_bytes(1, 32), prng_bytes(2, 12), 0),
             (M.CIPHER_AES_128_GCM, M.VERSION_TLS1_2, prng_bytes(3, 16), prng_bytes(4, 12), 0),
             (M.CIPHER_CHACHA20_POLY1305, M.VERSION_TLS1_3, prng_bytes(5, 32), prng_bytes(6, 12), 0)]
    c = Conns(slots)
    conns = []
    for slot in range(3):
        t = c.ot[slot]
        _, w, n, _ = O.stream_encrypt(t, prng_bytes(10 + slot, 300), 23, bytes(8), 100)
        one = len(w) // 3
        conns += [(slot, w[:one] + bytes([24]) + w[one + 1:], 0, 0),                       # type
                  (slot, w[:one] + w[one:one + 1] + b"\x03\x05" + w[one + 3:], 0, 0),     # version
                  (slot, w[:one] + w[one:one + 3] + b"\x00\x00" + w[one + 5:], 0, 0),     # zero length
                  (slot, w[:one] + w[one:one + 3] + b"\x40\x21" + w[one + 5:], 0, 0),     # too long
                  (slot, w[:one + 20] + bytes([w[one + 20] ^ 0x80]) + w[one + 21:], 0, 0),  # MAC
                  (slot, w[:4], 0, 0), (slot, b"", 0, 0),                                  # incomplete
                  (slot, bytes([20, 3, 3, 0, 1, 1]) + w, 0, 0),                           # CCS first
                  (slot, b"".join(_empty_record(t, k) for k in range(4)), 0, 0),          # 4 empty
                  (slot, b"".join(_empty_record(t, k) for k in range(2)), 0, 2),          # nb_zero carried
                  (slot, _empty_record(t, (1 << 64) - 1), (1 << 64) - 1, 0),              # ctr wrap
                  (slot, _typed_record(t, 0, 24) + w, 0, 0)]                              # inner type 24
    a, recs, res, sres, offs = c.decrypt(conns)
    for i, (slot, data, ctr, nbz) in enumerate(conns):
        want, wrecs, _ = O.stream_decrypt(c.ot[slot], data, ctr.to_bytes(8, "big"), nbz)
        g = sres[i]
        assert (int(g["status"]), int(g["nrec"]), int(g["consumed"]), bytes(g["in_ctr"]), int(g["nb_zero"])) == \
            (want["status"], want["nrec"], want["consumed"], want["in_ctr"], want["nb_zero"]), (i, want)
    c.close()


def test_too_many_records_is_buffer_too_small():
    slots = [(M.CIPHER_AES_128_GCM, M.VERSION_TLS1_3, bytes(16), bytes(12), 0)]
    c = Conns(slots)
    _, w, n, _ = O.stream_encrypt(c.ot[0], bytes(500), 23, bytes(8), 100)
    dev = torch.device("cuda")
    d = np.zeros(1, dtype=S.STREAM_IN)
    d[0]["len"] = len(w)
    ta = torch.from_numpy(np.frombuffer(w, dtype=np.uint8).copy()).to(dev)
    recs = torch.zeros(4 * 40, dtype=torch.uint8, device=dev)
    res = torch.zeros(4 * 16, dtype=torch.uint8, device=dev)
    sres = torch.zeros(32, dtype=torch.uint8, device=dev)
    with pytest.raises(S.StreamError) as e:
        S.decrypt(c.kt, d, 1, ta, recs, res, 4, sres)
    assert e.value.code == M.ERR_SSL_BUFFER_TOO_SMALL
    assert ta.cpu().numpy().tobytes() == w          # nothing decrypted
    c.close()


def test_stream_read_matches_oracle():
    """tlsrec_stream_read (ssl_read_application_data over the accepted
    records) against the oracle: bytes handed out, zeroization in place,
    records consumed and bytes left, for several buffer sizes."""
    slots = _slots(77)
    c = Conns(slots)
    rng = np.random.default_rng(3)
    jobs = []
    for i in range(40):
        n = int(rng.choice([1, 300, 5000, 16384, 30000]))
        jobs.append((i % 20, prng_bytes(3000 + i, n), int(rng.integers(0, 1 << 30)), int(rng.choice([0, 1000])),
                     23 if i % 4 else 22))
    got = c.encrypt(jobs)
    conns = [(slot, out, ctr, 0) for (slot, _, ctr, _, _), (_, out) in zip(jobs, got)]
    a, recs, res, sres, offs = c.decrypt(conns)
    dev = torch.device("cuda")
    for cap_kind in (0, 1, 2):
        caps = [[0, 17, 1000][cap_kind] if k % 3 else len(j[1]) + 5 for k, j in enumerate(jobs)]
        req = np.zeros(len(jobs), dtype=S.STREAM_READ_REQ)
        pos, outs = 0, []
        for k, cap in enumerate(caps):
            req[k] = (pos, cap, 0)
            outs.append(pos)
            pos += (cap + 127) // 128 * 128 + 128
        ta = torch.from_numpy(a.copy()).to(dev)
        tout = torch.zeros(max(pos, 16), dtype=torch.uint8, device=dev)
        rres = torch.zeros(len(jobs) * 16, dtype=torch.uint8, device=dev)
        S.read(torch.from_numpy(sres.view(np.uint8).copy()).to(dev), len(jobs),
               torch.from_numpy(recs.view(np.uint8).copy()).to(dev), torch.from_numpy(res.view(np.uint8).copy()).to(dev),
               ta, req, tout, rres)
        torch.cuda.synchronize()
        a2, o2 = ta.cpu().numpy(), tout.cpu().numpy()
        rr = rres.cpu().numpy().view(S.STREAM_READ_RES)
        for k, (slot, data, ctr, nbz) in enumerate(conns):
            g = sres[k]
            f, nrec = int(g["first"]), int(g["nrec"])
            wrecs = [(int(recs[f + j]["buf_off"]) - offs[k], int(res[f + j]["data_offset"]),
                      int(res[f + j]["data_len"]), int(res[f + j]["type"])) for j in range(nrec)]
            region = a[offs[k]:offs[k] + len(data)].tobytes()
            out, full, left, after = O.stream_read(region, wrecs, caps[k])
            assert (int(rr["copied"][k]), int(rr["records"][k]), int(rr["left"][k])) == (len(out), full, left), k
            assert o2[outs[k]:outs[k] + len(out)].tobytes() == out
            assert a2[offs[k]:offs[k] + len(data)].tobytes() == after
    c.close()


@pytest.mark.parametrize("cipher", [M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM])
def test_many_keys_small_records_wave_passes(cipher):
    """640 connections x 16 records of 1 400 B: under 64 KiB of records per
    key, so the stream layer's record-size hint sends the GCM kernels into
    wave passes at 16 lanes (engine.hip `light`); every record stream and
    plaintext checked against the oracle."""
    kl = M.KEYLEN[cipher]
    slots = [(cipher, M.VERSION_TLS1_3, prng_bytes(9000 + i, kl), prng_bytes(19000 + i, 12), 0) for i in range(640)]
    c = Conns(slots)
    jobs = [(i, prng_bytes(29000 + i, 16 * 1400), i * 7919, 1400, 23) for i in range(640)]
    got = c.encrypt(jobs)
    for (slot, pt, ctr, frag, typ), (r, out) in zip(jobs, got):
        st, want, nrec, ctr2 = O.stream_encrypt(c.ot[slot], pt, typ, ctr.to_bytes(8, "big"), frag)
        assert (int(r["status"]), int(r["nrec"]), out, bytes(r["out_ctr"])) == (st, nrec, want, ctr2), slot
    conns = [(slot, out, ctr, 0) for (slot, _, ctr, _, _), (_, out) in zip(jobs, got)]
    a, recs, res, sres, offs = c.decrypt(conns)
    for i, (slot, data, ctr, nbz) in enumerate(conns):
        g = sres[i]
        assert (int(g["status"]), int(g["nrec"])) == (0, 16), i
        f = int(g["first"])
        pt = jobs[i][1]
        for k in range(16):
            o = int(recs[f + k]["buf_off"]) + int(res[f + k]["data_offset"])
            assert int(res[f + k]["data_len"]) == 1400
            assert a[o:o + 1400].tobytes() == pt[1400 * k:1400 * (k + 1)], (i, k)
    c.close()


def test_send_copy_path_matches_oracle(monkeypatch):
    """TLSREC_STREAM_SRC=0: the send path copies the application data into
    the record arena and encrypts there (the r04 path, still taken by CID
    and ARIA / Camellia tables) instead of reading it in place; the same
    streams as the default path, checked against the oracle."""
    monkeypatch.setenv("TLSREC_STREAM_SRC", "0")
    slots = _slots(43)
    c = Conns(slots)
    rng = np.random.default_rng(11)
    jobs = []
    for i in range(40):
        n = int(rng.choice([0, 1, 15, 1400, 16383, 16385, 40000]))
        frag = int(rng.choice([0, 1000, 4096]))
        jobs.append((i % 20, prng_bytes(3000 + i, n), int(rng.integers(0, 1 << 40)), frag, 23))
    got = c.encrypt(jobs)
    for (slot, pt, ctr, frag, typ), (r, out) in zip(jobs, got):
        st, want, nrec, ctr2 = O.stream_encrypt(c.ot[slot], pt, typ, ctr.to_bytes(8, "big"), frag or 16384)
        assert (int(r["status"]), int(r["nrec"]), out, bytes(r["out_ctr"])) == (st, nrec, want, ctr2)
    c.close()


def test_send_counter_wrap_encrypts_nothing_past_the_wrap():
    """out_ctr = 2^64 - 2, three records: the reference writes the records with
    sequence numbers 2^64-2 and 2^64-1, then stops with COUNTER_WRAPPING
    (ssl_msg.c:2749-2756) -- nothing is ever encrypted under sequence 0 again
    (a reused nonce).  The third record's bytes of the output stream stay zero."""
    slots = [(M.CIPHER_AES_256_GCM, M.VERSION_TLS1_3, prng_bytes(21, 32), prng_bytes(22, 12), 0),
             (M.CIPHER_CHACHA20_POLY1305, M.VERSION_TLS1_2, prng_bytes(23, 32), prng_bytes(24, 12), 0)]
    c = Conns(slots)
    start = (1 << 64) - 2
    pt = prng_bytes(25, 3000)
    got = c.encrypt([(0, pt, start, 1000, 23), (1, pt, start, 1000, 23)])
    for slot, (r, out) in enumerate(got):
        st, want, nrec, c2 = O.stream_encrypt(c.ot[slot], pt, 23, start.to_bytes(8, "big"), 1000)
        assert st == M.ERR_SSL_COUNTER_WRAPPING and nrec == 2 and c2 == bytes(8)
        assert (int(r["status"]), int(r["nrec"]), bytes(r["out_ctr"])) == (st, nrec, c2)
        assert out == want
        region = c.last_regions[slot]
        assert region[len(out):] == bytes(len(region) - len(out)), "bytes written past the wrap"
    c.close()
