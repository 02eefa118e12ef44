"""Helpers that lay out record batches in a device arena, run them through
libtlsrec (GPU) and through the oracle (CPU), and compare.  Test-side only."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

import mbedtls_amd as M
import oracle as O
from tests.prng import prng_bytes

CIPHERS = {"AES-128-GCM": M.CIPHER_AES_128_GCM, "AES-256-GCM": M.CIPHER_AES_256_GCM,
           "CHACHA20-POLY1305": M.CIPHER_CHACHA20_POLY1305, "AES-192-GCM": M.CIPHER_AES_192_GCM,
           "AES-128-CCM": M.CIPHER_AES_128_CCM, "AES-192-CCM": M.CIPHER_AES_192_CCM,
           "AES-256-CCM": M.CIPHER_AES_256_CCM, "AES-128-CCM-8": M.CIPHER_AES_128_CCM_8,
           "AES-192-CCM-8": M.CIPHER_AES_192_CCM_8, "AES-256-CCM-8": M.CIPHER_AES_256_CCM_8,
           "ARIA-128-GCM": M.CIPHER_ARIA_128_GCM, "ARIA-192-GCM": M.CIPHER_ARIA_192_GCM,
           "ARIA-256-GCM": M.CIPHER_ARIA_256_GCM, "ARIA-128-CCM": M.CIPHER_ARIA_128_CCM,
           "ARIA-192-CCM": M.CIPHER_ARIA_192_CCM, "ARIA-256-CCM": M.CIPHER_ARIA_256_CCM,
           "CAMELLIA-128-GCM": M.CIPHER_CAMELLIA_128_GCM, "CAMELLIA-192-GCM": M.CIPHER_CAMELLIA_192_GCM,
           "CAMELLIA-256-GCM": M.CIPHER_CAMELLIA_256_GCM, "CAMELLIA-128-CCM": M.CIPHER_CAMELLIA_128_CCM,
           "CAMELLIA-192-CCM": M.CIPHER_CAMELLIA_192_CCM, "CAMELLIA-256-CCM": M.CIPHER_CAMELLIA_256_CCM}
VERSIONS = {"TLS1.2": M.VERSION_TLS1_2, "TLS1.3": M.VERSION_TLS1_3}


def keylen(cipher):
    return M.KEYLEN[cipher]


def explicit(cipher, ver):
    return ver == M.VERSION_TLS1_2 and cipher != M.CIPHER_CHACHA20_POLY1305


@dataclass
class Rec:
    slot: int
    buf: bytearray          # the whole record buffer (rec->buf .. rec->buf + buf_len)
    data_offset: int
    data_len: int
    ctr: bytes
    type: int
    ver: bytes = b"\x03\x03"
    cid: bytes = b""        # decrypt: the record's DTLS connection ID


class Batch:
    def __init__(self, slots, recs, align=16, cids=None):
        """slots: list of (cipher, version, key, iv, granularity); cids: optional
        {slot: connection ID} (the slot's out_cid / in_cid)"""
        self.slots = slots
        self.recs = recs
        self.cids = cids or {}
        offs, pos = [], 0
        for r in recs:
            offs.append(pos)
            # the record's CID bytes (decrypt) sit after its buffer
            pos += (len(r.buf) + len(r.cid) + align - 1) // align * align + align
        self.offs = offs
        self.arena = np.zeros(max(pos, 16), dtype=np.uint8)
        for r, o in zip(recs, offs):
            self.arena[o:o + len(r.buf)] = np.frombuffer(bytes(r.buf), dtype=np.uint8)
            if r.cid:
                self.arena[o + len(r.buf):o + len(r.buf) + len(r.cid)] = np.frombuffer(r.cid, dtype=np.uint8)
        d = M.records(len(recs))
        for i, (r, o) in enumerate(zip(recs, offs)):
            d[i]["buf_off"] = o
            d[i]["buf_len"] = len(r.buf)
            d[i]["data_offset"] = r.data_offset
            d[i]["data_len"] = r.data_len
            d[i]["slot"] = r.slot
            d[i]["ctr"] = np.frombuffer(r.ctr, dtype=np.uint8)
            d[i]["type"] = r.type
            d[i]["ver"] = np.frombuffer(r.ver, dtype=np.uint8)
            d[i]["cid_len"] = len(r.cid)
            d[i]["cid_off"] = len(r.buf)
        self.desc = d

    def key_materials(self):
        km = np.concatenate([M.key_material(c, v, k, iv, g) for (c, v, k, iv, g) in self.slots])
        return km

    def run_gpu(self, decrypt: bool, lanes=0, inplace=True, kt=None, mean_bytes=0, stream=None):
        """kt: an already loaded key table (e.g. filled by keytab_derive);
        mean_bytes: the record-size hint of tlsrec_batch_*_sized; stream: a
        HIP stream handle other than torch's (e.g. 2 = hipStreamPerThread)."""
        import torch
        dev = torch.device("cuda")
        own = kt is None
        if own:
            kt = M.KeyTable(max(1, len(self.slots)))
            kt.load(self.key_materials())
            for slot, cid in self.cids.items():
                kt.set_cid(slot, cid)
        arena = torch.from_numpy(self.arena.copy()).to(dev)
        out = arena if inplace else torch.zeros_like(arena)
        recs = torch.from_numpy(self.desc.view(np.uint8).copy()).to(dev)
        res = torch.zeros(len(self.recs) * 16, dtype=torch.uint8, device=dev)
        fn = M.batch_decrypt if decrypt else M.batch_encrypt
        if stream is not None:
            torch.cuda.synchronize()      # torch's fills above ran on its own stream
        fn(kt, recs, res, len(self.recs), arena, out, lanes=lanes, mean_bytes=mean_bytes, stream=stream)
        torch.cuda.synchronize()
        out_np = out.cpu().numpy()
        res_np = res.cpu().numpy().view(M.BATCH_RES)
        if own:
            kt.close()
        return out_np, res_np

    def run_oracle(self, decrypt: bool):
        outs, stats = [], []
        ts = {}
        for r in self.recs:
            c, v, k, iv, g = self.slots[r.slot]
            if r.slot not in ts:
                ts[r.slot] = O.Transform(v, c, k, k, iv, iv, granularity=g or 16)
                if r.slot in self.cids:
                    ts[r.slot].set_cid(self.cids[r.slot], self.cids[r.slot])
            t = ts[r.slot]
            rec = O.Record(ctr=r.ctr, type=r.type, ver=r.ver, buf=bytearray(r.buf),
                           data_offset=r.data_offset, data_len=r.data_len, cid=r.cid if decrypt else b"")
            st = t.decrypt_buf(rec) if decrypt else t.encrypt_buf(rec)
            outs.append(rec)
            stats.append(st)
        return outs, stats

    def compare(self, decrypt: bool, gpu_out, gpu_res, inplace=True):
        """Return list of mismatch descriptions (empty = bit-exact)."""
        o_recs, o_stats = self.run_oracle(decrypt)
        bad = []
        for i, (r, orec, ost) in enumerate(zip(self.recs, o_recs, o_stats)):
            g = gpu_res[i]
            fields = (int(g["status"]), int(g["data_offset"]), int(g["data_len"]), int(g["type"]),
                      int(g["cid_len"]) if not decrypt else 0)
            want = (ost, orec.data_offset, orec.data_len, orec.type, len(orec.cid) if not decrypt else 0)
            if fields != want:
                bad.append(f"rec {i}: fields {fields} != oracle {want}")
                continue
            o = self.offs[i]
            gbuf = bytes(gpu_out[o:o + len(r.buf)])
            if inplace:
                if gbuf != bytes(orec.buf):
                    diff = next(j for j in range(len(gbuf)) if gbuf[j] != orec.buf[j])
                    bad.append(f"rec {i}: buffer differs from byte {diff} (len {len(gbuf)})")
            elif ost == 0:
                lo, hi = orec.data_offset, orec.data_offset + orec.data_len
                if gbuf[lo:hi] != bytes(orec.buf[lo:hi]):
                    bad.append(f"rec {i}: output region differs")
        return bad


def random_slots(rng_seed, ciphers, versions, count):
    slots = []
    for i in range(count):
        c = ciphers[i % len(ciphers)]
        v = versions[(i // len(ciphers)) % len(versions)]
        b = prng_bytes(rng_seed * 1000 + i, 48)
        slots.append((c, v, b[:keylen(c)], b[32:48], 0))
    return slots


def plaintext_records(slots, lengths, seed, head=8, tail=40):
    recs = []
    for i, L in enumerate(lengths):
        s = i % len(slots)
        payload = prng_bytes(seed + i, L)
        buf = bytearray(head + L + tail)
        buf[head:head + L] = payload
        ctr = int(prng_bytes(seed ^ (i + 77), 8).hex(), 16).to_bytes(8, "big")
        recs.append(Rec(slot=s, buf=buf, data_offset=head, data_len=L, ctr=ctr,
                        type=23 if i % 5 else 22))
    return recs


def sealed_records(slots, lengths, seed, head=8, tail=40):
    """Records encrypted by the oracle, ready for a decrypt batch."""
    pre = plaintext_records(slots, lengths, seed, head, tail)
    b = Batch(slots, pre)
    outs, stats = b.run_oracle(False)
    recs = []
    for r, o, st in zip(pre, outs, stats):
        assert st == 0
        recs.append(Rec(slot=r.slot, buf=bytearray(o.buf), data_offset=o.data_offset,
                        data_len=o.data_len, ctr=r.ctr, type=o.type, ver=r.ver))
    return recs, pre


def gcm_sealed_records(slots, lengths, seed, head=8, tail=40):
    """GCM records sealed with the oracle's raw AEAD (no OUT_CONTENT_LEN cap,
    unlike the record-layer encrypt), framed as ssl_msg.c frames them:
    TLS 1.2 explicit nonce = ctr, AAD = ctr|type|ver|len16(plaintext);
    TLS 1.3 nonce = iv ^ (0^4|ctr), AAD = 23|ver|len16(ct+tag), inner type byte.
    Used for records the encrypt side may not produce (counters past 2^16)."""
    recs = []
    for i, L in enumerate(lengths):
        s = i % len(slots)
        c, v, k, iv, _ = slots[s]
        payload = prng_bytes(seed + i, L)
        ctr = int(prng_bytes(seed ^ (i + 77), 8).hex(), 16).to_bytes(8, "big")
        rtype = 23 if i % 5 else 22
        if v == M.VERSION_TLS1_3:
            inner = payload + bytes([rtype])
            nonce = bytes(a ^ b for a, b in zip(iv[:12], bytes(4) + ctr))
            aad = bytes([23]) + b"\x03\x03" + ((len(inner) + 16) & 0xffff).to_bytes(2, "big")
            ct, tag = O.gcm_encrypt(k, nonce, aad, inner)
            body = ct + tag
            wire_type = 23
        else:
            nonce = iv[:4] + ctr
            aad = ctr + bytes([rtype]) + b"\x03\x03" + (L & 0xffff).to_bytes(2, "big")
            ct, tag = O.gcm_encrypt(k, nonce, aad, payload)
            body = ctr + ct + tag
            wire_type = rtype
        buf = bytearray(head + len(body) + tail)
        buf[head:head + len(body)] = body
        recs.append(Rec(slot=s, buf=buf, data_offset=head, data_len=len(body), ctr=ctr, type=wire_type))
    return recs
