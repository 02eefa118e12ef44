"""ctypes wrapper around oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of Mbed TLS 4.1.0's AEAD record path (see oracle.h for
the reference file:line map and README.md for how it is pinned).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / the timed CPU baseline -- the product
package ``mbedtls_amd`` never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

ERR_BAD_INPUT_DATA = -135
ERR_BUFFER_TOO_SMALL = -138
ERR_INVALID_MAC = -0x7180
ERR_INVALID_RECORD = -0x7200
ERR_INTERNAL_ERROR = -0x6C00

TLS1_2 = 0x0303
TLS1_3 = 0x0304
AES_128_GCM = 1
AES_256_GCM = 2
CHACHA20_POLY1305 = 3
AES_192_GCM = 4
AES_128_CCM, AES_192_CCM, AES_256_CCM = 5, 6, 7
AES_128_CCM_8, AES_192_CCM_8, AES_256_CCM_8 = 8, 9, 10
ARIA_128_GCM, ARIA_192_GCM, ARIA_256_GCM = 11, 12, 13
ARIA_128_CCM, ARIA_192_CCM, ARIA_256_CCM = 14, 15, 16
CAMELLIA_128_GCM, CAMELLIA_192_GCM, CAMELLIA_256_GCM = 17, 18, 19
CAMELLIA_128_CCM, CAMELLIA_192_CCM, CAMELLIA_256_CCM = 20, 21, 22
KEYLEN = {AES_128_GCM: 16, AES_256_GCM: 32, CHACHA20_POLY1305: 32, AES_192_GCM: 24, AES_128_CCM: 16,
          AES_192_CCM: 24, AES_256_CCM: 32, AES_128_CCM_8: 16, AES_192_CCM_8: 24, AES_256_CCM_8: 32,
          ARIA_128_GCM: 16, ARIA_192_GCM: 24, ARIA_256_GCM: 32,
          ARIA_128_CCM: 16, ARIA_192_CCM: 24, ARIA_256_CCM: 32,
          CAMELLIA_128_GCM: 16, CAMELLIA_192_GCM: 24, CAMELLIA_256_GCM: 32,
          CAMELLIA_128_CCM: 16, CAMELLIA_192_CCM: 24, CAMELLIA_256_CCM: 32}
TAGLEN = {c: (8 if AES_128_CCM_8 <= c <= AES_256_CCM_8 else 16) for c in KEYLEN}

_lib = None


def build() -> str:
    """Compile the restatement with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c_u8p = ctypes.c_char_p
        L.orc_aes_setkey_enc.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint]
        L.orc_aes_encrypt_block.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_void_p]
        L.orc_gcm_setkey.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_uint]
        L.orc_gcm_encrypt.argtypes = [ctypes.c_void_p, c_u8p, c_u8p, ctypes.c_size_t,
                                      c_u8p, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t]
        L.orc_gcm_decrypt.argtypes = [ctypes.c_void_p, c_u8p, c_u8p, ctypes.c_size_t,
                                      c_u8p, ctypes.c_size_t, ctypes.c_void_p,
                                      c_u8p, ctypes.c_size_t]
        L.orc_ghash.argtypes = [ctypes.c_void_p, c_u8p, ctypes.c_size_t, c_u8p,
                                ctypes.c_size_t, ctypes.c_void_p]
        L.orc_gf128_mul.argtypes = [c_u8p, c_u8p, ctypes.c_void_p]
        L.orc_chacha20_block.argtypes = [c_u8p, ctypes.c_uint32, c_u8p, ctypes.c_void_p]
        L.orc_poly1305.argtypes = [c_u8p, c_u8p, ctypes.c_size_t, ctypes.c_void_p]
        L.orc_chachapoly_encrypt.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_size_t, c_u8p,
                                             ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_chachapoly_decrypt.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_size_t, c_u8p,
                                             ctypes.c_size_t, ctypes.c_void_p, c_u8p]
        L.orc_transform_setup.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          c_u8p, c_u8p, c_u8p, c_u8p, ctypes.c_size_t]
        L.orc_encrypt_buf.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_decrypt_buf.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.orc_bench_records.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        L.orc_bench_records.restype = ctypes.c_double
        L.orc_bench_records_multi.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                              ctypes.c_void_p]
        L.orc_bench_records_multi.restype = ctypes.c_double
        L.orc_bench_stream_rows.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.orc_bench_stream_rows.restype = ctypes.c_double
        L.orc_bench_keysched.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_bench_keysched.restype = ctypes.c_double
        _lib = L
    return _lib


# struct sizes: generous opaque buffers (orc_gcm_ctx ~ 520 B, orc_transform ~ 1.2 KiB)
_GCM_CTX = 1024
_TRANSFORM = 4096


def _buf(n):
    return ctypes.create_string_buffer(n)


def aria_encrypt_block(key: bytes, block: bytes) -> bytes:
    """ARIA (RFC 5794), oracle/aria.c."""
    f = lib().orc_aria_setkey_enc
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint]
    ctx = _buf(1024)
    assert f(ctx, key, len(key) * 8) == 0
    out = _buf(16)
    g = lib().orc_aria_encrypt_block
    g.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    g(ctx, block, out)
    return out.raw


def camellia_encrypt_block(key: bytes, block: bytes) -> bytes:
    """Camellia (RFC 3713), oracle/camellia.c."""
    f = lib().orc_camellia_setkey_enc
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint]
    ctx = _buf(1024)
    assert f(ctx, key, len(key) * 8) == 0
    out = _buf(16)
    g = lib().orc_camellia_encrypt_block
    g.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    g(ctx, block, out)
    return out.raw


def aria_gcm_encrypt(key: bytes, iv: bytes, aad: bytes, pt: bytes, bc: int = 1):
    """GCM over ARIA (bc 1) or Camellia (bc 2)."""
    f = lib().orc_gcm_setkey_ex
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint, ctypes.c_int]
    ctx = _buf(_GCM_CTX)
    assert f(ctx, key, len(key) * 8, bc) == 0
    out, tag = _buf(max(1, len(pt))), _buf(16)
    lib().orc_gcm_encrypt(ctx, iv, aad, len(aad), pt, len(pt), out, tag, 16)
    return out.raw[:len(pt)], tag.raw


def aes_encrypt_block(key: bytes, block: bytes) -> bytes:
    ctx = _buf(1024)
    assert lib().orc_aes_setkey_enc(ctx, key, len(key) * 8) == 0
    out = _buf(16)
    lib().orc_aes_encrypt_block(ctx, block, out)
    return out.raw


def gcm_encrypt(key: bytes, iv: bytes, aad: bytes, pt: bytes, tag_len: int = 16):
    ctx = _buf(_GCM_CTX)
    assert lib().orc_gcm_setkey(ctx, key, len(key) * 8) == 0
    out = _buf(max(1, len(pt)))
    tag = _buf(16)
    lib().orc_gcm_encrypt(ctx, iv, aad, len(aad), pt, len(pt), out, tag, tag_len)
    return out.raw[:len(pt)], tag.raw[:tag_len]


def gcm_decrypt(key: bytes, iv: bytes, aad: bytes, ct: bytes, tag: bytes):
    ctx = _buf(_GCM_CTX)
    assert lib().orc_gcm_setkey(ctx, key, len(key) * 8) == 0
    out = _buf(max(1, len(ct)))
    r = lib().orc_gcm_decrypt(ctx, iv, aad, len(aad), ct, len(ct), out, tag, len(tag))
    return r, out.raw[:len(ct)]


def ghash(key: bytes, aad: bytes, ct: bytes) -> bytes:
    ctx = _buf(_GCM_CTX)
    assert lib().orc_gcm_setkey(ctx, key, len(key) * 8) == 0
    out = _buf(16)
    lib().orc_ghash(ctx, aad, len(aad), ct, len(ct), out)
    return out.raw


def gf128_mul(x: bytes, y: bytes) -> bytes:
    out = _buf(16)
    lib().orc_gf128_mul(x, y, out)
    return out.raw


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    out = _buf(64)
    lib().orc_chacha20_block(key, counter, nonce, out)
    return out.raw


def poly1305(key: bytes, msg: bytes) -> bytes:
    out = _buf(16)
    lib().orc_poly1305(key, msg, len(msg), out)
    return out.raw


def ccm_encrypt(key: bytes, nonce: bytes, aad: bytes, pt: bytes, tag_len: int = 16):
    ctx = _buf(_GCM_CTX)
    assert lib().orc_aes_setkey_enc(ctx, key, len(key) * 8) == 0
    f = lib().orc_ccm_encrypt
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                  ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    out, tag = _buf(max(1, len(pt))), _buf(16)
    f(ctx, nonce, aad, len(aad), pt, len(pt), out, tag, tag_len)
    return out.raw[:len(pt)], tag.raw[:tag_len]


def chachapoly_encrypt(key: bytes, nonce: bytes, aad: bytes, pt: bytes):
    out = _buf(max(1, len(pt)))
    tag = _buf(16)
    lib().orc_chachapoly_encrypt(key, nonce, aad, len(aad), pt, len(pt), out, tag)
    return out.raw[:len(pt)], tag.raw


def chachapoly_decrypt(key: bytes, nonce: bytes, aad: bytes, ct: bytes, tag: bytes):
    out = _buf(max(1, len(ct)))
    r = lib().orc_chachapoly_decrypt(key, nonce, aad, len(aad), ct, len(ct), out, tag)
    return r, out.raw[:len(ct)]


class _CRecord(ctypes.Structure):
    _fields_ = [("ctr", ctypes.c_uint8 * 8), ("type", ctypes.c_uint8),
                ("ver", ctypes.c_uint8 * 2), ("buf", ctypes.c_void_p),
                ("buf_len", ctypes.c_size_t), ("data_offset", ctypes.c_size_t),
                ("data_len", ctypes.c_size_t), ("cid_len", ctypes.c_uint8),
                ("cid", ctypes.c_uint8 * 32)]


@dataclass
class Record:
    """Python mirror of mbedtls_record (library/ssl_misc.h:1163-1188)."""
    ctr: bytes
    type: int
    ver: bytes
    buf: bytearray
    data_offset: int
    data_len: int
    buf_len: int = field(default=-1)
    cid: bytes = b""           # DTLS 1.2 connection ID (rec->cid / cid_len)

    def __post_init__(self):
        if self.buf_len < 0:
            self.buf_len = len(self.buf)

    def data(self) -> bytes:
        return bytes(self.buf[self.data_offset:self.data_offset + self.data_len])


class Transform:
    """Mirror of the AEAD fields of struct mbedtls_ssl_transform with raw keys."""

    def __init__(self, tls_version, cipher, key_enc, key_dec, iv_enc, iv_dec,
                 granularity=16):
        self._mem = _buf(_TRANSFORM)
        pad = lambda b: bytes(b) + bytes(32 - len(b))  # noqa: E731
        r = lib().orc_transform_setup(self._mem, tls_version, cipher, pad(key_enc),
                                      pad(key_dec), pad(iv_enc)[:16], pad(iv_dec)[:16],
                                      granularity)
        if r != 0:
            raise ValueError(f"orc_transform_setup failed: {r}")
        self.tls_version, self.cipher = tls_version, cipher

    def set_cid(self, in_cid: bytes, out_cid: bytes) -> None:
        """DTLS 1.2 connection IDs of the transform (in_cid / out_cid)."""
        f = lib().orc_transform_set_cid
        f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        r = f(self._mem, bytes(in_cid), len(in_cid), bytes(out_cid), len(out_cid))
        if r != 0:
            raise ValueError(f"orc_transform_set_cid failed: {r}")

    def _call(self, fn, rec: Record) -> int:
        c = _CRecord()
        c.ctr[:] = list(rec.ctr)
        c.type = rec.type
        c.ver[:] = list(rec.ver)
        cbuf = (ctypes.c_uint8 * max(1, len(rec.buf))).from_buffer(rec.buf) if len(rec.buf) else None
        c.buf = ctypes.addressof(cbuf) if cbuf is not None else None
        c.buf_len = rec.buf_len
        c.data_offset = rec.data_offset
        c.data_len = rec.data_len
        c.cid_len = len(rec.cid)
        c.cid[:len(rec.cid)] = list(rec.cid)
        r = fn(self._mem, ctypes.byref(c))
        del cbuf
        rec.type, rec.ver = c.type, bytes(c.ver)
        rec.data_offset, rec.data_len = c.data_offset, c.data_len
        rec.cid = bytes(c.cid[:c.cid_len])
        return r

    def encrypt_buf(self, rec: Record) -> int:
        return self._call(lib().orc_encrypt_buf, rec)

    def decrypt_buf(self, rec: Record) -> int:
        return self._call(lib().orc_decrypt_buf, rec)

    def bench(self, direction: int, arena, stride: int, data_len: int, n: int,
              seq0: int = 0, threads: int = 1, status=None) -> float:
        """Time orc_bench_records (CPU baseline).  `arena` is a writable buffer
        (numpy array) holding n records at `stride`."""
        import numpy as np
        a = np.ascontiguousarray(arena)
        st = status.ctypes.data if status is not None else None
        return lib().orc_bench_records(self._mem, direction, a.ctypes.data, stride,
                                       data_len, n, seq0, threads, st)


# ---- TLS 1.3 key schedule (oracle/keysched.c) ---------------------------------
SHA256 = 0x02000009          # PSA_ALG_SHA_256
SHA384 = 0x0200000a          # PSA_ALG_SHA_384
HASHES = {"sha256": SHA256, "sha384": SHA384}
CONTEXT_UNHASHED, CONTEXT_HASHED = 0, 1


def hash_len(alg: int) -> int:
    return {SHA256: 32, SHA384: 48}[alg]


def _ks(fn, argtypes):
    f = getattr(lib(), fn)
    f.argtypes = argtypes
    f.restype = ctypes.c_int
    return f


_P, _S = ctypes.c_char_p, ctypes.c_size_t


def _chk(r, what):
    if r != 0:
        raise ValueError(f"{what} failed: {r}")


def sha(alg: int, msg: bytes) -> bytes:
    out = _buf(64)
    _chk(_ks("orc_hash", [ctypes.c_int, _P, _S, ctypes.c_void_p])(alg, msg, len(msg), out), "orc_hash")
    return out.raw[:hash_len(alg)]


def hmac(alg: int, key: bytes, msg: bytes) -> bytes:
    out = _buf(64)
    _chk(_ks("orc_hmac", [ctypes.c_int, _P, _S, _P, _S, ctypes.c_void_p])(alg, key, len(key), msg, len(msg), out),
         "orc_hmac")
    return out.raw[:hash_len(alg)]


def hkdf_expand(alg: int, prk: bytes, info: bytes, n: int) -> bytes:
    out = _buf(max(1, n))
    _chk(_ks("orc_hkdf_expand", [ctypes.c_int, _P, _S, _P, _S, ctypes.c_void_p, _S])(
        alg, prk, len(prk), info, len(info), out, n), "orc_hkdf_expand")
    return out.raw[:n]


def tls13_encode_label(n: int, label: bytes, ctx: bytes) -> bytes:
    out = _buf(2 + 1 + 6 + 249 + 1 + 64)
    f = getattr(lib(), "orc_tls13_encode_label")
    f.argtypes = [_S, _P, _S, _P, _S, ctypes.c_void_p]
    f.restype = _S
    k = f(n, label, len(label), ctx, len(ctx), out)
    return out.raw[:k]


def tls13_hkdf_expand_label(alg: int, secret: bytes, label: bytes, ctx: bytes, n: int) -> bytes:
    out = _buf(max(1, n))
    _chk(_ks("orc_tls13_hkdf_expand_label", [ctypes.c_int, _P, _S, _P, _S, _P, _S, ctypes.c_void_p, _S])(
        alg, secret, len(secret), label, len(label), ctx, len(ctx), out, n), "expand_label")
    return out.raw[:n]


def tls13_derive_secret(alg: int, secret: bytes, label: bytes, ctx: bytes, ctx_hashed: int, n: int) -> bytes:
    out = _buf(max(1, n))
    _chk(_ks("orc_tls13_derive_secret", [ctypes.c_int, _P, _S, _P, _S, _P, _S, ctypes.c_int, ctypes.c_void_p, _S])(
        alg, secret, len(secret), label, len(label), ctx, len(ctx), ctx_hashed, out, n), "derive_secret")
    return out.raw[:n]


def tls13_evolve_secret(alg: int, secret_old: bytes | None, inp: bytes | None) -> bytes:
    out = _buf(64)
    _chk(_ks("orc_tls13_evolve_secret", [ctypes.c_int, _P, _P, _S, ctypes.c_void_p])(
        alg, secret_old or None, inp or None, len(inp or b""), out), "evolve_secret")
    return out.raw[:hash_len(alg)]


def tls13_make_traffic_keys(alg: int, client_secret: bytes, server_secret: bytes, key_len: int, iv_len: int):
    ck, ci, sk, si = _buf(32), _buf(16), _buf(32), _buf(16)
    _chk(_ks("orc_tls13_make_traffic_keys", [ctypes.c_int, _P, _P, _S, _S, _S] + [ctypes.c_void_p] * 4)(
        alg, client_secret, server_secret, len(client_secret), key_len, iv_len, ck, ci, sk, si), "make_traffic_keys")
    return ck.raw[:key_len], ci.raw[:iv_len], sk.raw[:key_len], si.raw[:iv_len]


def tls13_exporter(alg: int, secret: bytes, label: bytes, context: bytes, n: int) -> bytes:
    out = _buf(max(1, n))
    _chk(_ks("orc_tls13_exporter", [ctypes.c_int, _P, _S, _P, _S, _P, _S, ctypes.c_void_p, _S])(
        alg, secret, len(secret), label, len(label), context, len(context), out, n), "exporter")
    return out.raw[:n]


def tls13_update_traffic_secret(alg: int, secret: bytes) -> bytes:
    out = _buf(64)
    _chk(_ks("orc_tls13_update_traffic_secret", [ctypes.c_int, _P, ctypes.c_void_p])(alg, secret, out),
         "update_traffic_secret")
    return out.raw[:hash_len(alg)]


# ---- stream record loops (oracle/stream.c) -------------------------------------
ERR_COUNTER_WRAPPING = -0x6B80
MAX_IN_RECORD = 16421
OUT_BUF_SPACE = 16416


class _StreamRec(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint32), ("data_offset", ctypes.c_uint32), ("data_len", ctypes.c_uint32),
                ("type", ctypes.c_uint8)]


class _StreamRes(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("nrec", ctypes.c_uint32), ("consumed", ctypes.c_uint32),
                ("in_ctr", ctypes.c_uint8 * 8), ("nb_zero", ctypes.c_uint8)]


def stream_decrypt(t: "Transform", data: bytes, in_ctr: bytes = bytes(8), nb_zero: int = 0,
                   max_record: int = MAX_IN_RECORD, max_version: int = TLS1_3):
    """Returns (res dict, [(off, data_offset, data_len, type)], buffer after)."""
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    cap = len(data) // 6 + 1
    recs = (_StreamRec * cap)()
    res = _StreamRes()
    f = lib().orc_stream_decrypt
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _S, ctypes.c_char_p, ctypes.c_uint8, _S, ctypes.c_int,
                  ctypes.c_void_p, _S, ctypes.c_void_p]
    f.restype = ctypes.c_int
    f(t._mem, buf, len(data), bytes(in_ctr), nb_zero, max_record, max_version, recs, cap, ctypes.byref(res))
    out = [(r.off, r.data_offset, r.data_len, r.type) for r in recs[:res.nrec]]
    return ({"status": res.status, "nrec": res.nrec, "consumed": res.consumed, "in_ctr": bytes(res.in_ctr),
             "nb_zero": res.nb_zero}, out, buf.raw[:len(data)])


def stream_read(buf: bytes, recs, cap: int):
    """ssl_read_application_data over accepted records [(off, data_offset,
    data_len, type)]: returns (copied bytes, records fully consumed, bytes
    left in the last record, buffer after zeroization)."""
    b = ctypes.create_string_buffer(bytes(buf), max(1, len(buf)))
    arr = (_StreamRec * max(1, len(recs)))()
    for i, (o, d, L, t) in enumerate(recs):
        arr[i].off, arr[i].data_offset, arr[i].data_len, arr[i].type = o, d, L, t
    out = ctypes.create_string_buffer(max(1, cap))
    c, r, lft = _S(), _S(), _S()
    f = lib().orc_stream_read
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _S, ctypes.c_void_p, _S, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p]
    f(b, arr, len(recs), out, cap, ctypes.byref(c), ctypes.byref(r), ctypes.byref(lft))
    return out.raw[:c.value], r.value, lft.value, b.raw[:len(buf)]


def stream_record_wire(t: "Transform", n: int) -> int:
    f = lib().orc_stream_record_wire
    f.argtypes = [ctypes.c_void_p, _S]
    f.restype = _S
    return f(t._mem, n)


def stream_encrypt(t: "Transform", pt: bytes, rtype: int = 23, out_ctr: bytes = bytes(8), max_frag: int = 16384,
                   out_buf_space: int = OUT_BUF_SPACE):
    """Returns (status, record stream bytes, records, out_ctr after)."""
    cap = sum(stream_record_wire(t, min(max_frag, len(pt) - o)) for o in range(0, len(pt), max_frag)) + 16
    out = ctypes.create_string_buffer(cap)
    ctr = (ctypes.c_uint8 * 8)(*out_ctr)
    olen = _S()
    nrec = ctypes.c_uint32()
    f = lib().orc_stream_encrypt
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, _S, ctypes.c_uint8, ctypes.c_void_p, _S, _S, ctypes.c_void_p, _S,
                  ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_int
    r = f(t._mem, bytes(pt), len(pt), rtype, ctr, max_frag, out_buf_space, out, cap, ctypes.byref(olen),
          ctypes.byref(nrec))
    return r, out.raw[:olen.value], nrec.value, bytes(ctr)


# ---- DTLS 1.2 datagram record loops (oracle/dtls.c) ------------------------------
ERR_UNEXPECTED_RECORD = -0x6700
ERR_EARLY_MESSAGE = -0x6480
ERR_CONN_EOF = -0x7280
DTLS_MAX_DATAGRAM = 16477
DTLS_DROPPED, DTLS_NOT_REACHED = 1, 2


class DtlsState(ctypes.Structure):
    """The mbedtls_ssl_context / config fields of the DTLS read loop."""
    _fields_ = [("window_top", ctypes.c_uint64), ("window", ctypes.c_uint64), ("badmac_seen", ctypes.c_uint32),
                ("badmac_limit", ctypes.c_uint32), ("in_epoch", ctypes.c_uint16), ("cid_len", ctypes.c_uint8),
                ("anti_replay", ctypes.c_uint8), ("ignore_unexpected_cid", ctypes.c_uint8),
                ("nb_zero", ctypes.c_uint8)]


class _DtlsRec(ctypes.Structure):
    _fields_ = [("dgram", ctypes.c_uint32), ("off", ctypes.c_uint32), ("data_offset", ctypes.c_uint32),
                ("data_len", ctypes.c_uint32), ("disp", ctypes.c_int32), ("type", ctypes.c_uint8)]


class _DtlsRes(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("nrec", ctypes.c_uint32), ("naccepted", ctypes.c_uint32),
                ("dgrams_done", ctypes.c_uint32), ("invalid_dgrams", ctypes.c_uint32)]


def dtls_replay_check(st: DtlsState, ctr: bytes) -> int:
    f = lib().orc_dtls_replay_check
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    f.restype = ctypes.c_int
    return f(ctypes.byref(st), bytes(ctr))


def dtls_replay_update(st: DtlsState, ctr: bytes) -> None:
    f = lib().orc_dtls_replay_update
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    f.restype = None
    f(ctypes.byref(st), bytes(ctr))


def dtls_decrypt(t: "Transform", st: DtlsState, datagrams):
    """One connection's datagrams (list of bytes), in arrival order.  `st` is
    updated in place.  Returns (res dict, [(dgram, off, data_offset,
    data_len, disp, type)], [datagram bytes after])."""
    offs, pos = [], 0
    for d in datagrams:
        offs.append(pos)
        pos += len(d)
    buf = ctypes.create_string_buffer(b"".join(datagrams), max(1, pos))
    cap = pos // 13 + 1
    recs = (_DtlsRec * cap)()
    res = _DtlsRes()
    doff = (ctypes.c_uint64 * max(1, len(datagrams)))(*offs)
    dlen = (ctypes.c_uint32 * max(1, len(datagrams)))(*[len(d) for d in datagrams])
    f = lib().orc_dtls_decrypt
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _S,
                  ctypes.c_void_p, _S, ctypes.c_void_p]
    f.restype = ctypes.c_int
    f(t._mem, ctypes.byref(st), buf, doff, dlen, len(datagrams), recs, cap, ctypes.byref(res))
    out = [(r.dgram, r.off, r.data_offset, r.data_len, r.disp, r.type) for r in recs[:res.nrec]]
    raw = buf.raw
    return ({"status": res.status, "nrec": res.nrec, "naccepted": res.naccepted, "dgrams_done": res.dgrams_done,
             "invalid_dgrams": res.invalid_dgrams}, out,
            [raw[o:o + len(d)] for o, d in zip(offs, datagrams)])


def dtls_record_wire(t: "Transform", n: int) -> int:
    f = lib().orc_dtls_record_wire
    f.argtypes = [ctypes.c_void_p, _S]
    f.restype = _S
    return f(t._mem, n)


def dtls_encrypt(t: "Transform", pt: bytes, rtype: int = 23, out_ctr: bytes = bytes(8), max_frag: int = 16384):
    """Returns (status, datagrams back to back, records, out_ctr after)."""
    cap = sum(dtls_record_wire(t, min(max_frag, len(pt) - o)) for o in range(0, len(pt), max_frag)) + 16
    out = ctypes.create_string_buffer(cap)
    ctr = (ctypes.c_uint8 * 8)(*out_ctr)
    olen = _S()
    nrec = ctypes.c_uint32()
    f = lib().orc_dtls_encrypt
    f.argtypes = [ctypes.c_void_p, ctypes.c_char_p, _S, ctypes.c_uint8, ctypes.c_void_p, _S, ctypes.c_void_p, _S,
                  ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_int
    r = f(t._mem, bytes(pt), len(pt), rtype, ctr, max_frag, out, cap, ctypes.byref(olen), ctypes.byref(nrec))
    return r, out.raw[:olen.value], nrec.value, bytes(ctr)


# ---- session tickets (oracle/ticket.c) -------------------------------------------
ERR_SESSION_TICKET_EXPIRED = -0x6D80


class _TicketKey(ctypes.Structure):
    _fields_ = [("cipher", ctypes.c_int), ("key", ctypes.c_uint8 * 32), ("name", ctypes.c_uint8 * 4)]


def _tkeys(keys):
    arr = (_TicketKey * 2)()
    for i, (c, k, name) in enumerate(keys):
        arr[i].cipher = c
        arr[i].key[:len(k)] = list(k)
        arr[i].name[:] = list(name)
    return arr


def ticket_write(keys, active: int, iv: bytes, state: bytes, space: int):
    """keys: [(cipher, key, name4)] x 2.  Returns (status, ticket bytes)."""
    buf = ctypes.create_string_buffer(max(space, 18 + len(state), 16))
    buf[4:16] = bytes(iv)
    buf[18:18 + len(state)] = bytes(state)
    tlen = _S()
    f = lib().orc_ticket_write
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, _S, _S, ctypes.c_void_p]
    f.restype = ctypes.c_int
    r = f(_tkeys(keys), active, buf, space, len(state), ctypes.byref(tlen))
    return r, buf.raw[:tlen.value] if r == 0 else b""


def ticket_parse(keys, ticket: bytes):
    """Returns (status, clear state bytes, buffer after)."""
    buf = ctypes.create_string_buffer(bytes(ticket), max(1, len(ticket)))
    cl = _S()
    f = lib().orc_ticket_parse
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _S, ctypes.c_void_p]
    f.restype = ctypes.c_int
    r = f(_tkeys(keys), buf, len(ticket), ctypes.byref(cl))
    raw = buf.raw[:len(ticket)]
    return r, (raw[18:18 + cl.value] if r == 0 else b""), raw


# ---- CPU-baseline leg on OpenSSL EVP (oracle/evp_bench.c) ----------------------
EVP_LIB_PATH = os.path.join(HERE, "libevpbench.so")
_evp = None


def evp_lib():
    """libevpbench.so: the record framing around OpenSSL 3 EVP AEADs (AES-NI /
    VAES GCM, SIMD ChaCha20-Poly1305), the accelerated x86 stand-in for the
    reference's CPU path in bench.py's cpu_baseline (AES-128/256-GCM and
    ChaCha20-Poly1305 only)."""
    global _evp
    if _evp is None:
        if not os.path.exists(EVP_LIB_PATH):
            build()
        L = ctypes.CDLL(EVP_LIB_PATH)
        L.evp_bench_records.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        L.evp_bench_records.restype = ctypes.c_double
        L.evp_mixed_create.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.c_int]
        L.evp_mixed_create.restype = ctypes.c_void_p
        L.evp_mixed_free.argtypes = [ctypes.c_void_p]
        L.evp_mixed_free.restype = None
        L.evp_mixed_records.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_size_t, ctypes.c_uint64, ctypes.c_void_p]
        L.evp_mixed_records.restype = ctypes.c_double
        L.evp_mixed_stream.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.c_void_p]
        L.evp_mixed_stream.restype = ctypes.c_double
        L.evp_call_profile.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.evp_call_profile.restype = ctypes.c_int
        L.evp_check_records.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_void_p]
        L.evp_check_records.restype = ctypes.c_int
        _evp = L
    return _evp


EVP_CIPHERS = (AES_128_GCM, AES_256_GCM, CHACHA20_POLY1305)


def evp_bench(cipher: int, tls_version: int, key: bytes, iv: bytes, direction: int, arena, stride: int,
              data_len: int, n: int, seq0: int, threads: int, status) -> float:
    """Time evp_bench_records: n records at `stride` in the numpy `arena`,
    direction 1 = encrypt (data_len = content bytes, at offset 8 for TLS 1.2
    GCM), 0 = decrypt (data_len = protected body).  Returns seconds."""
    if cipher not in EVP_CIPHERS:
        raise ValueError("evp_bench: AES-128/256-GCM and ChaCha20-Poly1305 only")
    return evp_lib().evp_bench_records(cipher, int(tls_version == TLS1_3), bytes(key), bytes(iv), direction,
                                       arena.ctypes.data, stride, data_len, n, seq0, threads,
                                       status.ctypes.data)


def bench_multi(transforms, direction: int, arena, stride: int, data_len: int, n: int, threads: int,
                status) -> float:
    """Time orc_bench_records_multi: record i under transforms[i % len],
    sequence number i // len, one thread per connection subset.  Seconds."""
    arr = (ctypes.c_void_p * len(transforms))(*[ctypes.addressof(t._mem) for t in transforms])
    return lib().orc_bench_records_multi(arr, len(transforms), direction, arena.ctypes.data, stride, data_len, n,
                                         threads, status.ctypes.data)


def bench_stream_rows(transforms, dtls: bool, direction: int, inp, in_stride: int, in_len: int, out,
                      out_stride: int, max_frag: int, threads: int, status) -> float:
    """Time orc_bench_stream_rows (oracle/rows_bench.c): connection c under
    transforms[c] sends (direction 1) its in_len bytes of application data as
    max_frag records (orc_stream_encrypt / orc_dtls_encrypt) or receives (0)
    its in_len wire bytes in place (orc_stream_decrypt / orc_dtls_decrypt;
    DTLS: max_frag = one datagram's wire size).  Seconds."""
    arr = (ctypes.c_void_p * len(transforms))(*[ctypes.addressof(t._mem) for t in transforms])
    return lib().orc_bench_stream_rows(arr, len(transforms), int(bool(dtls)), direction, inp.ctypes.data, in_stride,
                                       in_len, out.ctypes.data if out is not None else None, out_stride, max_frag,
                                       threads, status.ctypes.data)


def bench_keysched(alg: int, secrets, count: int, update: bool, keylen: int, threads: int):
    """Time orc_bench_keysched: per connection KeyUpdate (optional) then
    HKDF-Expand-Label key / iv (ssl_tls13_keys.c:219-291).  Returns (seconds,
    out keys (count, keylen + 12), status)."""
    import numpy as np
    sec = np.ascontiguousarray(secrets, dtype=np.uint8)
    out = np.zeros((count, keylen + 12), dtype=np.uint8)
    st = np.zeros(count, dtype=np.int32)
    t = lib().orc_bench_keysched(alg, sec.ctypes.data, count, int(bool(update)), keylen, threads, out.ctypes.data,
                                 st.ctypes.data)
    return t, out, st


class EvpMixed:
    """evp_mixed_*: one OpenSSL EVP context per connection (the c4 / c4s CPU
    leg).  ciphers: uint8 array (AES_128_GCM / AES_256_GCM / CHACHA20_POLY1305
    per connection), keys (n, 32), ivs (n, 12) uint8 arrays."""

    def __init__(self, ciphers, keys, ivs, tls_version, threads: int = 1):
        import numpy as np
        c = np.ascontiguousarray(ciphers, dtype=np.uint8)
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(len(c), 32)
        v = np.ascontiguousarray(ivs, dtype=np.uint8).reshape(len(c), 12)
        if not set(np.unique(c).tolist()) <= set(EVP_CIPHERS):
            raise ValueError("EvpMixed: AES-128/256-GCM and ChaCha20-Poly1305 only")
        self.threads = threads
        self._h = evp_lib().evp_mixed_create(len(c), c.ctypes.data, k.ctypes.data, v.ctypes.data,
                                              int(tls_version == TLS1_3), threads)
        if not self._h:
            raise RuntimeError("evp_mixed_create failed")

    def run(self, direction: int, arena, stride: int, data_len: int, n: int, status) -> float:
        """n records on the threads given at construction"""
        return evp_lib().evp_mixed_records(self._h, direction, arena.ctypes.data, stride, data_len, n,
                                           status.ctypes.data)

    def stream(self, dtls: bool, direction: int, inp, in_stride: int, in_len: int, out, out_stride: int,
               max_frag: int, status) -> float:
        """evp_mixed_stream: connection c's records sent (direction 1: in_len
        bytes of application data -> max_frag records in `out`) or received
        (0: in_len wire bytes decrypted in place; DTLS: max_frag = one
        datagram's wire size), the stream (ssl_msg.c:4700-4907 / :2648-2793)
        or DTLS 1.2 framing around one EVP AEAD per record.  Seconds."""
        return evp_lib().evp_mixed_stream(self._h, int(bool(dtls)), direction, inp.ctypes.data, in_stride, in_len,
                                          out.ctypes.data if out is not None else None, out_stride, max_frag,
                                          status.ctypes.data)

    def close(self):
        if self._h:
            evp_lib().evp_mixed_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def evp_call_profile(cipher: int, length: int, iters: int = 20000):
    """Microseconds per record spent in each EVP call of the EVP leg:
    {init_aad, update, final, tag} (evp_call_profile in evp_bench.c)."""
    out = (ctypes.c_double * 4)()
    if evp_lib().evp_call_profile(cipher, length, iters, out) != 0:
        return None
    return {"init_aad_us": round(out[0], 3), "update_us": round(out[1], 3), "final_us": round(out[2], 3),
            "tag_us": round(out[3], 3)}


def evp_check_records(mode: int, cipher: int, tls_version: int, keys, ivs, keyidx, seq, off, lengths, plain,
                      got=None, threads: int = 8):
    """Bulk EVP check of variable-length records (evp_check_records in
    evp_bench.c): mode 0 seals `plain` in place, mode 1 compares `got` (GPU
    encrypt output) with EVP's seal of `plain`, mode 2 compares the content of
    `got` (GPU decrypt output) with `plain`.  Returns the per-record int32
    result (0 = match / status 0)."""
    import numpy as np
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    ivs = np.ascontiguousarray(ivs, dtype=np.uint8)
    keyidx = np.ascontiguousarray(keyidx, dtype=np.uint32)
    seq = np.ascontiguousarray(seq, dtype=np.uint64)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = len(off)
    res = np.zeros(n, dtype=np.int32)
    g = got.ctypes.data if got is not None else None
    r = evp_lib().evp_check_records(mode, cipher, int(tls_version == TLS1_3), len(keys), keys.ctypes.data,
                                    ivs.ctypes.data, n, keyidx.ctypes.data, seq.ctypes.data, off.ctypes.data,
                                    lengths.ctypes.data, plain.ctypes.data, g, threads, res.ctypes.data)
    if r != 0:
        raise RuntimeError("evp_check_records failed")
    return res
