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
        _lib = L
    return _lib


# struct sizes: generous opaque buffers (orc_gcm_ctx ~ 520 B, orc_transform ~ 1.2 KiB)
_GCM_CTX = 1024
_TRANSFORM = 4096


def _buf(n):
    return ctypes.create_string_buffer(n)


def aes_encrypt_block(key: bytes, block: bytes) -> bytes:
    ctx = _buf(512)
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
                ("data_len", ctypes.c_size_t)]


@dataclass
class Record:
    """Python mirror of mbedtls_record (library/ssl_misc.h:1163-1188), non-CID."""
    ctr: bytes
    type: int
    ver: bytes
    buf: bytearray
    data_offset: int
    data_len: int
    buf_len: int = field(default=-1)

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
        r = fn(self._mem, ctypes.byref(c))
        del cbuf
        rec.type, rec.ver = c.type, bytes(c.ver)
        rec.data_offset, rec.data_len = c.data_offset, c.data_len
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
