"""TLS 1.3 key schedule on the GPU (library/ssl_tls13_keys.c), through the
C ABI of include/tlsrec.h.  Same arguments, outputs and error codes as the
reference functions; every hash / HMAC / HKDF step runs in a HIP kernel.

    mbedtls_ssl_tls13_hkdf_expand_label  (:138)  -> hkdf_expand_label
    mbedtls_ssl_tls13_derive_secret      (:293)  -> derive_secret
    mbedtls_ssl_tls13_evolve_secret      (:332)  -> evolve_secret
    mbedtls_ssl_tls13_make_traffic_keys  (:262)  -> make_traffic_keys
    mbedtls_ssl_tls13_exporter           (:1828) -> exporter
    KeyUpdate, "traffic upd" (ssl_tls13_keys.h:16, RFC 8446 7.2) -> update_traffic_secret
    batch: secrets in HBM -> key-table slots       -> keytab_derive
"""
from __future__ import annotations

import ctypes

from . import _abi
from .batch import KeyTable, _ptr, _stream

ALG_SHA_256 = _abi.ALG_SHA_256
ALG_SHA_384 = _abi.ALG_SHA_384
CONTEXT_UNHASHED = _abi.TLS13_CONTEXT_UNHASHED
CONTEXT_HASHED = _abi.TLS13_CONTEXT_HASHED
HASH_LEN = {ALG_SHA_256: 32, ALG_SHA_384: 48}


class KeyScheduleError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed: {code}")
        self.code = code


def _chk(fn, r):
    if r != 0:
        raise KeyScheduleError(fn, r)


def _b(x):
    return None if x is None else bytes(x)


def hkdf_expand_label(hash_alg: int, secret: bytes, label: bytes, ctx: bytes, n: int) -> bytes:
    out = ctypes.create_string_buffer(max(1, n))
    _chk("tlsrec_tls13_hkdf_expand_label", _abi.load().tlsrec_tls13_hkdf_expand_label(
        hash_alg, _b(secret), len(secret), _b(label), len(label), _b(ctx), len(ctx), out, n))
    return out.raw[:n]


def derive_secret(hash_alg: int, secret: bytes, label: bytes, ctx: bytes, ctx_hashed: int, n: int) -> bytes:
    out = ctypes.create_string_buffer(max(1, n))
    _chk("tlsrec_tls13_derive_secret", _abi.load().tlsrec_tls13_derive_secret(
        hash_alg, _b(secret), len(secret), _b(label), len(label), _b(ctx), len(ctx), ctx_hashed, out, n))
    return out.raw[:n]


def evolve_secret(hash_alg: int, secret_old: bytes | None, inp: bytes | None) -> bytes:
    out = ctypes.create_string_buffer(64)
    _chk("tlsrec_tls13_evolve_secret", _abi.load().tlsrec_tls13_evolve_secret(
        hash_alg, _b(secret_old) or None, _b(inp) or None, len(inp or b""), out))
    return out.raw[:HASH_LEN[hash_alg]]


def make_traffic_keys(hash_alg: int, client_secret: bytes, server_secret: bytes, key_len: int, iv_len: int):
    ks = _abi.CKeySet()
    _chk("tlsrec_tls13_make_traffic_keys", _abi.load().tlsrec_tls13_make_traffic_keys(
        hash_alg, _b(client_secret), _b(server_secret), len(client_secret), key_len, iv_len, ctypes.byref(ks)))
    return (bytes(ks.client_write_key[:key_len]), bytes(ks.client_write_iv[:iv_len]),
            bytes(ks.server_write_key[:key_len]), bytes(ks.server_write_iv[:iv_len]))


def exporter(hash_alg: int, secret: bytes, label: bytes, context: bytes, n: int) -> bytes:
    out = ctypes.create_string_buffer(max(1, n))
    _chk("tlsrec_tls13_exporter", _abi.load().tlsrec_tls13_exporter(
        hash_alg, _b(secret), len(secret), _b(label), len(label), _b(context), len(context), out, n))
    return out.raw[:n]


def update_traffic_secret(hash_alg: int, secret: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    _chk("tlsrec_tls13_update_traffic_secret",
         _abi.load().tlsrec_tls13_update_traffic_secret(hash_alg, _b(secret), out))
    return out.raw[:HASH_LEN[hash_alg]]


def keytab_derive(kt: KeyTable, first: int, count: int, cipher: int, secrets, key_update: bool = False,
                  stream=None) -> None:
    """`secrets`: device buffer (uint8 tensor) of count x 48 bytes
    (tlsrec_tls13_secret); updated in place when key_update."""
    _chk("tlsrec_tls13_keytab_derive", _abi.load().tlsrec_tls13_keytab_derive(
        kt.handle, first, count, cipher, _ptr(secrets), int(bool(key_update)), _stream(stream)))
