"""ctypes binding of include/tlsrec.h (the C ABI of libtlsrec.so).

This is the same binding a maintainer would add to a Python caller of the
reference record path; it loads the in-tree HIP library
and raises if it is missing -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libtlsrec.so")

# ---- constants (include/tlsrec.h, values of include/mbedtls/ssl.h) ----------
ERR_SSL_BAD_INPUT_DATA = -135
ERR_SSL_BUFFER_TOO_SMALL = -138
ERR_SSL_ALLOC_FAILED = -141
ERR_SSL_FEATURE_UNAVAILABLE = -0x7080
ERR_SSL_INVALID_MAC = -0x7180
ERR_SSL_INVALID_RECORD = -0x7200
ERR_SSL_HW_ACCEL_FAILED = -0x7F80
ERR_SSL_INTERNAL_ERROR = -0x6C00
ERR_SSL_UNEXPECTED_CID = -0x6000
ERR_SSL_COUNTER_WRAPPING = -0x6B80
ERR_SSL_SESSION_TICKET_EXPIRED = -0x6D80
ERR_SSL_UNEXPECTED_RECORD = -0x6700
ERR_SSL_EARLY_MESSAGE = -0x6480
ERR_SSL_CONN_EOF = -0x7280
DTLS_MAX_DATAGRAM = 16477
DTLS_OUT_BUFFER_LEN = 16477
DTLS_DROPPED, DTLS_NOT_REACHED = 1, 2
DTLS_ANTI_REPLAY, DTLS_IGNORE_UNEXPECTED_CID = 1, 2
MAX_IN_RECORD = 16421
OUT_BUF_SPACE = 16416

VERSION_TLS1_2 = 0x0303
VERSION_TLS1_3 = 0x0304
CIPHER_AES_128_GCM = 1
CIPHER_AES_256_GCM = 2
CIPHER_CHACHA20_POLY1305 = 3
CIPHER_AES_192_GCM = 4
CIPHER_AES_128_CCM, CIPHER_AES_192_CCM, CIPHER_AES_256_CCM = 5, 6, 7
CIPHER_AES_128_CCM_8, CIPHER_AES_192_CCM_8, CIPHER_AES_256_CCM_8 = 8, 9, 10
CIPHER_ARIA_128_GCM, CIPHER_ARIA_192_GCM, CIPHER_ARIA_256_GCM = 11, 12, 13
CIPHER_ARIA_128_CCM, CIPHER_ARIA_192_CCM, CIPHER_ARIA_256_CCM = 14, 15, 16
CIPHER_CAMELLIA_128_GCM, CIPHER_CAMELLIA_192_GCM, CIPHER_CAMELLIA_256_GCM = 17, 18, 19
CIPHER_CAMELLIA_128_CCM, CIPHER_CAMELLIA_192_CCM, CIPHER_CAMELLIA_256_CCM = 20, 21, 22
KEYLEN = {1: 16, 2: 32, 3: 32, 4: 24, 5: 16, 6: 24, 7: 32, 8: 16, 9: 24, 10: 32, 11: 16, 12: 24, 13: 32,
          14: 16, 15: 24, 16: 32, 17: 16, 18: 24, 19: 32, 20: 16, 21: 24, 22: 32}
TAGLEN = {c: (8 if 8 <= c <= 10 else 16) for c in KEYLEN}
MSG_APPLICATION_DATA = 23
MSG_CID = 25
CID_LEN_MAX = 32
ALG_SHA_256 = 0x02000009      # PSA_ALG_SHA_256
ALG_SHA_384 = 0x0200000a      # PSA_ALG_SHA_384
TLS13_CONTEXT_UNHASHED = 0
TLS13_CONTEXT_HASHED = 1

# ---- layouts -----------------------------------------------------------------
KEY_MATERIAL = np.dtype([("cipher", "u1"), ("tls_minor", "u1"), ("fixed_ivlen", "u1"),
                         ("taglen", "u1"), ("granularity", "u1"), ("reserved", "u1", 11),
                         ("iv", "u1", 16), ("key", "u1", 32)])
BATCH_REC = np.dtype([("buf_off", "<u8"), ("buf_len", "<u4"), ("data_offset", "<u4"),
                      ("data_len", "<u4"), ("slot", "<u4"), ("ctr", "u1", 8), ("type", "u1"),
                      ("ver", "u1", 2), ("cid_len", "u1"), ("cid_off", "<u4")], align=False)
BATCH_RES = np.dtype([("status", "<i4"), ("data_offset", "<u4"), ("data_len", "<u4"),
                      ("type", "u1"), ("cid_len", "u1"), ("reserved", "u1", 2)])
STREAM_IN = np.dtype([("off", "<u8"), ("len", "<u4"), ("slot", "<u4"), ("in_ctr", "u1", 8),
                      ("nb_zero", "u1"), ("reserved", "u1", 7)])
STREAM_IN_RES = np.dtype([("status", "<i4"), ("first", "<u4"), ("nrec", "<u4"), ("consumed", "<u4"),
                          ("in_ctr", "u1", 8), ("nb_zero", "u1"), ("reserved", "u1", 3), ("nparsed", "<u4")])
STREAM_OUT = np.dtype([("in_off", "<u8"), ("in_len", "<u4"), ("slot", "<u4"), ("out_off", "<u8"),
                       ("out_ctr", "u1", 8), ("max_frag", "<u4"), ("type", "u1"), ("reserved", "u1", 3)])
STREAM_OUT_RES = np.dtype([("status", "<i4"), ("first", "<u4"), ("nrec", "<u4"), ("out_len", "<u4"),
                           ("out_ctr", "u1", 8), ("nparsed", "<u4"), ("reserved", "u1", 4)])
TICKET = np.dtype([("off", "<u8"), ("len", "<u4"), ("clear_len", "<u4")])
TICKET_RES = np.dtype([("status", "<i4"), ("tlen", "<u4"), ("reserved", "<u4", 2)])
assert TICKET.itemsize == 16 and TICKET_RES.itemsize == 16
STREAM_READ_REQ = np.dtype([("out_off", "<u8"), ("out_cap", "<u4"), ("reserved", "<u4")])
STREAM_READ_RES = np.dtype([("copied", "<u4"), ("records", "<u4"), ("left", "<u4"), ("reserved", "<u4")])
assert STREAM_READ_REQ.itemsize == 16 and STREAM_READ_RES.itemsize == 16
DGRAM = np.dtype([("off", "<u8"), ("len", "<u4"), ("reserved", "<u4")])
DTLS_IN = np.dtype([("window_top", "<u8"), ("window", "<u8"), ("first_dgram", "<u4"), ("ndgram", "<u4"),
                    ("slot", "<u4"), ("badmac_seen", "<u4"), ("badmac_limit", "<u4"), ("in_epoch", "<u2"),
                    ("cid_len", "u1"), ("flags", "u1"), ("nb_zero", "u1"), ("reserved", "u1", 7)])
DTLS_IN_RES = np.dtype([("window_top", "<u8"), ("window", "<u8"), ("status", "<i4"), ("first", "<u4"),
                        ("nrec", "<u4"), ("naccepted", "<u4"), ("dgrams_done", "<u4"), ("invalid_dgrams", "<u4"),
                        ("badmac_seen", "<u4"), ("nb_zero", "u1"), ("reserved", "u1", 3)])
assert DGRAM.itemsize == 16 and DTLS_IN.itemsize == 48 and DTLS_IN_RES.itemsize == 48
assert STREAM_IN.itemsize == 32 and STREAM_IN_RES.itemsize == 32
assert STREAM_OUT.itemsize == 40 and STREAM_OUT_RES.itemsize == 32
assert KEY_MATERIAL.itemsize == 64 and BATCH_REC.itemsize == 40 and BATCH_RES.itemsize == 16


class CTransform(ctypes.Structure):
    _fields_ = [("minlen", ctypes.c_size_t), ("ivlen", ctypes.c_size_t),
                ("fixed_ivlen", ctypes.c_size_t), ("maclen", ctypes.c_size_t),
                ("taglen", ctypes.c_size_t), ("iv_enc", ctypes.c_ubyte * 16),
                ("iv_dec", ctypes.c_ubyte * 16), ("tls_version", ctypes.c_int),
                ("cipher", ctypes.c_int), ("keylen", ctypes.c_size_t),
                ("key_enc", ctypes.c_ubyte * 32), ("key_dec", ctypes.c_ubyte * 32),
                ("slot_enc", ctypes.c_int32), ("slot_dec", ctypes.c_int32),
                ("granularity", ctypes.c_uint32), ("in_cid_len", ctypes.c_uint8),
                ("out_cid_len", ctypes.c_uint8), ("in_cid", ctypes.c_ubyte * 32),
                ("out_cid", ctypes.c_ubyte * 32)]


class CKeySet(ctypes.Structure):
    """struct mbedtls_ssl_key_set (library/ssl_misc.h:604-618)"""
    _fields_ = [("client_write_key", ctypes.c_ubyte * 32), ("server_write_key", ctypes.c_ubyte * 32),
                ("client_write_iv", ctypes.c_ubyte * 16), ("server_write_iv", ctypes.c_ubyte * 16),
                ("key_len", ctypes.c_size_t), ("iv_len", ctypes.c_size_t)]


class CTicketKeys(ctypes.Structure):
    """the keys[2] / active fields of mbedtls_ssl_ticket_context"""
    _fields_ = [("slot", ctypes.c_uint32 * 2), ("name", (ctypes.c_uint8 * 4) * 2), ("active", ctypes.c_uint32)]


class CRecord(ctypes.Structure):
    _fields_ = [("ctr", ctypes.c_ubyte * 8), ("type", ctypes.c_ubyte), ("ver", ctypes.c_ubyte * 2),
                ("buf", ctypes.c_void_p), ("buf_len", ctypes.c_size_t),
                ("data_offset", ctypes.c_size_t), ("data_len", ctypes.c_size_t),
                ("cid_len", ctypes.c_ubyte), ("cid", ctypes.c_ubyte * 32)]


# every function include/tlsrec.h declares, with its signature
_VP, _U32, _INT, _SZ = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
SIGNATURES = {
    "tlsrec_transform_setup": (_INT, [_VP, _INT, _INT, _VP, _VP, _VP, _VP]),
    "tlsrec_transform_setup_ex": (_INT, [_VP, _INT, _INT, _VP, _VP, _VP, _VP, ctypes.c_uint]),
    "tlsrec_transform_free": (None, [_VP]),
    "tlsrec_transform_set_cid": (_INT, [_VP, _VP, _SZ, _VP, _SZ]),
    "tlsrec_keytab_set_cid": (_INT, [_VP, _U32, _VP, _SZ, _VP]),
    "tlsrec_encrypt_buf": (_INT, [_VP, _VP, _VP]),
    "tlsrec_decrypt_buf": (_INT, [_VP, _VP, _VP]),
    "tlsrec_keytab_create": (_INT, [ctypes.POINTER(_VP), _U32]),
    "tlsrec_keytab_load": (_INT, [_VP, _U32, _U32, _VP, _INT, _VP]),
    "tlsrec_keytab_capacity": (_U32, [_VP]),
    "tlsrec_keytab_free": (None, [_VP]),
    "tlsrec_batch_encrypt": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _U32, _VP]),
    "tlsrec_batch_decrypt": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _U32, _VP]),
    "tlsrec_batch_encrypt_sized": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _U32, _VP]),
    "tlsrec_batch_decrypt_sized": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _U32, _VP]),
    "tlsrec_host_batch_encrypt": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _U32, ctypes.c_uint64]),
    "tlsrec_host_batch_decrypt": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _U32, ctypes.c_uint64]),
    "tlsrec_frame_check": (_INT, [_INT, _VP, _VP, _VP, _VP, _VP]),
    "tlsrec_shard_bounds": (_INT, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _VP, _VP]),
    "tlsrec_device_check": (_INT, []),
    "tlsrec_tls13_hkdf_expand_label": (_INT, [_INT, _VP, _SZ, _VP, _SZ, _VP, _SZ, _VP, _SZ]),
    "tlsrec_tls13_derive_secret": (_INT, [_INT, _VP, _SZ, _VP, _SZ, _VP, _SZ, _INT, _VP, _SZ]),
    "tlsrec_tls13_evolve_secret": (_INT, [_INT, _VP, _VP, _SZ, _VP]),
    "tlsrec_tls13_make_traffic_keys": (_INT, [_INT, _VP, _VP, _SZ, _SZ, _SZ, _VP]),
    "tlsrec_tls13_exporter": (_INT, [_INT, _VP, _SZ, _VP, _SZ, _VP, _SZ, _VP, _SZ]),
    "tlsrec_tls13_update_traffic_secret": (_INT, [_INT, _VP, _VP]),
    "tlsrec_tls13_keytab_derive": (_INT, [_VP, _U32, _U32, _INT, _VP, _INT, _VP]),
    "tlsrec_ticket_write": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _VP]),
    "tlsrec_ticket_parse": (_INT, [_VP, _VP, _VP, _U32, _VP, _VP, _VP]),
    "tlsrec_stream_decrypt": (_INT, [_VP, _VP, _U32, _VP, _VP, _VP, _U32, _VP, _VP, _VP]),
    "tlsrec_stream_read": (_INT, [_VP, _U32, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    "tlsrec_stream_out_size": (ctypes.c_uint64, [_INT, _INT, _U32, ctypes.c_uint64, _U32]),
    "tlsrec_stream_encrypt": (_INT, [_VP, _VP, _U32, _VP, _VP, _VP, _VP, _U32, _VP, _VP, _VP]),
    "tlsrec_dtls_decrypt": (_INT, [_VP, _VP, _U32, _VP, _U32, _VP, _VP, _VP, _VP, _U32, _VP, _VP, _VP]),
    "tlsrec_dtls_out_size": (ctypes.c_uint64, [_INT, _U32, _U32, ctypes.c_uint64, _U32]),
    "tlsrec_dtls_encrypt": (_INT, [_VP, _VP, _U32, _VP, _VP, _VP, _VP, _U32, _VP, _VP, _VP]),
    "tlsrec_version_string": (ctypes.c_char_p, []),
}

_lib = None


def load():
    """Load libtlsrec.so (HIP runtime linked).  torch, when importable, is
    imported first so that the process uses a single libamdhip64."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (shares its HIP runtime with us)
    except Exception:
        pass
    # TLSREC_LIBRARY: an alternative in-tree build of the same ABI (A/B runs)
    path = os.environ.get("TLSREC_LIBRARY") or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with `python -m mbedtls_amd.build` "
                          "(there is no CPU fallback)")
    L = ctypes.CDLL(path)
    alt = path != LIB_PATH
    for name, (res, args) in SIGNATURES.items():
        if alt and not hasattr(L, name):
            continue          # an older A/B build may predate an entry point
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


TEST_LIB_PATH = os.path.join(PKG, "libtlsrec_test.so")
_test_lib = None


def test_library():
    """The test-hooks build (tests/ only), loaded once, with the ABI's
    signatures bound."""
    global _test_lib
    if _test_lib is None:
        if not os.path.exists(TEST_LIB_PATH):
            raise ImportError(f"{TEST_LIB_PATH} is missing: build it with `python -m mbedtls_amd.build`")
        load()                       # torch first, as load() does
        L = ctypes.CDLL(TEST_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _test_lib = L
    return _test_lib


class use_library:
    """Context manager for tests/: route every binding to another in-tree
    build of the same ABI for the duration -- the test-hooks build
    libtlsrec_test.so (-DTLSREC_TEST_HOOKS, the only one exporting
    tlsrec__test_*).  Objects (KeyTable, Transform) keep the library they were
    created with, so create them inside the block."""

    def __init__(self):
        self.saved = None

    def __enter__(self):
        global _lib
        L = test_library()
        self.saved, _lib = _lib, L
        return L

    def __exit__(self, *exc):
        global _lib
        _lib = self.saved
        return False
