"""Independent AEAD cross-check through OpenSSL libcrypto (ctypes, EVP API).

Used only by tests and the golden-vector generator to cross-validate the CPU
restatement in oracle/ for AES-256-GCM and ChaCha20-Poly1305, for which the
reference ships no record-level KAT.  Returns None when the
library is not present.
"""
from __future__ import annotations

import ctypes
import ctypes.util

_lib = None


def lib():
    global _lib
    if _lib is None:
        for name in ("libcrypto.so.3", ctypes.util.find_library("crypto")):
            if not name:
                continue
            try:
                _lib = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _lib is None:
            return None
        L = _lib
        L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        for f in ("EVP_aria_128_gcm", "EVP_aria_192_gcm", "EVP_aria_256_gcm", "EVP_aria_128_ecb",
                  "EVP_aria_128_ccm", "EVP_aria_192_ccm", "EVP_aria_256_ccm",
                  "EVP_aes_128_gcm", "EVP_aes_192_gcm", "EVP_aes_256_gcm", "EVP_chacha20_poly1305",
                  "EVP_aes_128_ccm", "EVP_aes_192_ccm", "EVP_aes_256_ccm",
                  "EVP_camellia_128_ecb", "EVP_camellia_192_ecb", "EVP_camellia_256_ecb",
                  "EVP_camellia_128_cbc", "EVP_camellia_192_cbc", "EVP_camellia_256_cbc"):
            getattr(L, f).restype = ctypes.c_void_p
        L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_char_p, ctypes.c_char_p]
        L.EVP_DecryptInit_ex.argtypes = L.EVP_EncryptInit_ex.argtypes
        L.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        upd = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
               ctypes.c_char_p, ctypes.c_int]
        L.EVP_EncryptUpdate.argtypes = upd
        L.EVP_DecryptUpdate.argtypes = upd
        L.EVP_EncryptFinal_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.EVP_DecryptFinal_ex.argtypes = L.EVP_EncryptFinal_ex.argtypes
        L.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
    return _lib


EVP_CTRL_AEAD_SET_IVLEN = 0x9
EVP_CTRL_AEAD_GET_TAG = 0x10
EVP_CTRL_AEAD_SET_TAG = 0x11


def _cipher(name: str, keylen: int):
    L = lib()
    if name == "gcm":
        return {16: L.EVP_aes_128_gcm, 24: L.EVP_aes_192_gcm, 32: L.EVP_aes_256_gcm}[keylen]()
    if name == "aria-gcm":
        return {16: L.EVP_aria_128_gcm, 24: L.EVP_aria_192_gcm, 32: L.EVP_aria_256_gcm}[keylen]()
    if name == "aria-ccm":
        return {16: L.EVP_aria_128_ccm, 24: L.EVP_aria_192_ccm, 32: L.EVP_aria_256_ccm}[keylen]()
    if name == "ccm":
        return {16: L.EVP_aes_128_ccm, 24: L.EVP_aes_192_ccm, 32: L.EVP_aes_256_ccm}[keylen]()
    return L.EVP_chacha20_poly1305()


def seal(name: str, key: bytes, nonce: bytes, aad: bytes, pt: bytes):
    L = lib()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        c = _cipher(name, len(key))
        assert L.EVP_EncryptInit_ex(ctx, c, None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, len(nonce), None) == 1
        assert L.EVP_EncryptInit_ex(ctx, None, None, key, nonce) == 1
        n = ctypes.c_int(0)
        if aad:
            assert L.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(pt) + 32)
        total = 0
        if pt:
            assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
            total = n.value
        assert L.EVP_EncryptFinal_ex(ctx, ctypes.byref(out, total), ctypes.byref(n)) == 1
        total += n.value
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1
        return out.raw[:total], tag.raw
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def open_(name: str, key: bytes, nonce: bytes, aad: bytes, ct: bytes, tag: bytes):
    """Returns plaintext bytes, or None when the tag does not verify."""
    L = lib()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        c = _cipher(name, len(key))
        assert L.EVP_DecryptInit_ex(ctx, c, None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, len(nonce), None) == 1
        assert L.EVP_DecryptInit_ex(ctx, None, None, key, nonce) == 1
        n = ctypes.c_int(0)
        if aad:
            assert L.EVP_DecryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(ct) + 32)
        total = 0
        if ct:
            assert L.EVP_DecryptUpdate(ctx, out, ctypes.byref(n), ct, len(ct)) == 1
            total = n.value
        tbuf = ctypes.create_string_buffer(bytes(tag), 16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, 16, tbuf) == 1
        ok = L.EVP_DecryptFinal_ex(ctx, ctypes.byref(out, total), ctypes.byref(n))
        if ok != 1:
            return None
        return out.raw[:total]
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def ccm_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes, tag_len: int, name: str = "ccm"):
    """AES-CCM (or ARIA-CCM, name="aria-ccm") through EVP (length-first call
    sequence of the CCM mode)."""
    L = lib()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(ctx, _cipher(name, len(key)), None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, len(nonce), None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, tag_len, None) == 1
        assert L.EVP_EncryptInit_ex(ctx, None, None, key, nonce) == 1
        n = ctypes.c_int(0)
        assert L.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), None, len(pt)) == 1
        if aad:
            assert L.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) == 1
        out = ctypes.create_string_buffer(len(pt) + 32)
        assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
        total = n.value
        assert L.EVP_EncryptFinal_ex(ctx, ctypes.byref(out, total), ctypes.byref(n)) == 1
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, tag_len, tag) == 1
        return out.raw[:total], tag.raw[:tag_len]
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def camellia(key: bytes, data: bytes, mode: str = "ecb", iv: bytes | None = None) -> bytes:
    """Camellia-ECB / -CBC (no padding) with OpenSSL, for whole blocks.  OpenSSL
    has no Camellia-GCM / -CCM; the tests build those modes around this."""
    L = lib()
    c = getattr(L, f"EVP_camellia_{len(key) * 8}_{mode}")()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(ctx, c, None, key, iv) == 1
        L.EVP_CIPHER_CTX_set_padding(ctx, 0)
        out = ctypes.create_string_buffer(len(data) + 16)
        n = ctypes.c_int(0)
        assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), data, len(data)) == 1
        return out.raw[:n.value]
    finally:
        L.EVP_CIPHER_CTX_free(ctx)
