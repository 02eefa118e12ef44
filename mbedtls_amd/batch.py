"""Device-resident batch API: per-connection key table in HBM and
protect/unprotect of many records with one launch (tlsrec_batch_*).

Buffers are plain device pointers; torch tensors (uint8 on a HIP device) are
accepted and their data_ptr / current stream are passed through.  torch is
plumbing only -- no torch op touches record bytes.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take a pointer of {type(x)}")


def _stream(stream):
    if stream is None:
        try:
            import torch
            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except Exception:
            pass
        return None
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return stream


def key_material(cipher: int, tls_version: int, key: bytes, iv: bytes, granularity: int = 0):
    """One tlsrec_key_material record (numpy structured scalar array of 1)."""
    km = np.zeros(1, dtype=_abi.KEY_MATERIAL)
    km["cipher"] = cipher
    km["tls_minor"] = 4 if tls_version == _abi.VERSION_TLS1_3 else 3
    fixed = 12 if (tls_version == _abi.VERSION_TLS1_3 or cipher == _abi.CIPHER_CHACHA20_POLY1305) else 4
    km["fixed_ivlen"] = fixed
    km["taglen"] = _abi.TAGLEN[cipher]
    km["granularity"] = granularity
    km["iv"][0, :fixed] = np.frombuffer(bytes(iv)[:fixed], dtype=np.uint8)
    km["key"][0, :len(key)] = np.frombuffer(bytes(key), dtype=np.uint8)
    return km


class KeyTable:
    """tlsrec_keytab: `capacity` key slots on the current HIP device."""

    def __init__(self, capacity: int):
        self._lib = _abi.load()
        h = ctypes.c_void_p()
        r = self._lib.tlsrec_keytab_create(ctypes.byref(h), capacity)
        if r != 0:
            raise RuntimeError(f"tlsrec_keytab_create failed: {r:#x}")
        self.handle = h
        self.capacity = capacity

    def load(self, keys, first: int = 0, stream=None):
        """keys: numpy array of KEY_MATERIAL (host) or a uint8 device tensor
        holding count*64 bytes (e.g. the result of an RCCL broadcast)."""
        if isinstance(keys, np.ndarray):
            keys = np.ascontiguousarray(keys, dtype=_abi.KEY_MATERIAL)
            count, on_dev, p = len(keys), 0, keys.ctypes.data
        else:
            count, on_dev, p = keys.numel() // 64, 1, keys.data_ptr()
        r = self._lib.tlsrec_keytab_load(self.handle, first, count, p, on_dev, _stream(stream))
        if r != 0:
            raise RuntimeError(f"tlsrec_keytab_load failed: {r:#x}")

    def set_cid(self, slot: int, cid: bytes, stream=None):
        """DTLS 1.2 connection ID of one slot (tlsrec_keytab_set_cid)."""
        r = self._lib.tlsrec_keytab_set_cid(self.handle, slot, bytes(cid), len(cid), _stream(stream))
        if r != 0:
            raise RuntimeError(f"tlsrec_keytab_set_cid failed: {r:#x}")

    def close(self):
        if self.handle is not None:
            self._lib.tlsrec_keytab_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _batch(name: str, kt: KeyTable, recs, res, n: int, in_arena, out_arena, lanes: int, stream,
           mean_bytes: int) -> None:
    """tlsrec_batch_<dir> (lanes: 0 = auto), or tlsrec_batch_<dir>_sized when
    the caller passes its mean record size (then lanes are auto)."""
    out_arena = in_arena if out_arena is None else out_arena
    lib = _abi.load()
    if mean_bytes:
        if lanes:
            raise ValueError("mean_bytes is a hint for the automatic lane choice: pass lanes=0")
        fn, arg = getattr(lib, name + "_sized"), mean_bytes
    else:
        fn, arg = getattr(lib, name), lanes
    r = fn(kt.handle, _ptr(recs), _ptr(res), n, _ptr(in_arena), _ptr(out_arena), arg, _stream(stream))
    if r != 0:
        raise RuntimeError(f"{name} failed: {r:#x}")


def batch_encrypt(kt: KeyTable, recs, res, n: int, in_arena, out_arena=None, lanes: int = 0,
                  stream=None, mean_bytes: int = 0) -> None:
    _batch("tlsrec_batch_encrypt", kt, recs, res, n, in_arena, out_arena, lanes, stream, mean_bytes)


def batch_decrypt(kt: KeyTable, recs, res, n: int, in_arena, out_arena=None, lanes: int = 0,
                  stream=None, mean_bytes: int = 0) -> None:
    _batch("tlsrec_batch_decrypt", kt, recs, res, n, in_arena, out_arena, lanes, stream, mean_bytes)


def host_batch(decrypt: bool, kt: KeyTable, recs, res, n: int, in_arena, out_arena=None, lanes: int = 0,
               chunk_bytes: int = 0) -> None:
    """tlsrec_host_batch_encrypt / _decrypt: descriptors, results and arenas
    in HOST memory (numpy arrays or pinned CPU tensors); synchronous."""
    out_arena = in_arena if out_arena is None else out_arena
    fn = _abi.load().tlsrec_host_batch_decrypt if decrypt else _abi.load().tlsrec_host_batch_encrypt
    r = fn(kt.handle, _ptr(recs), _ptr(res), n, _ptr(in_arena), _ptr(out_arena), lanes, chunk_bytes)
    if r != 0:
        raise RuntimeError(f"tlsrec_host_batch_{'decrypt' if decrypt else 'encrypt'} failed: {r:#x}")


def frame_check(decrypt: bool, km, rec):
    """Host-only framing verdict for one record (tlsrec_frame_check)."""
    km = np.ascontiguousarray(km, dtype=_abi.KEY_MATERIAL)
    rec = np.ascontiguousarray(rec, dtype=_abi.BATCH_REC)
    early = np.zeros(1, dtype=_abi.BATCH_RES)
    pos = ctypes.c_uint32()
    ln = ctypes.c_uint32()
    go = _abi.load().tlsrec_frame_check(int(decrypt), km.ctypes.data, rec.ctypes.data,
                                        early.ctypes.data, ctypes.byref(pos), ctypes.byref(ln))
    return bool(go), early[0], pos.value, ln.value


def records(n: int) -> np.ndarray:
    return np.zeros(n, dtype=_abi.BATCH_REC)


def results(n: int) -> np.ndarray:
    return np.zeros(n, dtype=_abi.BATCH_RES)


def seq_bytes(seq: np.ndarray) -> np.ndarray:
    """uint64 sequence numbers -> (n, 8) big-endian bytes (rec->ctr)."""
    return seq.astype(">u8").view(np.uint8).reshape(-1, 8)
