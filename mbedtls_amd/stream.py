"""TLS record streams on the GPU (tlsrec_stream_decrypt / _encrypt): whole
connections' received bytes split at their record headers and decrypted in
place, or application data framed into records and encrypted -- the
ssl_get_next_record / mbedtls_ssl_write_record loops of library/ssl_msg.c
over many connections at once.  Arrays are device buffers (torch tensors);
numpy structured arrays are accepted for the per-connection descriptors and
copied to the device.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi
from .batch import KeyTable, _ptr, _stream

STREAM_IN, STREAM_IN_RES = _abi.STREAM_IN, _abi.STREAM_IN_RES
STREAM_OUT, STREAM_OUT_RES = _abi.STREAM_OUT, _abi.STREAM_OUT_RES
STREAM_READ_REQ, STREAM_READ_RES = _abi.STREAM_READ_REQ, _abi.STREAM_READ_RES


class StreamError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed: {code}")
        self.code = code


def _dev(x, device):
    if isinstance(x, np.ndarray):
        import torch
        return torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1).copy()).to(device)
    return x


def out_size(tls_version: int, cipher: int, granularity: int, in_len: int, max_frag: int = 0) -> int:
    return int(_abi.load().tlsrec_stream_out_size(tls_version, cipher, granularity, in_len, max_frag))


def decrypt(kt: KeyTable, streams, n: int, arena, recs, res, max_records: int, sres, stream=None) -> int:
    """Returns the number of records framed; per-connection results land in
    `sres` (STREAM_IN_RES), per-record ones in `recs` / `res`."""
    dev = arena.device if hasattr(arena, "device") else None
    streams = _dev(streams, dev)
    total = ctypes.c_uint32()
    r = _abi.load().tlsrec_stream_decrypt(kt.handle, _ptr(streams), n, _ptr(arena), _ptr(recs), _ptr(res),
                                          max_records, _ptr(sres), ctypes.byref(total), _stream(stream))
    if r != 0:
        raise StreamError("tlsrec_stream_decrypt", r)
    return total.value


def encrypt(kt: KeyTable, streams, n: int, in_arena, out_arena, recs, res, max_records: int, sres,
            stream=None) -> int:
    dev = out_arena.device if hasattr(out_arena, "device") else None
    streams = _dev(streams, dev)
    total = ctypes.c_uint32()
    r = _abi.load().tlsrec_stream_encrypt(kt.handle, _ptr(streams), n, _ptr(in_arena), _ptr(out_arena), _ptr(recs),
                                          _ptr(res), max_records, _ptr(sres), ctypes.byref(total), _stream(stream))
    if r != 0:
        raise StreamError("tlsrec_stream_encrypt", r)
    return total.value


def read(sres, n: int, recs, res, arena, req, out_arena, rres, stream=None) -> None:
    """ssl_read_application_data over the accepted records of each connection
    (tlsrec_stream_read): application data gathered into the callers'
    buffers, the plaintext handed out zeroized in the arena."""
    dev = arena.device if hasattr(arena, "device") else None
    req = _dev(req, dev)
    r = _abi.load().tlsrec_stream_read(_ptr(sres), n, _ptr(recs), _ptr(res), _ptr(arena), _ptr(req),
                                       _ptr(out_arena), _ptr(rres), _stream(stream))
    if r != 0:
        raise StreamError("tlsrec_stream_read", r)
