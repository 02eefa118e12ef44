"""DTLS 1.2 datagram record layer on the GPU (tlsrec_dtls_decrypt / _encrypt):
received datagrams split at their DTLS record headers, decrypted in place and
passed through ssl_get_next_record's datagram rules (epoch, anti-replay
window, dropped datagrams, badmac_limit) per connection; application data
written as one record per datagram.  Arrays are device buffers (torch
tensors); numpy structured arrays are accepted for the per-connection and
per-datagram descriptors and copied to the device.
"""
from __future__ import annotations

import ctypes

from . import _abi
from .batch import KeyTable, _ptr, _stream
from .stream import StreamError, _dev

DGRAM, DTLS_IN, DTLS_IN_RES = _abi.DGRAM, _abi.DTLS_IN, _abi.DTLS_IN_RES


def out_size(cipher: int, granularity: int, cid_len: int, in_len: int, max_frag: int = 0) -> int:
    return int(_abi.load().tlsrec_dtls_out_size(cipher, granularity, cid_len, in_len, max_frag))


def decrypt(kt: KeyTable, conns, n: int, dgrams, ndgrams: int, arena, recs, res, disp, max_records: int, cres,
            stream=None) -> int:
    """Returns the number of records listed; per-connection results land in
    `cres` (DTLS_IN_RES), per-record ones in `recs` / `res` / `disp` (int32)."""
    dev = arena.device if hasattr(arena, "device") else None
    conns, dgrams = _dev(conns, dev), _dev(dgrams, dev)
    total = ctypes.c_uint32()
    r = _abi.load().tlsrec_dtls_decrypt(kt.handle, _ptr(conns), n, _ptr(dgrams), ndgrams, _ptr(arena), _ptr(recs),
                                        _ptr(res), _ptr(disp), max_records, _ptr(cres), ctypes.byref(total),
                                        _stream(stream))
    if r != 0:
        raise StreamError("tlsrec_dtls_decrypt", r)
    return total.value


def encrypt(kt: KeyTable, streams, n: int, in_arena, out_arena, recs, res, max_records: int, sres,
            stream=None) -> int:
    dev = out_arena.device if hasattr(out_arena, "device") else None
    streams = _dev(streams, dev)
    total = ctypes.c_uint32()
    r = _abi.load().tlsrec_dtls_encrypt(kt.handle, _ptr(streams), n, _ptr(in_arena), _ptr(out_arena), _ptr(recs),
                                        _ptr(res), max_records, _ptr(sres), ctypes.byref(total), _stream(stream))
    if r != 0:
        raise StreamError("tlsrec_dtls_encrypt", r)
    return total.value
