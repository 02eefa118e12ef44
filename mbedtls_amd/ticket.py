"""Session tickets on the GPU (tlsrec_ticket_write / _parse): the
mbedtls_ssl_ticket_write / mbedtls_ssl_ticket_parse AEAD protection of
library/ssl_ticket.c for a batch of tickets in device memory."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _abi
from .batch import KeyTable, _ptr, _stream

TICKET, TICKET_RES = _abi.TICKET, _abi.TICKET_RES
MIN_LEN = 34


def ticket_keys(slots, names, active: int) -> _abi.CTicketKeys:
    k = _abi.CTicketKeys()
    for i in range(2):
        k.slot[i] = slots[i]
        k.name[i][:] = list(bytes(names[i]))
    k.active = active
    return k


def _run(fn, kt: KeyTable, keys, tickets, n: int, arena, res, stream):
    if isinstance(tickets, np.ndarray):
        import torch
        tickets = torch.from_numpy(np.ascontiguousarray(tickets).view(np.uint8).reshape(-1).copy()).to(arena.device)
    r = getattr(_abi.load(), fn)(kt.handle, ctypes.byref(keys), _ptr(tickets), n, _ptr(arena), _ptr(res),
                                 _stream(stream))
    if r != 0:
        raise RuntimeError(f"{fn} failed: {r}")


def write(kt, keys, tickets, n, arena, res, stream=None):
    _run("tlsrec_ticket_write", kt, keys, tickets, n, arena, res, stream)


def parse(kt, keys, tickets, n, arena, res, stream=None):
    _run("tlsrec_ticket_parse", kt, keys, tickets, n, arena, res, stream)
