"""Multi-GPU sharding of a record batch: one process per GPU, no data-path
collective.

TLS records are independent AEAD units: a batch is
split into contiguous record ranges, one per rank, and every rank runs the
batch kernels on its own range against its own copy of the key table.  The
only collective is the key-table broadcast from rank 0 when the table is
(re)loaded -- 64 B of key material per slot over RCCL/xGMI (gloo on CPU) --
plus an optional all-reduce of per-rank status counts for the control
plane.  Record bytes never cross GPUs.

Nothing here computes: the caller passes the shard to
:func:`mbedtls_amd.batch_encrypt` / :func:`mbedtls_amd.batch_decrypt`.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._abi import KEY_MATERIAL


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    start: int      # first record of this rank's range
    count: int      # records in the range

    @property
    def stop(self) -> int:
        return self.start + self.count


def shard_bounds(n_records: int, rank: int, world: int) -> Shard:
    """Balanced contiguous split: the first n % world ranks take one extra
    record, so ranks differ by at most one record and every record has
    exactly one owner."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    if n_records < 0:
        raise ValueError("negative record count")
    base, extra = divmod(n_records, world)
    start = rank * base + min(rank, extra)
    return Shard(rank, world, start, base + (1 if rank < extra else 0))


def broadcast_keys(key_material, device, src: int = 0, group=None):
    """Return rank `src`'s key-material array on every rank, as a uint8
    tensor on `device` (a CUDA device for RCCL, CPU for gloo), ready for
    :meth:`mbedtls_amd.KeyTable.load`.  Non-source ranks pass an array of the
    same shape (its contents are ignored)."""
    import torch
    import torch.distributed as dist

    km = np.ascontiguousarray(key_material)
    if km.dtype != KEY_MATERIAL:
        raise TypeError("key_material must have dtype KEY_MATERIAL")
    t = torch.from_numpy(km.view(np.uint8).copy()).to(device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(t, src=src, group=group)
    return t


def status_counts(results) -> np.ndarray:
    """[records, ok, INVALID_MAC, other errors] of one rank's result array."""
    st = np.asarray(results["status"])
    ok = int((st == 0).sum())
    from ._abi import ERR_SSL_INVALID_MAC
    bad_mac = int((st == ERR_SSL_INVALID_MAC).sum())
    return np.array([st.size, ok, bad_mac, st.size - ok - bad_mac], dtype=np.int64)


def reduce_status(results, device="cpu", group=None) -> np.ndarray:
    """Sum of :func:`status_counts` over all ranks (control plane only)."""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(status_counts(results)).to(device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
    return t.cpu().numpy()
