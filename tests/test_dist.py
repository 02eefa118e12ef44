"""Multi-rank sharding on CPU (gloo, world_size 2): the key table reaches
every rank from rank 0, the record shards cover the batch exactly once, and
per-rank processing of the shards reproduces the single-process results
record for record.  The per-rank compute here is the oracle (CPU-only test
box); on GPUs bench.py runs the same shard/broadcast path with the batch
kernels over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import mbedtls_amd as M
from tests import batchlib as B


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch():
    slots = B.random_slots(4242, [M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305],
                           [M.VERSION_TLS1_2, M.VERSION_TLS1_3], 6)
    lengths = [0, 1, 15, 16, 17, 100, 1000, 1400, 4096] + [37 * i for i in range(28)]
    return slots, B.sealed_records(slots, lengths, seed=77)[0]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        slots, recs = _batch()
        full = B.Batch(slots, recs)
        km = full.key_materials() if rank == 0 else np.zeros(len(slots), dtype=M.KEY_MATERIAL)
        keys = M.broadcast_keys(km, "cpu")
        got_km = keys.numpy().view(M.KEY_MATERIAL)
        sh = M.shard_bounds(len(recs), rank, world)
        part = B.Batch(slots, recs[sh.start:sh.stop])
        outs, stats = part.run_oracle(True)
        res = np.zeros(len(stats), dtype=M.BATCH_RES)
        res["status"] = stats
        totals = M.reduce_status(res)
        q.put((rank, sh.start, sh.count, got_km.tobytes(), [o.data() for o in outs], stats, totals.tolist()))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_match_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got.sort()
    slots, recs = _batch()
    ref_outs, ref_stats = B.Batch(slots, recs).run_oracle(True)
    ref_km = B.Batch(slots, recs).key_materials().tobytes()
    covered = []
    for rank, start, count, km, datas, stats, totals in got:
        assert km == ref_km, f"rank {rank} key table differs from rank 0's"
        covered += list(range(start, start + count))
        assert datas == [o.data() for o in ref_outs[start:start + count]]
        assert stats == ref_stats[start:start + count]
        assert totals[0] == len(recs) and totals[1] == sum(s == 0 for s in ref_stats)
    assert covered == list(range(len(recs)))


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 3), (1 << 20, 8), (37, 8)])
def test_shard_bounds_partition(n, world):
    shards = [M.shard_bounds(n, r, world) for r in range(world)]
    assert shards[0].start == 0 and shards[-1].stop == n
    for a, b in zip(shards, shards[1:]):
        assert a.stop == b.start
    counts = [s.count for s in shards]
    assert max(counts) - min(counts) <= 1
    with pytest.raises(ValueError):
        M.shard_bounds(n, world, world)
