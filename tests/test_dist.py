"""Multi-rank sharding on CPU (gloo, world_size 2): the key table reaches
every rank from rank 0, the record shards cover the batch exactly once, and
per-rank processing of the shards reproduces the single-process results
record for record.  Each rank runs the product's own host code on its shard
-- tlsrec_shard_bounds and tlsrec_frame_check (the framing verdict of
encrypt_buf / decrypt_buf, libtlsrec.so, no GPU needed) -- and the oracle as
the AEAD stand-in of this CPU-only box; on GPUs bench.py and
tests/c/mgpu_shard.c run the same shard/broadcast sequence with the batch
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
        import ctypes
        from mbedtls_amd import _abi
        cs, cc = ctypes.c_uint64(), ctypes.c_uint64()
        assert _abi.load().tlsrec_shard_bounds(len(recs), rank, world, ctypes.byref(cs), ctypes.byref(cc)) == 0
        assert (cs.value, cc.value) == (sh.start, sh.count)
        part = B.Batch(slots, recs[sh.start:sh.stop])
        frames = []
        for d in part.desc:
            go, early, pos, ln = M.frame_check(True, got_km[d["slot"]], d)
            frames.append((go, int(early["status"]), pos, ln))
        outs, stats = part.run_oracle(True)
        res = np.zeros(len(stats), dtype=M.BATCH_RES)
        res["status"] = stats
        totals = M.reduce_status(res)
        q.put((rank, sh.start, sh.count, got_km.tobytes(), [o.data() for o in outs], stats, totals.tolist(), frames))
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
    full = B.Batch(slots, recs)
    ref_km = full.key_materials().tobytes()
    kms = full.key_materials()
    ref_frames = []
    for d in full.desc:
        go, early, pos, ln = M.frame_check(True, kms[d["slot"]], d)
        ref_frames.append((go, int(early["status"]), pos, ln))
    covered = []
    for rank, start, count, km, datas, stats, totals, frames in got:
        assert km == ref_km, f"rank {rank} key table differs from rank 0's"
        assert frames == ref_frames[start:start + count]
        # the framing verdict agrees with the oracle's outcome: a record the
        # framing stops never reaches the AEAD
        for (go, st, _, _), ost in zip(frames, stats):
            assert go or ost == st
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


@pytest.mark.parametrize("n,world", [(0, 1), (5, 2), (1000, 3), (1 << 23, 8), (37, 8), (3, 16)])
def test_c_shard_bounds_matches_python(n, world):
    """tlsrec_shard_bounds (the C hosts' shard split, tlsrec_host.c) equals
    mbedtls_amd.shard_bounds for every rank, and rejects bad ranks."""
    import ctypes
    from mbedtls_amd import _abi
    lib = _abi.load()
    for r in range(world):
        s, c = ctypes.c_uint64(), ctypes.c_uint64()
        assert lib.tlsrec_shard_bounds(n, r, world, ctypes.byref(s), ctypes.byref(c)) == 0
        sh = M.shard_bounds(n, r, world)
        assert (s.value, c.value) == (sh.start, sh.count)
    s, c = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.tlsrec_shard_bounds(n, world, world, ctypes.byref(s), ctypes.byref(c)) == M.ERR_SSL_BAD_INPUT_DATA
    assert lib.tlsrec_shard_bounds(n, 0, 0, ctypes.byref(s), ctypes.byref(c)) == M.ERR_SSL_BAD_INPUT_DATA


def _evidence_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        km = np.zeros(5, dtype=M.KEY_MATERIAL)
        if rank == 0:
            km["cipher"] = M.CIPHER_AES_256_GCM
            km["key"] = np.arange(5 * 32, dtype=np.uint8).reshape(5, 32)
        keys = M.broadcast_keys(km, "cpu")
        q.put((rank, bench.rank_evidence(dist, keys, "cpu", rank)))
    finally:
        dist.destroy_process_group()


def test_bench_rank_evidence_two_ranks():
    """bench.py's record of what the process group formed (the driver's SCALE
    run checks it): world size and backend as torch.distributed reports them,
    every rank, and the key-table digest all-gathered and equal on all ranks."""
    import hashlib
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_evidence_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    km = np.zeros(5, dtype=M.KEY_MATERIAL)
    km["cipher"] = M.CIPHER_AES_256_GCM
    km["key"] = np.arange(5 * 32, dtype=np.uint8).reshape(5, 32)
    want = hashlib.sha256(km.tobytes()).hexdigest()
    for rank, ev in got:
        assert ev["world_size"] == 2 and ev["backend"] == "gloo"
        assert [r["rank"] for r in ev["ranks"]] == [0, 1]
        assert ev["key_table_equal_on_all_ranks"] and ev["key_table_sha256"] == want
