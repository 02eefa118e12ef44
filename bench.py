#!/usr/bin/env python3
"""bench.py -- device-resident TLS record AEAD throughput on MI355X.

Default workload = BASELINE.json configs[1]: TLS 1.3 AES-256-GCM *decrypt* of
2^20 records x 16 KiB (16383 B content + 1 B type = 16384 B inner plaintext,
16400 B ciphertext+tag) under one key, inputs resident in HBM.  One step = one
tlsrec_batch_decrypt call over the whole batch (one kernel launch).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]

Multi-GPU: `python bench.py --gpus N` starts N rank processes itself (one per
GPU, before any GPU call in the parent; launch_ranks), or runs as one rank of
an external `torch.distributed.run ... bench.py --gpus N`.  Either way every
rank checks that the process group really has N ranks.  Records shard by
contiguous range (2^20 per rank, weak scaling: BASELINE configs[4] = 8 M x
16 KiB over 8 GPUs at N = 8); the only collective is the RCCL broadcast of the
key table from rank 0 (plus the max-time reduction).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "TLS records/sec + GiB/s AEAD throughput (device-resident), 16 KiB records"
HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md)
SEED = 0x7115EC0DE

CONFIGS = {
    # name: (cipher, tls, direction, content bytes, records, keys, workload text)
    "c1": ("AES-128-GCM", "TLS1.2", "encrypt", 1400, 1024, 1,
           "AES-128-GCM encrypt, 1024 x 1.4 KiB TLS 1.2 records, single key (plumbing check; the CPU leg is the reference-path restatement)"),
    "c2": ("AES-256-GCM", "TLS1.3", "decrypt", 16383, 1 << 20, 1,
           "AES-256-GCM decrypt, 1M x 16 KiB TLS 1.3 application-data records, single key"),
    "c3": ("CHACHA20-POLY1305", "TLS1.3", "encrypt", 1400, 1 << 20, 1,
           "ChaCha20-Poly1305 encrypt, 1M x 1.4 KiB TLS 1.3 records, single key"),
    "c4": ("MIX", "TLS1.3", "decrypt", 16383, 1 << 22, 1 << 16,
           "64K keys x 64 records, AES-256-GCM (even keys) + ChaCha20-Poly1305 (odd keys), records round-robin over keys, 16 KiB TLS 1.3 decrypt"),
    # SURVEY 8(f)-2 rows, same shape as c2 (not BASELINE configs)
    "ccm": ("AES-128-CCM", "TLS1.3", "decrypt", 16383, 1 << 20, 1,
            "AES-128-CCM decrypt, 1M x 16 KiB TLS 1.3 records, single key (8(f)-2)"),
    "ccm8": ("AES-128-CCM-8", "TLS1.3", "decrypt", 16383, 1 << 20, 1,
             "AES-128-CCM_8 decrypt, 1M x 16 KiB TLS 1.3 records, single key (8(f)-2)"),
    "ccme": ("AES-128-CCM", "TLS1.3", "encrypt", 16383, 1 << 20, 1,
             "AES-128-CCM encrypt, 1M x 16 KiB TLS 1.3 records, single key (8(f)-2, ccm sent)"),
    "gcm192": ("AES-192-GCM", "TLS1.3", "decrypt", 16383, 1 << 20, 1,
               "AES-192-GCM decrypt, 1M x 16 KiB TLS 1.3 records, single key (8(f)-2)"),
    "aria256": ("ARIA-256-GCM", "TLS1.2", "decrypt", 16384, 1 << 20, 1,
                "ARIA-256-GCM decrypt, 1M x 16 KiB TLS 1.2 records, single key (8(f)-2)"),
    "camellia128": ("CAMELLIA-128-GCM", "TLS1.2", "decrypt", 16384, 1 << 20, 1,
                    "Camellia-128-GCM decrypt, 1M x 16 KiB TLS 1.2 records, single key (8(f)-2)"),
    "k4": ("AES-256-GCM", "TLS1.3", "decrypt", 16383, 1 << 18, 1 << 16,
           "64K keys x 4 records, AES-256-GCM, records round-robin over keys, 16 KiB TLS 1.3 decrypt (few records per key)"),
    "k4e": ("AES-256-GCM", "TLS1.3", "encrypt", 16383, 1 << 18, 1 << 16,
            "64K keys x 4 records, AES-256-GCM, records round-robin over keys, 16 KiB TLS 1.3 encrypt (k4 sent)"),
    "chacha16k": ("CHACHA20-POLY1305", "TLS1.3", "decrypt", 16383, 1 << 20, 1,
                  "ChaCha20-Poly1305 decrypt, 1M x 16 KiB TLS 1.3 records, single key (the c4 ChaCha share)"),
    "c3d": ("CHACHA20-POLY1305", "TLS1.3", "decrypt", 1400, 1 << 20, 1,
            "ChaCha20-Poly1305 decrypt, 1M x 1.4 KiB TLS 1.3 records, single key (c3 received)"),
    "chacha16ke": ("CHACHA20-POLY1305", "TLS1.3", "encrypt", 16383, 1 << 20, 1,
                   "ChaCha20-Poly1305 encrypt, 1M x 16 KiB TLS 1.3 records, single key (chacha16k sent)"),
    "c2s": ("AES-256-GCM", "TLS1.3", "decrypt", 1400, 1 << 20, 1,
            "AES-256-GCM decrypt, 1M x 1.4 KiB TLS 1.3 records, single key (the GCM half of c4s without the key passes)"),
    "c2se": ("AES-256-GCM", "TLS1.3", "encrypt", 1400, 1 << 20, 1,
             "AES-256-GCM encrypt, 1M x 1.4 KiB TLS 1.3 records, single key (c2s sent)"),
    "c4s": ("MIX", "TLS1.3", "decrypt", 1400, 1 << 22, 1 << 16,
            "64K keys x 64 records, AES-256-GCM (even keys) + ChaCha20-Poly1305 (odd keys), records round-robin over keys, 1.4 KiB TLS 1.3 decrypt"),
}


KERNEL_OF = {"CHACHA20-POLY1305": "tlsrec_chachapoly_kernel", "AES-128-CCM": "tlsrec_ccm_kernel",
             "AES-128-CCM-8": "tlsrec_ccm_kernel", "MIX": "tlsrec_gcm_kernel + tlsrec_chachapoly_kernel"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="c2 (default) = the metric's workload; c1/c3/c4/c4s = the other BASELINE configs")
    ap.add_argument("--records", type=int, default=0, help="override records per GPU")
    ap.add_argument("--keys", type=int, default=0, help="override the config's key count (records round-robin over keys)")
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--align", type=int, default=128, help="record slot alignment in the arena (bytes; 128 = HBM/L2 line)")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall-time target of the CPU sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (pinned H2D/D2H) leg")
    ap.add_argument("--dist", action="store_true",
                    help="use the process group even at WORLD_SIZE=1 (rehearses the RCCL path on one GPU)")
    ap.add_argument("--e2e-records", type=int, default=0, help="records of the end-to-end leg (0 = ~2 GiB worth)")
    ap.add_argument("--verify", type=int, default=64, help="records spot-checked against the oracle")
    ap.add_argument("--key-order", choices=["round-robin", "contiguous"], default="round-robin",
                    help="record i under key i %% keys (default, SURVEY 8(d)-4) or i // (records / keys) "
                         "(diagnostic: a key's descriptors adjacent in memory)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def rank_env(base, rank, world, port):
    """The environment of rank `rank` of a `world`-rank job on this node (the
    variables torch.distributed.run would set)."""
    e = dict(base)
    e.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
             GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return e


def count_gpus(nodes="/sys/class/kfd/kfd/topology/nodes", dri="/dev/dri", env=None):
    """GPUs this process can open, counted without a HIP call or torch (the
    launcher parent must not touch the GPU before it starts the ranks): KFD
    topology nodes with SIMDs (CPU nodes have none) whose DRM render node this
    process may open -- a container sees every node of the host in sysfs but
    only its own render nodes -- capped by the ROCR / HIP / CUDA
    *_VISIBLE_DEVICES lists when set."""
    env = os.environ if env is None else env
    n = 0
    try:
        names = sorted(os.listdir(nodes))
    except OSError:
        names = []
    for name in names:
        props = {}
        try:
            with open(os.path.join(nodes, name, "properties")) as f:
                for line in f:
                    kv = line.split()
                    if len(kv) == 2:
                        props[kv[0]] = kv[1]
        except OSError:
            continue
        try:
            simds, minor = int(props.get("simd_count", "0")), int(props.get("drm_render_minor", "-1"))
        except ValueError:
            continue
        if simds > 0 and minor >= 0 and os.access(os.path.join(dri, f"renderD{minor}"), os.R_OK | os.W_OK):
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(world, argv, script=None, env=None, poll_s=0.2):
    """Start `world` rank processes of `script` (this file) with `argv` and
    wait for them.  Children, never an exec: the parent has made no GPU call.
    Rank 0's JSON line reaches stdout directly (the children inherit it).  The
    first rank that fails ends the others (by their own PIDs) and its exit
    code is returned; a signal to the parent is passed on to the ranks."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = script or os.path.abspath(__file__)
    base = dict(os.environ if env is None else env)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=rank_env(base, r, world, port))
             for r in range(world)]

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = {sig: signal.signal(sig, lambda s, f: (stop(), sys.exit(128 + s))) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    log(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the other ranks")
                    stop()
            if live:
                time.sleep(poll_s)
    finally:
        stop()
        for p in procs:
            p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)
    return rc


def inner_len(content, tls):
    if tls == "TLS1.3":
        return content + 1 + (16 - (content + 1) % 16) % 16
    return content


ROOFLINE_SCOPE = ("per GPU: achieved / frac / kernel_ms_avg are rank 0's kernel; per_rank lists every rank's, "
                  "frac_min_over_ranks the slowest GPU's")


def rank_timing(dist, wall, kern_ms, dev):
    """The step wall time as the max over ranks, and every rank's average
    kernel time (HIP events on its own launch stream), all-gathered so that
    rank 0's line carries them.  dist None: one process."""
    import torch
    avg = float(np.mean(kern_ms)) if len(kern_ms) else 0.0
    if dist is None:
        return wall, [avg]
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    mine = torch.tensor([avg], dtype=torch.float64, device=dev)
    allk = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(allk, mine)
    return float(t.item()), [float(x.item()) for x in allk]


def per_rank_roofline(kern_ms_ranks, alg_bytes_per_launch):
    """Each rank's achieved GB/s and fraction of the HBM peak from its own
    average kernel time, plus the minimum fraction (the slowest GPU)."""
    rows = []
    for r, ms in enumerate(kern_ms_ranks):
        ach = alg_bytes_per_launch / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        rows.append({"rank": r, "kernel_ms_avg": round(ms, 4), "achieved": round(ach, 2),
                     "frac": round(ach / HBM_PEAK_GBS, 4)})
    return {"per_rank": rows, "frac_min": min(x["frac"] for x in rows) if rows else None,
            "kernel_ms_max": max(x["kernel_ms_avg"] for x in rows) if rows else None}


def rank0_legs(dist, rank, run_cpu, run_e2e):
    """The CPU baseline and the host-buffer (e2e) legs, on rank 0 at every
    world size, outside the timed region: all ranks meet at a barrier, rank 0
    runs the legs while the others wait at a second one (so the legs share
    the box with idle GPUs only).  run_* None: the leg is switched off."""
    if dist is not None:
        dist.barrier()
    cpu = e2e = None
    try:
        if rank == 0:
            cpu = run_cpu() if run_cpu else None
            e2e = run_e2e() if run_e2e else None
    finally:
        if dist is not None:
            dist.barrier()
    return cpu, e2e


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # this process is the launcher: count the devices without any HIP call
        # (nor torch) and start one rank per GPU
        have = count_gpus()
        if have < args.gpus:
            log(f"bench.py: --gpus {args.gpus} needs {args.gpus} HIP devices, {have} visible; "
                f"refusing to report a {have}-GPU run as {args.gpus} GPUs")
            sys.exit(2)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    import torch
    import torch.distributed as dist
    import mbedtls_amd as M

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"bench.py: WORLD_SIZE {world} but --gpus {args.gpus}")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.dist
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)

    cname, tls, direction, content, n_default, nkeys, workload = CONFIGS[args.config]
    n = args.records or n_default
    nkeys = args.keys or nkeys
    ver = M.VERSION_TLS1_3 if tls == "TLS1.3" else M.VERSION_TLS1_2
    inner = inner_len(content, tls)
    head = 8 if tls == "TLS1.2" and cname != "CHACHA20-POLY1305" else 0   # TLS 1.2 GCM explicit nonce
    taglen = 8 if cname.endswith("CCM-8") else 16
    wire = head + inner + taglen
    # TLS 1.2 GCM/CCM records carry an 8-byte explicit IV ahead of the
    # ciphertext: the record buffer starts `lead` bytes into its slot so that
    # the AEAD region, which the kernels stream, is line-aligned
    lead = (args.align - head % args.align) % args.align if head else 0
    stride = (lead + wire + args.align - 1) // args.align * args.align
    ciphers = {"AES-128-GCM": [M.CIPHER_AES_128_GCM], "AES-256-GCM": [M.CIPHER_AES_256_GCM],
               "AES-128-CCM": [M.CIPHER_AES_128_CCM], "AES-128-CCM-8": [M.CIPHER_AES_128_CCM_8],
               "AES-192-GCM": [M.CIPHER_AES_192_GCM], "CHACHA20-POLY1305": [M.CIPHER_CHACHA20_POLY1305],
               "ARIA-256-GCM": [M.CIPHER_ARIA_256_GCM], "CAMELLIA-128-GCM": [M.CIPHER_CAMELLIA_128_GCM],
               "MIX": [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305]}[cname]
    nkeys = min(nkeys, n)

    # ---- key table: generated on rank 0, broadcast over RCCL (xGMI) -------------
    from tests.prng import prng_array
    km = np.zeros(nkeys, dtype=M.KEY_MATERIAL)
    if rank == 0:
        raw = prng_array(SEED, nkeys * 48).reshape(nkeys, 48)
        km["cipher"] = np.array([ciphers[i % len(ciphers)] for i in range(nkeys)], dtype=np.uint8)
        km["tls_minor"] = 4 if ver == M.VERSION_TLS1_3 else 3
        km["fixed_ivlen"] = 4 if head else 12
        km["taglen"] = [M.TAGLEN[c] for c in km["cipher"]]
        km["key"] = raw[:, :32]
        km["iv"][:, :12] = raw[:, 32:44]
    keys_dev = M.broadcast_keys(km, dev)          # RCCL broadcast when world > 1
    kt = M.KeyTable(nkeys)
    kt.load(keys_dev)
    dist_info = None
    if distributed:
        dist_info = rank_evidence(dist, keys_dev, dev, local)

    # ---- synthetic records (this rank's shard) ---------------------------------
    # weak scaling: a global stream of n x world records, one contiguous range
    # per rank (mbedtls_amd.shard); record bytes never leave their GPU
    sh = M.shard_bounds(n * world, rank, world)
    assert sh.count == n
    shard0 = sh.start
    arena = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev)
    recs = M.records(n)
    recs["buf_off"] = np.arange(n, dtype=np.uint64) * stride + lead
    recs["buf_len"] = stride - lead
    recs["data_offset"] = head
    recs["data_len"] = content
    # records round-robin over keys: neighbours never share a
    # key; the engine's bucket pass groups them by key on the device
    if args.key_order == "contiguous":
        recs["slot"] = (np.arange(n, dtype=np.uint64) * nkeys // n).astype(np.uint32)
    else:
        recs["slot"] = (np.arange(n, dtype=np.uint64) % nkeys).astype(np.uint32)
    seq = np.arange(shard0, shard0 + n, dtype=np.uint64)
    recs["ctr"] = M.seq_bytes(seq)
    recs["type"] = 23
    recs["ver"] = (3, 3)
    recs_dev = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    res_dev = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    sample = list(range(0, n, max(1, n // max(1, args.verify))))[:args.verify]
    pt_sample = {i: arena[i * stride + lead + head:i * stride + lead + head + content].cpu().numpy().copy()
                 for i in sample}

    # the caller's record size as the launch hint of tlsrec_batch_*_sized
    # (lanes auto); an explicit --lanes takes the unhinted call
    hint = 0 if args.lanes else wire
    if direction == "decrypt":
        # produce the ciphertexts with the (separately verified) encrypt kernel
        M.batch_encrypt(kt, recs_dev, res_dev, n, arena, arena, lanes=args.lanes, mean_bytes=hint)
        torch.cuda.synchronize()
        enc_status = res_dev.view(torch.int32)[0::4]
        assert int((enc_status != 0).sum()) == 0, "encrypt of the synthetic batch failed"
        dec = recs.copy()
        dec["data_offset"] = 0
        dec["data_len"] = wire
        in_recs = torch.from_numpy(dec.view(np.uint8).copy()).to(dev)
        in_arena, out_arena = arena, torch.empty_like(arena)
        run = lambda: M.batch_decrypt(kt, in_recs, res_dev, n, in_arena, out_arena, lanes=args.lanes,  # noqa: E731
                                      mean_bytes=hint)
    else:
        in_recs = recs_dev
        in_arena, out_arena = arena, torch.empty_like(arena)
        run = lambda: M.batch_encrypt(kt, in_recs, res_dev, n, in_arena, out_arena, lanes=args.lanes,  # noqa: E731
                                      mean_bytes=hint)

    # ---- warmup, then K timed steps -----------------------------------------
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        run()
        b.record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    wall, kern_ranks = rank_timing(dist if distributed else None, wall, kern_ms, dev)

    # ---- correctness of what was timed ----------------------------------------
    st = res_dev.view(torch.int32)[0::4]
    bad = int((st != 0).sum())
    lens = res_dev.view(torch.int32)[2::4]
    if direction == "decrypt":
        bad += int((lens != content).sum())
        for i in sample:
            got = out_arena[i * stride + lead + head:i * stride + lead + head + content].cpu().numpy()
            bad += int(not np.array_equal(got, pt_sample[i]))
    bad_t = torch.tensor([bad], dtype=torch.int64, device=dev)
    if distributed:
        dist.all_reduce(bad_t)
    bad = int(bad_t.item())

    # oracle spot check of the bytes (rank 0, sample): the ciphertext the
    # GPU produced must equal the CPU restatement's for the same inputs
    oracle_ok = None
    if rank == 0 and args.verify:
        import oracle as O
        oc = {c: c for c in M.KEYLEN}      # the oracle shares the cipher ids
        oracle_ok = True
        src = arena if direction == "decrypt" else out_arena
        for i in sample[:16]:
            s = int(recs["slot"][i])
            k = km[s]
            klen = M.KEYLEN[int(k["cipher"])]
            ot = O.Transform(O.TLS1_3 if ver == M.VERSION_TLS1_3 else O.TLS1_2, oc[int(k["cipher"])],
                             bytes(k["key"][:klen]), bytes(k["key"][:klen]), bytes(k["iv"]), bytes(k["iv"]))
            buf = bytearray(stride - lead)
            buf[head:head + content] = pt_sample[i].tobytes()
            orec = O.Record(ctr=bytes(recs["ctr"][i]), type=23, ver=b"\x03\x03", buf=buf,
                            data_offset=head, data_len=content)
            assert ot.encrypt_buf(orec) == 0
            got = src[i * stride + lead:i * stride + lead + wire].cpu().numpy().tobytes()
            oracle_ok &= got == orec.data()

    # ---- roofline of the dominant kernel --------------------------------------
    # algorithmic bytes per record as SURVEY 8(d) counts them: decrypt reads
    # ciphertext+tag + the 5-B header (AAD) and writes the inner plaintext + a
    # 4-B status (16 KiB TLS 1.3: 32 793 B); encrypt reads content + the type
    # byte and writes ciphertext+tag + the 5-B header (1.4 KiB: 2 830 B).  The
    # engine's own I/O per record -- a 40-B descriptor read, a 16-B result
    # written -- is listed beside it (..._with_descriptors).
    if direction == "decrypt":
        alg_per_rec = wire + 5 + inner + 4
        alg_desc = wire + inner + 40 + 16
    else:
        alg_per_rec = content + 1 + wire + 5
        alg_desc = content + wire + 40 + 16
    kern_avg_s = float(np.mean(kern_ms)) / 1e3
    achieved = alg_per_rec * n / kern_avg_s / 1e9
    per_rank = per_rank_roofline(kern_ranks, alg_per_rec * n)
    # HBM traffic per launch: PMC FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE
    # per record, measured by profiles/run_profile.sh on this config and
    # committed as profiles/traffic_<config>.json, scaled to this launch (not
    # re-measured in this run: counters need their own rocprofv3 passes).
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("direction") == direction and tj.get("record_inner_bytes") == inner:
            # reads from the request-size-resolved L2->fabric counters when the
            # profile has them (calibrated), else FETCH_SIZE x 2
            per_rec = tj.get("hbm_bytes_per_record_sized", tj["hbm_bytes_per_record"])
            reads = tj.get("read_counters", "FETCH_SIZE x 2")
            if "hbm_bytes_per_record_sized" in tj:
                reads = "TCC_EA0_RDREQ_{32B,64B,128B}_sum x size"
            traffic = round(per_rec * n)
            traffic_src = (f"profiles/traffic_{args.config}.json (rocprofv3 --pmc, reads {reads}, writes WRITE_SIZE; "
                           f"run {tj.get('source', '?')}, {per_rec:.0f} B/record x {n} records)")
    # The unit that actually bounds the kernel (LDS for the table ciphers):
    # its busy fraction from the committed PMC run (profiles/ceiling_<config>.json)
    # and the rate this kernel would reach with that unit 100 % busy.
    ceiling = None
    cpath = os.path.join(ROOT, "profiles", f"ceiling_{args.config}.json")
    if os.path.exists(cpath):
        with open(cpath) as f:
            cj = json.load(f)
        busy = cj["limiter_busy_frac"]
        ceiling = {"limiter": cj["limiter"], "busy_frac": busy,
                   "ceiling_GBps": round(achieved / busy, 1) if busy > 0 else None,
                   "ceiling_frac_of_hbm": round(achieved / busy / HBM_PEAK_GBS, 4) if busy > 0 else None,
                   "clock_ghz": cj.get("effective_clock_ghz"), "units": cj.get("units"),
                   "valu_x4": cj.get("valu_x4"), "valu_model": cj.get("valu_model"),
                   "source": f"profiles/ceiling_{args.config}.json ({cj.get('source', '?')})"}

    steps_s = wall / args.steps
    payload_total = float(n) * inner * world
    value = payload_total / steps_s / 2**30

    # the CPU leg and the host-buffer leg run on rank 0 at every world size,
    # after the timed region (the other ranks wait at a barrier): records in
    # host memory are pinned socket buffers -> device -> pinned (the boundary
    # the reference's callers hand over, ssl_msg.c:1855 / :2058), reported
    # beside the device-resident value, never as it
    run_cpu = None if args.no_cpu else (
        lambda: cpu_baseline(cname, ver, content, inner, wire, stride, km, args.cpu_seconds, direction))
    run_e2e = None if args.no_e2e else (
        lambda: end_to_end(M, kt, recs, arena, out_arena, n, stride, lead, head, content, wire, inner, direction,
                           args.e2e_records))
    cpu, e2e = rank0_legs(dist if distributed else None, rank, run_cpu, run_e2e)

    if world > 1 and args.config == "c2":
        # BASELINE configs[4] (c5): the c2 shard on every rank, keys broadcast over RCCL
        workload = (f"AES-256-GCM decrypt, {n * world} x 16 KiB TLS 1.3 records sharded across {world} MI355X "
                    f"({n} per GPU), key broadcast over RCCL/xGMI (BASELINE c5: 8M records at N = 8)")
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(steps_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 keys/nonces, uniform random payload; decrypt inputs made by the verified encrypt kernel)",
        "config": {"workload": workload, "config": args.config, "records_per_gpu": n,
                   "record_inner_bytes": inner, "record_wire_bytes": wire, "keys": nkeys,
                   "lanes_per_record": args.lanes or "auto", "slot_align": args.align, "aead_region_offset": lead + head,
                   "parallelism": f"shard{world}"},
        "records_per_s": round(n * world / steps_s, 1),
        "roofline": {"bound": "hbm", "scope": ROOFLINE_SCOPE, "limiter": (f"{ceiling['limiter']} ({ceiling['busy_frac']:.0%} busy, measured)"
                                                 if ceiling else None),
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": KERNEL_OF.get(cname, "tlsrec_gcm_kernel"), "ceiling": ceiling,
                     "algorithmic_bytes_per_record": alg_per_rec,
                     "algorithmic_bytes_rule": "SURVEY 8(d): ct+tag + 5-B header read, inner plaintext + 4-B status "
                                               "written (decrypt); content + type byte read, ct+tag + 5-B header "
                                               "written (encrypt)",
                     "algorithmic_bytes_per_record_with_descriptors": alg_desc,
                     "frac_with_descriptors": round(alg_desc * n / kern_avg_s / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel_ms_avg": round(kern_avg_s * 1e3, 4),
                     "timing": "HIP events on the launch stream around each timed step",
                     "per_rank": per_rank["per_rank"], "frac_min_over_ranks": per_rank["frac_min"],
                     "kernel_ms_max_over_ranks": per_rank["kernel_ms_max"]},
        "cpu_baseline": cpu,
        "e2e": e2e,
        "check": {"bad_records": bad, "oracle_sample_ok": oracle_ok},
        "dist": dist_info,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


def rank_evidence(dist, keys_dev, dev, local):
    """What the process group really formed: the world size and backend as
    torch.distributed reports them, every rank's device, and the SHA-256 of the
    key table each rank holds after the RCCL broadcast (all-gathered and
    checked equal -- the only data any rank receives from another)."""
    import hashlib
    import torch
    digest = hashlib.sha256(keys_dev.cpu().numpy().tobytes()).digest()
    mine = torch.tensor(list(digest), dtype=torch.uint8, device=dev)
    allg = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(allg, mine)
    digests = [bytes(t.cpu().tolist()).hex() for t in allg]
    me = {"rank": dist.get_rank(), "local_rank": local, "device": str(dev)}
    if torch.device(dev).type == "cuda":
        props = torch.cuda.get_device_properties(dev)
        me.update(name=torch.cuda.get_device_name(dev), arch=getattr(props, "gcnArchName", None),
                  pci_bus_id=getattr(props, "pci_bus_id", None), pci_device_id=getattr(props, "pci_device_id", None),
                  hip_device=torch.cuda.current_device())
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me)
    ok = len(set(digests)) == 1
    if not ok:
        raise RuntimeError(f"key tables differ across ranks after the broadcast: {digests}")
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": ranks,
            "key_table_sha256": digests[0], "key_table_equal_on_all_ranks": ok}


def end_to_end(M, kt, recs, arena, out_arena, n, stride, lead, head, content, wire, inner, direction, e2e_records):
    """tlsrec_host_batch_* over pinned host buffers: chunked H2D -> kernels ->
    D2H on three streams (engine.hip).  Input = the first E records of the
    bench batch (ciphertexts for decrypt), output into a second pinned buffer;
    statuses and a byte sample are checked against the device-resident run."""
    import torch
    E = min(n, e2e_records or max(1, (2 << 30) // stride))
    span = E * stride
    host_in = torch.empty(span, dtype=torch.uint8).pin_memory()
    host_out = torch.empty(span, dtype=torch.uint8).pin_memory()
    host_in.copy_(arena[:span])
    d = recs[:E].copy()
    if direction == "decrypt":
        d["data_offset"] = 0
        d["data_len"] = wire
    res = M.results(E)
    chunk = int(os.environ.get("BENCH_E2E_CHUNK_MB", "64")) << 20    # pipeline chunk (measurement override)
    dec = direction == "decrypt"
    M.host_batch(dec, kt, d, res, E, host_in, host_out, chunk_bytes=chunk)      # warm-up
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        M.host_batch(dec, kt, d, res, E, host_in, host_out, chunk_bytes=chunk)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    ok = bool((res["status"] == 0).all())
    lo, hi = (lead + head, lead + head + content) if dec else (lead, lead + wire)
    ref = out_arena                  # the device-resident run of the same records
    for i in sorted({0, E // 2, E - 1}):
        ok &= bool(torch.equal(host_out[i * stride + lo:i * stride + hi], ref[i * stride + lo:i * stride + hi].cpu()))
    dev = torch.empty(span, dtype=torch.uint8, device=arena.device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev.copy_(host_in, non_blocking=True)
    torch.cuda.synchronize()
    h2d = span / (time.perf_counter() - t0) / 1e9
    t0 = time.perf_counter()
    host_out.copy_(dev, non_blocking=True)
    torch.cuda.synchronize()
    d2h = span / (time.perf_counter() - t0) / 1e9
    del dev
    return {"value": round(E * inner / best / 2**30, 3), "unit": "GiB/s", "records_per_s": round(E / best, 1),
            "records": E, "chunk_bytes": chunk, "device_slots": 3, "streams": "H2D / kernels / D2H",
            "h2d_only_GBps": round(h2d, 2), "d2h_only_GBps": round(d2h, 2), "check_ok": ok,
            "what": "pinned host records -> device -> pinned host (tlsrec_host_batch_%s); PCIe-inclusive, "
                    "not the device-resident headline" % direction}


def host_cores():
    """Threads the CPU legs use: the host CPUs this process may run on
    (affinity), capped by a cgroup CPU quota and by OMP_NUM_THREADS, which the
    GPU pool sets to the box's CPU share (os.cpu_count() there shows the whole
    machine).  Returns (threads, how they were determined)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    n, why = aff, [f"affinity {aff} CPUs", f"os.cpu_count {os.cpu_count()}"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            qc = max(1, -(-int(q) // int(per)))
            n = min(n, qc)
            why.append(f"cgroup quota {qc} CPUs")
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
        why.append(f"OMP_NUM_THREADS {omp} (the box's CPU share)")
    return max(1, n), "; ".join(why)


def _timed_sample(target_s, stride, n0, seal, run):
    """Grow the sample (up to a 512 MiB arena) until one pass takes about
    target_s, then repeat passes until target_s of wall time; seal() prepares
    the arena untimed before each pass (decrypt inputs)."""
    cap = 512 << 20
    n = n0
    while True:
        arena = seal(n, None)
        el = run(arena, n)
        if el >= target_s or n * stride * 2 > cap:
            break
        n = min(int(n * max(2.0, min(8.0, target_s / max(el, 1e-3)))), cap // stride)
    reps = 1
    while el < target_s:
        seal(n, arena)
        el += run(arena, n)
        reps += 1
    return n, reps, el


def cpu_baseline(cname, ver, content, inner, wire, stride, km, target_s, direction):
    """Two CPU legs on the same record shape, timed on this host's cores
    (threads = host_cores()): 'evp' -- the record framing around OpenSSL 3
    EVP AEADs (AES-NI/VAES GCM, SIMD ChaCha20-Poly1305), the stand-in for the
    reference's default x86 path (AES-NI on by default, ChangeLog:1021-1024);
    'port' -- this repository's C restatement (oracle/, table AES + 4-bit
    Shoup GHASH, the Mbed TLS builtin design).  Multi-connection configs (c4,
    c4s, k4: any config with more than one key) run both legs with one key
    context per connection, record i under connection i % keys
    (ssl_misc.h:1073-1120: one transform per connection).
    The headline value is the faster leg (the stronger CPU baseline); both are
    listed, with the EVP leg's per-call time split."""
    import oracle as O
    from tests.prng import prng_array
    mix = len(km) > 1      # one transform per connection (c4, c4s, k4)
    cipher = {"CHACHA20-POLY1305": O.CHACHA20_POLY1305, "AES-128-GCM": O.AES_128_GCM, "AES-128-CCM": O.AES_128_CCM,
              "AES-128-CCM-8": O.AES_128_CCM_8, "AES-192-GCM": O.AES_192_GCM,
              "ARIA-256-GCM": O.ARIA_256_GCM, "CAMELLIA-128-GCM": O.CAMELLIA_128_GCM}.get(cname, O.AES_256_GCM)
    k = km[0]
    klen = O.KEYLEN[cipher]
    key, iv = bytes(k["key"][:klen]), bytes(k["iv"])
    tls = O.TLS1_3 if ver == 0x0304 else O.TLS1_2
    head = 8 if tls == O.TLS1_2 and cipher != O.CHACHA20_POLY1305 else 0
    threads, how = host_cores()
    payload = prng_array(SEED ^ 0xC0FFEE, 4096 * content).reshape(4096, content) if content else None
    st_cache = {}
    nconn = len(km) if mix else 1

    def fresh(n, arena):
        if arena is None:
            arena = np.zeros(n * stride, dtype=np.uint8)
        if content:
            v = arena.reshape(n, stride)
            for lo in range(0, n, 4096):
                hi = min(n, lo + 4096)
                v[lo:hi, head:head + content] = payload[:hi - lo]
        st_cache[n] = np.zeros(n, dtype=np.int32)
        return arena

    legs = []
    enc_len = wire if direction == "decrypt" else content
    dflag = 0 if direction == "decrypt" else 1
    if mix:
        ciph = km["cipher"].astype(np.uint8)
        keys = np.ascontiguousarray(km["key"][:, :32])
        ivs = np.ascontiguousarray(km["iv"][:, :12])
        ts = [O.Transform(tls, int(c), bytes(kk[:O.KEYLEN[int(c)]]), bytes(kk[:O.KEYLEN[int(c)]]),
                          bytes(v), bytes(v)) for c, kk, v in zip(ciph, km["key"], km["iv"])]
        port_do = lambda d, a, ln, n: O.bench_multi(ts, d, a, stride, ln, n, threads, st_cache[n])  # noqa: E731
        what = f"{nconn} connections (one transform each), record i under connection i % {nconn}"
    else:
        t = O.Transform(tls, cipher, key, key, iv, iv)
        port_do = lambda d, a, ln, n: t.bench(d, a, stride, ln, n, 0, threads, st_cache[n])  # noqa: E731
        what = "one key"
    impls = {"CHACHA20-POLY1305": "ChaCha20 + 44-bit-limb Poly1305",
             "ARIA-256-GCM": "byte-wise ARIA + 4-bit Shoup GHASH",
             "CAMELLIA-128-GCM": "byte-wise Camellia (unoptimised oracle port) + 4-bit Shoup GHASH",
             "MIX": "table AES + 4-bit Shoup GHASH / ChaCha20 + 44-bit-limb Poly1305"}

    def port_seal(n, arena):
        arena = fresh(n, arena)
        if direction == "decrypt":
            port_do(1, arena, content, n)
            assert (st_cache[n] == 0).all()
        return arena

    def port_run(arena, n):
        el = port_do(dflag, arena, enc_len, n)
        assert (st_cache[n] == 0).all()
        return el

    evp_ok = all(int(c) in O.EVP_CIPHERS for c in km["cipher"]) if mix else cipher in O.EVP_CIPHERS
    if evp_ok:
        if mix:
            em = O.EvpMixed(km["cipher"], keys, ivs, tls, threads)
            evp_do = lambda d, a, ln, n: em.run(d, a, stride, ln, n, st_cache[n])  # noqa: E731
        else:
            evp_do = lambda d, a, ln, n: O.evp_bench(cipher, tls, key, iv, d, a, stride, ln, n, 0,  # noqa: E731
                                                     threads, st_cache[n])

        def evp_seal(n, arena):
            arena = fresh(n, arena)
            if direction == "decrypt":
                evp_do(1, arena, content, n)
                assert (st_cache[n] == 0).all()
            return arena

        def evp_run(arena, n):
            el = evp_do(dflag, arena, enc_len, n)
            assert (st_cache[n] == 0).all()
            return el

        n, reps, el = _timed_sample(target_s, stride, 1024, evp_seal, evp_run)
        names = {O.AES_128_GCM: "AES-128-GCM", O.AES_256_GCM: "AES-256-GCM", O.CHACHA20_POLY1305: "CHACHA20-POLY1305"}
        prof = {names[c]: O.evp_call_profile(c, inner)
                for c in sorted(set(int(x) for x in (km["cipher"] if mix else [cipher])))}
        legs.append({"value": round(n * reps * inner / el / 2**30, 3), "unit": "GiB/s", "cores": threads,
                     "kind": "port", "leg": "evp",
                     "sample": f"{n} records ({reps} passes) x {inner} B inner plaintext, {direction}, {what}: "
                               f"ssl_msg.c record framing around OpenSSL 3 EVP AEAD (AES-NI/VAES GCM, SIMD "
                               f"ChaCha20-Poly1305; oracle/libevpbench.so), nonce-only re-init per record as libssl "
                               f"does for TLS 1.3, one OpenSSL library context per thread, {el:.2f} s wall on "
                               f"{threads} threads",
                     "evp_us_per_record_one_thread": prof})
        if mix:
            em.close()
    n, reps, el = _timed_sample(target_s, stride, 1024, port_seal, port_run)
    impl = impls.get(cname, "table AES + 4-bit Shoup GHASH" if "GCM" in cname else "table AES CCM")
    legs.append({"value": round(n * reps * inner / el / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
                 "leg": "port",
                 "sample": f"{n} records ({reps} passes) x {inner} B inner plaintext, {direction}, {what}: "
                           f"oracle/liboracle.so C restatement ({impl}), {el:.2f} s wall on {threads} threads"})
    out = dict(max(legs, key=lambda x: x["value"]))
    out.pop("evp_us_per_record_one_thread", None)
    out["cores_how"] = how
    out["headline"] = "the faster of the legs"
    out["legs"] = legs
    return out


if __name__ == "__main__":
    main()
