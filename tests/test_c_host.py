"""A plain C program (tests/c/abi_host.c, gcc, include/tlsrec.h only) as the
host of libtlsrec.so -- the way Mbed TLS C code would call the engine.

  - not gpu: tlsrec_record's field offsets equal a mirror of mbedtls_record
    (ssl_misc.h:1163-1188), and the batch structs have the kernels' sizes;
  - gpu: the reference's 4 TLS 1.3 record KATs (test_suite_ssl.data:2776-2834)
    through tlsrec_encrypt_buf / tlsrec_decrypt_buf from C, single-record
    round trips with latency percentiles, and concurrent C threads each with
    its own transform (every payload checked).
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c", "abi_host")


def _exe():
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(os.path.join(ROOT, "tests", "c", "abi_host.c")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c")], check=True)
    return EXE


def _run(*args, timeout=120):
    p = subprocess.run([_exe(), *map(str, args)], capture_output=True, text=True, timeout=timeout)
    out = json.loads(p.stdout.strip().splitlines()[-1]) if p.stdout.strip() else {}
    return p.returncode, out, p.stderr


def test_c_layout_matches_mbedtls_record():
    rc, out, err = _run("layout")
    assert rc == 0, (out, err)
    assert out["ok"] is True
    for field, (a, b) in out["layout"].items():
        assert a == b, field


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.gpu
def test_c_reference_kats():
    if not _gpu():
        pytest.skip("needs a GPU")
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        kats = json.load(f)
    for k in kats:
        rc, out, err = _run("kat", k["endpoint"], k["ctr"], k["server_key"], k["server_iv"], k["client_key"],
                            k["client_iv"], k["plaintext"], k["ciphertext"])
        assert rc == 0, (k["name"], out, err)
        assert out["ciphertext_equal"] and out["plaintext_equal"]


@pytest.mark.gpu
@pytest.mark.parametrize("cipher,tls,content", [(2, "1.3", 16383), (2, "1.3", 1400), (3, "1.3", 1400),
                                                (1, "1.2", 1400), (5, "1.3", 1400)])
def test_c_single_record_latency(cipher, tls, content):
    if not _gpu():
        pytest.skip("needs a GPU")
    rc, out, err = _run("latency", cipher, tls, content, 200)
    assert rc == 0, (out, err)
    assert out["bad"] == 0
    lat = out["latency_us"]
    print(json.dumps(lat))
    assert lat["encrypt_p50"] > 0 and lat["decrypt_p50"] > 0


@pytest.mark.gpu
def test_c_threads_concurrent_transforms():
    if not _gpu():
        pytest.skip("needs a GPU")
    rc, out, err = _run("threads", 12, 100)
    assert rc == 0, (out, err)
    assert out["bad"] == 0


MGPU = os.path.join(ROOT, "tests", "c", "mgpu_shard")


@pytest.mark.gpu
@pytest.mark.parametrize("records,content", [(4096, 1400), (777, 16383), (1, 0)])
def test_c_multi_gpu_host_one_rank(records, content):
    """tests/c/mgpu_shard.c at world 1 (one GPU per box here): rank 0's key
    table through ncclBroadcast into tlsrec_keytab_load(keys_on_device=1),
    tlsrec_shard_bounds, an encrypt/decrypt round trip of the shard and the
    ncclAllReduce of status counts -- the C multi-GPU sequence of DESIGN.md
    section 6.  World > 1 needs one GPU per rank (the driver's 8-GPU node)."""
    assert _gpu(), "needs a GPU"
    if not os.path.exists(MGPU):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c"), "mgpu_shard"], check=True)
    p = subprocess.run([MGPU, "1", str(records), str(content)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.stdout, p.stderr)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["pass"] is True and out["records"] == records and out["round_trip_ok"] == records
    assert out["ranks_with_rank0_keys"] == 1 and out["shard0"] == [0, records]


@pytest.mark.gpu
@pytest.mark.parametrize("fill", ["0x55", "0"])
@pytest.mark.parametrize("mode", ["pageable", "memset", "pinned"])
def test_system_runtime_direction_switches(mode, fill):
    """Batch calls alternating encrypt / decrypt over a 256-key table on the
    system HIP runtime (no torch in the process: what a C host links).  Every
    call must write every result -- with the stream-ordered allocator for the
    bucket scratch, the first call after a direction change wrote none.  With
    a zero pre-fill (which reads as success) every result must still carry the
    kernel's verdict: the fail-closed contract (ssl_msg.c:1260 / :1804)."""
    assert _gpu(), "needs a GPU"
    env = dict(os.environ)
    p = subprocess.run(["python3", os.path.join(ROOT, "tests", "sysrt_seq.py"), "64", "256", "eddeedde", mode, fill],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["verdicts"] == [64] * 8, out
    if fill != "0":
        assert out["written"] == [64] * 8, out


DTLS = os.path.join(ROOT, "tests", "c", "dtls_host")


@pytest.mark.gpu
@pytest.mark.parametrize("conns,dgrams,content,cipher", [(64, 8, 1200, 1), (300, 3, 16384, 2), (17, 40, 100, 3),
                                                          (32, 6, 1400, 8)])
def test_c_dtls_host(conns, dgrams, content, cipher):
    """tests/c/dtls_host.c: a C program (gcc, include/tlsrec.h + the HIP
    runtime API) sends datagrams with tlsrec_dtls_encrypt and receives them,
    plus a replay and a bad-MAC datagram per connection, with
    tlsrec_dtls_decrypt -- every plaintext, disposition and window checked."""
    assert _gpu(), "needs a GPU"
    if not os.path.exists(DTLS):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c"), "dtls_host"], check=True)
    p = subprocess.run([DTLS, str(conns), str(dgrams), str(content), str(cipher)], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, (p.stdout, p.stderr)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["pass"] is True and out["accepted"] == conns * dgrams == out["plaintext_ok"]
    assert out["replays_skipped"] == conns and out["bad_mac_dropped"] == conns
