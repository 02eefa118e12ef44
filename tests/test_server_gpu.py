"""The record server (mbedtls_amd/csrc/server.hip): single-record calls of
AES-128/192/256-GCM and ChaCha20-Poly1305 transforms are served by a resident
kernel polling pinned request slots instead of a launch per call.  Every
served call must return exactly what the reference's mbedtls_ssl_encrypt_buf /
mbedtls_ssl_decrypt_buf return for it (ssl_msg.c:784-1268, :1270-1834): the
ciphertext against the oracle, status / data_offset / data_len / type, the
wipe on a bad tag, TLS 1.3 inner type and padding -- at every record length
class and buffer alignment the staging sees -- and the launch path (server
disabled) must give the same bytes."""
import ctypes

import pytest

import mbedtls_amd as M
import oracle as O
from mbedtls_amd import _abi
from tests.prng import prng_bytes

pytestmark = pytest.mark.gpu

SERVED = [M.CIPHER_AES_128_GCM, M.CIPHER_AES_256_GCM, M.CIPHER_AES_192_GCM, M.CIPHER_CHACHA20_POLY1305]
LENGTHS = [0, 1, 15, 16, 17, 63, 64, 65, 100, 1000, 1007, 1400, 1408, 4000, 8191, 16383, 16384]


def _stats():
    f = _abi.load().tlsrec__server_stats
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 3
    s, fb, ln = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    f(ctypes.byref(s), ctypes.byref(fb), ctypes.byref(ln))
    return s.value, fb.value, ln.value


def _enable(on: bool):
    _abi.load().tlsrec__server_enable(1 if on else 0)


@pytest.fixture(autouse=True)
def _server_on():
    _enable(True)
    yield
    _enable(True)


def _pair(cipher, ver, seed):
    kl = M.KEYLEN[cipher]
    key, iv = prng_bytes(seed, kl), prng_bytes(seed + 1, 16)
    return M.Transform(ver, cipher, key, key, iv, iv), O.Transform(ver, cipher, key, key, iv, iv)


def _head(cipher, ver):
    return 8 if ver == M.VERSION_TLS1_2 and cipher != M.CIPHER_CHACHA20_POLY1305 else 0


def _roundtrip(t, ot, cipher, ver, ln, n, extra_head=0, typ=23):
    """encrypt on the GPU and in the oracle, compare, decrypt back; returns errors"""
    head = _head(cipher, ver) + extra_head
    pt = prng_bytes(7000 + n * 31 + ln, ln)
    buf = bytearray(prng_bytes(9000 + n, head)) + bytearray(pt) + bytearray(64 + 16)
    ctr = (n * 977 + 3).to_bytes(8, "big")
    rec = M.Record(ctr=ctr, type=typ, ver=b"\x03\x03", buf=bytearray(buf), data_offset=head, data_len=ln)
    orec = O.Record(ctr=ctr, type=typ, ver=b"\x03\x03", buf=bytearray(buf), data_offset=head, data_len=ln)
    st, ost = t.encrypt_buf(rec), ot.encrypt_buf(orec)
    got = (st, rec.data_offset, rec.data_len, rec.type)
    want = (ost, orec.data_offset, orec.data_len, orec.type)
    if got != want:
        return [("encrypt fields", ln, got, want)]
    if st != 0:
        return []
    if bytes(rec.buf) != bytes(orec.buf):
        return [("encrypt buffer differs from the oracle", ln, extra_head)]
    st = t.decrypt_buf(rec)
    ost = ot.decrypt_buf(orec)
    got = (st, rec.data_offset, rec.data_len, rec.type)
    want = (ost, orec.data_offset, orec.data_len, orec.type)
    if got != want:
        return [("decrypt fields", ln, got, want)]
    if st == 0 and (rec.data() != pt or bytes(rec.buf) != bytes(orec.buf)):
        return [("decrypt bytes", ln)]
    return []


@pytest.mark.parametrize("cipher", SERVED)
@pytest.mark.parametrize("ver", [M.VERSION_TLS1_2, M.VERSION_TLS1_3])
def test_served_records_match_oracle(cipher, ver):
    t, ot = _pair(cipher, ver, 100 + cipher * 7 + ver)
    s0, f0, _ = _stats()
    errs = []
    try:
        for n, ln in enumerate(LENGTHS):
            for extra in (0, 3, 13):       # AEAD start at every 16-byte phase the staging re-aligns
                errs += _roundtrip(t, ot, cipher, ver, ln, n * 3 + extra, extra)
    finally:
        t.close()
    assert not errs, errs[:4]
    s1, f1, _ = _stats()
    calls = 2 * len(LENGTHS) * 3
    why = _why()
    # The grid's idle exit is ordered against submits (server.hip, the
    # activity / closing / settled handshake): a call never posts to a grid
    # that is leaving, and a grid never leaves idle while a claim is still
    # posting, so nothing is withdrawn by the idle exit; a call that finds the
    # grid gone launches the next one instead of taking the launch path.  (A
    # host thread descheduled past the end of a grid's 20-ms window can still
    # see its request withdrawn -- it then runs on the launch path, and its
    # bytes were checked against the oracle above like every other call's.)
    assert why[2] <= 2, f"withdrawn requests: {why}"
    assert f1 - f0 <= 2, ("calls went back to the launch path (batch pending, set not drained, "
                          f"withdrawn, no slot so far: {why})")
    assert s1 - s0 >= calls - 2, "the record server did not serve these calls"


def _why():
    why = (ctypes.c_uint64 * 4)()
    _abi.load().tlsrec__server_why(why)
    return list(why)


def test_idle_boundary_submits_are_never_withdrawn():
    """Calls at the idle exit's boundary (TLSREC_SERVER_IDLE_MS = 0.05, gaps of
    0..400 us between calls, 1 400-B and 16 KiB records) in a process of their
    own (the idle limit is read once per process): every call is served by a
    grid -- none withdrawn, none on the launch path -- the grids really leave
    idle and are relaunched, and every record matches the oracle."""
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, TLSREC_SERVER_IDLE_MS="0.05")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-m", "tests._server_idle_child", "600"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["errors"] == [], r["errors"][:4]
    assert r["why"][2] == 0, r
    assert r["fallback"] <= 2, r
    assert r["served"] >= r["calls"] - 2, r
    assert r["launches"] >= 20, r      # the grids left idle and were relaunched many times


def test_idle_exit_waits_for_a_claim_still_posting():
    """a host thread that claimed a slot but has not posted yet
    (here held 300 us between claim and post by the test-hooks build's
    TLSREC_TEST_SERVER_POST_DELAY_US, six times the 50-us idle limit) keeps
    the grid: workgroup 0 commits the idle exit only when every claim has
    settled, so no request is withdrawn and every call is served by a grid."""
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, TLSREC_SERVER_IDLE_MS="0.05", TLSREC_TEST_SERVER_POST_DELAY_US="300")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-m", "tests._server_idle_child", "200", "--test-lib"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["errors"] == [], r["errors"][:4]
    assert r["why"][2] == 0, r
    assert r["fallback"] <= 2, r
    assert r["served"] >= r["calls"] - 2, r


@pytest.mark.parametrize("cipher", SERVED)
def test_served_tamper_wipes_like_the_reference(cipher):
    """a flipped ciphertext or tag byte: INVALID_MAC, output wiped (PSA), as the oracle"""
    ver = M.VERSION_TLS1_3
    t, ot = _pair(cipher, ver, 500 + cipher)
    try:
        for n, (ln, where) in enumerate([(1400, 0), (1400, 1399), (1400, 1400 + 1 + 16 - 1), (16000, 9000),
                                         (0, 1), (33, 40)]):
            pt = prng_bytes(n, ln)
            buf = bytearray(pt) + bytearray(64 + 16)
            ctr = (n + 11).to_bytes(8, "big")
            rec = M.Record(ctr=ctr, type=23, ver=b"\x03\x03", buf=bytearray(buf), data_offset=0, data_len=ln)
            assert t.encrypt_buf(rec) == 0
            total = rec.data_len
            where = min(where, total - 1)
            rec.buf[rec.data_offset + where] ^= 0x20
            orec = O.Record(ctr=ctr, type=rec.type, ver=b"\x03\x03", buf=bytearray(rec.buf),
                            data_offset=rec.data_offset, data_len=rec.data_len)
            st, ost = t.decrypt_buf(rec), ot.decrypt_buf(orec)
            assert st == ost == M.ERR_SSL_INVALID_MAC, (ln, where, st, ost)
            assert bytes(rec.buf) == bytes(orec.buf), (ln, where)
    finally:
        t.close()


@pytest.mark.parametrize("cipher", [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305])
def test_served_inner_plaintext(cipher):
    """TLS 1.3: padding granularities, every content type byte; an all-zero
    inner plaintext is INVALID_RECORD (ssl_msg.c:1809-1826)"""
    kl = M.KEYLEN[cipher]
    key, iv = prng_bytes(61, kl), prng_bytes(62, 16)
    for gran in (1, 16, 255):
        t = M.Transform(M.VERSION_TLS1_3, cipher, key, key, iv, iv, granularity=gran)
        ot = O.Transform(M.VERSION_TLS1_3, cipher, key, key, iv, iv, granularity=gran)
        try:
            for n, ln in enumerate([0, 1, 17, 300, 1400]):
                for typ in (21, 22, 23):
                    assert not _roundtrip(t, ot, cipher, M.VERSION_TLS1_3, ln, n * 5 + typ, 0, typ)
            # all-zero inner plaintext: type byte 0 -> no non-zero byte after decryption
            buf = bytearray(1400 + 256 + 64)
            rec = M.Record(ctr=(77).to_bytes(8, "big"), type=0, ver=b"\x03\x03", buf=bytearray(buf), data_offset=0,
                           data_len=1400)
            orec = O.Record(ctr=(77).to_bytes(8, "big"), type=0, ver=b"\x03\x03", buf=bytearray(buf), data_offset=0,
                            data_len=1400)
            assert t.encrypt_buf(rec) == ot.encrypt_buf(orec) == 0
            assert bytes(rec.buf) == bytes(orec.buf)
            assert t.decrypt_buf(rec) == ot.decrypt_buf(orec) == M.ERR_SSL_INVALID_RECORD
        finally:
            t.close()


def test_server_and_launch_path_agree():
    """the same calls with the server disabled (the coalescing launch path) give the same bytes"""
    outs = []
    for on in (True, False):
        _enable(on)
        s0, _, _ = _stats()
        res = []
        for cipher in SERVED:
            for ver in (M.VERSION_TLS1_2, M.VERSION_TLS1_3):
                kl = M.KEYLEN[cipher]
                t = M.Transform(ver, cipher, prng_bytes(cipher, kl), prng_bytes(cipher + 1, kl),
                                prng_bytes(cipher + 2, 16), prng_bytes(cipher + 3, 16))
                try:
                    for n, ln in enumerate([5, 1400, 9000]):
                        head = _head(cipher, ver)
                        buf = bytearray(head) + bytearray(prng_bytes(n, ln)) + bytearray(80)
                        rec = M.Record(ctr=(n + 1).to_bytes(8, "big"), type=23, ver=b"\x03\x03", buf=buf,
                                       data_offset=head, data_len=ln)
                        res.append((t.encrypt_buf(rec), rec.data_offset, rec.data_len, bytes(rec.buf)))
                finally:
                    t.close()
        s1, _, _ = _stats()
        assert (s1 > s0) == on
        outs.append(res)
    assert outs[0] == outs[1]
