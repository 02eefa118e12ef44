"""CPU-side checks of the drop-in boundary: libtlsrec.so loads, exports every
function include/tlsrec.h declares, and its struct layouts match; the host
framing decisions (everything mbedtls_ssl_{en,de}crypt_buf decide before the
AEAD) agree with the oracle restatement.  No compute call needs a GPU here.
"""
import ctypes
import os
import re

import numpy as np
import pytest

import mbedtls_amd as M
from mbedtls_amd import _abi
import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "tlsrec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tlsrec_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_symbol():
    L = M.load()
    names = _declared()
    assert len(names) >= 14
    for n in names:
        assert hasattr(L, n), f"libtlsrec.so does not export {n}"
        assert n in _abi.SIGNATURES, f"python binding lacks {n}"


def _exports(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_test_hooks_only_in_the_test_build():
    """The release library carries no test hook (the reference compiles its
    own only under MBEDTLS_TEST_HOOKS, library/ssl_misc.h:2685); the
    test-hooks build exports them and every entry point of the ABI."""
    rel = _exports(_abi.LIB_PATH)
    tst = _exports(_abi.TEST_LIB_PATH)
    assert not [s for s in rel if s.startswith("tlsrec__test_")], sorted(s for s in rel if "test" in s)
    for s in ("tlsrec__test_skip_record", "tlsrec__test_fail_staging", "tlsrec__test_server_shadow",
              "tlsrec__test_lane_ops", "tlsrec__test_scan"):
        assert s in tst, s
    for n in _declared():
        assert n in tst, n


def test_struct_layouts():
    assert ctypes.sizeof(_abi.CRecord) == 88       # + cid_len, cid[32]
    assert ctypes.sizeof(_abi.CTransform) == 232   # + in/out_cid_len, in/out_cid[32]
    assert M.BATCH_REC.itemsize == 40 and M.BATCH_RES.itemsize == 16 and M.KEY_MATERIAL.itemsize == 64


def test_version_string():
    assert "gfx950" in M.version()


CIPHERS = sorted(M.KEYLEN)      # every AEAD id of include/tlsrec.h
VERSIONS = [M.VERSION_TLS1_2, M.VERSION_TLS1_3]


@pytest.mark.parametrize("cipher", CIPHERS)
@pytest.mark.parametrize("ver", VERSIONS)
def test_frame_check_matches_oracle(cipher, ver):
    """Early exits (INTERNAL_ERROR, BAD_INPUT_DATA, BUFFER_TOO_SMALL,
    INVALID_MAC) and the fields they leave, over a sweep of buffer shapes."""
    kl = M.KEYLEN[cipher]
    key, iv = bytes([5]) * kl, bytes([6]) * 16
    km = M.key_material(cipher, ver, key, iv)
    ot = O.Transform(ver, cipher, key, key, iv, iv)
    rng = np.random.default_rng(cipher * 10 + ver)
    for trial in range(600):
        buf_len = int(rng.integers(0, 120)) if trial % 3 else int(rng.integers(16380, 16450))
        do = int(rng.integers(0, buf_len + 3))
        dl = int(rng.integers(0, buf_len + 3))
        rec = M.records(1)
        rec["buf_len"], rec["data_offset"], rec["data_len"] = buf_len, do, dl
        rec["type"] = 23
        rec["ver"] = (3, 3)
        for dec in (False, True):
            go, early, pos, ln = M.frame_check(dec, km, rec)
            orec = O.Record(ctr=bytes(8), type=23, ver=b"\x03\x03", buf=bytearray(max(buf_len, do + dl, 1) + 64),
                            data_offset=do, data_len=dl, buf_len=buf_len)
            if dec:
                # make sure a record that passes the checks fails only at the tag
                st = ot.decrypt_buf(orec)
                if go:
                    assert st == O.ERR_INVALID_MAC
                else:
                    assert int(early["status"]) == st
                    assert (int(early["data_offset"]), int(early["data_len"])) == (orec.data_offset, orec.data_len)
            else:
                st = ot.encrypt_buf(orec)
                if go:
                    assert st in (0, O.ERR_BUFFER_TOO_SMALL)   # the latter: explicit IV after the AEAD
                else:
                    assert int(early["status"]) == st, (buf_len, do, dl)
                    assert (int(early["data_offset"]), int(early["data_len"]), int(early["type"])) == \
                        (orec.data_offset, orec.data_len, orec.type)


def test_no_gpu_means_loud_failure():
    """Without a device every data path reports HW_ACCEL_FAILED, never a CPU result."""
    L = M.load()
    if L.tlsrec_device_check() == 0:
        pytest.skip("a device is present")
    t = _abi.CTransform()
    r = L.tlsrec_transform_setup(ctypes.byref(t), M.VERSION_TLS1_3, M.CIPHER_AES_256_GCM,
                                 bytes(32), bytes(32), bytes(12), bytes(12))
    assert r == M.ERR_SSL_HW_ACCEL_FAILED
    h = ctypes.c_void_p()
    assert L.tlsrec_keytab_create(ctypes.byref(h), 4) == M.ERR_SSL_HW_ACCEL_FAILED


def test_pair_small_lane_model():
    """the paired passes' lanes per record for small records (engine.hip
    tlsrec__gcm_pair_small_l, a host function: no GPU needed) -- the round-fill
    model picks the lane count that measured best at every records-per-key
    point of the r05 sweep (profiles/archive/r05/small_rpk/)"""
    import ctypes
    from mbedtls_amd import _abi
    f = _abi.load().tlsrec__gcm_pair_small_l
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32]
    best = {16: 8, 23: 4, 32: 4, 47: 8, 64: 2, 95: 4, 128: 2, 191: 2}
    assert {r: f(r) for r in best} == best
    assert all(f(r) in (2, 4, 8) for r in range(12, 256))
