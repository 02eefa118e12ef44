"""The TLS 1.3 key-schedule oracle (oracle/keysched.c) against the
reference's own vectors (tests/golden/tls13_keys.json, transcribed from
test_suite_ssl.data by tests/golden/make_tls13_keys.py) and against Python's
hashlib/hmac as an independent SHA-2 / HMAC implementation."""
import hashlib
import hmac as pyhmac
import json
import os

import pytest

import oracle as O
from tests.prng import prng_bytes

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tls13_keys.json")))
X = bytes.fromhex


@pytest.mark.parametrize("v", G["expand_label"], ids=lambda v: v["where"])
def test_expand_label_reference_vectors(v):
    got = O.tls13_hkdf_expand_label(O.HASHES[v["hash"]], X(v["secret"]), v["label"].encode(), X(v["ctx"]), v["len"])
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("v", G["derive_secret"], ids=lambda v: v["name"])
def test_derive_secret_reference_vectors(v):
    got = O.tls13_derive_secret(O.HASHES[v["hash"]], X(v["secret"]), v["label"].encode(), X(v["ctx"]),
                                v["ctx_hashed"], v["len"])
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("v", G["evolve"], ids=lambda v: v["where"])
def test_evolve_secret_reference_vectors(v):
    got = O.tls13_evolve_secret(O.HASHES[v["hash"]], X(v["secret"]) or None, X(v["input"]) or None)
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("v", G["traffic_keys"], ids=lambda v: v["where"])
def test_traffic_keys_reference_vectors(v):
    ck, ci, sk, si = O.tls13_make_traffic_keys(O.HASHES[v["hash"]], X(v["client_secret"]), X(v["server_secret"]),
                                               v["key_len"], v["iv_len"])
    assert (ck.hex(), ci.hex(), sk.hex(), si.hex()) == (v["client_key"], v["client_iv"], v["server_key"],
                                                        v["server_iv"])


@pytest.mark.parametrize("v", G["exporter"], ids=lambda v: v["where"])
def test_exporter_reference_vectors(v):
    got = O.tls13_exporter(O.HASHES[v["hash"]], X(v["secret"]), v["label"].encode(), v["context"].encode(), v["len"])
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("alg,name", [(O.SHA256, "sha256"), (O.SHA384, "sha384")])
@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 111, 112, 127, 128, 129, 1000])
def test_sha_hmac_vs_hashlib(alg, name, n):
    msg = prng_bytes(0x5EED + n, n)
    assert O.sha(alg, msg) == hashlib.new(name, msg).digest()
    for kl in (0, 32, 48, 64, 128, 200):
        key = prng_bytes(0xBEEF + kl, kl)
        assert O.hmac(alg, key, msg) == pyhmac.new(key, msg, name).digest()


def test_hkdf_expand_multi_block_and_update():
    prk = prng_bytes(7, 32)
    info = b"ctx"
    # RFC 5869 expand, independently
    t, out = b"", b""
    for i in range(1, 5):
        t = pyhmac.new(prk, t + info + bytes([i]), "sha256").digest()
        out += t
    assert O.hkdf_expand(O.SHA256, prk, info, 100) == out[:100]
    nxt = O.tls13_update_traffic_secret(O.SHA384, prng_bytes(9, 48))
    assert nxt == O.tls13_hkdf_expand_label(O.SHA384, prng_bytes(9, 48), b"traffic upd", b"", 48)
