"""GPU parity of the TLS 1.3 key schedule (keysched.hip, through the C ABI):
the reference's own vectors (tests/golden/tls13_keys.json), the oracle on
random inputs, the reference's argument checks, and the batch derivation
into a key table checked end to end by record encryption."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import mbedtls_amd as M  # noqa: E402
from mbedtls_amd import keysched as K  # noqa: E402
import oracle as O  # noqa: E402
from tests import batchlib as B  # noqa: E402
from tests.prng import prng_bytes  # noqa: E402

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "tls13_keys.json")))
X = bytes.fromhex
ALG = {"sha256": K.ALG_SHA_256, "sha384": K.ALG_SHA_384}


@pytest.mark.parametrize("v", G["expand_label"], ids=lambda v: v["where"])
def test_expand_label_vectors(v):
    got = K.hkdf_expand_label(ALG[v["hash"]], X(v["secret"]), v["label"].encode(), X(v["ctx"]), v["len"])
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("v", G["derive_secret"], ids=lambda v: v["name"])
def test_derive_secret_vectors(v):
    got = K.derive_secret(ALG[v["hash"]], X(v["secret"]), v["label"].encode(), X(v["ctx"]), v["ctx_hashed"], v["len"])
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("v", G["evolve"], ids=lambda v: v["where"])
def test_evolve_vectors(v):
    got = K.evolve_secret(ALG[v["hash"]], X(v["secret"]) or None, X(v["input"]) or None)
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("v", G["traffic_keys"], ids=lambda v: v["where"])
def test_traffic_key_vectors(v):
    ck, ci, sk, si = K.make_traffic_keys(ALG[v["hash"]], X(v["client_secret"]), X(v["server_secret"]),
                                         v["key_len"], v["iv_len"])
    assert (ck.hex(), ci.hex(), sk.hex(), si.hex()) == (v["client_key"], v["client_iv"], v["server_key"],
                                                        v["server_iv"])


@pytest.mark.parametrize("v", G["exporter"], ids=lambda v: v["where"])
def test_exporter_vectors(v):
    got = K.exporter(ALG[v["hash"]], X(v["secret"]), v["label"].encode(), v["context"].encode(), v["len"])
    assert got.hex() == v["expected"]


@pytest.mark.parametrize("alg", [K.ALG_SHA_256, K.ALG_SHA_384])
def test_random_vs_oracle(alg):
    H = K.HASH_LEN[alg]
    for i, (ll, cl, n, sl) in enumerate([(0, 0, 1, H), (1, 0, 12, H), (11, 32, 16, H), (249, 64, 100, H),
                                         (5, 48, 255, 200), (7, 0, 3 * H + 5, 10), (30, 1, 1000, 129)]):
        sec, lab, ctx = prng_bytes(100 + i, sl), prng_bytes(200 + i, ll), prng_bytes(300 + i, cl)
        assert K.hkdf_expand_label(alg, sec, lab, ctx, n) == O.tls13_hkdf_expand_label(alg, sec, lab, ctx, n)
        for hashed in (0, 1):
            c2 = prng_bytes(400 + i, 300) if hashed == 0 else ctx
            assert (K.derive_secret(alg, sec[:H], lab, c2, hashed, H) ==
                    O.tls13_derive_secret(alg, sec[:H], lab, c2, hashed, H))
        assert K.update_traffic_secret(alg, sec[:H]) == O.tls13_update_traffic_secret(alg, sec[:H])
        inp = prng_bytes(500 + i, 3 * i)
        assert K.evolve_secret(alg, sec[:H], inp) == O.tls13_evolve_secret(alg, sec[:H], inp)
        assert K.exporter(alg, sec[:H], lab[:40], ctx, 40) == O.tls13_exporter(alg, sec[:H], lab[:40], ctx, 40)


def test_argument_checks():
    """ssl_tls13_keys.c:152-171: oversized label / context / length are
    INTERNAL_ERROR, a non-hash algorithm BAD_INPUT_DATA."""
    s = bytes(32)
    with pytest.raises(K.KeyScheduleError) as e:
        K.hkdf_expand_label(K.ALG_SHA_256, s, bytes(250), b"", 16)
    assert e.value.code == M.ERR_SSL_INTERNAL_ERROR
    with pytest.raises(K.KeyScheduleError) as e:
        K.hkdf_expand_label(K.ALG_SHA_256, s, b"key", bytes(65), 16)
    assert e.value.code == M.ERR_SSL_INTERNAL_ERROR
    with pytest.raises(K.KeyScheduleError) as e:
        K.hkdf_expand_label(K.ALG_SHA_256, s, b"key", b"", 255 * 64 + 1)
    assert e.value.code == M.ERR_SSL_INTERNAL_ERROR
    with pytest.raises(K.KeyScheduleError) as e:
        K.hkdf_expand_label(0x05500200, s, b"key", b"", 16)
    assert e.value.code == M.ERR_SSL_BAD_INPUT_DATA


@pytest.mark.parametrize("cipher", list(B.CIPHERS.values()))
@pytest.mark.parametrize("update", [False, True])
def test_keytab_derive_end_to_end(cipher, update):
    """Device secrets -> (KeyUpdate) -> key/iv -> key table -> record
    encryption, against the oracle's key schedule + record layer."""
    n = 300
    alg = K.ALG_SHA_384 if cipher == M.CIPHER_AES_256_GCM else K.ALG_SHA_256
    H = K.HASH_LEN[alg]
    raw = prng_bytes(0xD0 + cipher + 7 * update, n * 48)
    secrets = torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).cuda()
    kt = M.KeyTable(n + 5)
    K.keytab_derive(kt, 5, n, cipher, secrets, key_update=update)
    torch.cuda.synchronize()
    got_secrets = secrets.cpu().numpy().tobytes()
    slots = [(cipher, M.VERSION_TLS1_3, bytes(16), bytes(12), 0)] * 5
    klen = M.KEYLEN[cipher]
    for i in range(n):
        s = raw[48 * i:48 * i + H]
        if update:
            s = O.tls13_update_traffic_secret(alg, s)
            assert got_secrets[48 * i:48 * i + H] == s
        else:
            assert got_secrets[48 * i:48 * i + 48] == raw[48 * i:48 * i + 48]
        key = O.tls13_hkdf_expand_label(alg, s, b"key", b"", klen)
        iv = O.tls13_hkdf_expand_label(alg, s, b"iv", b"", 12)
        slots.append((cipher, M.VERSION_TLS1_3, key, iv, 0))
    lengths = [int(x) % 1500 for x in np.frombuffer(prng_bytes(9, 2 * n), dtype=np.uint16)]
    recs = B.plaintext_records(slots[5:], lengths, seed=77)
    for r in recs:
        r.slot += 5
    b = B.Batch(slots, recs)
    out, res = b.run_gpu(False, kt=kt)
    assert b.compare(False, out, res) == []
    kt.close()
