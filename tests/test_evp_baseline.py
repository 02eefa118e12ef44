"""The OpenSSL-EVP CPU-baseline leg (oracle/evp_bench.c) computes exactly what
the oracle restatement computes: same ciphertext bytes for encrypt, same
plaintext / status for decrypt (incl. a tampered record), TLS 1.2 and 1.3.
CPU only; it pins the bench's cpu_baseline to the reference semantics."""
import numpy as np
import pytest

import oracle as O
from tests.prng import prng_bytes


@pytest.mark.parametrize("cipher", O.EVP_CIPHERS)
@pytest.mark.parametrize("ver", [O.TLS1_2, O.TLS1_3])
@pytest.mark.parametrize("content", [0, 1, 100, 1400, 16383])
def test_evp_leg_matches_oracle(cipher, ver, content):
    kl = O.KEYLEN[cipher]
    key, iv = prng_bytes(cipher * 3 + ver, kl), prng_bytes(cipher * 5 + ver, 16)
    head = 8 if ver == O.TLS1_2 and cipher != O.CHACHA20_POLY1305 else 0
    inner = content + 1 + (16 - (content + 1) % 16) % 16 if ver == O.TLS1_3 else content
    wire = head + inner + 16
    stride = (wire + 127) // 128 * 128
    n, seq0 = 9, 1000
    arena = np.zeros(n * stride, dtype=np.uint8)
    for i in range(n):
        arena[i * stride + head:i * stride + head + content] = np.frombuffer(prng_bytes(i + content, content), np.uint8)
    plain = arena.copy()
    st = np.zeros(n, dtype=np.int32)
    O.evp_bench(cipher, ver, key, iv, 1, arena, stride, content, n, seq0, 3, st)
    assert (st == 0).all()
    t = O.Transform(ver, cipher, key, key, iv, iv)
    for i in range(n):
        buf = bytearray(plain[i * stride:(i + 1) * stride].tobytes())
        seq = (seq0 + i).to_bytes(8, "big")
        rec = O.Record(ctr=seq, type=23, ver=b"\x03\x03", buf=buf, data_offset=head, data_len=content)
        assert t.encrypt_buf(rec) == 0
        assert rec.data_offset == 0 and rec.data_len == wire
        assert arena[i * stride:i * stride + wire].tobytes() == rec.data(), i
    arena[2 * stride + wire - 3] ^= 1                  # tamper record 2's tag
    O.evp_bench(cipher, ver, key, iv, 0, arena, stride, wire, n, seq0, 2, st)
    assert st[2] == O.ERR_INVALID_MAC
    assert all(st[i] == 0 for i in range(n) if i != 2)
    for i in range(n):
        if i != 2:
            got = arena[i * stride + head:i * stride + head + content]
            assert got.tobytes() == plain[i * stride + head:i * stride + head + content].tobytes()
