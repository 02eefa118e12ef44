"""CPU test of the table-free GF(2^128) multiply (mbedtls_amd/csrc/tlsrec_clmul.h):
tests/c/libclmul_check.so (gcc; and ROCm's clang) against the oracle's bitwise orc_gf128_mul
(the GCM multiply of SP 800-38D 6.3) on random and edge operands, the
identity element and commutativity."""
import ctypes
import os
import subprocess

import pytest

from tests.prng import prng_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang"


@pytest.fixture(scope="module", params=["libclmul_check.so", "libclmul_check_clang.so"], ids=["gcc", "clang"])
def libs(request):
    """gcc builds the portable branches of tlsrec_clmul.h; ROCm's clang the
    __clang__ ones the kernels compile (the bit reversal by builtins)"""
    if request.param.endswith("_clang.so") and not os.path.exists(CLANG):
        pytest.skip("no ROCm clang")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c"), request.param], check=True)
    c = ctypes.CDLL(os.path.join(ROOT, "tests", "c", request.param))
    import oracle as O
    return c, O


def _mul(lib, fn, x, y):
    if fn == "orc_gf128_mul":
        return lib.gf128_mul(x, y)
    out = ctypes.create_string_buffer(16)
    getattr(lib, fn)(x, y, out)
    return out.raw


def test_clmul_vs_oracle(libs):
    c, o = libs
    edge = [bytes(16), b"\x80" + bytes(15), bytes(15) + b"\x01", b"\xff" * 16, b"\x01" + bytes(15)]
    vals = edge + [prng_bytes(9100 + i, 16) for i in range(400)]
    for i, x in enumerate(vals):
        y = vals[(7 * i + 3) % len(vals)]
        assert _mul(c, "clmul_check_mul", x, y) == _mul(o, "orc_gf128_mul", x, y), (x.hex(), y.hex())


def test_clmul_identity_and_commutes(libs):
    c, _ = libs
    one = b"\x80" + bytes(15)          # the GCM string of the polynomial 1
    for i in range(50):
        x, y = prng_bytes(9600 + i, 16), prng_bytes(9700 + i, 16)
        assert _mul(c, "clmul_check_mul", x, one) == x
        assert _mul(c, "clmul_check_mul", x, y) == _mul(c, "clmul_check_mul", y, x)


def _xpow_string(bits):
    """the GCM string of sum X^j over j in bits (bit j = MSB-first bit j)"""
    v = bytearray(16)
    for j in bits:
        v[j // 8] |= 0x80 >> (j % 8)
    return bytes(v)


@pytest.mark.parametrize("fn", ["clmul_check_gtab4", "clmul_check_gtab4_quad"], ids=["entry", "quad"])
def test_gtab4_table_vs_oracle(libs, fn):
    """the 4-bit position table built from P alone (tlsrec_gtab4_*, what the
    paired GCM passes build in LDS from H^L): entry n of window k = P * sum of
    X^(4k+i) over the set bits 3-i of n, against the oracle's multiply --
    every window and entry, for H-like and edge values of P; built entry by
    entry (r05) and a quarter window per lane (r06, tlsrec_gtab4_quad)"""
    c, o = libs
    vals = [b"\x80" + bytes(15), bytes(15) + b"\x01", b"\xff" * 16] + [prng_bytes(9800 + i, 16) for i in range(12)]
    out = ctypes.create_string_buffer(8192)
    for p in vals:
        getattr(c, fn)(p, out)
        for k in range(32):
            for n in range(16):
                want = _mul(o, "orc_gf128_mul", p, _xpow_string([4 * k + i for i in range(4) if (n >> (3 - i)) & 1]))
                assert out.raw[k * 256 + 16 * n:k * 256 + 16 * n + 16] == want, (p.hex(), k, n)
