"""The engine's exclusive scan (kernels.hip tlsrec__exclusive_scan: the
bucket pass's per-key offsets and the stream / DTLS record offsets; it
replaced hipcub::DeviceScan) against numpy, at chunk edges and at the sizes
the engine scans (10 classes x 64 K keys + 2; 256 K connections + 1)."""
import ctypes

import numpy as np
import pytest

from mbedtls_amd import _abi

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 2, 255, 256, 4095, 4096, 4097, 8192 + 17, 10 * 65536 + 2, 262145, 1 << 21])
def test_exclusive_scan_matches_numpy(n):
    lib = _abi.test_library()     # self-test entry points: the test-hooks build
    f = lib.tlsrec__test_scan
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    rng = np.random.default_rng(n)
    # sparse like the bucket counts (most keys of most classes empty), with bursts
    x = np.where(rng.random(n) < 0.2, rng.integers(0, 300, n), 0).astype(np.uint32)
    x[rng.integers(0, n, 3)] = 4096
    out = np.zeros(n, dtype=np.uint32)
    assert f(x.ctypes.data, n, out.ctypes.data) == 0
    want = np.concatenate([[0], np.cumsum(x.astype(np.uint64))[:-1]]).astype(np.uint32)
    assert np.array_equal(out, want), np.flatnonzero(out != want)[:5]
