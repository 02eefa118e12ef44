"""The cross-lane helpers of tlsrec_recdev.h (DPP quad_perm / row_shl /
row_mirror / row_half_mirror and v_permlane16/32_swap, which replaced
ds_bpermute in the GHASH lane tree, the wave reductions and the Poly1305 lane
sum) against their intended lane maps, through the library's self-test kernel
tlsrec__test_lane_ops."""
import ctypes

import numpy as np
import pytest

from mbedtls_amd import _abi

pytestmark = pytest.mark.gpu


def test_lane_ops_match_their_lane_maps():
    lib = _abi.test_library()     # self-test entry points: the test-hooks build
    out = np.zeros(17 * 64, dtype=np.uint32)
    f = lib.tlsrec__test_lane_ops
    f.argtypes = [ctypes.c_void_p]
    assert f(out.ctypes.data) == 0
    o = out.reshape(17, 64)
    lane = np.arange(64)
    v = ((lane * 37 + 11) & 63) + 100 * lane
    # butterfly partners: xor 1, xor 2, mirror in 8, mirror in 16, xor 16, xor 32
    assert (o[0] == v[lane ^ 1]).all()
    assert (o[1] == v[lane ^ 2]).all()
    assert (o[2] == v[(lane & ~7) | (7 - (lane & 7))]).all()
    assert (o[3] == v[(lane & ~15) | (15 - (lane & 15))]).all()
    assert (o[4] == v[lane ^ 16]).all()
    assert (o[5] == v[lane ^ 32]).all()
    # from_up<SH>: lane i gets lane i + SH for the lanes the tree reads
    for k, sh in enumerate((1, 2, 4, 8, 16, 32)):
        q = lane % (2 * sh)
        use = q < sh
        assert (o[6 + k][use] == v[lane[use] + sh]).all(), sh
    assert (o[12] == v.max()).all() and (o[13] == v.min()).all()
    assert (o[14] == v.reshape(8, 8).max(axis=1).repeat(8)).all()
    bits = (1 << (lane & 31)).astype(np.uint64)
    assert (o[15] == np.bitwise_or.reduce(bits.reshape(16, 4), axis=1).repeat(4)).all()
    assert (o[16] == v.reshape(8, 8).sum(axis=1).repeat(8)).all()
