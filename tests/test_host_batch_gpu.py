"""tlsrec_host_batch_encrypt / _decrypt: records in host memory (the
socket-buffer boundary), chunked H2D -> kernels -> D2H on three streams.
Bit-exact against the oracle for every record, with chunks small enough that
a batch spans many chunks and every device slot is reused, pinned arenas
(kernels write the output straight into host memory) and pageable ones
(chunks copied back), in place and into a second arena; out-of-order
descriptors are refused."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import mbedtls_amd as M  # noqa: E402
from tests import batchlib as B  # noqa: E402
from tests.prng import prng_bytes  # noqa: E402


def _host_run(b, decrypt, chunk, pinned, inplace, lanes=0):
    kt = M.KeyTable(len(b.slots))
    kt.load(b.key_materials())
    if pinned:
        arena = torch.from_numpy(b.arena.copy()).pin_memory()
        out = arena if inplace else torch.zeros_like(arena).pin_memory()
        a_np, o_np = arena.numpy(), out.numpy()
    else:
        a_np = b.arena.copy()
        o_np = a_np if inplace else np.zeros_like(a_np)
    res = M.results(len(b.recs))
    M.host_batch(decrypt, kt, b.desc, res, len(b.recs), a_np, o_np, lanes=lanes, chunk_bytes=chunk)
    kt.close()
    return o_np.copy(), res


@pytest.mark.parametrize("decrypt", [False, True], ids=["enc", "dec"])
@pytest.mark.parametrize("pinned", [True, False], ids=["pinned", "pageable"])
def test_host_batch_vs_oracle(decrypt, pinned):
    ciphers = [M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305, M.CIPHER_AES_128_CCM_8, M.CIPHER_CAMELLIA_128_GCM]
    slots = B.random_slots(0x4057, ciphers, [M.VERSION_TLS1_2, M.VERSION_TLS1_3], 12)
    lengths = [int(x) for x in np.frombuffer(prng_bytes(0x4058, 2 * 300), np.uint16) % 5000] + [16383, 0, 1]
    recs = B.sealed_records(slots, lengths, seed=91)[0] if decrypt else B.plaintext_records(slots, lengths, seed=91)
    if decrypt:
        for i in range(0, len(recs), 13):
            recs[i].buf[recs[i].data_offset + 3] ^= 0x20
    b = B.Batch(slots, recs, align=128)
    for chunk in (0, 64 << 10, 300 << 10):
        out, res = _host_run(b, decrypt, chunk, pinned, inplace=True)
        bad = b.compare(decrypt, out, res)
        assert not bad, f"chunk={chunk}: " + "; ".join(bad[:5])
    out, res = _host_run(b, decrypt, 100 << 10, pinned, inplace=False)
    # pinned output: the kernels write into it directly (the bytes the device
    # batch API writes out of place); pageable: whole chunks copied back
    bad = b.compare(decrypt, out, res, inplace=not pinned)
    assert not bad, "; ".join(bad[:5])


def test_host_batch_rejects_unordered():
    slots = B.random_slots(0x4059, [M.CIPHER_AES_128_GCM], [M.VERSION_TLS1_3], 1)
    b = B.Batch(slots, B.plaintext_records(slots, [100, 200, 300], seed=1))
    d = b.desc.copy()
    d["buf_off"][[0, 1]] = d["buf_off"][[1, 0]]
    kt = M.KeyTable(1)
    kt.load(b.key_materials())
    with pytest.raises(RuntimeError):
        M.host_batch(False, kt, d, M.results(3), 3, b.arena.copy(), None)
    kt.close()
