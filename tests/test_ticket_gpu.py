"""GPU parity of the session-ticket batch (ticket.hip through the C ABI)
against the oracle's restatement of ssl_ticket.c: byte-exact tickets,
statuses and lengths, parse results, every check."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import mbedtls_amd as M  # noqa: E402
from mbedtls_amd import ticket as T  # noqa: E402
import oracle as O  # noqa: E402
from tests.prng import prng_bytes  # noqa: E402

KEYSETS = [(M.CIPHER_AES_256_GCM, M.CIPHER_CHACHA20_POLY1305), (M.CIPHER_AES_128_GCM, M.CIPHER_AES_128_CCM),
           (M.CIPHER_AES_256_CCM, M.CIPHER_AES_192_GCM),
           # every AEAD key type of mbedtls_ssl_ticket_setup (ssl_ticket.c:188-209), incl. the
           # kernel's LDS-image variants: ARIA only, Camellia only, ARIA + Camellia, AES + Camellia
           (M.CIPHER_ARIA_128_GCM, M.CIPHER_ARIA_256_CCM), (M.CIPHER_CAMELLIA_256_GCM, M.CIPHER_CAMELLIA_128_CCM),
           (M.CIPHER_ARIA_192_GCM, M.CIPHER_CAMELLIA_192_GCM), (M.CIPHER_AES_128_GCM, M.CIPHER_CAMELLIA_256_CCM)]
KEYSET_IDS = ["gcm256-chacha", "gcm128-ccm128", "ccm256-gcm192", "aria", "camellia", "aria-camellia", "aes-camellia"]


def _setup(ciphers, seed):
    okeys = [(c, prng_bytes(seed + i, M.KEYLEN[c]), bytes([80 + i, 81, 82, 83 + seed % 7])) for i, c in
             enumerate(ciphers)]
    kt = M.KeyTable(4)
    km = np.concatenate([M.key_material(c, M.VERSION_TLS1_3, k, bytes(12)) for c, k, _ in okeys])
    kt.load(km, first=1)
    return okeys, kt


def _arena(items, space_of):
    offs, pos = [], 0
    for it in items:
        offs.append(pos)
        pos += (space_of(it) + 127) // 128 * 128 + 128
    return offs, np.zeros(max(pos, 16), dtype=np.uint8)


@pytest.mark.parametrize("ciphers", KEYSETS, ids=KEYSET_IDS)
def test_write_parse_batch(ciphers):
    okeys, kt = _setup(ciphers, 3)
    rng = np.random.default_rng(11)
    jobs = []   # (iv, state, space)
    for i in range(700):
        n = int(rng.choice([0, 1, 15, 16, 17, 64, 100, 257, 1000]))
        space = 34 + n + int(rng.integers(0, 40))
        if i % 50 == 7:
            space = int(rng.integers(0, 34))              # CHK_BUF_PTR
        elif i % 50 == 9:
            space = 34 + n - int(rng.integers(1, 16)) if n > 16 else space   # no room for the tag
        jobs.append((prng_bytes(100 + i, 12), prng_bytes(200 + i, n), space))
    dev = torch.device("cuda")
    for active in (0, 1):
        keys = T.ticket_keys([1, 2], [okeys[0][2], okeys[1][2]], active)
        offs, a = _arena(jobs, lambda j: max(j[2], 18 + len(j[1])))
        d = np.zeros(len(jobs), dtype=T.TICKET)
        for i, ((iv, st, space), o) in enumerate(zip(jobs, offs)):
            a[o + 4:o + 16] = np.frombuffer(iv, np.uint8)
            a[o + 18:o + 18 + len(st)] = np.frombuffer(st, np.uint8)
            d[i] = (o, space, len(st))
        ta = torch.from_numpy(a).to(dev)
        res = torch.zeros(len(jobs) * 16, dtype=torch.uint8, device=dev)
        T.write(kt, keys, d, len(jobs), ta, res)
        torch.cuda.synchronize()
        out = ta.cpu().numpy()
        r = res.cpu().numpy().view(T.TICKET_RES)
        tickets = []
        for i, ((iv, st, space), o) in enumerate(zip(jobs, offs)):
            want_st, want = O.ticket_write(okeys, active, iv, st, space)
            assert int(r["status"][i]) == want_st, i
            if want_st == 0:
                assert int(r["tlen"][i]) == len(want)
                assert out[o:o + len(want)].tobytes() == want, i
                tickets.append((o, len(want), want))
        # parse what the GPU wrote, plus damaged copies
        pj = []
        for k, (o, tl, w) in enumerate(tickets):
            t = w
            if k % 9 == 1:
                t = w[:20] + bytes([w[20] ^ 4]) + w[21:] if tl > 20 else w
            elif k % 9 == 2:
                t = b"nope" + w[4:]
            elif k % 9 == 3:
                t = w[:-1]
            pj.append(t)
        offs2, a2 = _arena(pj, len)
        d2 = np.zeros(len(pj), dtype=T.TICKET)
        for i, (t, o) in enumerate(zip(pj, offs2)):
            a2[o:o + len(t)] = np.frombuffer(t, np.uint8)
            d2[i] = (o, len(t), 0)
        ta2 = torch.from_numpy(a2).to(dev)
        res2 = torch.zeros(len(pj) * 16, dtype=torch.uint8, device=dev)
        T.parse(kt, keys, d2, len(pj), ta2, res2)
        torch.cuda.synchronize()
        out2 = ta2.cpu().numpy()
        r2 = res2.cpu().numpy().view(T.TICKET_RES)
        for i, (t, o) in enumerate(zip(pj, offs2)):
            want_st, clear, after = O.ticket_parse(okeys, t)
            assert int(r2["status"][i]) == want_st, (i, int(r2["status"][i]), want_st)
            assert out2[o:o + len(t)].tobytes() == after, i
            if want_st == 0:
                assert int(r2["tlen"][i]) == len(clear)
    kt.close()
