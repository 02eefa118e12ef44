"""Session-ticket oracle (oracle/ticket.c) against OpenSSL as an independent
AEAD and the checks of library/ssl_ticket.c (the reference has no ticket KAT:
its IV is random, so parity is pinned through the AEAD primitives)."""
import pytest

import oracle as O
from tests import _openssl as S
from tests import test_camellia_oracle as CAM
from tests.prng import prng_bytes

KEYSETS = [(O.AES_256_GCM, O.CHACHA20_POLY1305), (O.AES_128_GCM, O.AES_128_CCM), (O.AES_256_CCM, O.AES_192_GCM),
           (O.ARIA_128_GCM, O.ARIA_256_CCM), (O.CAMELLIA_256_GCM, O.CAMELLIA_128_CCM)]


def _keys(ciphers, seed=1):
    return [(c, prng_bytes(seed + i, O.KEYLEN[c]), bytes([65 + i, 66, 67, 68 + seed])) for i, c in enumerate(ciphers)]


@pytest.mark.parametrize("ciphers", KEYSETS)
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 100, 300, 1000])
def test_write_vs_openssl_and_parse(ciphers, n):
    keys = _keys(ciphers)
    for active in (0, 1):
        iv, st = prng_bytes(10 + n, 12), prng_bytes(20 + n, n)
        r, t = O.ticket_write(keys, active, iv, st, 34 + n + 7)
        assert r == 0 and len(t) == 34 + n and t[:4] == keys[active][2] and t[4:16] == iv
        c, k = keys[active][0], keys[active][1]
        if c == O.CHACHA20_POLY1305:
            ct, tag = S.seal("chacha", k, iv, t[:18], st)
        elif c in (O.AES_128_CCM, O.AES_192_CCM, O.AES_256_CCM):
            ct, tag = S.ccm_seal(k, iv, t[:18], st, 16)
        elif c in (O.ARIA_128_GCM, O.ARIA_192_GCM, O.ARIA_256_GCM):
            ct, tag = S.seal("aria-gcm", k, iv, t[:18], st)
        elif c in (O.ARIA_128_CCM, O.ARIA_192_CCM, O.ARIA_256_CCM):
            ct, tag = S.ccm_seal(k, iv, t[:18], st, 16, name="aria-ccm")
        elif c in (O.CAMELLIA_128_GCM, O.CAMELLIA_192_GCM, O.CAMELLIA_256_GCM):
            ct, tag = CAM.gcm_ref(k, iv, t[:18], st)     # SP 800-38D over OpenSSL Camellia-ECB
        elif c in (O.CAMELLIA_128_CCM, O.CAMELLIA_192_CCM, O.CAMELLIA_256_CCM):
            ct, tag = CAM.ccm_ref(k, iv, t[:18], st)     # SP 800-38C over OpenSSL Camellia
        else:
            ct, tag = S.seal("gcm", k, iv, t[:18], st)
        assert t[18:] == ct + tag
        r2, clear, _ = O.ticket_parse(keys, t)
        assert r2 == 0 and clear == st


def test_checks():
    keys = _keys(KEYSETS[0])
    st = prng_bytes(5, 50)
    assert O.ticket_write(keys, 0, bytes(12), st, 33)[0] == O.ERR_BUFFER_TOO_SMALL      # CHK_BUF_PTR
    assert O.ticket_write(keys, 0, bytes(12), st, 34 + 49)[0] == O.ERR_BUFFER_TOO_SMALL  # no tag room
    r, t = O.ticket_write(keys, 1, bytes(12), st, 200)
    assert O.ticket_parse(keys, t[:33])[0] == O.ERR_BAD_INPUT_DATA                       # < TICKET_MIN_LEN
    assert O.ticket_parse(keys, t + b"x")[0] == O.ERR_BAD_INPUT_DATA                     # length field mismatch
    assert O.ticket_parse(keys, b"zzzz" + t[4:])[0] == O.ERR_SESSION_TICKET_EXPIRED      # unknown key name
    bad = t[:40] + bytes([t[40] ^ 1]) + t[41:]
    r2, _, after = O.ticket_parse(keys, bad)
    assert r2 == O.ERR_INVALID_MAC and after[18:18 + 50] == bytes(50)                   # output cleared
