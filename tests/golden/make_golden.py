#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py

Sources of truth, in order:
  1. reference_kats.json -- the reference's own TLS 1.3 record KATs,
     transcribed (data only) from /root/reference/tests/suites/
     test_suite_ssl.data:2776-2834 (ssl_tls13_record_protection).  Those
     vectors originate from tls13.ulfheim.net and RFC 8448 section 3.
  2. standard_vectors.json -- FIPS-197 C.1/C.3, the GCM specification test
     cases 2/4/14 and RFC 8439 2.3.2/2.5.2/2.8.2 (transcribed from the
     published standards).
  3. records.json -- record-layer vectors for every (cipher, TLS version) pair
     at the SURVEY.md 8c lengths, produced by the oracle restatement and
     accepted only if OpenSSL libcrypto (an independent implementation)
     reproduces the AEAD output bit for bit.

This script needs the oracle (gcc-built) and libcrypto; the GPU box only
reads the resulting JSON.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402
from tests import _openssl as S  # noqa: E402
from tests.test_camellia_oracle import ccm_ref, gcm_ref  # noqa: E402
from tests.prng import prng_bytes  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

REFERENCE_KATS = [
    # name, endpoint, ctr, server_key, server_iv, client_key, client_iv, plaintext, ciphertext
    ("ulfheim_1", "client", 0, "0b6d22c8ff68097ea871c672073773bf", "1b13dd9f8d8f17091d34b349",
     "49134b95328f279f0183860589ac6707", "bc4dd5f7b98acff85466261d", "70696e67",
     "c74061535eb12f5f25a781957874742ab7fb305dd5"),
    ("ulfheim_2", "server", 1, "0b6d22c8ff68097ea871c672073773bf", "1b13dd9f8d8f17091d34b349",
     "49134b95328f279f0183860589ac6707", "bc4dd5f7b98acff85466261d", "706f6e67",
     "370e5f168afa7fb16b663ecdfca3dbb81931a90ca7"),
    ("rfc8448_1", "client", 0, "9f02283b6c9c07efc26bb9f2ac92e356", "cf782b88dd83549aadf1e984",
     "17422dda596ed5d9acd890e3c63f5051", "5b78923dee08579033e523d9",
     "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f202122232425262728292a2b2c2d2e2f3031",
     "a23f7054b62c94d0affafe8228ba55cbefacea42f914aa66bcab3f2b9819a8a5b46b395bd54a9a20441e2b62974e1f5a6292a2977014bd1e3deae63aeebb21694915e4"),
    ("rfc8448_2", "server", 1, "9f02283b6c9c07efc26bb9f2ac92e356", "cf782b88dd83549aadf1e984",
     "17422dda596ed5d9acd890e3c63f5051", "5b78923dee08579033e523d9",
     "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f202122232425262728292a2b2c2d2e2f3031",
     "2e937e11ef4ac740e538ad36005fc4a46932fc3225d05f82aa1b36e30efaf97d90e6dffc602dcb501a59a8fcc49c4bf2e5f0a21c0047c2abf332540dd032e167c2955d"),
]

STANDARD = {
    "aes_block": [
        # FIPS-197 Appendix C.1 / C.3
        {"key": "000102030405060708090a0b0c0d0e0f", "pt": "00112233445566778899aabbccddeeff",
         "ct": "69c4e0d86a7b0430d8cdb78070b4c55a"},
        {"key": "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
         "pt": "00112233445566778899aabbccddeeff", "ct": "8ea2b7ca516745bfeafc49904b496089"},
    ],
    "gcm": [
        # GCM specification (McGrew & Viega) test cases 2, 4 and 14
        {"key": "00000000000000000000000000000000", "iv": "000000000000000000000000", "aad": "",
         "pt": "00000000000000000000000000000000", "ct": "0388dace60b6a392f328c2b971b2fe78",
         "tag": "ab6e47d42cec13bdf53a67b21257bddf"},
        {"key": "feffe9928665731c6d6a8f9467308308", "iv": "cafebabefacedbaddecaf888",
         "aad": "feedfacedeadbeeffeedfacedeadbeefabaddad2",
         "pt": "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a721c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b39",
         "ct": "42831ec2217774244b7221b784d0d49ce3aa212f2c02a4e035c17e2329aca12e21d514b25466931c7d8f6a5aac84aa051ba30b396a0aac973d58e091",
         "tag": "5bc94fbc3221a5db94fae95ae7121a47"},
        {"key": "0000000000000000000000000000000000000000000000000000000000000000",
         "iv": "000000000000000000000000", "aad": "",
         "pt": "00000000000000000000000000000000", "ct": "cea7403d4d606b6e074ec5d3baf39d18",
         "tag": "d0d1c8a799996bf0265b98b5d48ab919"},
    ],
    "ccm": [
        # NIST SP 800-38C Appendix C, Example 3 (12-byte nonce, 8-byte tag)
        {"key": "404142434445464748494a4b4c4d4e4f", "nonce": "101112131415161718191a1b",
         "aad": "000102030405060708090a0b0c0d0e0f10111213",
         "pt": "202122232425262728292a2b2c2d2e2f3031323334353637",
         "ct": "e3b201a9f5b71a7a9b1ceaeccd97e70b6176aad9a4428aa5", "tag": "484392fbc1b09951"},
    ],
    "chacha20_block": [
        # RFC 8439 2.3.2 (first 16 bytes of the serialized block)
        {"key": "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
         "counter": 1, "nonce": "000000090000004a00000000", "out16": "10f1e7e4d13b5915500fdd1fa32071c4"},
    ],
    "poly1305": [
        # RFC 8439 2.5.2
        {"key": "85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b",
         "msg": "43727970746f6772617068696320466f72756d2052657365617263682047726f7570",
         "tag": "a8061dc1305136c6c22b8baf0c0127a9"},
    ],
    "chachapoly": [
        # RFC 8439 2.8.2
        {"key": "808182838485868788898a8b8c8d8e8f909192939495969798999a9b9c9d9e9f",
         "nonce": "070000004041424344454647", "aad": "50515253c0c1c2c3c4c5c6c7",
         "pt": ("4c616469657320616e642047656e746c656d656e206f662074686520636c617373206f66202739393a"
                "204966204920636f756c64206f6666657220796f75206f6e6c79206f6e652074697020666f722074"
                "6865206675747572652c2073756e73637265656e20776f756c642062652069742e"),
         "ct16": "d31a8d34648e60db7b86afbc53ef7ec2", "tag": "1ae10b594f09e26a7e902ecbd0600691"},
    ],
}

CIPHERS = {"AES-128-GCM": O.AES_128_GCM, "AES-256-GCM": O.AES_256_GCM,
           "CHACHA20-POLY1305": O.CHACHA20_POLY1305,
           # SURVEY 8(f)-2 (appended: the seeds of the cases above stay unchanged)
           "AES-192-GCM": O.AES_192_GCM, "AES-128-CCM": O.AES_128_CCM, "AES-192-CCM": O.AES_192_CCM,
           "AES-256-CCM": O.AES_256_CCM, "AES-128-CCM-8": O.AES_128_CCM_8, "AES-192-CCM-8": O.AES_192_CCM_8,
           "AES-256-CCM-8": O.AES_256_CCM_8,
           # ARIA-GCM / ARIA-CCM (appended likewise)
           "ARIA-128-GCM": O.ARIA_128_GCM, "ARIA-192-GCM": O.ARIA_192_GCM, "ARIA-256-GCM": O.ARIA_256_GCM,
           "ARIA-128-CCM": O.ARIA_128_CCM, "ARIA-192-CCM": O.ARIA_192_CCM, "ARIA-256-CCM": O.ARIA_256_CCM,
           # Camellia-GCM / Camellia-CCM (appended likewise; OpenSSL has no Camellia AEAD, so the
           # cross-check is SP 800-38D / 38C assembled on OpenSSL Camellia-ECB/-CBC,
           # tests/test_camellia_oracle.py gcm_ref / ccm_ref)
           "CAMELLIA-128-GCM": O.CAMELLIA_128_GCM, "CAMELLIA-192-GCM": O.CAMELLIA_192_GCM,
           "CAMELLIA-256-GCM": O.CAMELLIA_256_GCM, "CAMELLIA-128-CCM": O.CAMELLIA_128_CCM,
           "CAMELLIA-192-CCM": O.CAMELLIA_192_CCM, "CAMELLIA-256-CCM": O.CAMELLIA_256_CCM}
VERSIONS = {"TLS1.2": O.TLS1_2, "TLS1.3": O.TLS1_3}
LENGTHS = [0, 1, 15, 16, 17, 1400, 16383]
SEED = 0x7115EC0DE


def _keylen(c):
    return O.KEYLEN[c]


def make_records():
    out = []
    case = 0
    for cname, c in CIPHERS.items():
        for vname, v in VERSIONS.items():
            for L in LENGTHS:
                for rep in range(2):
                    seed = SEED + case
                    case += 1
                    rnd = prng_bytes(seed, 32 + 32 + 16 + 16 + 8)
                    key_enc = rnd[:_keylen(c)]
                    key_dec = rnd[32:32 + _keylen(c)]
                    iv_enc, iv_dec = rnd[64:80], rnd[80:96]
                    ctr = rnd[96:104]
                    payload = prng_bytes(seed ^ 0xA5A5, L)
                    rtype = 23 if rep == 0 else 22
                    t = O.Transform(v, c, key_enc, key_dec, iv_enc, iv_dec)
                    head = 8 if (v == O.TLS1_2 and c != O.CHACHA20_POLY1305) else 0
                    buf = bytearray(head + L + 64)
                    buf[head:head + L] = payload
                    rec = O.Record(ctr=ctr, type=rtype, ver=b"\x03\x03", buf=buf,
                                   data_offset=head, data_len=L)
                    r = t.encrypt_buf(rec)
                    assert r == 0, (cname, vname, L, r)
                    wire = rec.data()
                    # independent AEAD cross-check (OpenSSL)
                    if v == O.TLS1_3:
                        g = 16
                        pad = (g - (L + 1) % g) % g
                        inner = payload + bytes([rtype]) + bytes(pad)
                        aad = bytes([23, 3, 3]) + (len(inner) + O.TAGLEN[c]).to_bytes(2, "big")
                        nonce = bytes(a ^ b for a, b in zip(iv_enc[:12], bytes(4) + ctr))
                        body = wire
                    else:
                        inner = payload
                        aad = ctr + bytes([rtype, 3, 3]) + L.to_bytes(2, "big")
                        if c == O.CHACHA20_POLY1305:
                            nonce = bytes(a ^ b for a, b in zip(iv_enc[:12], bytes(4) + ctr))
                            body = wire
                        else:
                            nonce = iv_enc[:4] + ctr
                            assert wire[:8] == ctr
                            body = wire[8:]
                    tl = O.TAGLEN[c]
                    if c >= O.CAMELLIA_128_CCM:
                        ct, tag = ccm_ref(key_enc, nonce, aad, inner, tl)
                    elif c >= O.CAMELLIA_128_GCM:
                        ct, tag = gcm_ref(key_enc, nonce, aad, inner)
                    elif O.AES_128_CCM <= c <= O.AES_256_CCM_8:
                        ct, tag = S.ccm_seal(key_enc, nonce, aad, inner, tl)
                    elif c >= O.ARIA_128_CCM:
                        ct, tag = S.ccm_seal(key_enc, nonce, aad, inner, tl, name="aria-ccm")
                    elif c >= O.ARIA_128_GCM:
                        ct, tag = S.seal("aria-gcm", key_enc, nonce, aad, inner)
                    else:
                        name = "gcm" if c != O.CHACHA20_POLY1305 else "chacha"
                        ct, tag = S.seal(name, key_enc, nonce, aad, inner)
                    assert body == ct + tag, (cname, vname, L)
                    ent = {"cipher": cname, "version": vname, "len": L, "seed": seed,
                           "key_enc": key_enc.hex(), "key_dec": key_dec.hex(),
                           "iv_enc": iv_enc.hex(), "iv_dec": iv_dec.hex(),
                           "ctr": ctr.hex(), "type": rtype,
                           "out_offset": rec.data_offset, "out_len": rec.data_len,
                           "out_type": rec.type,
                           "wire_sha256": hashlib.sha256(wire).hexdigest(),
                           "tag": wire[-O.TAGLEN[c]:].hex()}
                    if L <= 64:
                        ent["payload"] = payload.hex()
                        ent["wire"] = wire.hex()
                    out.append(ent)
    return out


def main():
    assert S.lib() is not None, "libcrypto needed to generate fixtures"
    kats = [dict(zip(("name", "endpoint", "ctr", "server_key", "server_iv", "client_key",
                      "client_iv", "plaintext", "ciphertext"), k)) for k in REFERENCE_KATS]
    for k in kats:
        k["source"] = "/root/reference/tests/suites/test_suite_ssl.data:2776-2834"
    with open(os.path.join(OUT, "reference_kats.json"), "w") as f:
        json.dump(kats, f, indent=1)
    with open(os.path.join(OUT, "standard_vectors.json"), "w") as f:
        json.dump(STANDARD, f, indent=1)
    recs = make_records()
    with open(os.path.join(OUT, "records.json"), "w") as f:
        json.dump({"seed": SEED, "prng": "splitmix64 (tests/prng.py)", "cases": recs}, f, indent=0)
    print(f"wrote {len(kats)} KATs, {len(recs)} record vectors")


if __name__ == "__main__":
    main()
