/*
 * camellia.c -- Camellia block cipher (RFC 3713), TEST INFRASTRUCTURE ONLY.
 *
 * The reference reaches Camellia through PSA (PSA_KEY_TYPE_CAMELLIA with
 * PSA_ALG_GCM / PSA_ALG_CCM, mbedtls_ssl_cipher_to_psa, library/ssl_tls.c:
 * 2290-2345); the implementation lives in the absent TF-PSA-Crypto, so this
 * restates the published cipher (RFC 3713 section 2):
 *   - SBOX1 (the 256-byte table of RFC 3713 2.4.4), SBOX2 = SBOX1 <<< 1,
 *     SBOX3 = SBOX1 <<< 7, SBOX4(x) = SBOX1(x <<< 1);
 *   - F = S-layer (SBOX 1 2 3 4 2 3 4 1 on bytes t1..t8) then the P-layer;
 *   - FL / FL^-1 between every 6 rounds;
 *   - key schedule: KA / KB from Sigma1..Sigma6, subkeys by 128-bit rotations
 *     of KL, KR, KA, KB (RFC 3713 2.2, 2.3).
 * 18 rounds for 128-bit keys, 24 for 192 / 256.  Pinned by the RFC 3713
 * Appendix A vectors and OpenSSL's EVP Camellia (tests/test_camellia_oracle.py).
 *
 * Context: orc_aes_ctx with kind = 2, nr = 18 / 24, and the 64-bit subkeys in
 * ark as big-endian 8-byte strings in use order:
 *   kw1 kw2 | k1..k6 | ke1 ke2 | k7..k12 | ke3 ke4 | k13..k18
 *   [| ke5 ke6 | k19..k24] | kw3 kw4       (26 or 34 subkeys)
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

static const uint8_t SBOX1[256] = {
    112, 130,  44, 236, 179,  39, 192, 229, 228, 133,  87,  53, 234,  12, 174,  65,
     35, 239, 107, 147,  69,  25, 165,  33, 237,  14,  79,  78,  29, 101, 146, 189,
    134, 184, 175, 143, 124, 235,  31, 206,  62,  48, 220,  95,  94, 197,  11,  26,
    166, 225,  57, 202, 213,  71,  93,  61, 217,   1,  90, 214,  81,  86, 108,  77,
    139,  13, 154, 102, 251, 204, 176,  45, 116,  18,  43,  32, 240, 177, 132, 153,
    223,  76, 203, 194,  52, 126, 118,   5, 109, 183, 169,  49, 209,  23,   4, 215,
     20,  88,  58,  97, 222,  27,  17,  28,  50,  15, 156,  22,  83,  24, 242,  34,
    254,  68, 207, 178, 195, 181, 122, 145,  36,   8, 232, 168,  96, 252, 105,  80,
    170, 208, 160, 125, 161, 137,  98, 151,  84,  91,  30, 149, 224, 255, 100, 210,
     16, 196,   0,  72, 163, 247, 117, 219, 138,   3, 230, 218,   9,  63, 221, 148,
    135,  92, 131,   2, 205,  74, 144,  51, 115, 103, 246, 243, 157, 127, 191, 226,
     82, 155, 216,  38, 200,  55, 198,  59, 129, 150, 111,  75,  19, 190,  99,  46,
    233, 121, 167, 140, 159, 110, 188, 142,  41, 245, 249, 182,  47, 253, 180,  89,
    120, 152,   6, 106, 231,  70, 113, 186, 212,  37, 171,  66, 136, 162, 141, 250,
    114,   7, 185,  85, 248, 238, 172,  10,  54,  73,  42, 104,  60,  56, 241, 164,
     64,  40, 211, 123, 187, 201,  67, 193,  21, 227, 173, 244, 119, 199, 128, 158,
};

static uint8_t rol8(uint8_t x, int n) { return (uint8_t) ((x << n) | (x >> (8 - n))); }
static uint8_t sb(int i, uint8_t x)
{
    switch (i) {
        case 1: return SBOX1[x];
        case 2: return rol8(SBOX1[x], 1);
        case 3: return rol8(SBOX1[x], 7);
        default: return SBOX1[rol8(x, 1)];
    }
}

const uint8_t *orc_camellia_sbox1(void) { return SBOX1; }

/* F-function (RFC 3713 2.4.1) */
static uint64_t cam_f(uint64_t in, uint64_t ke)
{
    static const int which[8] = { 1, 2, 3, 4, 2, 3, 4, 1 };
    uint64_t x = in ^ ke;
    uint8_t t[8];
    for (int i = 0; i < 8; i++) t[i] = sb(which[i], (uint8_t) (x >> (56 - 8 * i)));
    /* P-layer: which t's feed y1..y8 */
    static const uint8_t p[8] = { 0xB7 /* t1 t3 t4 t6 t7 t8 */, 0xDB, 0xED, 0x7E, 0xC7, 0x6B, 0x3D, 0x9E };
    uint64_t out = 0;
    for (int j = 0; j < 8; j++) {
        uint8_t y = 0;
        for (int i = 0; i < 8; i++)
            if (p[j] & (0x80 >> i)) y ^= t[i];
        out = (out << 8) | y;
    }
    return out;
}

static uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static uint64_t cam_fl(uint64_t in, uint64_t ke)
{
    uint32_t x1 = (uint32_t) (in >> 32), x2 = (uint32_t) in;
    const uint32_t k1 = (uint32_t) (ke >> 32), k2 = (uint32_t) ke;
    x2 ^= rol32(x1 & k1, 1);
    x1 ^= (x2 | k2);
    return ((uint64_t) x1 << 32) | x2;
}

static uint64_t cam_flinv(uint64_t in, uint64_t ke)
{
    uint32_t y1 = (uint32_t) (in >> 32), y2 = (uint32_t) in;
    const uint32_t k1 = (uint32_t) (ke >> 32), k2 = (uint32_t) ke;
    y1 ^= (y2 | k2);
    y2 ^= rol32(y1 & k1, 1);
    return ((uint64_t) y1 << 32) | y2;
}

typedef struct { uint64_t hi, lo; } u128;

static u128 rol128(u128 v, int n)
{
    u128 r;
    n &= 127;
    if (n >= 64) { uint64_t t = v.hi; v.hi = v.lo; v.lo = t; n -= 64; }
    if (n == 0) return v;
    r.hi = (v.hi << n) | (v.lo >> (64 - n));
    r.lo = (v.lo << n) | (v.hi >> (64 - n));
    return r;
}

static uint64_t ld64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return v;
}

static void st64(uint8_t *p, uint64_t v)
{
    for (int i = 7; i >= 0; i--) { p[i] = (uint8_t) v; v >>= 8; }
}

int orc_camellia_setkey_enc(orc_aes_ctx *ctx, const uint8_t *key, unsigned keybits)
{
    static const uint64_t SIGMA[6] = {
        0xA09E667F3BCC908BULL, 0xB67AE8584CAA73B2ULL, 0xC6EF372FE94F82BEULL,
        0x54FF53A5F1D36F1CULL, 0x10E527FADE682D1DULL, 0xB05688C2B3E6C1FDULL };
    u128 kl, kr, ka, kb;
    kl.hi = ld64(key); kl.lo = ld64(key + 8);
    switch (keybits) {
        case 128: kr.hi = kr.lo = 0; break;
        case 192: kr.hi = ld64(key + 16); kr.lo = ~kr.hi; break;
        case 256: kr.hi = ld64(key + 16); kr.lo = ld64(key + 24); break;
        default: return -1;
    }
    uint64_t d1 = kl.hi ^ kr.hi, d2 = kl.lo ^ kr.lo;
    d2 ^= cam_f(d1, SIGMA[0]);
    d1 ^= cam_f(d2, SIGMA[1]);
    d1 ^= kl.hi; d2 ^= kl.lo;
    d2 ^= cam_f(d1, SIGMA[2]);
    d1 ^= cam_f(d2, SIGMA[3]);
    ka.hi = d1; ka.lo = d2;
    d1 = ka.hi ^ kr.hi; d2 = ka.lo ^ kr.lo;
    d2 ^= cam_f(d1, SIGMA[4]);
    d1 ^= cam_f(d2, SIGMA[5]);
    kb.hi = d1; kb.lo = d2;

    /* subkeys in use order as (source, rotation, halves: 3 both, 1 hi, 2 lo),
     * RFC 3713 2.2 tables; 128-bit keys take k9 from KA<<<45 and k10 from KL<<<60 */
    enum { L, R, A, B };
    static const uint8_t s128[14][3] = {
        { L, 0, 3 }, { A, 0, 3 }, { L, 15, 3 }, { A, 15, 3 }, { A, 30, 3 }, { L, 45, 3 }, { A, 45, 1 },
        { L, 60, 2 }, { A, 60, 3 }, { L, 77, 3 }, { L, 94, 3 }, { A, 94, 3 }, { L, 111, 3 }, { A, 111, 3 } };
    static const uint8_t s256[17][3] = {
        { L, 0, 3 }, { B, 0, 3 }, { R, 15, 3 }, { A, 15, 3 }, { R, 30, 3 }, { B, 30, 3 }, { L, 45, 3 },
        { A, 45, 3 }, { L, 60, 3 }, { R, 60, 3 }, { B, 60, 3 }, { L, 77, 3 }, { A, 77, 3 }, { R, 94, 3 },
        { A, 94, 3 }, { L, 111, 3 }, { B, 111, 3 } };
    const u128 src[4] = { kl, kr, ka, kb };
    const uint8_t (*tab)[3] = keybits == 128 ? s128 : s256;
    const int rows = keybits == 128 ? 14 : 17;
    uint64_t sk[34];
    int n = 0;
    for (int i = 0; i < rows; i++) {
        const u128 v = rol128(src[tab[i][0]], tab[i][1]);
        if (tab[i][2] & 1) sk[n++] = v.hi;
        if (tab[i][2] & 2) sk[n++] = v.lo;
    }
    ctx->nr = keybits == 128 ? 18 : 24;
    ctx->kind = 2;
    memset(ctx->ark, 0, sizeof(ctx->ark));
    for (int i = 0; i < n; i++) st64(ctx->ark[i / 2] + 8 * (i & 1), sk[i]);
    return 0;
}

/* RFC 3713 2.3.1 / 2.3.2: whitening, 6-round groups separated by FL / FL^-1 */
void orc_camellia_encrypt_block(const orc_aes_ctx *ctx, const uint8_t in[16], uint8_t out[16])
{
#define SK(i) ld64(ctx->ark[(i) / 2] + 8 * ((i) & 1))
    uint64_t d1 = ld64(in) ^ SK(0), d2 = ld64(in + 8) ^ SK(1);
    int i = 2;
    const int groups = ctx->nr / 6;
    for (int g = 0; g < groups; g++) {
        for (int r = 0; r < 3; r++) {
            d2 ^= cam_f(d1, SK(i)); i++;
            d1 ^= cam_f(d2, SK(i)); i++;
        }
        if (g != groups - 1) {
            d1 = cam_fl(d1, SK(i)); i++;
            d2 = cam_flinv(d2, SK(i)); i++;
        }
    }
    d2 ^= SK(i); i++;
    d1 ^= SK(i);
    st64(out, d2);
    st64(out + 8, d1);
#undef SK
}
