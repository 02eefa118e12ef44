/*
 * aria.c -- ARIA block cipher (RFC 5794 / KS X 1213), TEST INFRASTRUCTURE ONLY.
 *
 * The reference reaches ARIA through PSA (PSA_KEY_TYPE_ARIA with PSA_ALG_GCM,
 * mbedtls_ssl_cipher_to_psa, library/ssl_tls.c:2248-2289); the implementation
 * lives in the absent TF-PSA-Crypto, so this restates the published cipher:
 *   - S-boxes: SB1 = the AES S-box, SB2(x) = B * x^247 ^ 0xE2 in GF(2^8) mod
 *     x^8+x^4+x^3+x+1 (B given below by the images of the 8 basis bits),
 *     SB3 = SB1^-1, SB4 = SB2^-1 (RFC 5794 2.4.2);
 *   - substitution layers SL1 = (SB1,SB2,SB3,SB4)x4, SL2 = (SB3,SB4,SB1,SB2)x4;
 *   - diffusion layer A, the involutory 16x16 binary matrix of RFC 5794 2.4.3;
 *   - key schedule with C1..C3 (fractional bits of 1/pi) and the 128-bit
 *     rotations of RFC 5794 2.2.
 * Pinned by the RFC 5794 Appendix A vectors and by OpenSSL's EVP ARIA
 * (tests/test_aria_oracle.py).
 */
#include <stdint.h>
#include <string.h>
#include <pthread.h>

#include "oracle.h"

static uint8_t sb[4][256];
static pthread_once_t g_aria_once = PTHREAD_ONCE_INIT;

static uint8_t gf8mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t) ((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

static void aria_tables_init(void)
{
    /* B * y for the SB2 affine map: column k = B applied to bit k */
    static const uint8_t bcol[8] = { 0xac, 0xc5, 0x12, 0xcf, 0x5b, 0x5f, 0x85, 0xee };
    const uint8_t *s1 = orc_aes_sbox();
    for (int x = 0; x < 256; x++) {
        /* y = x^247 */
        uint8_t y = 1, base = (uint8_t) x;
        for (int e = 247; e; e >>= 1) {
            if (e & 1) y = gf8mul(y, base);
            base = gf8mul(base, base);
        }
        if (x == 0) y = 0;
        uint8_t v = 0xe2;
        for (int k = 0; k < 8; k++)
            if ((y >> k) & 1) v ^= bcol[k];
        sb[0][x] = s1[x];
        sb[1][x] = v;
    }
    for (int x = 0; x < 256; x++) {
        sb[2][sb[0][x]] = (uint8_t) x;
        sb[3][sb[1][x]] = (uint8_t) x;
    }
}

const uint8_t *orc_aria_sbox(int i)
{
    pthread_once(&g_aria_once, aria_tables_init);
    return sb[i & 3];
}

/* RFC 5794 2.4.3: y_i = XOR of x_j over the row's seven j */
static const uint8_t A_rows[16][7] = {
    { 3, 4, 6, 8, 9, 13, 14 },  { 2, 5, 7, 8, 9, 12, 15 },  { 1, 4, 6, 10, 11, 12, 15 }, { 0, 5, 7, 10, 11, 13, 14 },
    { 0, 2, 5, 8, 11, 14, 15 }, { 1, 3, 4, 9, 10, 14, 15 }, { 0, 2, 7, 9, 10, 12, 13 },  { 1, 3, 6, 8, 11, 12, 13 },
    { 0, 1, 4, 7, 10, 13, 15 }, { 0, 1, 5, 6, 11, 12, 14 }, { 2, 3, 5, 6, 8, 13, 15 },   { 2, 3, 4, 7, 9, 12, 14 },
    { 1, 2, 6, 7, 9, 11, 12 },  { 0, 3, 6, 7, 8, 10, 13 },  { 0, 3, 4, 5, 9, 11, 14 },   { 1, 2, 4, 5, 8, 10, 15 },
};

static void layer_a(uint8_t x[16])
{
    uint8_t y[16];
    for (int i = 0; i < 16; i++) {
        uint8_t v = 0;
        for (int j = 0; j < 7; j++) v ^= x[A_rows[i][j]];
        y[i] = v;
    }
    memcpy(x, y, 16);
}

static void sl_apply(uint8_t x[16], int odd)
{
    /* SL1: SB1 SB2 SB3 SB4 ...  SL2: SB3 SB4 SB1 SB2 ... */
    static const int p1[4] = { 0, 1, 2, 3 }, p2[4] = { 2, 3, 0, 1 };
    for (int i = 0; i < 16; i++) x[i] = sb[(odd ? p1 : p2)[i & 3]][x[i]];
}

static void fo(uint8_t d[16], const uint8_t rk[16])
{
    for (int i = 0; i < 16; i++) d[i] ^= rk[i];
    sl_apply(d, 1);
    layer_a(d);
}

static void fe(uint8_t d[16], const uint8_t rk[16])
{
    for (int i = 0; i < 16; i++) d[i] ^= rk[i];
    sl_apply(d, 0);
    layer_a(d);
}

/* out = x rotated right by n bits (128-bit big-endian string) */
static void rotr128(uint8_t out[16], const uint8_t x[16], int n)
{
    n &= 127;
    const int by = n / 8, bi = n % 8;
    for (int i = 0; i < 16; i++) {
        const uint8_t a = x[(i - by + 16) % 16], b = x[(i - by - 1 + 32) % 16];
        out[i] = (uint8_t) (bi ? ((a >> bi) | (b << (8 - bi))) : a);
    }
}

int orc_aria_setkey_enc(orc_aes_ctx *ctx, const uint8_t *key, unsigned keybits)
{
    static const uint8_t C[3][16] = {
        { 0x51, 0x7c, 0xc1, 0xb7, 0x27, 0x22, 0x0a, 0x94, 0xfe, 0x13, 0xab, 0xe8, 0xfa, 0x9a, 0x6e, 0xe0 },
        { 0x6d, 0xb1, 0x4a, 0xcc, 0x9e, 0x21, 0xc8, 0x20, 0xff, 0x28, 0xb1, 0xd5, 0xef, 0x5d, 0xe2, 0xb0 },
        { 0xdb, 0x92, 0x37, 0x1d, 0x21, 0x26, 0xe9, 0x70, 0x03, 0x24, 0x97, 0x75, 0x04, 0xe8, 0xc9, 0x0e },
    };
    pthread_once(&g_aria_once, aria_tables_init);
    int first;
    switch (keybits) {
        case 128: ctx->nr = 12; first = 0; break;
        case 192: ctx->nr = 14; first = 1; break;
        case 256: ctx->nr = 16; first = 2; break;
        default: return -1;
    }
    uint8_t w[4][16], t[16], kr[16];
    memcpy(w[0], key, 16);
    memset(kr, 0, 16);
    memcpy(kr, key + 16, keybits / 8 - 16);
    memcpy(t, w[0], 16); fo(t, C[first]);           for (int i = 0; i < 16; i++) w[1][i] = t[i] ^ kr[i];
    memcpy(t, w[1], 16); fe(t, C[(first + 1) % 3]); for (int i = 0; i < 16; i++) w[2][i] = t[i] ^ w[0][i];
    memcpy(t, w[2], 16); fo(t, C[(first + 2) % 3]); for (int i = 0; i < 16; i++) w[3][i] = t[i] ^ w[1][i];
    /* ek(4g+j+1) = W_j ^ (W_(j+1) >>> r_g), r = 19, 31, -61, -31, -19 (RFC 5794 2.2) */
    static const int rot[5] = { 19, 31, 128 - 61, 128 - 31, 128 - 19 };
    for (int e = 0; e < ctx->nr + 1; e++) {
        const int g = e / 4, j = e % 4;
        rotr128(t, w[(j + 1) % 4], rot[g]);
        for (int i = 0; i < 16; i++) ctx->ark[e][i] = w[j][i] ^ t[i];
    }
    ctx->kind = 1;
    return 0;
}

void orc_aria_encrypt_block(const orc_aes_ctx *ctx, const uint8_t in[16], uint8_t out[16])
{
    uint8_t d[16];
    memcpy(d, in, 16);
    for (int r = 1; r < ctx->nr; r++) {
        if (r & 1) fo(d, ctx->ark[r - 1]);
        else fe(d, ctx->ark[r - 1]);
    }
    for (int i = 0; i < 16; i++) d[i] ^= ctx->ark[ctx->nr - 1][i];
    sl_apply(d, 0);
    for (int i = 0; i < 16; i++) out[i] = d[i] ^ ctx->ark[ctx->nr][i];
}
