/*
 * oracle.c -- CPU restatement of the Mbed TLS 4.1.0 AEAD record path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h for scope, citations and pinning).
 * The product (mbedtls_amd/) never links or calls this file; it is the
 * checker the GPU path is compared against and the CPU baseline bench.py
 * times beside it.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <string.h>
#include <time.h>

/* ======================================================================
 * AES (FIPS-197).  The S-box is derived from its definition (multiplicative
 * inverse in GF(2^8) mod x^8+x^4+x^3+x+1 followed by the affine map), not
 * transcribed.  Encryption uses four 1 KiB "T" tables that fold SubBytes,
 * ShiftRows and MixColumns -- the same algorithm class as the Mbed TLS
 * builtin aes.c without AES-NI.
 * ==================================================================== */
static uint8_t g_sbox[256];
static uint32_t g_te[4][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static uint8_t gf8_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t) ((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void aes_tables_init(void)
{
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; y++) {
                if (gf8_mul((uint8_t) x, (uint8_t) y) == 1) { inv = (uint8_t) y; break; }
            }
        }
        uint8_t s = inv;
        uint8_t r = inv;
        for (int i = 1; i <= 4; i++) {
            r = (uint8_t) ((r << 1) | (r >> 7));
            s ^= r;
        }
        g_sbox[x] = (uint8_t) (s ^ 0x63);
    }
    for (int x = 0; x < 256; x++) {
        uint8_t s = g_sbox[x];
        uint8_t s2 = gf8_mul(s, 2), s3 = gf8_mul(s, 3);
        /* column contributed by a byte in row 0: (2s, s, s, 3s), little-endian
         * packed so that output row i sits in byte i of the word */
        uint32_t t0 = (uint32_t) s2 | ((uint32_t) s << 8) | ((uint32_t) s << 16) |
                      ((uint32_t) s3 << 24);
        g_te[0][x] = t0;
        g_te[1][x] = rotl32(t0, 8);
        g_te[2][x] = rotl32(t0, 16);
        g_te[3][x] = rotl32(t0, 24);
    }
}

static void ensure_tables(void) { pthread_once(&g_once, aes_tables_init); }

const uint8_t *orc_aes_sbox(void)
{
    ensure_tables();
    return g_sbox;
}

static uint32_t ld32le(const uint8_t *p)
{
    return (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16) |
           ((uint32_t) p[3] << 24);
}

static void st32le(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t) v; p[1] = (uint8_t) (v >> 8);
    p[2] = (uint8_t) (v >> 16); p[3] = (uint8_t) (v >> 24);
}

static uint32_t sub_word(uint32_t w)
{
    return (uint32_t) g_sbox[w & 0xff] | ((uint32_t) g_sbox[(w >> 8) & 0xff] << 8) |
           ((uint32_t) g_sbox[(w >> 16) & 0xff] << 16) |
           ((uint32_t) g_sbox[w >> 24] << 24);
}

/* FIPS-197 5.2 KeyExpansion; words kept little-endian (byte 4i in bits 0-7). */
int orc_aes_setkey_enc(orc_aes_ctx *ctx, const uint8_t *key, unsigned keybits)
{
    ensure_tables();
    int nk;
    switch (keybits) {
        case 128: nk = 4; ctx->nr = 10; break;
        case 192: nk = 6; ctx->nr = 12; break;
        case 256: nk = 8; ctx->nr = 14; break;
        default: return -1;
    }
    ctx->kind = 0;
    int total = 4 * (ctx->nr + 1);
    for (int i = 0; i < nk; i++) ctx->rk[i] = ld32le(key + 4 * i);
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = ctx->rk[i - 1];
        if (i % nk == 0) {
            t = sub_word((t >> 8) | (t << 24)) ^ rcon;   /* RotWord = rotate bytes left */
            rcon = gf8_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = sub_word(t);
        }
        ctx->rk[i] = ctx->rk[i - nk] ^ t;
    }
    return 0;
}

void orc_aes_encrypt_block(const orc_aes_ctx *ctx, const uint8_t in[16], uint8_t out[16])
{
    if (ctx->kind == 1) {               /* ARIA (aria.c) under the same GCM / CCM code */
        orc_aria_encrypt_block(ctx, in, out);
        return;
    }
    if (ctx->kind == 2) {               /* Camellia (camellia.c) */
        orc_camellia_encrypt_block(ctx, in, out);
        return;
    }
    const uint32_t *rk = ctx->rk;
    uint32_t s[4], t[4];
    for (int c = 0; c < 4; c++) s[c] = ld32le(in + 4 * c) ^ rk[c];
    for (int r = 1; r < ctx->nr; r++) {
        rk += 4;
        for (int c = 0; c < 4; c++) {
            /* ShiftRows: row i of column c comes from column c+i */
            t[c] = g_te[0][s[c] & 0xff] ^ g_te[1][(s[(c + 1) & 3] >> 8) & 0xff] ^
                   g_te[2][(s[(c + 2) & 3] >> 16) & 0xff] ^ g_te[3][s[(c + 3) & 3] >> 24] ^ rk[c];
        }
        memcpy(s, t, sizeof(s));
    }
    rk += 4;
    for (int c = 0; c < 4; c++) {
        uint32_t w = (uint32_t) g_sbox[s[c] & 0xff] |
                     ((uint32_t) g_sbox[(s[(c + 1) & 3] >> 8) & 0xff] << 8) |
                     ((uint32_t) g_sbox[(s[(c + 2) & 3] >> 16) & 0xff] << 16) |
                     ((uint32_t) g_sbox[s[(c + 3) & 3] >> 24] << 24);
        st32le(out + 4 * c, w ^ rk[c]);
    }
}

/* ======================================================================
 * GCM (NIST SP 800-38D).  Field elements are 128-bit strings whose bit 0
 * (MSB of byte 0) is the coefficient of x^0; multiplication by x is a right
 * shift with reduction by R = 0xE1 || 0^120.  GHASH uses Shoup's 4-bit table
 * method: 16 multiples of H plus a 16-entry reduction table.
 * ==================================================================== */
static uint64_t ld64be(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return v;
}

static void st64be(uint8_t *p, uint64_t v)
{
    for (int i = 7; i >= 0; i--) { p[i] = (uint8_t) v; v >>= 8; }
}

static void gf_shr1(uint64_t *hi, uint64_t *lo)
{
    uint64_t lsb = *lo & 1;
    *lo = (*lo >> 1) | (*hi << 63);
    *hi >>= 1;
    if (lsb) *hi ^= 0xE100000000000000ULL;
}

static uint64_t g_last4[16];
static pthread_once_t g_once4 = PTHREAD_ONCE_INIT;
static void last4_init(void)
{
    for (int rem = 0; rem < 16; rem++) {
        uint64_t hi = 0, lo = (uint64_t) rem;
        for (int k = 0; k < 4; k++) gf_shr1(&hi, &lo);
        g_last4[rem] = hi;
    }
}

int orc_gcm_setkey(orc_gcm_ctx *ctx, const uint8_t *key, unsigned keybits)
{
    return orc_gcm_setkey_ex(ctx, key, keybits, 0);
}

int orc_gcm_setkey_ex(orc_gcm_ctx *ctx, const uint8_t *key, unsigned keybits, int bc)
{
    static const uint8_t zero[16] = { 0 };
    pthread_once(&g_once4, last4_init);
    if ((bc == 2 ? orc_camellia_setkey_enc(&ctx->aes, key, keybits)
         : bc ? orc_aria_setkey_enc(&ctx->aes, key, keybits) : orc_aes_setkey_enc(&ctx->aes, key, keybits)) != 0)
        return -1;
    orc_aes_encrypt_block(&ctx->aes, zero, ctx->h);
    uint64_t hi = ld64be(ctx->h), lo = ld64be(ctx->h + 8);
    /* table index n = raw nibble; its bit 3 is the lowest power in the window */
    ctx->hh[0] = ctx->hl[0] = 0;
    ctx->hh[8] = hi; ctx->hl[8] = lo;
    for (int n = 4; n > 0; n >>= 1) {
        gf_shr1(&hi, &lo);
        ctx->hh[n] = hi; ctx->hl[n] = lo;
    }
    for (int n = 2; n < 16; n <<= 1) {
        for (int j = 1; j < n; j++) {
            ctx->hh[n + j] = ctx->hh[n] ^ ctx->hh[j];
            ctx->hl[n + j] = ctx->hl[n] ^ ctx->hl[j];
        }
    }
    return 0;
}

/* out = x * H.  Horner over the 32 nibble windows from the highest power:
 * window 2b is the high nibble of byte b, window 2b+1 its low nibble. */
void orc_ghash_mult(const orc_gcm_ctx *ctx, const uint8_t x[16], uint8_t out[16])
{
    uint64_t zh = 0, zl = 0;
    for (int b = 15; b >= 0; b--) {
        for (int half = 0; half < 2; half++) {
            uint8_t n = half == 0 ? (x[b] & 0x0f) : (x[b] >> 4);
            uint8_t rem = (uint8_t) (zl & 0x0f);
            zl = (zl >> 4) | (zh << 60);
            zh = (zh >> 4) ^ g_last4[rem];
            zh ^= ctx->hh[n];
            zl ^= ctx->hl[n];
        }
    }
    st64be(out, zh);
    st64be(out + 8, zl);
}

/* generic bitwise product (used by tests to derive powers of H) */
void orc_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16])
{
    uint64_t zh = 0, zl = 0, vh = ld64be(y), vl = ld64be(y + 8);
    for (int i = 0; i < 128; i++) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1) { zh ^= vh; zl ^= vl; }
        gf_shr1(&vh, &vl);
    }
    st64be(out, zh);
    st64be(out + 8, zl);
}

static void ghash_update(const orc_gcm_ctx *ctx, uint8_t y[16], const uint8_t *p, size_t len)
{
    uint8_t blk[16];
    while (len > 0) {
        size_t n = len < 16 ? len : 16;
        memset(blk, 0, 16);
        memcpy(blk, p, n);
        for (int i = 0; i < 16; i++) y[i] ^= blk[i];
        orc_ghash_mult(ctx, y, y);
        p += n;
        len -= n;
    }
}

void orc_ghash(const orc_gcm_ctx *ctx, const uint8_t *aad, size_t aad_len,
               const uint8_t *ct, size_t ct_len, uint8_t out[16])
{
    uint8_t y[16] = { 0 }, lb[16];
    ghash_update(ctx, y, aad, aad_len);
    ghash_update(ctx, y, ct, ct_len);
    st64be(lb, (uint64_t) aad_len * 8);
    st64be(lb + 8, (uint64_t) ct_len * 8);
    ghash_update(ctx, y, lb, 16);
    memcpy(out, y, 16);
}

static void gcm_ctr(const orc_gcm_ctx *ctx, const uint8_t j0[16], const uint8_t *in,
                    uint8_t *out, size_t len)
{
    uint8_t cb[16], ks[16];
    memcpy(cb, j0, 16);
    uint32_t ctr = (uint32_t) ld64be(j0 + 8);   /* low 32 bits of the BE block */
    while (len > 0) {
        ctr++;                                   /* inc32 */
        cb[12] = (uint8_t) (ctr >> 24); cb[13] = (uint8_t) (ctr >> 16);
        cb[14] = (uint8_t) (ctr >> 8);  cb[15] = (uint8_t) ctr;
        orc_aes_encrypt_block(&ctx->aes, cb, ks);
        size_t n = len < 16 ? len : 16;
        for (size_t i = 0; i < n; i++) out[i] = in[i] ^ ks[i];
        in += n; out += n; len -= n;
    }
}

void orc_gcm_encrypt(const orc_gcm_ctx *ctx, const uint8_t iv[12],
                     const uint8_t *aad, size_t aad_len,
                     const uint8_t *in, size_t len, uint8_t *out,
                     uint8_t *tag, size_t tag_len)
{
    uint8_t j0[16], s[16], ek[16];
    memcpy(j0, iv, 12);
    j0[12] = j0[13] = j0[14] = 0; j0[15] = 1;
    gcm_ctr(ctx, j0, in, out, len);
    orc_ghash(ctx, aad, aad_len, out, len, s);
    orc_aes_encrypt_block(&ctx->aes, j0, ek);
    for (size_t i = 0; i < tag_len; i++) tag[i] = s[i] ^ ek[i];
}

int orc_gcm_decrypt(const orc_gcm_ctx *ctx, const uint8_t iv[12],
                    const uint8_t *aad, size_t aad_len,
                    const uint8_t *in, size_t len, uint8_t *out,
                    const uint8_t *tag, size_t tag_len)
{
    uint8_t j0[16], s[16], ek[16];
    memcpy(j0, iv, 12);
    j0[12] = j0[13] = j0[14] = 0; j0[15] = 1;
    orc_ghash(ctx, aad, aad_len, in, len, s);
    orc_aes_encrypt_block(&ctx->aes, j0, ek);
    uint8_t diff = 0;
    for (size_t i = 0; i < tag_len; i++) diff |= (uint8_t) (tag[i] ^ s[i] ^ ek[i]);
    if (diff != 0) return ORC_ERR_SSL_INVALID_MAC;
    gcm_ctr(ctx, j0, in, out, len);
    return 0;
}

/* ======================================================================
 * CCM (NIST SP 800-38C, RFC 3610 formatting) with a 12-byte nonce:
 *   B0 = flags(Adata, t, q=3) || N || Q(3)      (A.2.1)
 *   AAD block(s) = len16(a) || a || 0-pad       (A.2.2, a < 2^16 - 2^8)
 *   payload blocks zero-padded                  (A.2.3)
 *   T = MSB_t(CBC-MAC), C = P ^ S_1.., U = T ^ MSB_t(S_0), S_i = E(ctr_i),
 *   ctr_i = (q-1) || N || i(3)                  (A.3)
 * ==================================================================== */
static void ccm_mac(const orc_aes_ctx *aes, const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                    const uint8_t *pt, size_t len, size_t tag_len, uint8_t x[16])
{
    uint8_t b[16];
    b[0] = (uint8_t) ((aad_len ? 0x40 : 0) | (((tag_len - 2) / 2) << 3) | 2);
    memcpy(b + 1, nonce, 12);
    b[13] = (uint8_t) (len >> 16);
    b[14] = (uint8_t) (len >> 8);
    b[15] = (uint8_t) len;
    orc_aes_encrypt_block(aes, b, x);
    if (aad_len) {
        /* len16 || aad, then zero padding, in 16-byte blocks */
        uint8_t buf[16];
        size_t fill = 2, i = 0;
        memset(buf, 0, 16);
        buf[0] = (uint8_t) (aad_len >> 8);
        buf[1] = (uint8_t) aad_len;
        while (i < aad_len) {
            buf[fill++] = aad[i++];
            if (fill == 16) {
                for (int k = 0; k < 16; k++) x[k] ^= buf[k];
                orc_aes_encrypt_block(aes, x, x);
                memset(buf, 0, 16);
                fill = 0;
            }
        }
        if (fill) {
            for (int k = 0; k < 16; k++) x[k] ^= buf[k];
            orc_aes_encrypt_block(aes, x, x);
        }
    }
    for (size_t off = 0; off < len; off += 16) {
        size_t n = len - off < 16 ? len - off : 16;
        for (size_t k = 0; k < n; k++) x[k] ^= pt[off + k];
        orc_aes_encrypt_block(aes, x, x);
    }
}

static void ccm_ctr(const orc_aes_ctx *aes, const uint8_t nonce[12], uint32_t i, uint8_t s[16])
{
    uint8_t a[16];
    a[0] = 2;
    memcpy(a + 1, nonce, 12);
    a[13] = (uint8_t) (i >> 16);
    a[14] = (uint8_t) (i >> 8);
    a[15] = (uint8_t) i;
    orc_aes_encrypt_block(aes, a, s);
}

static void ccm_crypt(const orc_aes_ctx *aes, const uint8_t nonce[12], const uint8_t *in, size_t len, uint8_t *out)
{
    uint8_t s[16];
    uint32_t i = 1;
    for (size_t off = 0; off < len; off += 16, i++) {
        ccm_ctr(aes, nonce, i, s);
        size_t n = len - off < 16 ? len - off : 16;
        for (size_t k = 0; k < n; k++) out[off + k] = in[off + k] ^ s[k];
    }
}

void orc_ccm_encrypt(const orc_aes_ctx *aes, const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                     const uint8_t *in, size_t len, uint8_t *out, uint8_t *tag, size_t tag_len)
{
    uint8_t x[16], s0[16];
    ccm_mac(aes, nonce, aad, aad_len, in, len, tag_len, x);
    ccm_crypt(aes, nonce, in, len, out);
    ccm_ctr(aes, nonce, 0, s0);
    for (size_t k = 0; k < tag_len; k++) tag[k] = x[k] ^ s0[k];
}

int orc_ccm_decrypt(const orc_aes_ctx *aes, const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                    const uint8_t *in, size_t len, uint8_t *out, const uint8_t *tag, size_t tag_len)
{
    uint8_t x[16], s0[16];
    ccm_crypt(aes, nonce, in, len, out);
    ccm_mac(aes, nonce, aad, aad_len, out, len, tag_len, x);
    ccm_ctr(aes, nonce, 0, s0);
    uint8_t diff = 0;
    for (size_t k = 0; k < tag_len; k++) diff |= (uint8_t) (tag[k] ^ x[k] ^ s0[k]);
    return diff ? ORC_ERR_SSL_INVALID_MAC : 0;
}

/* ======================================================================
 * ChaCha20 (RFC 8439 2.3) and Poly1305 (RFC 8439 2.5) with 44-bit limbs.
 * ==================================================================== */
#define QR(a, b, c, d) do { \
        a += b; d ^= a; d = rotl32(d, 16); \
        c += d; b ^= c; b = rotl32(b, 12); \
        a += b; d ^= a; d = rotl32(d, 8);  \
        c += d; b ^= c; b = rotl32(b, 7);  \
} while (0)

void orc_chacha20_block(const uint8_t key[32], uint32_t counter,
                        const uint8_t nonce[12], uint8_t out[64])
{
    uint32_t in[16], x[16];
    in[0] = 0x61707865; in[1] = 0x3320646e; in[2] = 0x79622d32; in[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) in[4 + i] = ld32le(key + 4 * i);
    in[12] = counter;
    for (int i = 0; i < 3; i++) in[13 + i] = ld32le(nonce + 4 * i);
    memcpy(x, in, sizeof(x));
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) st32le(out + 4 * i, x[i] + in[i]);
}

void orc_chacha20_xor(const uint8_t key[32], uint32_t counter,
                      const uint8_t nonce[12], const uint8_t *in,
                      uint8_t *out, size_t len)
{
    uint8_t ks[64];
    while (len > 0) {
        orc_chacha20_block(key, counter++, nonce, ks);
        size_t n = len < 64 ? len : 64;
        for (size_t i = 0; i < n; i++) out[i] = in[i] ^ ks[i];
        in += n; out += n; len -= n;
    }
}

typedef struct {
    uint64_t r0, r1, r2, s1, s2;
    uint64_t h0, h1, h2;
    uint64_t pad0, pad1;
} poly_state;

#define M44 0xfffffffffffULL
#define M42 0x3ffffffffffULL

static uint64_t ld64le(const uint8_t *p)
{
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

static void st64le(uint8_t *p, uint64_t v)
{
    for (int i = 0; i < 8; i++) { p[i] = (uint8_t) v; v >>= 8; }
}

static void poly_init(poly_state *st, const uint8_t key[32])
{
    uint64_t t0 = ld64le(key) & 0x0ffffffc0fffffffULL;      /* clamp r */
    uint64_t t1 = ld64le(key + 8) & 0x0ffffffc0ffffffcULL;
    st->r0 = t0 & M44;
    st->r1 = ((t0 >> 44) | (t1 << 20)) & M44;
    st->r2 = (t1 >> 24) & M42;
    st->s1 = st->r1 * 20;                 /* 2^132 = 4 * 2^130 == 4*5 (mod p) */
    st->s2 = st->r2 * 20;
    st->h0 = st->h1 = st->h2 = 0;
    st->pad0 = ld64le(key + 16);
    st->pad1 = ld64le(key + 24);
}

/* h = (h + m + 2^128) * r  mod 2^130-5, for one full 16-byte block */
static void poly_block(poly_state *st, const uint8_t m[16])
{
    typedef unsigned __int128 u128;
    uint64_t t0 = ld64le(m), t1 = ld64le(m + 8);
    uint64_t h0 = st->h0 + (t0 & M44);
    uint64_t h1 = st->h1 + (((t0 >> 44) | (t1 << 20)) & M44);
    uint64_t h2 = st->h2 + (((t1 >> 24) & M42) | (1ULL << 40));
    u128 d0 = (u128) h0 * st->r0 + (u128) h1 * st->s2 + (u128) h2 * st->s1;
    u128 d1 = (u128) h0 * st->r1 + (u128) h1 * st->r0 + (u128) h2 * st->s2;
    u128 d2 = (u128) h0 * st->r2 + (u128) h1 * st->r1 + (u128) h2 * st->r0;
    uint64_t c = (uint64_t) (d0 >> 44); h0 = (uint64_t) d0 & M44;
    d1 += c; c = (uint64_t) (d1 >> 44); h1 = (uint64_t) d1 & M44;
    d2 += c; c = (uint64_t) (d2 >> 42); h2 = (uint64_t) d2 & M42;
    h0 += c * 5; c = h0 >> 44; h0 &= M44;
    h1 += c;
    st->h0 = h0; st->h1 = h1; st->h2 = h2;
}

/* absorb `len` bytes zero-padded to a multiple of 16 (RFC 8439 2.8 pad16) */
static void poly_padded(poly_state *st, const uint8_t *p, size_t len)
{
    uint8_t blk[16];
    while (len >= 16) { poly_block(st, p); p += 16; len -= 16; }
    if (len) {
        memset(blk, 0, 16);
        memcpy(blk, p, len);
        poly_block(st, blk);
    }
}

static void poly_finish(poly_state *st, uint8_t tag[16])
{
    uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2, c;
    c = h1 >> 44; h1 &= M44; h2 += c;
    c = h2 >> 42; h2 &= M42; h0 += c * 5;
    c = h0 >> 44; h0 &= M44; h1 += c;
    c = h1 >> 44; h1 &= M44; h2 += c;
    c = h2 >> 42; h2 &= M42; h0 += c * 5;
    c = h0 >> 44; h0 &= M44; h1 += c;
    /* g = h + 5 - 2^130; take g if it did not borrow, i.e. h >= p */
    uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= M44;
    uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= M44;
    uint64_t g2 = h2 + c - (1ULL << 42);
    uint64_t mask = (g2 >> 63) - 1;   /* all ones when no borrow */
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask & M42);
    uint64_t t0 = h0 | (h1 << 44);
    uint64_t t1 = (h1 >> 20) | (h2 << 24);
    uint64_t s0 = t0 + st->pad0;
    c = s0 < t0;
    uint64_t s1 = t1 + st->pad1 + c;
    st64le(tag, s0);
    st64le(tag + 8, s1);
}

void orc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16])
{
    poly_state st;
    poly_init(&st, key);
    uint8_t blk[16];
    while (len >= 16) { poly_block(&st, msg); msg += 16; len -= 16; }
    if (len) {
        /* RFC 8439 2.5.1: a short final block gets its 0x01 byte right after
         * the message bytes; it is not counted as 2^128 */
        poly_state tmp = st;
        memset(blk, 0, 16);
        memcpy(blk, msg, len);
        blk[len] = 1;
        /* emulate by absorbing with the hibit removed */
        typedef unsigned __int128 u128;
        uint64_t t0 = ld64le(blk), t1 = ld64le(blk + 8);
        uint64_t h0 = tmp.h0 + (t0 & M44);
        uint64_t h1 = tmp.h1 + (((t0 >> 44) | (t1 << 20)) & M44);
        uint64_t h2 = tmp.h2 + ((t1 >> 24) & M42);
        u128 d0 = (u128) h0 * st.r0 + (u128) h1 * st.s2 + (u128) h2 * st.s1;
        u128 d1 = (u128) h0 * st.r1 + (u128) h1 * st.r0 + (u128) h2 * st.s2;
        u128 d2 = (u128) h0 * st.r2 + (u128) h1 * st.r1 + (u128) h2 * st.r0;
        uint64_t c = (uint64_t) (d0 >> 44); h0 = (uint64_t) d0 & M44;
        d1 += c; c = (uint64_t) (d1 >> 44); h1 = (uint64_t) d1 & M44;
        d2 += c; c = (uint64_t) (d2 >> 42); h2 = (uint64_t) d2 & M42;
        h0 += c * 5; c = h0 >> 44; h0 &= M44; h1 += c;
        st.h0 = h0; st.h1 = h1; st.h2 = h2;
    }
    poly_finish(&st, tag);
}

static void chachapoly_tag(const uint8_t key[32], const uint8_t nonce[12],
                           const uint8_t *aad, size_t aad_len,
                           const uint8_t *ct, size_t len, uint8_t tag[16])
{
    uint8_t otk[64], lens[16];
    orc_chacha20_block(key, 0, nonce, otk);        /* RFC 8439 2.6 */
    poly_state st;
    poly_init(&st, otk);
    poly_padded(&st, aad, aad_len);
    poly_padded(&st, ct, len);
    st64le(lens, (uint64_t) aad_len);
    st64le(lens + 8, (uint64_t) len);
    poly_block(&st, lens);
    poly_finish(&st, tag);
}

void orc_chachapoly_encrypt(const uint8_t key[32], const uint8_t nonce[12],
                            const uint8_t *aad, size_t aad_len,
                            const uint8_t *in, size_t len, uint8_t *out,
                            uint8_t tag[16])
{
    orc_chacha20_xor(key, 1, nonce, in, out, len);
    chachapoly_tag(key, nonce, aad, aad_len, out, len, tag);
}

int orc_chachapoly_decrypt(const uint8_t key[32], const uint8_t nonce[12],
                           const uint8_t *aad, size_t aad_len,
                           const uint8_t *in, size_t len, uint8_t *out,
                           const uint8_t tag[16])
{
    uint8_t t[16], diff = 0;
    chachapoly_tag(key, nonce, aad, aad_len, in, len, t);
    for (int i = 0; i < 16; i++) diff |= (uint8_t) (t[i] ^ tag[i]);
    if (diff) return ORC_ERR_SSL_INVALID_MAC;
    orc_chacha20_xor(key, 1, nonce, in, out, len);
    return 0;
}

/* ======================================================================
 * Record layer: restatement of library/ssl_msg.c (Mbed TLS 4.1.0).
 * ==================================================================== */

/* ssl_tls13_keys.c:974-998 (TLS 1.3) and ssl_tls.c:7768-7797 (TLS 1.2 AEAD) */
int orc_transform_setup(orc_transform *t, int tls_version, int cipher,
                        const uint8_t *key_enc, const uint8_t *key_dec,
                        const uint8_t *iv_enc, const uint8_t *iv_dec,
                        size_t granularity)
{
    memset(t, 0, sizeof(*t));
    t->tls_version = tls_version;
    t->cipher = cipher;
    t->granularity = granularity ? granularity : 16;
    switch (cipher) {                 /* mbedtls_ssl_cipher_to_psa, ssl_tls.c:2168-2363 */
        case ORC_CIPHER_AES_128_GCM: case ORC_CIPHER_AES_128_CCM: case ORC_CIPHER_AES_128_CCM_8:
            t->keylen = 16; break;
        case ORC_CIPHER_AES_192_GCM: case ORC_CIPHER_AES_192_CCM: case ORC_CIPHER_AES_192_CCM_8:
            t->keylen = 24; break;
        case ORC_CIPHER_AES_256_GCM: case ORC_CIPHER_AES_256_CCM: case ORC_CIPHER_AES_256_CCM_8:
        case ORC_CIPHER_CHACHA20_POLY1305: t->keylen = 32; break;
        /* ARIA-GCM (PSA_KEY_TYPE_ARIA + PSA_ALG_GCM, ssl_tls.c:2248-2289) */
        case ORC_CIPHER_ARIA_128_GCM: case ORC_CIPHER_ARIA_128_CCM: t->keylen = 16; break;
        case ORC_CIPHER_ARIA_192_GCM: case ORC_CIPHER_ARIA_192_CCM: t->keylen = 24; break;
        case ORC_CIPHER_ARIA_256_GCM: case ORC_CIPHER_ARIA_256_CCM: t->keylen = 32; break;
        /* Camellia-GCM / -CCM (PSA_KEY_TYPE_CAMELLIA, ssl_tls.c:2297-2345) */
        case ORC_CIPHER_CAMELLIA_128_GCM: case ORC_CIPHER_CAMELLIA_128_CCM: t->keylen = 16; break;
        case ORC_CIPHER_CAMELLIA_192_GCM: case ORC_CIPHER_CAMELLIA_192_CCM: t->keylen = 24; break;
        case ORC_CIPHER_CAMELLIA_256_GCM: case ORC_CIPHER_CAMELLIA_256_CCM: t->keylen = 32; break;
        default: return ORC_ERR_SSL_FEATURE_UNAVAILABLE;
    }
    t->ivlen = 12;
    /* MBEDTLS_CIPHERSUITE_SHORT_TAG: ssl_tls.c:7707-7708, ssl_tls13_keys.c:981-985 */
    t->taglen = (cipher >= ORC_CIPHER_AES_128_CCM_8 && cipher <= ORC_CIPHER_AES_256_CCM_8) ? 8 : 16;
    t->maclen = 0;
    if (tls_version == ORC_VERSION_TLS1_3) {
        t->fixed_ivlen = t->ivlen;
        t->minlen = t->taglen + t->granularity;
    } else if (tls_version == ORC_VERSION_TLS1_2) {
        t->fixed_ivlen = (cipher == ORC_CIPHER_CHACHA20_POLY1305) ? 12 : 4;
        t->minlen = (t->ivlen - t->fixed_ivlen) + t->taglen;
    } else {
        return ORC_ERR_SSL_BAD_INPUT_DATA;
    }
    memcpy(t->key_enc, key_enc, t->keylen);
    memcpy(t->key_dec, key_dec, t->keylen);
    memcpy(t->iv_enc, iv_enc, 16);
    memcpy(t->iv_dec, iv_dec, 16);
    if (cipher != ORC_CIPHER_CHACHA20_POLY1305) {
        const int bc = cipher >= ORC_CIPHER_CAMELLIA_128_GCM ? 2 : cipher >= ORC_CIPHER_ARIA_128_GCM ? 1 : 0;
        orc_gcm_setkey_ex(&t->gcm_enc, key_enc, (unsigned) t->keylen * 8, bc);
        orc_gcm_setkey_ex(&t->gcm_dec, key_dec, (unsigned) t->keylen * 8, bc);
    }
    return 0;
}

/* ssl_msg.c:768-781: IV := (fixed_iv || 0) XOR (0 || dynamic_iv) */
static void build_nonce(uint8_t nonce[12], const uint8_t *fixed, size_t fixed_len,
                        const uint8_t dyn[8])
{
    memset(nonce, 0, 12);
    memcpy(nonce, fixed, fixed_len);
    for (int i = 0; i < 8; i++) nonce[4 + i] ^= dyn[i];
}

/* ssl_msg.c:568-735.  Non-CID: TLS 1.3 type || ver || len(TLSCiphertext),
 * TLS 1.2 seq || type || ver || len.  DTLS 1.2 + CID (RFC 9146, :683-724):
 * 0xff x 8 || type || cid_len || type || ver || epoch+seq || cid || len. */
static size_t build_aad(uint8_t aad[23 + ORC_CID_LEN_MAX], const orc_record *rec, int tls_version, size_t taglen)
{
    size_t n = 0, len_field = rec->data_len;
    if (tls_version == ORC_VERSION_TLS1_3) {
        len_field += taglen;           /* :671-677 */
    } else if (rec->cid_len != 0) {
        memset(aad, 0xff, 8);          /* seq_num_placeholder, :685-687 */
        n = 8;
        aad[n++] = rec->type;          /* tls12_cid, :690-691 */
        aad[n++] = rec->cid_len;       /* :694-695 */
    } else {
        memcpy(aad, rec->ctr, 8);      /* :700-703 */
        n = 8;
    }
    aad[n++] = rec->type;              /* :707-709 */
    aad[n++] = rec->ver[0];            /* :711-713 */
    aad[n++] = rec->ver[1];
    if (tls_version != ORC_VERSION_TLS1_3 && rec->cid_len != 0) {
        memcpy(aad + n, rec->ctr, 8);  /* :717-720 */
        n += 8;
        memcpy(aad + n, rec->cid, rec->cid_len);   /* :722-724 */
        n += rec->cid_len;
    }
    aad[n++] = (uint8_t) (len_field >> 8);         /* :727-731 */
    aad[n++] = (uint8_t) len_field;
    return n;
}

int orc_transform_set_cid(orc_transform *t, const uint8_t *in_cid, size_t in_len,
                          const uint8_t *out_cid, size_t out_len)
{
    if (in_len > ORC_CID_LEN_MAX || out_len > ORC_CID_LEN_MAX) return ORC_ERR_SSL_BAD_INPUT_DATA;
    t->in_cid_len = (uint8_t) in_len;
    t->out_cid_len = (uint8_t) out_len;
    memset(t->in_cid, 0, sizeof(t->in_cid));
    memset(t->out_cid, 0, sizeof(t->out_cid));
    if (in_len) memcpy(t->in_cid, in_cid, in_len);
    if (out_len) memcpy(t->out_cid, out_cid, out_len);
    return 0;
}

/* ssl_build_inner_plaintext (ssl_msg.c:466-491) with the padding of
 * ssl_compute_padding_length (:431-435) */
static int build_inner(uint8_t *data, size_t *len, size_t remaining, uint8_t type, size_t g)
{
    size_t pad = (g - (*len + 1) % g) % g, n = *len;
    if (remaining == 0) return -1;
    data[n++] = type;
    remaining--;
    if (remaining < pad) return -1;
    memset(data + n, 0, pad);
    *len = n + pad;
    return 0;
}

/* ssl_parse_inner_plaintext (ssl_msg.c:496-514) */
static int parse_inner(const uint8_t *data, size_t *len, uint8_t *type)
{
    size_t remaining = *len;
    do {
        if (remaining == 0) return -1;
        remaining--;
    } while (data[remaining] == 0);
    *len = remaining;
    *type = data[remaining];
    return 0;
}

static int is_ccm(int c)
{
    return (c >= ORC_CIPHER_AES_128_CCM && c <= ORC_CIPHER_AES_256_CCM_8) ||
           (c >= ORC_CIPHER_ARIA_128_CCM && c <= ORC_CIPHER_ARIA_256_CCM) ||
           (c >= ORC_CIPHER_CAMELLIA_128_CCM && c <= ORC_CIPHER_CAMELLIA_256_CCM);
}

static void aead_seal(const orc_transform *t, const uint8_t nonce[12],
                      const uint8_t *aad, size_t aad_len, uint8_t *data, size_t len)
{
    if (t->cipher == ORC_CIPHER_CHACHA20_POLY1305) {
        orc_chachapoly_encrypt(t->key_enc, nonce, aad, aad_len, data, len, data, data + len);
    } else if (is_ccm(t->cipher)) {
        orc_ccm_encrypt(&t->gcm_enc.aes, nonce, aad, aad_len, data, len, data, data + len, t->taglen);
    } else {
        orc_gcm_encrypt(&t->gcm_enc, nonce, aad, aad_len, data, len, data, data + len, 16);
    }
}

static int aead_open(const orc_transform *t, const uint8_t nonce[12],
                     const uint8_t *aad, size_t aad_len, uint8_t *data, size_t len)
{
    if (t->cipher == ORC_CIPHER_CHACHA20_POLY1305) {
        return orc_chachapoly_decrypt(t->key_dec, nonce, aad, aad_len, data, len, data, data + len);
    }
    if (is_ccm(t->cipher))
        return orc_ccm_decrypt(&t->gcm_dec.aes, nonce, aad, aad_len, data, len, data, data + len, t->taglen);
    return orc_gcm_decrypt(&t->gcm_dec, nonce, aad, aad_len, data, len, data, data + len, 16);
}

/* mbedtls_ssl_encrypt_buf, ssl_msg.c:784-1268, AEAD branch */
int orc_encrypt_buf(const orc_transform *t, orc_record *rec)
{
    if (t == NULL) return ORC_ERR_SSL_INTERNAL_ERROR;                   /* :810-813 */
    if (rec == NULL || rec->buf == NULL || rec->buf_len < rec->data_offset ||
        rec->buf_len - rec->data_offset < rec->data_len) {
        return ORC_ERR_SSL_INTERNAL_ERROR;                               /* :814-823 */
    }
    uint8_t *data = rec->buf + rec->data_offset;
    size_t post_avail = rec->buf_len - (rec->data_len + rec->data_offset);
    if (rec->data_len > ORC_OUT_CONTENT_LEN) return ORC_ERR_SSL_BAD_INPUT_DATA; /* :831-839 */

    if (t->tls_version == ORC_VERSION_TLS1_3) {                          /* :853-868 */
        if (build_inner(data, &rec->data_len, post_avail, rec->type, t->granularity) != 0)
            return ORC_ERR_SSL_BUFFER_TOO_SMALL;
        rec->type = 23;                                                  /* APPLICATION_DATA */
    }
    rec->cid_len = t->out_cid_len;                                       /* :874-875 */
    memcpy(rec->cid, t->out_cid, t->out_cid_len);
    if (rec->cid_len != 0) {                                             /* :878-897 */
        if (build_inner(data, &rec->data_len, post_avail, rec->type, t->granularity) != 0)
            return ORC_ERR_SSL_BUFFER_TOO_SMALL;
        rec->type = ORC_SSL_MSG_CID;
    }
    post_avail = rec->buf_len - (rec->data_len + rec->data_offset);

    if (post_avail < t->taglen) return ORC_ERR_SSL_BUFFER_TOO_SMALL;    /* :995-998 */
    uint8_t nonce[12], aad[23 + ORC_CID_LEN_MAX];
    build_nonce(nonce, t->iv_enc, t->fixed_ivlen, rec->ctr);             /* :1012-1019 */
    size_t aad_len = build_aad(aad, rec, t->tls_version, t->taglen);    /* :1025-1027 */
    aead_seal(t, nonce, aad, aad_len, data, rec->data_len);             /* :1043-1049 */
    rec->data_len += t->taglen;
    if (t->ivlen != t->fixed_ivlen) {                                   /* :1066-1075 */
        if (rec->data_offset < 8) return ORC_ERR_SSL_BUFFER_TOO_SMALL;
        memcpy(data - 8, rec->ctr, 8);
        rec->data_offset -= 8;
        rec->data_len += 8;
    }
    return 0;
}

/* mbedtls_ssl_decrypt_buf, ssl_msg.c:1270-1834, AEAD branch */
int orc_decrypt_buf(const orc_transform *t, orc_record *rec)
{
    if (rec == NULL || rec->buf == NULL || rec->buf_len < rec->data_offset ||
        rec->buf_len - rec->data_offset < rec->data_len) {
        return ORC_ERR_SSL_INTERNAL_ERROR;                               /* :1301-1307 */
    }
    if (rec->cid_len != t->in_cid_len ||                                 /* :1313-1320 */
        memcmp(rec->cid, t->in_cid, rec->cid_len) != 0) {
        return ORC_ERR_SSL_UNEXPECTED_CID;
    }
    uint8_t *data = rec->buf + rec->data_offset;
    const uint8_t *dyn = rec->ctr;
    if (t->ivlen != t->fixed_ivlen) {                                   /* :1352-1365 */
        if (rec->data_len < 8) return ORC_ERR_SSL_INVALID_MAC;
        dyn = data;
        data += 8;
        rec->data_offset += 8;
        rec->data_len -= 8;
    }
    if (rec->data_len < t->taglen) return ORC_ERR_SSL_INVALID_MAC;      /* :1371-1377 */
    rec->data_len -= t->taglen;
    uint8_t nonce[12], aad[23 + ORC_CID_LEN_MAX];
    build_nonce(nonce, t->iv_dec, t->fixed_ivlen, dyn);
    size_t aad_len = build_aad(aad, rec, t->tls_version, t->taglen);
    if (aead_open(t, nonce, aad, aad_len, data, rec->data_len) != 0) {   /* :1412-1424 */
        /* PSA core wipes the whole output buffer on failure */
        memset(data, 0, rec->buf_len - (size_t) (data - rec->buf));
        return ORC_ERR_SSL_INVALID_MAC;
    }
    if (t->tls_version == ORC_VERSION_TLS1_3) {                          /* :1809-1818 */
        if (parse_inner(data, &rec->data_len, &rec->type) != 0) return ORC_ERR_SSL_INVALID_RECORD;
    }
    if (rec->cid_len != 0) {                                             /* :1821-1829 */
        if (parse_inner(data, &rec->data_len, &rec->type) != 0) return ORC_ERR_SSL_INVALID_RECORD;
    }
    return 0;
}

/* ======================================================================
 * CPU baseline driver
 * ==================================================================== */
typedef struct {
    const orc_transform *t;
    int dir;
    uint8_t *arena;
    size_t stride, data_len;
    uint64_t lo, hi, seq0;
    int32_t *status;
} bench_job;

static void *bench_worker(void *arg)
{
    bench_job *j = (bench_job *) arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        orc_record rec;
        rec.cid_len = 0;   /* no DTLS connection ID on this path */
        uint64_t seq = j->seq0 + i;
        for (int k = 7; k >= 0; k--) { rec.ctr[k] = (uint8_t) seq; seq >>= 8; }
        rec.type = 23;   /* application data (inner type on encrypt, outer on decrypt) */
        rec.ver[0] = 3; rec.ver[1] = 3;
        rec.buf = j->arena + i * j->stride;
        rec.buf_len = j->stride;
        rec.data_offset = (j->dir && j->t->ivlen != j->t->fixed_ivlen) ? 8 : 0;
        rec.data_len = j->data_len;
        int r = j->dir ? orc_encrypt_buf(j->t, &rec) : orc_decrypt_buf(j->t, &rec);
        if (j->status) j->status[i] = r;
    }
    return NULL;
}

double orc_bench_records(const orc_transform *t, int dir, uint8_t *arena,
                         size_t stride, size_t data_len, uint64_t n,
                         uint64_t seq0, int threads, int32_t *status)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    bench_job jobs[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < threads; i++) {
        jobs[i] = (bench_job) { t, dir, arena, stride, data_len,
                                n * (uint64_t) i / (uint64_t) threads,
                                n * (uint64_t) (i + 1) / (uint64_t) threads, seq0, status };
        if (pthread_create(&tid[i], NULL, bench_worker, &jobs[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);   /* started workers use the caller's buffers */
            return -1.0;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double) (b.tv_sec - a.tv_sec) + 1e-9 * (double) (b.tv_nsec - a.tv_nsec);
}

/* Many connections (the c4 / c4s CPU leg): record i belongs to connection
 * i % nconn with the connection's own sequence number i / nconn, and each
 * connection is served by one thread (connection % threads), as
 * evp_mixed_records in evp_bench.c. */
typedef struct {
    const orc_transform *const *ts;
    uint32_t nconn;
    int dir, t, threads;
    uint8_t *arena;
    size_t stride, data_len;
    uint64_t n;
    int32_t *status;
} bench_mjob;

static void *bench_mworker(void *arg)
{
    bench_mjob *j = (bench_mjob *) arg;
    for (uint64_t i = 0; i < j->n; i++) {
        const uint32_t c = (uint32_t) (i % j->nconn);
        if ((int) (c % (uint32_t) j->threads) != j->t) continue;
        const orc_transform *t = j->ts[c];
        orc_record rec;
        rec.cid_len = 0;
        uint64_t seq = i / j->nconn;
        for (int k = 7; k >= 0; k--) { rec.ctr[k] = (uint8_t) seq; seq >>= 8; }
        rec.type = 23;
        rec.ver[0] = 3; rec.ver[1] = 3;
        rec.buf = j->arena + i * j->stride;
        rec.buf_len = j->stride;
        rec.data_offset = (j->dir && t->ivlen != t->fixed_ivlen) ? 8 : 0;
        rec.data_len = j->data_len;
        const int r = j->dir ? orc_encrypt_buf(t, &rec) : orc_decrypt_buf(t, &rec);
        if (j->status) j->status[i] = r;
    }
    return NULL;
}

double orc_bench_records_multi(const orc_transform *const *ts, uint32_t nconn, int dir, uint8_t *arena,
                               size_t stride, size_t data_len, uint64_t n, int threads, int32_t *status)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    bench_mjob jobs[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < threads; i++) {
        jobs[i] = (bench_mjob) { ts, nconn, dir, i, threads, arena, stride, data_len, n, status };
        if (pthread_create(&tid[i], NULL, bench_mworker, &jobs[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);   /* started workers use the caller's buffers */
            return -1.0;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double) (b.tv_sec - a.tv_sec) + 1e-9 * (double) (b.tv_nsec - a.tv_nsec);
}
