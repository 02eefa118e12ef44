/*
 * keysched.c -- CPU restatement of the TLS 1.3 key schedule of Mbed TLS 4.1.0.
 *
 * TEST INFRASTRUCTURE ONLY (scope and pinning: oracle.h, oracle/README.md).
 *
 * Reference functions restated (library/ssl_tls13_keys.c):
 *   ssl_tls13_hkdf_encode_label            :98-136  (HkdfLabel, RFC 8446 7.1)
 *   mbedtls_ssl_tls13_hkdf_expand_label    :138-217 (HKDF-Expand over HkdfLabel)
 *   ssl_tls13_make_traffic_key             :219-246 ("key" / "iv" with empty context)
 *   mbedtls_ssl_tls13_make_traffic_keys    :262-291
 *   mbedtls_ssl_tls13_derive_secret        :293-330 (context hashed unless CONTEXT_HASHED)
 *   mbedtls_ssl_tls13_evolve_secret        :332-419 (Derive-Secret(., "derived", "") then
 *                                                    HKDF-Extract; zero IKM when input is empty)
 *   mbedtls_ssl_tls13_exporter             :1828-1858
 *   labels                                  library/ssl_tls13_keys.h:13-33 ("traffic upd" :16)
 * Key update (RFC 8446 7.2): the label "traffic upd" is declared at
 * ssl_tls13_keys.h:16; application_traffic_secret_N+1 =
 * HKDF-Expand-Label(secret_N, "traffic upd", "", Hash.length).
 *
 * The hash / HMAC / HKDF primitives live in the absent TF-PSA-Crypto
 * (psa_hash_compute, PSA_ALG_HKDF_EXTRACT / _EXPAND); they are restated from
 * FIPS 180-4 (SHA-256, SHA-384/512), RFC 2104 (HMAC) and RFC 5869 (HKDF).
 */
#include "oracle.h"

#include <string.h>

/* ---------------- SHA-256 (FIPS 180-4 6.2) ------------------------------ */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2 };

static uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void sha256_block(uint32_t h[8], const uint8_t *p)
{
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t) p[4 * i] << 24) | ((uint32_t) p[4 * i + 1] << 16) | ((uint32_t) p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = hh + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* ---------------- SHA-512 / SHA-384 (FIPS 180-4 6.4, 6.5) --------------- */
static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL };

static void sha512_block(uint64_t h[8], const uint8_t *p)
{
    uint64_t w[80];
    for (int i = 0; i < 16; i++) {
        uint64_t v = 0;
        for (int j = 0; j < 8; j++) v = (v << 8) | p[8 * i + j];
        w[i] = v;
    }
    for (int i = 16; i < 80; i++) {
        uint64_t s0 = ror64(w[i - 15], 1) ^ ror64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        uint64_t s1 = ror64(w[i - 2], 19) ^ ror64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 80; i++) {
        uint64_t t1 = hh + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + w[i];
        uint64_t t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* Incremental hash over SHA-256 or SHA-384. */
typedef struct {
    int alg;                  /* ORC_HASH_SHA256 / ORC_HASH_SHA384 */
    uint32_t h32[8];
    uint64_t h64[8];
    uint8_t buf[128];
    size_t fill;
    uint64_t total;
} hctx;

static size_t blk_of(int alg) { return alg == ORC_HASH_SHA384 ? 128 : 64; }

size_t orc_hash_len(int alg)
{
    return alg == ORC_HASH_SHA256 ? 32 : alg == ORC_HASH_SHA384 ? 48 : 0;
}

static void h_init(hctx *c, int alg)
{
    static const uint32_t iv256[8] = { 0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                       0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19 };
    static const uint64_t iv384[8] = { 0xcbbb9d5dc1059ed8ULL, 0x629a292a367cd507ULL, 0x9159015a3070dd17ULL,
                                       0x152fecd8f70e5939ULL, 0x67332667ffc00b31ULL, 0x8eb44a8768581511ULL,
                                       0xdb0c2e0d64f98fa7ULL, 0x47b5481dbefa4fa4ULL };
    memset(c, 0, sizeof(*c));
    c->alg = alg;
    memcpy(c->h32, iv256, sizeof(iv256));
    memcpy(c->h64, iv384, sizeof(iv384));
}

static void h_compress(hctx *c, const uint8_t *p)
{
    if (c->alg == ORC_HASH_SHA384) sha512_block(c->h64, p);
    else sha256_block(c->h32, p);
}

static void h_update(hctx *c, const uint8_t *p, size_t n)
{
    const size_t B = blk_of(c->alg);
    c->total += n;
    while (n) {
        size_t take = B - c->fill < n ? B - c->fill : n;
        memcpy(c->buf + c->fill, p, take);
        c->fill += take; p += take; n -= take;
        if (c->fill == B) { h_compress(c, c->buf); c->fill = 0; }
    }
}

static void h_final(hctx *c, uint8_t *out)
{
    const size_t B = blk_of(c->alg), L = B == 128 ? 16 : 8;
    uint64_t bits = c->total * 8;
    uint8_t pad = 0x80;
    h_update(c, &pad, 1);
    c->total--;                                   /* padding is not message */
    uint8_t z = 0;
    while (c->fill != B - L) { h_update(c, &z, 1); c->total--; }
    uint8_t len[16] = { 0 };
    for (int i = 0; i < 8; i++) len[L - 1 - i] = (uint8_t) (bits >> (8 * i));
    h_update(c, len, L);
    if (c->alg == ORC_HASH_SHA384) {
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 8; j++) out[8 * i + j] = (uint8_t) (c->h64[i] >> (56 - 8 * j));
    } else {
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t) (c->h32[i] >> (24 - 8 * j));
    }
}

int orc_hash(int alg, const uint8_t *msg, size_t len, uint8_t *out)
{
    if (!orc_hash_len(alg)) return ORC_ERR_SSL_BAD_INPUT_DATA;
    hctx c;
    h_init(&c, alg);
    h_update(&c, msg, len);
    h_final(&c, out);
    return 0;
}

/* ---------------- HMAC (RFC 2104) / HKDF (RFC 5869) ---------------------- */
/* HMAC over the concatenation m1 || m2 || m3 (any may be empty). */
static void hmac3(int alg, const uint8_t *key, size_t klen, const uint8_t *m1, size_t l1, const uint8_t *m2,
                  size_t l2, const uint8_t *m3, size_t l3, uint8_t *out)
{
    const size_t B = blk_of(alg), H = orc_hash_len(alg);
    uint8_t k0[128] = { 0 }, pad[128], inner[64];
    if (klen > B) orc_hash(alg, key, klen, k0);
    else if (klen) memcpy(k0, key, klen);
    hctx c;
    for (size_t i = 0; i < B; i++) pad[i] = k0[i] ^ 0x36;
    h_init(&c, alg);
    h_update(&c, pad, B);
    if (l1) h_update(&c, m1, l1);
    if (l2) h_update(&c, m2, l2);
    if (l3) h_update(&c, m3, l3);
    h_final(&c, inner);
    for (size_t i = 0; i < B; i++) pad[i] = k0[i] ^ 0x5c;
    h_init(&c, alg);
    h_update(&c, pad, B);
    h_update(&c, inner, H);
    h_final(&c, out);
}

int orc_hmac(int alg, const uint8_t *key, size_t klen, const uint8_t *msg, size_t len, uint8_t *out)
{
    if (!orc_hash_len(alg)) return ORC_ERR_SSL_BAD_INPUT_DATA;
    hmac3(alg, key, klen, msg, len, NULL, 0, NULL, 0, out);
    return 0;
}

/* HKDF-Extract(salt, IKM) = HMAC(salt, IKM), RFC 5869 2.2 */
int orc_hkdf_extract(int alg, const uint8_t *salt, size_t salt_len, const uint8_t *ikm, size_t ikm_len,
                     uint8_t *prk)
{
    return orc_hmac(alg, salt, salt_len, ikm, ikm_len, prk);
}

/* HKDF-Expand(PRK, info, L), RFC 5869 2.3: T(i) = HMAC(PRK, T(i-1) | info | i) */
int orc_hkdf_expand(int alg, const uint8_t *prk, size_t prk_len, const uint8_t *info, size_t info_len,
                    uint8_t *out, size_t out_len)
{
    const size_t H = orc_hash_len(alg);
    if (!H || out_len > 255 * H) return ORC_ERR_SSL_BAD_INPUT_DATA;
    uint8_t t[64];
    size_t done = 0;
    for (uint8_t i = 1; done < out_len; i++) {
        hmac3(alg, prk, prk_len, t, i == 1 ? 0 : H, info, info_len, &i, 1, t);
        size_t take = out_len - done < H ? out_len - done : H;
        memcpy(out + done, t, take);
        done += take;
    }
    return 0;
}

/* ---------------- TLS 1.3 (library/ssl_tls13_keys.c) --------------------- */
#define ORC_TLS13_MAX_LABEL 249                       /* ssl_tls13_keys.h:66 */
#define ORC_TLS13_MAX_CONTEXT 64                      /* PSA_HASH_MAX_SIZE, ssl_tls13_keys.h:71 */

/* ssl_tls13_hkdf_encode_label, ssl_tls13_keys.c:98-136:
 *   uint16 length || uint8 len("tls13 " + label) || "tls13 " || label || uint8 len(ctx) || ctx */
size_t orc_tls13_encode_label(size_t desired, const uint8_t *label, size_t label_len, const uint8_t *ctx,
                              size_t ctx_len, uint8_t *dst)
{
    uint8_t *p = dst;
    *p++ = (uint8_t) (desired >> 8);
    *p++ = (uint8_t) desired;
    *p++ = (uint8_t) (6 + label_len);
    memcpy(p, "tls13 ", 6);
    p += 6;
    if (label_len) memcpy(p, label, label_len);
    p += label_len;
    *p++ = (uint8_t) ctx_len;
    if (ctx_len) memcpy(p, ctx, ctx_len);
    p += ctx_len;
    return (size_t) (p - dst);
}

/* mbedtls_ssl_tls13_hkdf_expand_label, ssl_tls13_keys.c:138-217 */
int orc_tls13_hkdf_expand_label(int alg, const uint8_t *secret, size_t secret_len, const uint8_t *label,
                                size_t label_len, const uint8_t *ctx, size_t ctx_len, uint8_t *buf, size_t buf_len)
{
    if (label_len > ORC_TLS13_MAX_LABEL || ctx_len > ORC_TLS13_MAX_CONTEXT) return ORC_ERR_SSL_INTERNAL_ERROR;
    if (buf_len > 255 * 64) return ORC_ERR_SSL_INTERNAL_ERROR;   /* MAX_EXPANSION_LEN = 255 * PSA_HASH_MAX_SIZE, ssl_tls13_keys.h:78 */
    if (!orc_hash_len(alg)) return ORC_ERR_SSL_BAD_INPUT_DATA;
    uint8_t info[2 + 1 + 6 + ORC_TLS13_MAX_LABEL + 1 + ORC_TLS13_MAX_CONTEXT];
    size_t n = orc_tls13_encode_label(buf_len, label, label_len, ctx, ctx_len, info);
    return orc_hkdf_expand(alg, secret, secret_len, info, n, buf, buf_len);
}

/* mbedtls_ssl_tls13_derive_secret, ssl_tls13_keys.c:293-330 */
int orc_tls13_derive_secret(int alg, const uint8_t *secret, size_t secret_len, const uint8_t *label,
                            size_t label_len, const uint8_t *ctx, size_t ctx_len, int ctx_hashed, uint8_t *dst,
                            size_t dst_len)
{
    uint8_t hashed[64];
    if (ctx_hashed == ORC_TLS13_CONTEXT_UNHASHED) {
        int r = orc_hash(alg, ctx, ctx_len, hashed);
        if (r) return r;
        ctx_len = orc_hash_len(alg);
    } else {
        if (ctx_len > sizeof(hashed)) return ORC_ERR_SSL_INTERNAL_ERROR;
        if (ctx_len) memcpy(hashed, ctx, ctx_len);
    }
    return orc_tls13_hkdf_expand_label(alg, secret, secret_len, label, label_len, hashed, ctx_len, dst, dst_len);
}

/* mbedtls_ssl_tls13_evolve_secret, ssl_tls13_keys.c:332-419 */
int orc_tls13_evolve_secret(int alg, const uint8_t *secret_old, const uint8_t *input, size_t input_len,
                            uint8_t *secret_new)
{
    const size_t H = orc_hash_len(alg);
    if (!H) return ORC_ERR_SSL_BAD_INPUT_DATA;
    uint8_t tmp[64] = { 0 }, zeros[64] = { 0 };
    if (secret_old) {
        int r = orc_tls13_derive_secret(alg, secret_old, H, (const uint8_t *) "derived", 7, NULL, 0,
                                        ORC_TLS13_CONTEXT_UNHASHED, tmp, H);
        if (r) return r;
    }
    const uint8_t *ikm = (input && input_len) ? input : zeros;
    size_t ikm_len = (input && input_len) ? input_len : H;
    return orc_hkdf_extract(alg, tmp, H, ikm, ikm_len, secret_new);
}

/* mbedtls_ssl_tls13_make_traffic_keys, ssl_tls13_keys.c:219-291 */
int orc_tls13_make_traffic_keys(int alg, const uint8_t *client_secret, const uint8_t *server_secret,
                                size_t secret_len, size_t key_len, size_t iv_len, uint8_t *client_key,
                                uint8_t *client_iv, uint8_t *server_key, uint8_t *server_iv)
{
    int r;
    if ((r = orc_tls13_hkdf_expand_label(alg, client_secret, secret_len, (const uint8_t *) "key", 3, NULL, 0,
                                         client_key, key_len)) ||
        (r = orc_tls13_hkdf_expand_label(alg, client_secret, secret_len, (const uint8_t *) "iv", 2, NULL, 0,
                                         client_iv, iv_len)) ||
        (r = orc_tls13_hkdf_expand_label(alg, server_secret, secret_len, (const uint8_t *) "key", 3, NULL, 0,
                                         server_key, key_len)) ||
        (r = orc_tls13_hkdf_expand_label(alg, server_secret, secret_len, (const uint8_t *) "iv", 2, NULL, 0,
                                         server_iv, iv_len)))
        return r;
    return 0;
}

/* mbedtls_ssl_tls13_exporter, ssl_tls13_keys.c:1828-1858 */
int orc_tls13_exporter(int alg, const uint8_t *secret, size_t secret_len, const uint8_t *label, size_t label_len,
                       const uint8_t *context, size_t context_len, uint8_t *out, size_t out_len)
{
    const size_t H = orc_hash_len(alg);
    uint8_t s[64];
    int r = orc_tls13_derive_secret(alg, secret, secret_len, label, label_len, NULL, 0, ORC_TLS13_CONTEXT_UNHASHED,
                                    s, H);
    if (r) return r;
    return orc_tls13_derive_secret(alg, s, H, (const uint8_t *) "exporter", 8, context, context_len,
                                   ORC_TLS13_CONTEXT_UNHASHED, out, out_len);
}

/* Key update, RFC 8446 7.2 (label ssl_tls13_keys.h:16). */
int orc_tls13_update_traffic_secret(int alg, const uint8_t *secret, uint8_t *next)
{
    const size_t H = orc_hash_len(alg);
    if (!H) return ORC_ERR_SSL_BAD_INPUT_DATA;
    return orc_tls13_hkdf_expand_label(alg, secret, H, (const uint8_t *) "traffic upd", 11, NULL, 0, next, H);
}
