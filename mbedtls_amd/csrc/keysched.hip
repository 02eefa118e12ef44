/*
 * keysched.hip -- TLS 1.3 key schedule on the GPU.
 *
 * HKDF-SHA256 / HKDF-SHA384 (RFC 5869 over FIPS 180-4, HMAC per RFC 2104)
 * with the TLS 1.3 label encoding of library/ssl_tls13_keys.c:
 *
 *   reference                                   here
 *   ssl_tls13_hkdf_encode_label      :98-136    encode_label()       (host: framing only)
 *   mbedtls_ssl_tls13_hkdf_expand_label :138    tlsrec_tls13_hkdf_expand_label
 *   mbedtls_ssl_tls13_make_traffic_keys :262    tlsrec_tls13_make_traffic_keys
 *   mbedtls_ssl_tls13_derive_secret     :293    tlsrec_tls13_derive_secret
 *   mbedtls_ssl_tls13_evolve_secret     :332    tlsrec_tls13_evolve_secret
 *   mbedtls_ssl_tls13_exporter          :1828   tlsrec_tls13_exporter
 *   "traffic upd" (ssl_tls13_keys.h:16)         tlsrec_tls13_update_traffic_secret (RFC 8446 7.2)
 *   (batch)                                     tlsrec_tls13_keytab_derive: secrets in HBM ->
 *                                               key material -> key-table slots, no host round trip
 *
 * Every hash, HMAC and HKDF step runs in a kernel; the host only encodes the
 * HkdfLabel byte string (length, "tls13 " + label, context length), moves
 * bytes and checks arguments the way the reference does.  One thread per
 * derivation: this is per-connection control work (a few SHA compressions),
 * not the bulk path, so lanes are independent and the message buffers live
 * in per-lane scratch.
 */
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "tlsrec.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"

namespace tlsks {

/* ---------------- SHA-2 round constants (FIPS 180-4 4.2.2, 4.2.3) ------- */
__constant__ const uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2 };

__constant__ const uint64_t kK512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL };

enum { H_SHA256 = 0, H_SHA384 = 1 };

__device__ __forceinline__ uint32_t ror32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

/* The message block is kept as big-endian words (16 x 32 bit for SHA-256,
 * 16 x 64 bit for SHA-384), filled a byte at a time. */
struct Hash {
    uint32_t alg;
    uint32_t fill;            /* bytes in the current block */
    uint64_t total;           /* message bytes absorbed */
    uint64_t st[8];           /* SHA-256 uses the low 32 bits */
    uint64_t w[16];           /* SHA-256 uses the low 32 bits of w[0..15] */
};

__device__ __forceinline__ uint32_t blk_bytes(uint32_t alg) { return alg == H_SHA384 ? 128u : 64u; }
__device__ __forceinline__ uint32_t out_bytes(uint32_t alg) { return alg == H_SHA384 ? 48u : 32u; }

__device__ void compress(Hash &h)
{
    if (h.alg == H_SHA384) {
        uint64_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = h.w[i];
        uint64_t a = h.st[0], b = h.st[1], c = h.st[2], d = h.st[3], e = h.st[4], f = h.st[5], g = h.st[6],
                 k = h.st[7];
        for (int i = 0; i < 80; i++) {
            uint64_t wi;
            if (i < 16) {
                wi = w[i & 15];
            } else {
                const uint64_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
                wi = w[i & 15] + (ror64(w15, 1) ^ ror64(w15, 8) ^ (w15 >> 7)) + w[(i - 7) & 15] +
                     (ror64(w2, 19) ^ ror64(w2, 61) ^ (w2 >> 6));
                w[i & 15] = wi;
            }
            const uint64_t t1 = k + (ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41)) + ((e & f) ^ (~e & g)) + kK512[i] + wi;
            const uint64_t t2 = (ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
            k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h.st[0] += a; h.st[1] += b; h.st[2] += c; h.st[3] += d;
        h.st[4] += e; h.st[5] += f; h.st[6] += g; h.st[7] += k;
    } else {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = (uint32_t) h.w[i];
        uint32_t a = (uint32_t) h.st[0], b = (uint32_t) h.st[1], c = (uint32_t) h.st[2], d = (uint32_t) h.st[3];
        uint32_t e = (uint32_t) h.st[4], f = (uint32_t) h.st[5], g = (uint32_t) h.st[6], k = (uint32_t) h.st[7];
        for (int i = 0; i < 64; i++) {
            uint32_t wi;
            if (i < 16) {
                wi = w[i & 15];
            } else {
                const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
                wi = w[i & 15] + (ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3)) + w[(i - 7) & 15] +
                     (ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10));
                w[i & 15] = wi;
            }
            const uint32_t t1 = k + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + kK256[i] + wi;
            const uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h.st[0] = (uint32_t) (h.st[0] + a); h.st[1] = (uint32_t) (h.st[1] + b);
        h.st[2] = (uint32_t) (h.st[2] + c); h.st[3] = (uint32_t) (h.st[3] + d);
        h.st[4] = (uint32_t) (h.st[4] + e); h.st[5] = (uint32_t) (h.st[5] + f);
        h.st[6] = (uint32_t) (h.st[6] + g); h.st[7] = (uint32_t) (h.st[7] + k);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) h.w[i] = 0;
    h.fill = 0;
}

__device__ void hinit(Hash &h, uint32_t alg)
{
    /* FIPS 180-4 5.3.3 (SHA-256) and 5.3.4 (SHA-384) */
    const uint64_t iv256[8] = { 0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19 };
    const uint64_t iv384[8] = { 0xcbbb9d5dc1059ed8ULL, 0x629a292a367cd507ULL, 0x9159015a3070dd17ULL,
                                0x152fecd8f70e5939ULL, 0x67332667ffc00b31ULL, 0x8eb44a8768581511ULL,
                                0xdb0c2e0d64f98fa7ULL, 0x47b5481dbefa4fa4ULL };
    h.alg = alg;
    h.fill = 0;
    h.total = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) h.st[i] = alg == H_SHA384 ? iv384[i] : iv256[i];
#pragma unroll
    for (int i = 0; i < 16; i++) h.w[i] = 0;
}

/* absorb one byte (no length accounting) */
__device__ __forceinline__ void put(Hash &h, uint32_t byte)
{
    const uint32_t wb = h.alg == H_SHA384 ? 8u : 4u;
    const uint32_t idx = h.fill / wb, sh = 8 * (wb - 1 - h.fill % wb);
    h.w[idx] |= (uint64_t) (byte & 0xff) << sh;
    if (++h.fill == blk_bytes(h.alg)) compress(h);
}

__device__ void update(Hash &h, const uint8_t *p, uint32_t n, uint8_t x = 0)
{
    for (uint32_t i = 0; i < n; i++) put(h, p[i] ^ x);
    h.total += n;
}

/* n copies of byte b (key padding) */
__device__ void update_fill(Hash &h, uint8_t b, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) put(h, b);
    h.total += n;
}

__device__ void finish(Hash &h, uint8_t *out)
{
    const uint64_t bits = h.total * 8;
    const uint32_t B = blk_bytes(h.alg), L = h.alg == H_SHA384 ? 16u : 8u;
    put(h, 0x80);
    while (h.fill != B - L) put(h, 0);
    for (uint32_t i = 0; i < L; i++) put(h, i < L - 8 ? 0u : (uint32_t) (bits >> (8 * (L - 1 - i))));
    const uint32_t n = out_bytes(h.alg);
    for (uint32_t i = 0; i < n; i++) {
        if (h.alg == H_SHA384) out[i] = (uint8_t) (h.st[i / 8] >> (56 - 8 * (i % 8)));
        else out[i] = (uint8_t) (h.st[i / 4] >> (24 - 8 * (i % 4)));
    }
}

/* HMAC (RFC 2104) with a key already reduced to <= one block. */
struct Hmac {
    Hash in;
    uint8_t k0[128];
    uint32_t klen;
};

__device__ void hmac_start(Hmac &m, uint32_t alg, const uint8_t *key, uint32_t klen)
{
    const uint32_t B = blk_bytes(alg);
    if (klen > B) {                     /* RFC 2104 2: hash keys longer than the block */
        Hash t;
        hinit(t, alg);
        update(t, key, klen);
        finish(t, m.k0);
        klen = out_bytes(alg);
    } else {
        for (uint32_t i = 0; i < klen; i++) m.k0[i] = key[i];
    }
    m.klen = klen;
    hinit(m.in, alg);
    update(m.in, m.k0, klen, 0x36);
    update_fill(m.in, 0x36, B - klen);
}

__device__ void hmac_end(Hmac &m, uint8_t *out)
{
    uint8_t inner[64];
    finish(m.in, inner);
    const uint32_t alg = m.in.alg, B = blk_bytes(alg);
    Hash o;
    hinit(o, alg);
    update(o, m.k0, m.klen, 0x5c);
    update_fill(o, 0x5c, B - m.klen);
    update(o, inner, out_bytes(alg));
    finish(o, out);
}

/* HKDF-Expand (RFC 5869 2.3) with info = info1 || info2:
 * T(i) = HMAC(PRK, T(i-1) || info || i), OKM = first L bytes of T(1)||T(2)... */
__device__ void hkdf_expand(uint32_t alg, const uint8_t *prk, uint32_t prk_len, const uint8_t *info1,
                            uint32_t len1, const uint8_t *info2, uint32_t len2, uint8_t *out, uint32_t out_len)
{
    const uint32_t H = out_bytes(alg);
    uint8_t t[64];
    uint32_t done = 0;
    for (uint32_t i = 1; done < out_len; i++) {
        Hmac m;
        hmac_start(m, alg, prk, prk_len);
        if (i > 1) update(m.in, t, H);
        update(m.in, info1, len1);
        update(m.in, info2, len2);
        const uint8_t ctr = (uint8_t) i;
        update(m.in, &ctr, 1);
        hmac_end(m, t);
        const uint32_t take = out_len - done < H ? out_len - done : H;
        for (uint32_t j = 0; j < take; j++) out[done + j] = t[j];
        done += take;
    }
}

/* ---------------- kernels ---------------------------------------------- */
enum { OP_HASH = 0, OP_HMAC = 1, OP_EXPAND = 2 };

struct Job {
    uint32_t op, alg;
    const uint8_t *key;
    uint32_t key_len;
    const uint8_t *msg;       /* message / info (first part) */
    uint32_t msg_len;
    const uint8_t *msg2;      /* info, second part (a context computed on the device) */
    uint32_t msg2_len;
    uint8_t *out;
    uint32_t out_len;
};

__global__ void __launch_bounds__(64) kdf_job_kernel(const Job *jobs, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Job j = jobs[i];
    if (j.op == OP_HASH) {
        Hash h;
        hinit(h, j.alg);
        update(h, j.msg, j.msg_len);
        update(h, j.msg2, j.msg2_len);
        finish(h, j.out);
    } else if (j.op == OP_HMAC) {
        Hmac m;
        hmac_start(m, j.alg, j.key, j.key_len);
        update(m.in, j.msg, j.msg_len);
        update(m.in, j.msg2, j.msg2_len);
        hmac_end(m, j.out);
    } else {
        hkdf_expand(j.alg, j.key, j.key_len, j.msg, j.msg_len, j.msg2, j.msg2_len, j.out, j.out_len);
    }
}

/* Batch traffic-key derivation: one thread per connection direction.
 * infos = HkdfLabel("traffic upd", "", H) || HkdfLabel("key", "", key_len)
 *         || HkdfLabel("iv", "", 12), encoded on the host (same for all). */
struct DeriveArgs {
    tlsrec_tls13_secret *secrets;
    tlsrec_key_material *out;
    uint8_t infos[96];        /* the three encoded HkdfLabels, by value (no host staging buffer) */
    uint32_t len_upd, len_key, len_iv;
    uint32_t count, alg, cipher, key_len, update;
};

__global__ void __launch_bounds__(64) tls13_derive_kernel(DeriveArgs a)
{
    /* the encoded labels (kernel argument) staged once per workgroup */
    __shared__ uint8_t infos[96];
    for (int k = threadIdx.x; k < 96; k += blockDim.x) infos[k] = a.infos[k];
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.count) return;
    const uint32_t H = out_bytes(a.alg);
    uint8_t s[48];
    for (uint32_t k = 0; k < H; k++) s[k] = a.secrets[i].secret[k];
    if (a.update) {
        /* RFC 8446 7.2: secret_N+1 = HKDF-Expand-Label(secret_N, "traffic upd", "", H) */
        uint8_t nx[48];
        hkdf_expand(a.alg, s, H, infos, a.len_upd, nullptr, 0, nx, H);
        for (uint32_t k = 0; k < H; k++) {
            s[k] = nx[k];
            a.secrets[i].secret[k] = nx[k];
        }
    }
    tlsrec_key_material km;
    uint8_t *raw = (uint8_t *) &km;
    for (int k = 0; k < 64; k++) raw[k] = 0;
    km.cipher = (uint8_t) a.cipher;
    km.tls_minor = 4;
    km.fixed_ivlen = 12;      /* TLS 1.3: fixed_ivlen = ivlen = 12, ssl_tls13_keys.c:985-998 */
    km.taglen = (uint8_t) tlsrec_cipher_taglen((int) a.cipher);
    /* ssl_tls13_make_traffic_key, ssl_tls13_keys.c:219-246 */
    hkdf_expand(a.alg, s, H, infos + a.len_upd, a.len_key, nullptr, 0, km.key, a.key_len);
    hkdf_expand(a.alg, s, H, infos + a.len_upd + a.len_key, a.len_iv, nullptr, 0, km.iv, 12);
    uint4 *dst = reinterpret_cast<uint4 *>(a.out + i);
    const uint4 *src = reinterpret_cast<const uint4 *>(&km);
#pragma unroll
    for (int k = 0; k < 4; k++) dst[k] = src[k];
}

} /* namespace tlsks */

using namespace tlsks;

/* ======================================================================
 * host side
 * ==================================================================== */
static const size_t MAX_LABEL = 249;        /* MBEDTLS_SSL_TLS1_3_HKDF_LABEL_MAX_LABEL_LEN, ssl_tls13_keys.h:66 */
static const size_t MAX_CONTEXT = 64;       /* MBEDTLS_SSL_TLS1_3_KEY_SCHEDULE_MAX_CONTEXT_LEN = PSA_HASH_MAX_SIZE */
static const size_t MAX_EXPANSION = 255 * 64;   /* ..._MAX_EXPANSION_LEN = 255 * MBEDTLS_TLS1_3_MD_MAX_SIZE */

static int alg_index(int hash_alg)
{
    return hash_alg == TLSREC_ALG_SHA_256 ? H_SHA256 : hash_alg == TLSREC_ALG_SHA_384 ? H_SHA384 : -1;
}

static size_t alg_len(int idx) { return idx == H_SHA384 ? 48 : 32; }

/* ssl_tls13_hkdf_encode_label, ssl_tls13_keys.c:98-136 (without the context
 * bytes when ctx == NULL: the caller appends a device-computed context) */
static size_t encode_label(size_t desired, const unsigned char *label, size_t label_len, const unsigned char *ctx,
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
    if (ctx && ctx_len) {
        memcpy(p, ctx, ctx_len);
        p += ctx_len;
    }
    return (size_t) (p - dst);
}

/* A device arena for single-shot calls: inputs are packed into one host
 * buffer, copied once, the job chain runs, the outputs come back. */
namespace {
struct Arena {
    uint8_t host[32768];
    size_t used = 0;
    size_t put(const void *p, size_t n)
    {
        size_t off = used;
        if (n && p) memcpy(host + off, p, n);
        else if (n) memset(host + off, 0, n);
        used = (used + n + 15) & ~(size_t) 15;
        return off;
    }
};
}

static pthread_mutex_t g_ks_mu = PTHREAD_MUTEX_INITIALIZER;
static hipStream_t g_ks_stream = nullptr;
static uint8_t *g_ks_dev = nullptr;          /* 32 KiB arena + job array */
static const size_t KS_DEV_BYTES = 32768 + 16 * sizeof(Job);

static int ks_init_locked(void)
{
    if (g_ks_dev) return 0;
    if (tlsrec_device_check() != 0) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    if (hipStreamCreateWithFlags(&g_ks_stream, hipStreamNonBlocking) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    if (hipMalloc((void **) &g_ks_dev, KS_DEV_BYTES) != hipSuccess) {
        g_ks_dev = nullptr;
        return TLSREC_ERR_SSL_ALLOC_FAILED;
    }
    return 0;
}

/* Run `stages` dependent launches; stage s runs jobs [first[s], first[s+1]).
 * Job pointers are arena offsets (tagged with bit 63) rebased to the device. */
static const uint64_t OFF = 1ull << 62;
static inline const uint8_t *dev_off(size_t off) { return (const uint8_t *) (uintptr_t) (OFF | off); }

static int run_jobs(Arena &ar, Job *jobs, const int *first, int stages, const size_t *outs, void *const *host_out,
                    const size_t *out_len, int nouts)
{
    pthread_mutex_lock(&g_ks_mu);
    int r = ks_init_locked();
    if (r == 0) {
        const int njobs = first[stages];
        auto fix = [](const uint8_t *p) -> const uint8_t * {
            const uint64_t v = (uint64_t) (uintptr_t) p;
            return (v & OFF) ? g_ks_dev + (v & ~OFF) : p;
        };
        for (int i = 0; i < njobs; i++) {
            jobs[i].key = fix(jobs[i].key);
            jobs[i].msg = fix(jobs[i].msg);
            jobs[i].msg2 = fix(jobs[i].msg2);
            jobs[i].out = (uint8_t *) fix(jobs[i].out);
        }
        Job *djobs = (Job *) (g_ks_dev + 32768);
        hipError_t e = hipMemcpyAsync(g_ks_dev, ar.host, ar.used, hipMemcpyHostToDevice, g_ks_stream);
        if (e == hipSuccess) e = hipMemcpyAsync(djobs, jobs, sizeof(Job) * njobs, hipMemcpyHostToDevice, g_ks_stream);
        for (int s = 0; s < stages && e == hipSuccess; s++) {
            const uint32_t n = (uint32_t) (first[s + 1] - first[s]);
            hipLaunchKernelGGL(kdf_job_kernel, dim3(1), dim3(64), 0, g_ks_stream, djobs + first[s], n);
            e = hipGetLastError();
        }
        for (int o = 0; o < nouts && e == hipSuccess; o++)
            e = hipMemcpyAsync(host_out[o], g_ks_dev + outs[o], out_len[o], hipMemcpyDeviceToHost, g_ks_stream);
        if (e == hipSuccess) e = hipStreamSynchronize(g_ks_stream);
        /* wipe secrets from the device arena (ssl_tls13_keys.c zeroizes its temporaries) */
        hipMemsetAsync(g_ks_dev, 0, ar.used, g_ks_stream);
        hipStreamSynchronize(g_ks_stream);
        if (e != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    pthread_mutex_unlock(&g_ks_mu);
    memset(ar.host, 0, ar.used);
    return r;
}

static Job job(uint32_t op, int alg, size_t key, uint32_t key_len, size_t msg, uint32_t msg_len, size_t out,
               uint32_t out_len)
{
    Job j;
    memset(&j, 0, sizeof(j));
    j.op = op;
    j.alg = (uint32_t) alg;
    j.key = dev_off(key);
    j.key_len = key_len;
    j.msg = dev_off(msg);
    j.msg_len = msg_len;
    j.msg2 = dev_off(0);
    j.msg2_len = 0;
    j.out = (uint8_t *) dev_off(out);
    j.out_len = out_len;
    return j;
}

extern "C" int tlsrec_tls13_hkdf_expand_label(int hash_alg, const unsigned char *secret, size_t secret_len,
                                              const unsigned char *label, size_t label_len,
                                              const unsigned char *ctx, size_t ctx_len, unsigned char *buf,
                                              size_t buf_len)
{
    /* argument checks in the order of ssl_tls13_keys.c:152-171 */
    if (label_len > MAX_LABEL) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (ctx_len > MAX_CONTEXT) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (buf_len > MAX_EXPANSION) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    const int a = alg_index(hash_alg);
    if (a < 0) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (buf_len > 255 * alg_len(a)) return TLSREC_ERR_SSL_BAD_INPUT_DATA;   /* HKDF-Expand limit (PSA: INVALID_ARGUMENT) */
    if (secret_len > 4096) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (buf_len == 0) return 0;
    Arena ar;
    uint8_t info[2 + 1 + 6 + 249 + 1 + 64];
    const size_t il = encode_label(buf_len, label, label_len, ctx, ctx_len, info);
    const size_t o_sec = ar.put(secret, secret_len), o_info = ar.put(info, il), o_out = ar.put(nullptr, buf_len);
    memset(info, 0, sizeof(info));
    if (ar.used > 32768) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    Job j[1] = { job(OP_EXPAND, a, o_sec, (uint32_t) secret_len, o_info, (uint32_t) il, o_out, (uint32_t) buf_len) };
    const int first[2] = { 0, 1 };
    void *ho[1] = { buf };
    return run_jobs(ar, j, first, 1, &o_out, ho, &buf_len, 1);
}

/* Derive-Secret with the context hashed on the device: HASH(ctx) -> EXPAND
 * with info = HkdfLabel prefix || Hash(ctx). */
static int derive_secret_impl(int a, const unsigned char *secret, size_t secret_len, const unsigned char *label,
                              size_t label_len, const unsigned char *ctx, size_t ctx_len, int ctx_hashed,
                              unsigned char *dst, size_t dst_len)
{
    if (label_len > MAX_LABEL) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (ctx_hashed != TLSREC_TLS13_CONTEXT_UNHASHED && ctx_len > MAX_CONTEXT) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (dst_len > MAX_EXPANSION) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (dst_len > 255 * alg_len(a)) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (secret_len > 4096 || (ctx_hashed == TLSREC_TLS13_CONTEXT_UNHASHED && ctx_len > 16384))
        return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (dst_len == 0) return 0;
    Arena ar;
    const size_t H = alg_len(a);
    uint8_t info[2 + 1 + 6 + 249 + 1 + 64];
    const size_t ctx_out = ctx_hashed == TLSREC_TLS13_CONTEXT_UNHASHED ? H : ctx_len;
    /* prefix up to and including the context-length byte */
    const size_t il = encode_label(dst_len, label, label_len, nullptr, ctx_out, info);
    const size_t o_sec = ar.put(secret, secret_len), o_info = ar.put(info, il);
    const size_t o_ctx = ar.put(ctx, ctx_len), o_hash = ar.put(nullptr, 64), o_out = ar.put(nullptr, dst_len);
    memset(info, 0, sizeof(info));
    if (ar.used > 32768) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    Job j[2];
    int first[3];
    int stages;
    if (ctx_hashed == TLSREC_TLS13_CONTEXT_UNHASHED) {
        j[0] = job(OP_HASH, a, 0, 0, o_ctx, (uint32_t) ctx_len, o_hash, (uint32_t) H);
        j[1] = job(OP_EXPAND, a, o_sec, (uint32_t) secret_len, o_info, (uint32_t) il, o_out, (uint32_t) dst_len);
        j[1].msg2 = dev_off(o_hash);
        j[1].msg2_len = (uint32_t) H;
        first[0] = 0; first[1] = 1; first[2] = 2;
        stages = 2;
    } else {
        j[0] = job(OP_EXPAND, a, o_sec, (uint32_t) secret_len, o_info, (uint32_t) il, o_out, (uint32_t) dst_len);
        j[0].msg2 = dev_off(o_ctx);
        j[0].msg2_len = (uint32_t) ctx_len;
        first[0] = 0; first[1] = 1;
        stages = 1;
    }
    void *ho[1] = { dst };
    return run_jobs(ar, j, first, stages, &o_out, ho, &dst_len, 1);
}

extern "C" int tlsrec_tls13_derive_secret(int hash_alg, const unsigned char *secret, size_t secret_len,
                                          const unsigned char *label, size_t label_len, const unsigned char *ctx,
                                          size_t ctx_len, int ctx_hashed, unsigned char *dstbuf, size_t dstbuf_len)
{
    const int a = alg_index(hash_alg);
    if (a < 0) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    return derive_secret_impl(a, secret, secret_len, label, label_len, ctx, ctx_len, ctx_hashed, dstbuf, dstbuf_len);
}

extern "C" int tlsrec_tls13_evolve_secret(int hash_alg, const unsigned char *secret_old, const unsigned char *input,
                                          size_t input_len, unsigned char *secret_new)
{
    const int a = alg_index(hash_alg);
    if (a < 0) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    const size_t H = alg_len(a);
    if (input_len > 16384) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    Arena ar;
    uint8_t info[32];
    const size_t il = encode_label(H, (const unsigned char *) "derived", 7, nullptr, H, info);
    const size_t o_old = ar.put(secret_old, secret_old ? H : 0), o_info = ar.put(info, il);
    const size_t o_empty = ar.put(nullptr, 0), o_hash = ar.put(nullptr, 64), o_tmp = ar.put(nullptr, 64);
    const bool have_in = input != NULL && input_len != 0;
    const size_t o_in = ar.put(have_in ? input : nullptr, have_in ? input_len : H);   /* zeros when absent */
    const size_t o_out = ar.put(nullptr, 64);
    Job j[3];
    int first[4];
    int stages = 0, k = 0;
    first[0] = 0;
    if (secret_old) {
        /* Derive-Secret(secret_old, "derived", "") -> tmp (ssl_tls13_keys.c:358-369) */
        j[k++] = job(OP_HASH, a, 0, 0, o_empty, 0, o_hash, (uint32_t) H);
        first[++stages] = k;
        j[k] = job(OP_EXPAND, a, o_old, (uint32_t) H, o_info, (uint32_t) il, o_tmp, (uint32_t) H);
        j[k].msg2 = dev_off(o_hash);
        j[k++].msg2_len = (uint32_t) H;
        first[++stages] = k;
    }
    /* HKDF-Extract(salt = tmp (zeros for the first stage), IKM) */
    j[k++] = job(OP_HMAC, a, o_tmp, (uint32_t) H, o_in, (uint32_t) (have_in ? input_len : H), o_out, (uint32_t) H);
    first[++stages] = k;
    void *ho[1] = { secret_new };
    return run_jobs(ar, j, first, stages, &o_out, ho, &H, 1);
}

extern "C" int tlsrec_tls13_make_traffic_keys(int hash_alg, const unsigned char *client_secret,
                                              const unsigned char *server_secret, size_t secret_len, size_t key_len,
                                              size_t iv_len, tlsrec_key_set *keys)
{
    const int a = alg_index(hash_alg);
    if (a < 0) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (!keys || key_len > sizeof(keys->client_write_key) || iv_len > sizeof(keys->client_write_iv))
        return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (secret_len > 4096) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    Arena ar;
    uint8_t ik[32], iv[32];
    const size_t lk = encode_label(key_len, (const unsigned char *) "key", 3, nullptr, 0, ik);
    const size_t lv = encode_label(iv_len, (const unsigned char *) "iv", 2, nullptr, 0, iv);
    const size_t o_c = ar.put(client_secret, secret_len), o_s = ar.put(server_secret, secret_len);
    const size_t o_ik = ar.put(ik, lk), o_iv = ar.put(iv, lv);
    const size_t o_ck = ar.put(nullptr, 32), o_ci = ar.put(nullptr, 16), o_sk = ar.put(nullptr, 32),
                 o_si = ar.put(nullptr, 16);
    Job j[4] = { job(OP_EXPAND, a, o_c, (uint32_t) secret_len, o_ik, (uint32_t) lk, o_ck, (uint32_t) key_len),
                 job(OP_EXPAND, a, o_c, (uint32_t) secret_len, o_iv, (uint32_t) lv, o_ci, (uint32_t) iv_len),
                 job(OP_EXPAND, a, o_s, (uint32_t) secret_len, o_ik, (uint32_t) lk, o_sk, (uint32_t) key_len),
                 job(OP_EXPAND, a, o_s, (uint32_t) secret_len, o_iv, (uint32_t) lv, o_si, (uint32_t) iv_len) };
    const int first[2] = { 0, 4 };
    const size_t outs[4] = { o_ck, o_ci, o_sk, o_si };
    void *ho[4] = { keys->client_write_key, keys->client_write_iv, keys->server_write_key, keys->server_write_iv };
    const size_t ol[4] = { key_len, iv_len, key_len, iv_len };
    int r = run_jobs(ar, j, first, 1, outs, ho, ol, 4);
    if (r == 0) {
        keys->key_len = key_len;
        keys->iv_len = iv_len;
    }
    return r;
}

extern "C" int tlsrec_tls13_exporter(int hash_alg, const unsigned char *secret, size_t secret_len,
                                     const unsigned char *label, size_t label_len,
                                     const unsigned char *context_value, size_t context_len, unsigned char *out,
                                     size_t out_len)
{
    const int a = alg_index(hash_alg);
    if (a < 0) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    const size_t H = alg_len(a);
    uint8_t s[64];
    /* ssl_tls13_keys.c:1836-1852: two Derive-Secret steps, unhashed contexts */
    int r = derive_secret_impl(a, secret, secret_len, label, label_len, nullptr, 0, TLSREC_TLS13_CONTEXT_UNHASHED,
                               s, H);
    if (r == 0)
        r = derive_secret_impl(a, s, H, (const unsigned char *) "exporter", 8, context_value, context_len,
                               TLSREC_TLS13_CONTEXT_UNHASHED, out, out_len);
    volatile uint8_t *v = s;
    for (size_t i = 0; i < sizeof(s); i++) v[i] = 0;
    return r;
}

extern "C" int tlsrec_tls13_update_traffic_secret(int hash_alg, const unsigned char *secret, unsigned char *next)
{
    const int a = alg_index(hash_alg);
    if (a < 0) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    const size_t H = alg_len(a);
    return tlsrec_tls13_hkdf_expand_label(hash_alg, secret, H, (const unsigned char *) "traffic upd", 11, nullptr, 0,
                                          next, H);
}

/* engine.hip: key-table bookkeeping + key setup of slots whose material was
 * written to the table's device staging area by a kernel */
extern "C" tlsrec_key_material *tlsrec__keytab_stage(tlsrec_keytab *kt);
extern "C" int tlsrec__keytab_commit_staged(tlsrec_keytab *kt, uint32_t first, uint32_t count, int cipher,
                                            hipStream_t st);

extern "C" int tlsrec_tls13_keytab_derive(tlsrec_keytab *kt, uint32_t first, uint32_t count, int cipher,
                                          tlsrec_tls13_secret *secrets, int key_update, void *stream)
{
    if (!kt || (!secrets && count)) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (first > tlsrec_keytab_capacity(kt) || count > tlsrec_keytab_capacity(kt) - first)
        return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    uint32_t key_len, alg;
    /* TLS 1.3 suites fix the hash with the AEAD (RFC 8446 B.4):
     * TLS_AES_256_GCM_SHA384, every other suite SHA-256 */
    key_len = tlsrec_cipher_keylen(cipher);
    if (key_len == 0) return TLSREC_ERR_SSL_FEATURE_UNAVAILABLE;
    alg = cipher == TLSREC_CIPHER_AES_256_GCM ? H_SHA384 : H_SHA256;
    if (count == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    uint8_t infos[96];
    const uint32_t H = (uint32_t) alg_len((int) alg);
    const size_t lu = encode_label(H, (const unsigned char *) "traffic upd", 11, nullptr, 0, infos);
    const size_t lk = encode_label(key_len, (const unsigned char *) "key", 3, nullptr, 0, infos + lu);
    const size_t lv = encode_label(12, (const unsigned char *) "iv", 2, nullptr, 0, infos + lu + lk);
    DeriveArgs a;
    a.secrets = secrets;
    a.out = tlsrec__keytab_stage(kt) + first;
    memcpy(a.infos, infos, sizeof(a.infos));
    a.len_upd = (uint32_t) lu;
    a.len_key = (uint32_t) lk;
    a.len_iv = (uint32_t) lv;
    a.count = count;
    a.alg = alg;
    a.cipher = (uint32_t) cipher;
    a.key_len = key_len;
    a.update = key_update ? 1u : 0u;
    hipLaunchKernelGGL(tls13_derive_kernel, dim3((count + 63) / 64), dim3(64), 0, st, a);
    int r = hipGetLastError() == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    if (r == 0) r = tlsrec__keytab_commit_staged(kt, first, count, cipher, st);
    return r;
}
