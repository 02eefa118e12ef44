/*
 * tlsrec_clmul.h -- GF(2^128) multiply of two variable elements in the GCM
 * convention (SP 800-38D 6.3) on 32-bit integer arithmetic, no tables: a
 * carry-less 32x32 -> 64 product from four integer multiplies per bit class
 * ("holes" every fourth bit keep the integer carries out of the bits that are
 * read), Karatsuba 128 = 2 x 64 = 4 x 32 (nine 32-bit products), and the
 * reduction by x^128 + x^7 + x^2 + x + 1.
 *
 * Host and device: the kernels use it where a power of H is needed whose
 * position table is not in LDS; gcc builds it for the CPU test
 * (tests/c/clmul_check.c against the oracle's bitwise orc_gf128_mul).
 * Blocks are the 16-byte GCM strings as four little-endian words (the
 * kernels' uint4 layout).
 */
#ifndef TLSREC_CLMUL_H
#define TLSREC_CLMUL_H

#include <stdint.h>

#if defined(__HIPCC__)
#define TLSREC_CLMUL_FN __host__ __device__ __forceinline__
#else
#define TLSREC_CLMUL_FN static inline
#endif

/* a ^ b ^ c ^ d on 64-bit values: two three-input XORs per word on the
 * device (gfx950 v_bitop3_b32), which the compiler does not form itself here */
TLSREC_CLMUL_FN uint64_t tlsrec_xor4_64(uint64_t a, uint64_t b, uint64_t c, uint64_t d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_bitop3_b32(
        __builtin_amdgcn_bitop3_b32((uint32_t) a, (uint32_t) b, (uint32_t) c, 0x96), (uint32_t) d, 0u, 0x96);
    const uint32_t hi = __builtin_amdgcn_bitop3_b32(
        __builtin_amdgcn_bitop3_b32((uint32_t) (a >> 32), (uint32_t) (b >> 32), (uint32_t) (c >> 32), 0x96),
        (uint32_t) (d >> 32), 0u, 0x96);
    return ((uint64_t) hi << 32) | lo;
#else
    return a ^ b ^ c ^ d;
#endif
}

/* carry-less 32 x 32 -> 64: bit class c of x (bits = c mod 4) times bit
 * class d of y lands on class c + d; at most 8 terms meet at a bit, so their
 * integer sum stays below 16 and never carries into the next bit of the
 * same class */
TLSREC_CLMUL_FN uint64_t tlsrec_clmul32(uint32_t x, uint32_t y)
{
    const uint64_t x0 = x & 0x11111111u, x1 = x & 0x22222222u, x2 = x & 0x44444444u, x3 = x & 0x88888888u;
    const uint64_t y0 = y & 0x11111111u, y1 = y & 0x22222222u, y2 = y & 0x44444444u, y3 = y & 0x88888888u;
    const uint64_t z0 = tlsrec_xor4_64(x0 * y0, x1 * y3, x2 * y2, x3 * y1);
    const uint64_t z1 = tlsrec_xor4_64(x0 * y1, x1 * y0, x2 * y3, x3 * y2);
    const uint64_t z2 = tlsrec_xor4_64(x0 * y2, x1 * y1, x2 * y0, x3 * y3);
    const uint64_t z3 = tlsrec_xor4_64(x0 * y3, x1 * y2, x2 * y1, x3 * y0);
    /* class c of the product from z_c: three masked merges under the disjoint
     * class masks (one v_bitop3_b32 per word each) instead of four ANDs and
     * three ORs */
    uint64_t r = z3;
    r = (z2 & 0x4444444444444444ull) | (r & ~0x4444444444444444ull);
    r = (z1 & 0x2222222222222222ull) | (r & ~0x2222222222222222ull);
    r = (z0 & 0x1111111111111111ull) | (r & ~0x1111111111111111ull);
    return r;
}

/* GCM bytes (little-endian word of bytes 4k..4k+3) <-> polynomial word k
 * (bit j = coefficient of x^(32k+j)): reverse the bits of each byte */
TLSREC_CLMUL_FN uint32_t tlsrec_brev8x4(uint32_t w)
{
#if defined(__clang__)
    return __builtin_bswap32(__builtin_bitreverse32(w));     /* v_bfrev_b32 + v_perm_b32 */
#else
    w = ((w >> 1) & 0x55555555u) | ((w & 0x55555555u) << 1);
    w = ((w >> 2) & 0x33333333u) | ((w & 0x33333333u) << 2);
    w = ((w >> 4) & 0x0F0F0F0Fu) | ((w & 0x0F0F0F0Fu) << 4);
    return w;
#endif
}

/* 64 x 64 -> 128 (Karatsuba over 32-bit halves); a, b: 2 words, r: 4 words */
TLSREC_CLMUL_FN void tlsrec_clmul64(const uint32_t a[2], const uint32_t b[2], uint32_t r[4])
{
    const uint64_t lo = tlsrec_clmul32(a[0], b[0]);
    const uint64_t hi = tlsrec_clmul32(a[1], b[1]);
    const uint64_t mid = tlsrec_clmul32(a[0] ^ a[1], b[0] ^ b[1]) ^ lo ^ hi;
    r[0] = (uint32_t) lo;
    r[1] = (uint32_t) (lo >> 32) ^ (uint32_t) mid;
    r[2] = (uint32_t) hi ^ (uint32_t) (mid >> 32);
    r[3] = (uint32_t) (hi >> 32);
}

/* x * y in GF(2^128), GCM strings as little-endian words */
TLSREC_CLMUL_FN void tlsrec_gf128_mul(const uint32_t x[4], const uint32_t y[4], uint32_t out[4])
{
    uint32_t a[4], b[4];
    for (int i = 0; i < 4; i++) {
        a[i] = tlsrec_brev8x4(x[i]);
        b[i] = tlsrec_brev8x4(y[i]);
    }
    /* 128 x 128 -> 256, Karatsuba over 64-bit halves */
    uint32_t l[4], h[4], m[4];
    tlsrec_clmul64(a, b, l);
    tlsrec_clmul64(a + 2, b + 2, h);
    const uint32_t as[2] = { a[0] ^ a[2], a[1] ^ a[3] }, bs[2] = { b[0] ^ b[2], b[1] ^ b[3] };
    tlsrec_clmul64(as, bs, m);
    uint32_t c[8];
    for (int i = 0; i < 4; i++) {
        m[i] ^= l[i] ^ h[i];
        c[i] = l[i];
        c[4 + i] = h[i];
    }
    for (int i = 0; i < 4; i++) c[2 + i] ^= m[i];
    /* reduce: x^128 = x^7 + x^2 + x + 1; H = c[4..7] (degree <= 126) */
    uint32_t r[4];
    for (int i = 0; i < 4; i++) {
        const uint32_t hp = i ? c[3 + i] : 0u;       /* word below, for the carries of the shifts */
        r[i] = c[i] ^ c[4 + i] ^ (c[4 + i] << 1) ^ (hp >> 31) ^ (c[4 + i] << 2) ^ (hp >> 30) ^ (c[4 + i] << 7) ^
               (hp >> 25);
    }
    /* the bits the shifts moved past x^127, folded once more (degree < 14) */
    const uint32_t o = (c[7] >> 31) ^ (c[7] >> 30) ^ (c[7] >> 25);
    r[0] ^= o ^ (o << 1) ^ (o << 2) ^ (o << 7);
    for (int i = 0; i < 4; i++) out[i] = tlsrec_brev8x4(r[i]);
}

/* x * X^s for 0 <= s <= 63 (X the field's generator): with the GCM string
 * as a 128-bit big-endian number V (X^0 the most significant bit), V >> s,
 * and the s bits that fall off (X^128 .. X^(127+s)) folded back with
 * X^128 = X^7 + X^2 + X + 1 -- their product by that stays below X^(s+7) <=
 * X^70, so one fold is enough.  hi / lo are V's two 64-bit halves. */
TLSREC_CLMUL_FN void tlsrec_gf128_shr(uint64_t *hi, uint64_t *lo, uint32_t s)
{
    const uint64_t h = *hi, l = *lo;
    const uint64_t d = s ? l << (64 - s) : 0;              /* the dropped bits, at the top of a word */
    uint64_t rl = s ? (l >> s) | (h << (64 - s)) : l;
    uint64_t rh = h >> s;
    rh ^= d ^ (d >> 1) ^ (d >> 2) ^ (d >> 7);
    rl ^= (d << 63) ^ (d << 62) ^ (d << 57);
    *hi = rh;
    *lo = rl;
}

TLSREC_CLMUL_FN uint32_t tlsrec_bswap32(uint32_t v)
{
    return (v >> 24) | ((v >> 8) & 0xff00u) | ((v << 8) & 0xff0000u) | (v << 24);
}

/* The 4-bit position table of P (the layout of the key-setup kernel and of
 * tlsrec_device.h gmul): window k, entry n = sum over the set bits 3-i of n
 * of P * X^(4k+i), i.e. B_k * poly_n with B_k = P * X^(4k) and poly_n the
 * degree-3 polynomial of n's bits.  The paired GCM passes build a key's
 * Horner table in LDS this way from P = H^L alone instead of reading its
 * 8 KiB from HBM: a lane starts at B_k = P * X^(4k) (two shifts), makes its
 * entry n, and steps to window k + 4 by X^16. */
TLSREC_CLMUL_FN void tlsrec_gtab4_entry(uint64_t bh, uint64_t bl, uint32_t n, uint64_t *rh, uint64_t *rl)
{
    uint64_t ah = 0, al = 0;
    for (int i = 0; i < 4; i++) {
        const uint64_t m = 0 - (uint64_t) ((n >> (3 - i)) & 1u);   /* masks: P is secret */
        ah ^= bh & m;
        al ^= bl & m;
        tlsrec_gf128_shr(&bh, &bl, 1);
    }
    *rh = ah;
    *rl = al;
}

/* words (the kernels' uint4 layout) <-> the 128-bit big-endian halves */
TLSREC_CLMUL_FN void tlsrec_g_from_words(const uint32_t w[4], uint64_t *hi, uint64_t *lo)
{
    *hi = (uint64_t) tlsrec_bswap32(w[0]) << 32 | tlsrec_bswap32(w[1]);
    *lo = (uint64_t) tlsrec_bswap32(w[2]) << 32 | tlsrec_bswap32(w[3]);
}

TLSREC_CLMUL_FN void tlsrec_g_to_words(uint64_t hi, uint64_t lo, uint32_t w[4])
{
    w[0] = tlsrec_bswap32((uint32_t) (hi >> 32));
    w[1] = tlsrec_bswap32((uint32_t) hi);
    w[2] = tlsrec_bswap32((uint32_t) (lo >> 32));
    w[3] = tlsrec_bswap32((uint32_t) lo);
}

/* B_k = P * X^(4k), 0 <= k < 32 */
TLSREC_CLMUL_FN void tlsrec_gtab4_base(const uint32_t p[4], uint32_t k, uint64_t *bh, uint64_t *bl)
{
    tlsrec_g_from_words(p, bh, bl);
    const uint32_t sh = 4 * k, s1 = sh > 63 ? 63 : sh;
    tlsrec_gf128_shr(bh, bl, s1);
    tlsrec_gf128_shr(bh, bl, sh - s1);
}

/* V * X (V >> 1 as the big-endian number, the bit falling off X^127 folded
 * back as X^128 = X^7 + X^2 + X + 1, i.e. 0xE1 at the top) -- a masked
 * constant instead of tlsrec_gf128_shr's general fold */
TLSREC_CLMUL_FN void tlsrec_gf128_mulx(uint64_t *hi, uint64_t *lo)
{
    const uint64_t m = 0 - (*lo & 1u);
    *lo = (*lo >> 1) | (*hi << 63);
    *hi = (*hi >> 1) ^ (m & 0xE100000000000000ull);
}

/* Entries 4q .. 4q + 3 of window k of P's 4-bit position table (the layout
 * of tlsrec_gtab4_entry), as the paired GCM passes build it (r06): one lane
 * per (window, quarter), B_k = P X^(4k) and its multiples by X, X^2, X^3
 * once, the quarter's two high bits selecting its base, the four entries
 * the base plus the 0 / X^3 / X^2 / X^2 + X^3 multiples (with tlsrec_gtab4_entry
 * per entry, 16 general shifts a lane).  out: 4 entries in the kernels' word
 * layout. */
TLSREC_CLMUL_FN void tlsrec_gtab4_quad(const uint32_t p[4], uint32_t k, uint32_t q, uint32_t out[4][4])
{
    uint64_t h0, l0;
    tlsrec_gtab4_base(p, k, &h0, &l0);                 /* B X^0: n bit 3 */
    uint64_t h1 = h0, l1 = l0;
    tlsrec_gf128_mulx(&h1, &l1);                       /* B X^1: n bit 2 */
    uint64_t h2 = h1, l2 = l1;
    tlsrec_gf128_mulx(&h2, &l2);                       /* B X^2: n bit 1 */
    uint64_t h3 = h2, l3 = l2;
    tlsrec_gf128_mulx(&h3, &l3);                       /* B X^3: n bit 0 */
    const uint64_t m3 = 0 - (uint64_t) ((q >> 1) & 1u), m2 = 0 - (uint64_t) (q & 1u);   /* masks: P is secret */
    const uint64_t bh = (h0 & m3) ^ (h1 & m2), bl = (l0 & m3) ^ (l1 & m2);
    tlsrec_g_to_words(bh, bl, out[0]);
    tlsrec_g_to_words(bh ^ h3, bl ^ l3, out[1]);
    tlsrec_g_to_words(bh ^ h2, bl ^ l2, out[2]);
    tlsrec_g_to_words(bh ^ h2 ^ h3, bl ^ l2 ^ l3, out[3]);
}

#endif /* TLSREC_CLMUL_H */
