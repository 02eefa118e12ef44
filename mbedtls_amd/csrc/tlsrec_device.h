/*
 * tlsrec_device.h -- CDNA4 (gfx950) device primitives for the record engine.
 *
 *  - AES forward cipher with two 256-entry "T" tables in LDS, replicated 32x
 *    so that lane l always reads bank (l & 31): data-dependent indices never
 *    conflict.  One v_perm_b32 builds each LDS address from a state byte.
 *  - GHASH multiply by a fixed power of H with 4-bit position tables in LDS
 *    (32 windows x 16 entries x 16 B = 8 KiB per power); one ds_read_b128
 *    per nibble, conflict-free because a window's 16 entries span exactly the
 *    64 banks.
 *  - ChaCha20 block per lane (RFC 8439 2.3), v_alignbit rotates.
 *  - Poly1305 arithmetic mod 2^130-5 in five 26-bit limbs with 64-bit
 *    multiply-adds (v_mad_u64_u32).
 *
 * The AES S-box is generated at compile time from its FIPS-197 definition.
 */
#ifndef TLSREC_DEVICE_H
#define TLSREC_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tlsrec {

/* ---------------- AES S-box (constexpr, FIPS-197 5.1.1) ---------------- */
struct SboxGen {
    uint8_t v[256];
    constexpr SboxGen() : v() {
        uint8_t ex[256] = {};
        uint8_t lg[256] = {};
        uint8_t x = 1;
        for (int i = 0; i < 255; i++) {
            ex[i] = x;
            lg[x] = (uint8_t) i;
            uint8_t x2 = (uint8_t) ((x << 1) ^ ((x & 0x80) ? 0x1b : 0));
            x = (uint8_t) (x2 ^ x);               /* generator 3 */
        }
        for (int a = 0; a < 256; a++) {
            uint8_t inv = a ? ex[(255 - lg[a]) % 255] : 0;
            uint8_t s = inv, r = inv;
            for (int k = 0; k < 4; k++) {
                r = (uint8_t) ((r << 1) | (r >> 7));
                s = (uint8_t) (s ^ r);
            }
            v[a] = (uint8_t) (s ^ 0x63);
        }
    }
};

__constant__ const SboxGen kSbox{};

__device__ __forceinline__ uint32_t xtime8(uint32_t s) { return ((s << 1) ^ (0x1bu & (0u - ((s >> 7) & 1u)))) & 0xff; }
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rotr16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
/* gfx950 v_bitop3_b32: one VALU op for a ^ b ^ c */
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

/* ---------------- LDS T-tables ----------------------------------------- */
/* Entry x of table j (j = 0: T0 = (2s,s,s,3s), j = 1: T1 = rotl8(T0)),
 * copy c, lives at lds_aes + x*256 + j*128 + c*4.  T2 = rotl16(T0) and
 * T3 = rotl16(T1) are formed with one v_alignbit per column. */
__device__ __forceinline__ void aes_fill_tables(uint8_t *lds_aes, int tid, int nthreads)
{
    for (int t = tid; t < 256 * 4; t += nthreads) {
        uint32_t x = t & 255, part = t >> 8;          /* part: copies 8*part .. 8*part+7 */
        uint32_t s = kSbox.v[x];
        uint32_t s2 = xtime8(s), s3 = s2 ^ s;
        uint32_t t0 = s2 | (s << 8) | (s << 16) | (s3 << 24);
        uint32_t t1 = rotl32(t0, 8);
        uint4 v0 = make_uint4(t0, t0, t0, t0), v1 = make_uint4(t1, t1, t1, t1);
        uint8_t *row = lds_aes + x * 256 + part * 32;
        *reinterpret_cast<uint4 *>(row) = v0;
        *reinterpret_cast<uint4 *>(row + 16) = v0;
        *reinterpret_cast<uint4 *>(row + 128) = v1;
        *reinterpret_cast<uint4 *>(row + 144) = v1;
    }
}

/* v_perm selector: byte0 <- lanebase byte 0 (= (lane&31)*4), byte1 <- state
 * byte k, bytes 2,3 <- 0.  The result is the LDS address x*256 + (lane&31)*4. */
/* constant address space: read-only for the kernel's lifetime, scalar loads */
typedef const __attribute__((address_space(4))) uint32_t kconst_u32;

/* Record payload access through the global address space.  Through generic
 * pointers (struct members) these compile to flat_load/flat_store, which
 * count on lgkmcnt as well as vmcnt: the first LDS wait after the load then
 * becomes vmcnt(0) lgkmcnt(0) and the wave stalls for the full HBM latency
 * in every step. */
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 glob_u32x4;
/* TLSREC_NT_DATA (A/B builds): bit 0 loads, bit 1 stores of record payload
 * with the non-temporal hint */
#ifndef TLSREC_NT_DATA
#define TLSREC_NT_DATA 0
#endif
__device__ __forceinline__ uint4 gload16(const uint8_t *p)
{
#if TLSREC_NT_DATA & 1
    const u32x4 v = __builtin_nontemporal_load((const glob_u32x4 *) (uintptr_t) p);
#else
    const u32x4 v = *(const glob_u32x4 *) (uintptr_t) p;
#endif
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gstore16(uint8_t *p, uint4 v)
{
    u32x4 w = { v.x, v.y, v.z, v.w };
#if TLSREC_NT_DATA & 2
    __builtin_nontemporal_store(w, (glob_u32x4 *) (uintptr_t) p);
#else
    *(glob_u32x4 *) (uintptr_t) p = w;
#endif
}

#define TLSREC_PSEL(k) (0x0C0C0000u | ((4u + (k)) << 8))

template <int AES_OFF>
__device__ __forceinline__ uint32_t tlook(const uint8_t *lds, uint32_t w, uint32_t lb, int k, int tab)
{
    uint32_t a = __builtin_amdgcn_perm(w, lb, TLSREC_PSEL(k));
    return *reinterpret_cast<const uint32_t *>(lds + a + AES_OFF + tab * 128);
}

/* AES-128 (NR=10) / AES-256 (NR=14) forward cipher of one block per lane.
 * Words are little-endian columns: byte r of word c is row r of column c.
 * `rk` holds the key schedule in the engine's "rotated" form: words of the
 * middle rounds 1..NR-1 are stored rotr16(rk) so that each output column is
 *     xor3(T0[a], T1[b], rotl16(xor3(T0[c], T1[d], rotr16(rk))))
 * = 4 lookups + 3 VALU ops (rotl16(x ^ rotr16(k)) = rotl16(x) ^ k). */
template <int NR, int AES_OFF, typename RK>
__device__ __forceinline__ uint4 aes_encrypt(const uint8_t *lds, uint32_t lb, RK rk,
                                             uint4 in)
{
    uint32_t s0 = in.x ^ rk[0], s1 = in.y ^ rk[1], s2 = in.z ^ rk[2], s3 = in.w ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t t0 = xor3(tlook<AES_OFF>(lds, s0, lb, 0, 0), tlook<AES_OFF>(lds, s1, lb, 1, 1),
                           rotl16(xor3(tlook<AES_OFF>(lds, s2, lb, 2, 0), tlook<AES_OFF>(lds, s3, lb, 3, 1), rk[4 * r + 0])));
        uint32_t t1 = xor3(tlook<AES_OFF>(lds, s1, lb, 0, 0), tlook<AES_OFF>(lds, s2, lb, 1, 1),
                           rotl16(xor3(tlook<AES_OFF>(lds, s3, lb, 2, 0), tlook<AES_OFF>(lds, s0, lb, 3, 1), rk[4 * r + 1])));
        uint32_t t2 = xor3(tlook<AES_OFF>(lds, s2, lb, 0, 0), tlook<AES_OFF>(lds, s3, lb, 1, 1),
                           rotl16(xor3(tlook<AES_OFF>(lds, s0, lb, 2, 0), tlook<AES_OFF>(lds, s1, lb, 3, 1), rk[4 * r + 2])));
        uint32_t t3 = xor3(tlook<AES_OFF>(lds, s3, lb, 0, 0), tlook<AES_OFF>(lds, s0, lb, 1, 1),
                           rotl16(xor3(tlook<AES_OFF>(lds, s1, lb, 2, 0), tlook<AES_OFF>(lds, s2, lb, 3, 1), rk[4 * r + 3])));
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    /* last round: S[x] is byte 1 (and byte 2) of T0[x] */
    uint32_t o[4];
    const uint32_t s[4] = { s0, s1, s2, s3 };
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t a = tlook<AES_OFF>(lds, s[c], lb, 0, 0);
        uint32_t b = tlook<AES_OFF>(lds, s[(c + 1) & 3], lb, 1, 0);
        uint32_t d2 = tlook<AES_OFF>(lds, s[(c + 2) & 3], lb, 2, 0);
        uint32_t d3 = tlook<AES_OFF>(lds, s[(c + 3) & 3], lb, 3, 0);
        uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0C0C0501u);   /* [a.b1, b.b1, 0, 0] */
        uint32_t hi = __builtin_amdgcn_perm(d3, d2, 0x06020C0Cu);  /* [0, 0, d2.b2, d3.b2] */
        o[c] = __builtin_amdgcn_bitop3_b32(lo, hi, rk[4 * NR + c], 0x56);   /* (lo | hi) ^ k */
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

/* ---------------- ARIA (RFC 5794) --------------------------------------- */
/* SB1 = AES S-box, SB2(x) = B x^247 ^ 0xE2 (B by the images of the 8 basis
 * bits), SB3 = SB1^-1, SB4 = SB2^-1; generated at compile time. */
struct AriaSboxGen {
    uint8_t v[4][256];
    static constexpr uint8_t mul(uint8_t a, uint8_t b)
    {
        uint8_t r = 0;
        for (int i = 0; i < 8; i++) {
            if ((b >> i) & 1) r = (uint8_t) (r ^ a);
            a = (uint8_t) ((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        }
        return r;
    }
    constexpr AriaSboxGen() : v()
    {
        const SboxGen aes{};
        const uint8_t bcol[8] = { 0xac, 0xc5, 0x12, 0xcf, 0x5b, 0x5f, 0x85, 0xee };
        for (int x = 0; x < 256; x++) {
            uint8_t y = 1, base = (uint8_t) x;
            for (int e = 247; e; e >>= 1) {
                if (e & 1) y = mul(y, base);
                base = mul(base, base);
            }
            if (x == 0) y = 0;
            uint8_t t = 0xe2;
            for (int k = 0; k < 8; k++)
                if ((y >> k) & 1) t = (uint8_t) (t ^ bcol[k]);
            v[0][x] = aes.v[x];
            v[1][x] = t;
        }
        for (int x = 0; x < 256; x++) {
            v[2][v[0][x]] = (uint8_t) x;
            v[3][v[1][x]] = (uint8_t) x;
        }
    }
};

__constant__ const AriaSboxGen kAriaSbox{};

/* Diffusion layer A (RFC 5794 2.4.3), on 16 bytes held in the low bits of
 * 16 registers: y_i = x_a ^ x_b ^ ... (7 terms, two xor3 + one xor). */
#define TLSREC_ARIA_A(y, x)                                                                  \
    do {                                                                                     \
        y[0] = xor3(xor3(x[3], x[4], x[6]), xor3(x[8], x[9], x[13]), x[14]);                 \
        y[1] = xor3(xor3(x[2], x[5], x[7]), xor3(x[8], x[9], x[12]), x[15]);                 \
        y[2] = xor3(xor3(x[1], x[4], x[6]), xor3(x[10], x[11], x[12]), x[15]);               \
        y[3] = xor3(xor3(x[0], x[5], x[7]), xor3(x[10], x[11], x[13]), x[14]);               \
        y[4] = xor3(xor3(x[0], x[2], x[5]), xor3(x[8], x[11], x[14]), x[15]);                \
        y[5] = xor3(xor3(x[1], x[3], x[4]), xor3(x[9], x[10], x[14]), x[15]);                \
        y[6] = xor3(xor3(x[0], x[2], x[7]), xor3(x[9], x[10], x[12]), x[13]);                \
        y[7] = xor3(xor3(x[1], x[3], x[6]), xor3(x[8], x[11], x[12]), x[13]);                \
        y[8] = xor3(xor3(x[0], x[1], x[4]), xor3(x[7], x[10], x[13]), x[15]);                \
        y[9] = xor3(xor3(x[0], x[1], x[5]), xor3(x[6], x[11], x[12]), x[14]);                \
        y[10] = xor3(xor3(x[2], x[3], x[5]), xor3(x[6], x[8], x[13]), x[15]);                \
        y[11] = xor3(xor3(x[2], x[3], x[4]), xor3(x[7], x[9], x[12]), x[14]);                \
        y[12] = xor3(xor3(x[1], x[2], x[6]), xor3(x[7], x[9], x[11]), x[12]);                \
        y[13] = xor3(xor3(x[0], x[3], x[6]), xor3(x[7], x[8], x[10]), x[13]);                \
        y[14] = xor3(xor3(x[0], x[3], x[4]), xor3(x[5], x[9], x[11]), x[14]);                \
        y[15] = xor3(xor3(x[1], x[2], x[4]), xor3(x[5], x[8], x[10]), x[15]);                \
    } while (0)

/* LDS S-box image of the LDS-table block ciphers (ARIA, Camellia): for each
 * byte value x, 32 copies (copy = lane & 31) of one dword holding the four
 * S-box outputs S_0[x] .. S_3[x] in its bytes 0..3, at OFF + x*128 + copy*4
 * (32 KiB).  A lookup is ds_read_u8 at OFF + (x << 7) + (lane & 31)*4 + t:
 * each lane of a 32-lane ds_read group owns its bank ((a/4) mod 32 = lane &
 * 31), so reads never conflict and their timing does not depend on the key
 * or the data. */
template <typename GEN>
__device__ __forceinline__ void sbox_fill_tables(uint8_t *lds, int tid, int nthreads, const GEN &g)
{
    for (int i = tid; i < 256 * 8; i += nthreads) {
        const int x = i >> 3, part = i & 7;   /* part: copies 4*part .. 4*part+3 */
        const uint32_t v = (uint32_t) g.v[0][x] | ((uint32_t) g.v[1][x] << 8) | ((uint32_t) g.v[2][x] << 16) |
                           ((uint32_t) g.v[3][x] << 24);
        *reinterpret_cast<uint4 *>(lds + x * 128 + part * 16) = make_uint4(v, v, v, v);
    }
}

template <int OFF>
__device__ __forceinline__ uint32_t sbox_lds(const uint8_t *lds, uint32_t lb, int t, uint32_t x)
{
    return lds[OFF + (x << 7) + lb + t];
}

__device__ __forceinline__ void aria_fill_tables(uint8_t *lds, int tid, int nthreads)
{
    sbox_fill_tables(lds, tid, nthreads, kAriaSbox);
}

/* ARIA forward cipher (NR = 12/14/16 rounds) of one block per lane.  Words
 * are little-endian (byte i of the block = byte i%4 of word i/4); rk = the
 * NR + 1 round keys as 4 words each.  lb = (lane & 31) * 4. */
template <int NR, int ARIA_OFF, typename RK>
__device__ __forceinline__ uint4 aria_encrypt(const uint8_t *lds, uint32_t lb, RK rk, uint4 in)
{
    const uint32_t w[4] = { in.x, in.y, in.z, in.w };
    uint32_t x[16], y[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = (w[i >> 2] >> (8 * (i & 3))) & 0xffu;
#pragma unroll
    for (int r = 1; r <= NR; r++) {
        /* AddRoundKey, then SL1 (odd rounds: SB1 SB2 SB3 SB4) or SL2 (even and
         * the last round: SB3 SB4 SB1 SB2) */
        const bool odd = (r & 1) && r != NR;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t kb = (rk[4 * (r - 1) + (i >> 2)] >> (8 * (i & 3))) & 0xffu;
            const int t = odd ? (i & 3) : ((i & 3) ^ 2);
            x[i] = sbox_lds<ARIA_OFF>(lds, lb, t, x[i] ^ kb);
        }
        if (r != NR) {
            TLSREC_ARIA_A(y, x);
#pragma unroll
            for (int i = 0; i < 16; i++) x[i] = y[i];
        }
    }
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 4; c++)
        o[c] = (x[4 * c] | (x[4 * c + 1] << 8) | (x[4 * c + 2] << 16) | (x[4 * c + 3] << 24)) ^ rk[4 * NR + c];
    return make_uint4(o[0], o[1], o[2], o[3]);
}

/* ---------------- Camellia (RFC 3713) ----------------------------------- */
/* SBOX1 (RFC 3713 2.4.4); SBOX2 = SBOX1 <<< 1, SBOX3 = SBOX1 <<< 7,
 * SBOX4(x) = SBOX1(x <<< 1); staged as the four bytes of the S-box image
 * (sbox_fill_tables). */
struct CamSboxGen {
    uint8_t v[4][256];
    constexpr CamSboxGen() : v()
    {
        constexpr uint8_t s1[256] = {
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
        for (int x = 0; x < 256; x++) {
            const uint32_t a = s1[x];
            v[0][x] = (uint8_t) a;
            v[1][x] = (uint8_t) ((a << 1) | (a >> 7));                /* SBOX2 */
            v[2][x] = (uint8_t) ((a << 7) | (a >> 1));                /* SBOX3 */
            v[3][x] = s1[((x << 1) | (x >> 7)) & 0xff];               /* SBOX4 */
        }
    }
};

__constant__ const CamSboxGen kCamSbox{};

__device__ __forceinline__ void cam_fill_tables(uint8_t *lds, int tid, int nthreads)
{
    sbox_fill_tables(lds, tid, nthreads, kCamSbox);
}

/* F(x ^ k) on the 64-bit half (h = the high word): S-boxes 1234 / 2341 on
 * the bytes t1..t8 of x ^ k (t1 = the top byte of h), then the P-layer on
 * A = z1..z4, B = z5..z8 (big-endian words) as word rotations:
 *   U = A ^ (B <<< 8),  V = B ^ (U <<< 16),  U' = U ^ (V >>> 8),
 *   y1..y4 = V ^ (U' >>> 8),  y5..y8 = U'
 * (each y_i the XOR of the RFC 3713 2.4.3 terms). */
template <int OFF>
__device__ __forceinline__ void cam_f(const uint8_t *lds, uint32_t lb, uint32_t xh, uint32_t xl, uint32_t kh,
                                      uint32_t kl, uint32_t &oh, uint32_t &ol)
{
    xh ^= kh;
    xl ^= kl;
    const uint32_t z1 = sbox_lds<OFF>(lds, lb, 0, xh >> 24), z2 = sbox_lds<OFF>(lds, lb, 1, (xh >> 16) & 0xffu);
    const uint32_t z3 = sbox_lds<OFF>(lds, lb, 2, (xh >> 8) & 0xffu), z4 = sbox_lds<OFF>(lds, lb, 3, xh & 0xffu);
    const uint32_t z5 = sbox_lds<OFF>(lds, lb, 1, xl >> 24), z6 = sbox_lds<OFF>(lds, lb, 2, (xl >> 16) & 0xffu);
    const uint32_t z7 = sbox_lds<OFF>(lds, lb, 3, (xl >> 8) & 0xffu), z8 = sbox_lds<OFF>(lds, lb, 0, xl & 0xffu);
    const uint32_t A = (z1 << 24) | (z2 << 16) | (z3 << 8) | z4;
    const uint32_t B = (z5 << 24) | (z6 << 16) | (z7 << 8) | z8;
    const uint32_t U = A ^ __builtin_amdgcn_alignbit(B, B, 24);
    const uint32_t V = B ^ __builtin_amdgcn_alignbit(U, U, 16);
    const uint32_t U2 = U ^ __builtin_amdgcn_alignbit(V, V, 8);
    oh = V ^ __builtin_amdgcn_alignbit(U2, U2, 8);
    ol = U2;
}

/* Camellia forward cipher (NR = 18 / 24 rounds) of one block per lane.  Words
 * of in/out are little-endian byte quadruples of the block; rk = the 64-bit
 * subkeys in use order (kw1 kw2 | k1..k6 | ke1 ke2 | ... | kw3 kw4) as
 * (high, low) word pairs.  lb = (lane & 31) * 4. */
template <int NR, int OFF, typename RK>
__device__ __forceinline__ uint4 cam_encrypt(const uint8_t *lds, uint32_t lb, RK rk, uint4 in)
{
    uint32_t d1h = bswap32(in.x) ^ rk[0], d1l = bswap32(in.y) ^ rk[1];
    uint32_t d2h = bswap32(in.z) ^ rk[2], d2l = bswap32(in.w) ^ rk[3];
    constexpr int G = NR / 6;
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int base = 4 + g * 16;     /* 6 round keys + 2 FL keys per group, 2 words each */
#pragma unroll
        for (int r = 0; r < 3; r++) {
            uint32_t fh, fl;
            cam_f<OFF>(lds, lb, d1h, d1l, rk[base + 4 * r], rk[base + 4 * r + 1], fh, fl);
            d2h ^= fh;
            d2l ^= fl;
            cam_f<OFF>(lds, lb, d2h, d2l, rk[base + 4 * r + 2], rk[base + 4 * r + 3], fh, fl);
            d1h ^= fh;
            d1l ^= fl;
        }
        if (g != G - 1) {
            /* FL(d1, ke_a), FL^-1(d2, ke_b) (RFC 3713 2.4.2) */
            const uint32_t k1 = rk[base + 12], k2 = rk[base + 13], k3 = rk[base + 14], k4 = rk[base + 15];
            d1l ^= __builtin_amdgcn_alignbit(d1h & k1, d1h & k1, 31);
            d1h ^= (d1l | k2);
            d2h ^= (d2l | k4);
            d2l ^= __builtin_amdgcn_alignbit(d2h & k3, d2h & k3, 31);
        }
    }
    constexpr int W = 4 + 16 * G - 4;    /* kw3 kw4 */
    d2h ^= rk[W];
    d2l ^= rk[W + 1];
    d1h ^= rk[W + 2];
    d1l ^= rk[W + 3];
    return make_uint4(bswap32(d2h), bswap32(d2l), bswap32(d1h), bswap32(d1l));
}

/* The LDS-table block ciphers behind the GCM / CCM kernels' ARIA slot:
 * NR 12 / 14 / 16 = ARIA, NR 18 / 24 = Camellia. */
template <int NR>
__device__ __forceinline__ void alt_fill_tables(uint8_t *lds, int tid, int nthreads)
{
    if constexpr (NR >= 18)
        cam_fill_tables(lds, tid, nthreads);
    else
        aria_fill_tables(lds, tid, nthreads);
}

template <int NR, int OFF, typename RK>
__device__ __forceinline__ uint4 alt_encrypt(const uint8_t *lds, uint32_t lb, RK rk, uint4 in)
{
    if constexpr (NR >= 18)
        return cam_encrypt<NR, OFF>(lds, lb, rk, in);
    else
        return aria_encrypt<NR, OFF>(lds, lb, rk, in);
}

/* ---------------- GHASH with LDS position tables ----------------------- */
/* Table PI (a power of H) holds T_k[n] = sum_{i<4} bit(3-i of n) * P * x^(4k+i)
 * at PI*8192 + k*256 + n*16, as the 16-byte GCM string.  Window k = 2b is the
 * high nibble of byte b, k = 2b+1 its low nibble. */
/* G = table-read groups per multiply (8 reads each when G = 4); MEM = whether
 * a group boundary also orders memory (stops later LDS reads -- including
 * unrelated AES lookups -- from moving above it). */
template <int PI, int G = 4, bool MEM = true>
__device__ __forceinline__ uint4 gmul(const uint8_t *lds, uint4 y)
{
    const uint32_t w[4] = { y.x, y.y, y.z, y.w };
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int d = 0; d < 4; d++) {
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int b = 4 * d + e;
            uint32_t ahi = (e == 0) ? (w[d] & 0xf0u) : ((w[d] >> (8 * e)) & 0xf0u);
            uint32_t alo = (e == 0) ? ((w[d] << 4) & 0xf0u) : ((w[d] >> (8 * e - 4)) & 0xf0u);
            uint4 th = *reinterpret_cast<const uint4 *>(lds + ahi + PI * 8192 + (2 * b) * 256);
            uint4 tl = *reinterpret_cast<const uint4 *>(lds + alo + PI * 8192 + (2 * b + 1) * 256);
            acc.x = xor3(acc.x, th.x, tl.x);
            acc.y = xor3(acc.y, th.y, tl.y);
            acc.z = xor3(acc.z, th.z, tl.z);
            acc.w = xor3(acc.w, th.w, tl.w);
        }
        /* bound the table reads in flight: the opaque acc (+ memory clobber)
         * keeps the next group's ds_read_b128 below this group's XORs;
         * otherwise all 32 reads are hoisted and the multiply needs 128 VGPRs */
        if ((d + 1) % (4 / G) == 0) {
            if constexpr (MEM)
                asm volatile("" : "+v"(acc.x), "+v"(acc.y), "+v"(acc.z), "+v"(acc.w) : : "memory");
            else
                asm volatile("" : "+v"(acc.x), "+v"(acc.y), "+v"(acc.z), "+v"(acc.w));
        }
    }
    return acc;
}

/* Part of gmul: the table reads of bytes e0 .. e0+NE-1 of 32-bit word d of y. */
template <int PI, int NE = 4>
__device__ __forceinline__ void gmul_word(const uint8_t *lds, uint32_t wd, int d, uint4 &acc, int e0 = 0)
{
#pragma unroll
    for (int i = 0; i < NE; i++) {
        const int e = e0 + i;
        const int b = 4 * d + e;
        uint32_t ahi = (e == 0) ? (wd & 0xf0u) : ((wd >> (8 * e)) & 0xf0u);
        uint32_t alo = (e == 0) ? ((wd << 4) & 0xf0u) : ((wd >> (8 * e - 4)) & 0xf0u);
        uint4 th = *reinterpret_cast<const uint4 *>(lds + ahi + PI * 8192 + (2 * b) * 256);
        uint4 tl = *reinterpret_cast<const uint4 *>(lds + alo + PI * 8192 + (2 * b + 1) * 256);
        acc.x = xor3(acc.x, th.x, tl.x);
        acc.y = xor3(acc.y, th.y, tl.y);
        acc.z = xor3(acc.z, th.z, tl.z);
        acc.w = xor3(acc.w, th.w, tl.w);
    }
}

/* gmul_word with the table at LDS offset base (a multiple of 256) of the
 * kernel's LDS array lds: the entry address as base | (nibble x 16) --
 * one v_and_or per read where lds-relative pointer arithmetic took a shift,
 * a mask and an add (r06; the paired passes' tables sit at a per-pair base) */
#ifndef TLSREC_GH_OR
#define TLSREC_GH_OR 1
#endif
template <int PI, int NE = 4>
__device__ __forceinline__ void gmul_word_or(const uint8_t *lds, uint32_t base, uint32_t wd, int d, uint4 &acc,
                                             int e0 = 0)
{
#pragma unroll
    for (int i = 0; i < NE; i++) {
        const int e = e0 + i;
        const int b = 4 * d + e;
        const uint32_t ahi = base | ((e == 0) ? (wd & 0xf0u) : ((wd >> (8 * e)) & 0xf0u));
        const uint32_t alo = base | ((e == 0) ? ((wd << 4) & 0xf0u) : ((wd >> (8 * e - 4)) & 0xf0u));
        uint4 th = *reinterpret_cast<const uint4 *>(lds + ahi + PI * 8192 + (2 * b) * 256);
        uint4 tl = *reinterpret_cast<const uint4 *>(lds + alo + PI * 8192 + (2 * b + 1) * 256);
        acc.x = xor3(acc.x, th.x, tl.x);
        acc.y = xor3(acc.y, th.y, tl.y);
        acc.z = xor3(acc.z, th.z, tl.z);
        acc.w = xor3(acc.w, th.w, tl.w);
    }
}

/* ---------------- GHASH with 5-bit position tables (G5) ------------------ *
 * ds_read_b64 serves 32 lanes per LDS cycle over all 64 banks, so a 256-byte
 * image of 32 eight-byte entries is conflict-free for any index: a 5-bit
 * window read as two 8-byte halves costs the LDS what one 4-bit window's
 * ds_read_b128 costs.  26 windows cover the 128 bits (24 of 5 bits, 2 of 4
 * that straddle a word boundary): 104 LDS cycles per multiply instead of 128.
 * Windows take contiguous bits of the little-endian block words; the lo
 * halves (8 B) of window k's 32 entries sit at k*256, the hi halves at
 * G5_HI + k*256 -- more than ds_read2_b64's offset range apart, so the two
 * reads of a window stay ds_read_b64 (the fused ds_read2_b64 takes 8 LDS
 * cycles over 32 banks and would conflict).  Entry n of window
 * k = sum over set bits i of n of P * x^j(bit i), j the GCM bit index of that
 * word bit (tlsrec_keysetup_kernel writes the tables). */
constexpr int G5_HI = 26 * 256;
struct G5Win { uint8_t d, s, cross; };
__host__ __device__ constexpr G5Win g5_win(int k)
{
    return k < 6 ? G5Win{ 0, (uint8_t) (5 * k), 0 }
         : k == 6 ? G5Win{ 0, 30, 1 }
         : k < 13 ? G5Win{ 1, (uint8_t) (2 + 5 * (k - 7)), 0 }
         : k < 19 ? G5Win{ 2, (uint8_t) (5 * (k - 13)), 0 }
         : k == 19 ? G5Win{ 2, 30, 1 }
         : G5Win{ 3, (uint8_t) (2 + 5 * (k - 20)), 0 };
}
/* word / bit of bit i (0 = LSB) of window k's index */
__host__ __device__ constexpr int g5_word(int k, int i) { return g5_win(k).cross && i >= 2 ? g5_win(k).d + 1 : g5_win(k).d; }
__host__ __device__ constexpr int g5_bit(int k, int i)
{
    return g5_win(k).cross ? (i < 2 ? 30 + i : i - 2) : g5_win(k).s + i;
}
__host__ __device__ constexpr int g5_bits(int k) { return g5_win(k).cross ? 4 : 5; }

/* byte offset (index * 8) of window k's entry for the block words w */
template <int K>
__device__ __forceinline__ uint32_t g5_addr(const uint32_t (&w)[4])
{
    constexpr G5Win W = g5_win(K);
    if constexpr (W.cross)
        return __builtin_amdgcn_alignbit(w[W.d + 1], w[W.d], 27) & 0x78u;
    else if constexpr (W.s >= 3)
        return (w[W.d] >> (W.s - 3)) & 0xF8u;
    else
        return (w[W.d] << (3 - W.s)) & 0xF8u;
}

/* the hi-half address as a register the compiler cannot relate to the lo
 * one: otherwise it fuses the pair into ds_read2st64_b64 (8 LDS cycles over
 * 32 banks, conflicting) */
__device__ __forceinline__ uint32_t g5_hi(uint32_t a)
{
    uint32_t h;
    asm("v_mov_b32 %0, %1" : "=v"(h) : "v"(a));
    return h;
}

/* acc ^= the products of windows K0 .. K0+NK-1 (table at lds) */
template <int K0, int NK>
__device__ __forceinline__ void gmul5_part(const uint8_t *lds, const uint32_t (&w)[4], uint4 &acc)
{
    if constexpr (NK >= 2) {
        const uint32_t a0 = g5_addr<K0>(w), a1 = g5_addr<K0 + 1>(w);
        const uint2 l0 = *reinterpret_cast<const uint2 *>(lds + a0 + K0 * 256);
        const uint2 h0 = *reinterpret_cast<const uint2 *>(lds + g5_hi(a0) + G5_HI + K0 * 256);
        const uint2 l1 = *reinterpret_cast<const uint2 *>(lds + a1 + (K0 + 1) * 256);
        const uint2 h1 = *reinterpret_cast<const uint2 *>(lds + g5_hi(a1) + G5_HI + (K0 + 1) * 256);
        acc.x = xor3(acc.x, l0.x, l1.x);
        acc.y = xor3(acc.y, l0.y, l1.y);
        acc.z = xor3(acc.z, h0.x, h1.x);
        acc.w = xor3(acc.w, h0.y, h1.y);
        gmul5_part<K0 + 2, NK - 2>(lds, w, acc);
    } else if constexpr (NK == 1) {
        const uint32_t a0 = g5_addr<K0>(w);
        const uint2 l0 = *reinterpret_cast<const uint2 *>(lds + a0 + K0 * 256);
        const uint2 h0 = *reinterpret_cast<const uint2 *>(lds + g5_hi(a0) + G5_HI + K0 * 256);
        acc.x ^= l0.x;
        acc.y ^= l0.y;
        acc.z ^= h0.x;
        acc.w ^= h0.y;
    }
}

/* phase g (0..7) of a G5 multiply: windows [3g + min(g, 2), ...): 4,4,3,3,3,3,3,3 */
template <int G>
__device__ __forceinline__ void gmul5_phase(const uint8_t *lds, const uint32_t (&w)[4], uint4 &acc)
{
    constexpr int K0 = G < 2 ? 4 * G : 8 + 3 * (G - 2);
    constexpr int NK = G < 2 ? 4 : 3;
    gmul5_part<K0, NK>(lds, w, acc);
}

/* y * P with P's G5 table at lds (whole multiply, four phases of 6-7 windows) */
__device__ __forceinline__ uint4 gmul5(const uint8_t *lds, uint4 y)
{
    const uint32_t w[4] = { y.x, y.y, y.z, y.w };
    uint4 acc = make_uint4(0, 0, 0, 0);
    gmul5_part<0, 7>(lds, w, acc);
    asm volatile("" : "+v"(acc.x), "+v"(acc.y), "+v"(acc.z), "+v"(acc.w) : : "memory");
    gmul5_part<7, 6>(lds, w, acc);
    asm volatile("" : "+v"(acc.x), "+v"(acc.y), "+v"(acc.z), "+v"(acc.w) : : "memory");
    gmul5_part<13, 7>(lds, w, acc);
    asm volatile("" : "+v"(acc.x), "+v"(acc.y), "+v"(acc.z), "+v"(acc.w) : : "memory");
    gmul5_part<20, 6>(lds, w, acc);
    return acc;
}

/* AES middle round r on (s0..s3), rotated round keys (see aes_encrypt). */
template <int AES_OFF, typename RK>
__device__ __forceinline__ void aes_round(const uint8_t *lds, uint32_t lb, RK rk, int r,
                                          uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3)
{
    uint32_t t0 = xor3(tlook<AES_OFF>(lds, s0, lb, 0, 0), tlook<AES_OFF>(lds, s1, lb, 1, 1),
                       rotl16(xor3(tlook<AES_OFF>(lds, s2, lb, 2, 0), tlook<AES_OFF>(lds, s3, lb, 3, 1), rk[4 * r + 0])));
    uint32_t t1 = xor3(tlook<AES_OFF>(lds, s1, lb, 0, 0), tlook<AES_OFF>(lds, s2, lb, 1, 1),
                       rotl16(xor3(tlook<AES_OFF>(lds, s3, lb, 2, 0), tlook<AES_OFF>(lds, s0, lb, 3, 1), rk[4 * r + 1])));
    uint32_t t2 = xor3(tlook<AES_OFF>(lds, s2, lb, 0, 0), tlook<AES_OFF>(lds, s3, lb, 1, 1),
                       rotl16(xor3(tlook<AES_OFF>(lds, s0, lb, 2, 0), tlook<AES_OFF>(lds, s1, lb, 3, 1), rk[4 * r + 2])));
    uint32_t t3 = xor3(tlook<AES_OFF>(lds, s3, lb, 0, 0), tlook<AES_OFF>(lds, s0, lb, 1, 1),
                       rotl16(xor3(tlook<AES_OFF>(lds, s1, lb, 2, 0), tlook<AES_OFF>(lds, s2, lb, 3, 1), rk[4 * r + 3])));
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
}

/* ---------------- counter-mode round caching -------------------------- *
 * Within one record the GCM counter block is (N0, N1, N2, BE32(ctr)) with
 * ctr < 2^16, so after whitening only rows 2 and 3 of column 3 vary: round 1
 * has one varying lookup in columns 0 and 1 and none in columns 2 and 3, and
 * round 2 has two varying lookups per column.  ctr_cache() folds everything
 * else into six per-record words (rotated round-key form, see aes_encrypt):
 *   t0 = rotl16(k0r ^ T1[s3.b3])          t1 = rotl16(k1r ^ T0[s3.b2])
 *   u0 = T0[t0.b0] ^ T1[t1.b1] ^ d0       u1 = T0[t1.b0] ^ d1 ^ rotl16(T1[t0.b3])
 *   u2 = rotl16(T0[t0.b2] ^ T1[t1.b3] ^ d2r)
 *   u3 = T1[t0.b1] ^ d3 ^ rotl16(T0[t1.b2])
 * (10 lookups instead of 32 for rounds 1-2). */
struct CtrCache { uint32_t k0r, k1r, d0, d1, d2r, d3; };

template <int AES_OFF, typename RK>
__device__ __forceinline__ CtrCache ctr_cache(const uint8_t *lds, uint32_t lb, RK rk, uint32_t n0, uint32_t n1,
                                              uint32_t n2)
{
#define TA(x, k) tlook<AES_OFF>(lds, (x), lb, (k), 0)
#define TB(x, k) tlook<AES_OFF>(lds, (x), lb, (k), 1)
    const uint32_t s0 = n0 ^ rk[0], s1 = n1 ^ rk[1], s2 = n2 ^ rk[2], s3 = rk[3];   /* ctr rows 0,1 = 0 */
    CtrCache c;
    c.k0r = rotr16(xor3(TA(s0, 0), TB(s1, 1), rotl16(TA(s2, 2) ^ rk[4])));
    c.k1r = rotr16(xor3(TA(s1, 0), TB(s2, 1), rotl16(TB(s0, 3) ^ rk[5])));
    const uint32_t t2 = xor3(TA(s2, 0), TB(s3, 1), rotl16(xor3(TA(s0, 2), TB(s1, 3), rk[6])));
    const uint32_t t3 = xor3(TA(s3, 0), TB(s0, 1), rotl16(xor3(TA(s1, 2), TB(s2, 3), rk[7])));
    c.d0 = rotl16(xor3(TA(t2, 2), TB(t3, 3), rk[8]));
    c.d1 = TB(t2, 1) ^ rotl16(TA(t3, 2) ^ rk[9]);
    c.d2r = rotr16(TA(t2, 0) ^ TB(t3, 1)) ^ rk[10];
    c.d3 = TA(t3, 0) ^ rotl16(TB(t2, 3) ^ rk[11]);
    return c;
#undef TA
#undef TB
}

/* Fused counter-block encryption and one GHASH multiply, for a step whose
 * GHASH input does not depend on this step's keystream:
 *     ks = E_K(N0, N1, N2, ctrw),  prod = y * P_PI
 * (ctrw = BE32(ctr) as a little-endian word, ctr < 2^16, rounds 1-2 from `cc`).
 * The 32 GHASH table reads are issued in 8 groups of 4 (a half word of y),
 * group g after AES round R0 + g*RS, each sharing its phase with that
 * round's T-table reads so the LDS sees both streams at once.  The empty
 * asm statements are the phase boundaries: they re-define the AES state, the
 * accumulator and the source words still to be read, so no read moves into an
 * earlier phase (bounded reads in flight and VGPRs, no memory clobber). */
template <int NR, int AES_OFF, int PI, int R0 = 2, int RS = 1, bool G5 = false, typename RK>
__device__ __forceinline__ void aes_ghash(const uint8_t *lds, const uint8_t *gh, uint32_t lb, RK rk,
                                          const CtrCache &cc, uint32_t ctrw, uint4 y, uint4 &ks, uint4 &prod)
{
    static_assert(R0 >= 2 && R0 + 7 * RS <= NR - 1, "GHASH groups must fall on middle rounds 2..NR-1");
#define TA(x, k) tlook<AES_OFF>(lds, (x), lb, (k), 0)
#define TB(x, k) tlook<AES_OFF>(lds, (x), lb, (k), 1)
    uint32_t s0, s1, s2, s3;
    {
        const uint32_t w3 = ctrw ^ rk[3];
        const uint32_t t0 = rotl16(cc.k0r ^ TB(w3, 3));
        const uint32_t t1 = rotl16(cc.k1r ^ TA(w3, 2));
        s0 = xor3(TA(t0, 0), TB(t1, 1), cc.d0);
        s1 = xor3(TA(t1, 0), cc.d1, rotl16(TB(t0, 3)));
        s2 = rotl16(xor3(TA(t0, 2), TB(t1, 3), cc.d2r));
        s3 = xor3(TB(t0, 1), cc.d3, rotl16(TA(t1, 2)));
    }
#undef TA
#undef TB
    uint32_t w[4] = { y.x, y.y, y.z, y.w };
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int r = 2; r < NR; r++) {
        if (r > 2) aes_round<AES_OFF>(lds, lb, rk, r, s0, s1, s2, s3);
        const int g = (r - R0) / RS;
        if (r >= R0 && (r - R0) % RS == 0 && g < 8) {
            if constexpr (G5) {
                /* G5 phases read windows across word boundaries: every word
                 * still read enters the next phase through the barrier */
                switch (g) {
                    case 0: gmul5_phase<0>(gh, w, acc); break;
                    case 1: gmul5_phase<1>(gh, w, acc); break;
                    case 2: gmul5_phase<2>(gh, w, acc); break;
                    case 3: gmul5_phase<3>(gh, w, acc); break;
                    case 4: gmul5_phase<4>(gh, w, acc); break;
                    case 5: gmul5_phase<5>(gh, w, acc); break;
                    case 6: gmul5_phase<6>(gh, w, acc); break;
                    default: gmul5_phase<7>(gh, w, acc); break;
                }
                asm volatile("" : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(acc.x), "+v"(acc.y), "+v"(acc.z),
                             "+v"(acc.w));
                if (g < 2) asm volatile("" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
                else if (g < 4) asm volatile("" : "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
                else if (g < 6) asm volatile("" : "+v"(w[2]), "+v"(w[3]));
                else asm volatile("" : "+v"(w[3]));
            } else {
                if constexpr (TLSREC_GH_OR)
                    gmul_word_or<PI, 2>(lds, (uint32_t) (gh - lds), w[g >> 1], g >> 1, acc, 2 * (g & 1));
                else
                    gmul_word<PI, 2>(gh, w[g >> 1], g >> 1, acc, 2 * (g & 1));
                asm volatile("" : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(acc.x), "+v"(acc.y), "+v"(acc.z),
                             "+v"(acc.w));
                /* the words still to be read enter the next phase through the barrier */
                if (g < 2) asm volatile("" : "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
                else if (g < 4) asm volatile("" : "+v"(w[2]), "+v"(w[3]));
                else if (g < 6) asm volatile("" : "+v"(w[3]));
            }
        }
    }
    uint32_t o[4];
    const uint32_t s[4] = { s0, s1, s2, s3 };
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t a = tlook<AES_OFF>(lds, s[c], lb, 0, 0);
        uint32_t b = tlook<AES_OFF>(lds, s[(c + 1) & 3], lb, 1, 0);
        uint32_t d2 = tlook<AES_OFF>(lds, s[(c + 2) & 3], lb, 2, 0);
        uint32_t d3 = tlook<AES_OFF>(lds, s[(c + 3) & 3], lb, 3, 0);
        uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0C0C0501u);
        uint32_t hi = __builtin_amdgcn_perm(d3, d2, 0x06020C0Cu);
        o[c] = __builtin_amdgcn_bitop3_b32(lo, hi, rk[4 * NR + c], 0x56);
    }
    ks = make_uint4(o[0], o[1], o[2], o[3]);
    prod = acc;
}

/* NB independent counter blocks of one record and NB independent GHASH
 * multiplies per call (NB Horner chains per lane), phase-interleaved as in
 * aes_ghash: chain b's group g of 4 table reads follows AES round 2 + g. */
template <int NR, int AES_OFF, int PI, int NB, typename RK>
__device__ __forceinline__ void aes_ghash_n(const uint8_t *lds, uint32_t lb, RK rk, const CtrCache &cc,
                                            const uint32_t (&ctrw)[NB], const uint4 (&y)[NB], uint4 (&ks)[NB],
                                            uint4 (&prod)[NB])
{
    static_assert(NR >= 10, "rounds 2..9 carry the GHASH groups");
#define TA(x, k) tlook<AES_OFF>(lds, (x), lb, (k), 0)
#define TB(x, k) tlook<AES_OFF>(lds, (x), lb, (k), 1)
    uint32_t s[NB][4];
    uint32_t w[NB][4];
    uint4 acc[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const uint32_t w3 = ctrw[b] ^ rk[3];
        const uint32_t t0 = rotl16(cc.k0r ^ TB(w3, 3));
        const uint32_t t1 = rotl16(cc.k1r ^ TA(w3, 2));
        s[b][0] = xor3(TA(t0, 0), TB(t1, 1), cc.d0);
        s[b][1] = xor3(TA(t1, 0), cc.d1, rotl16(TB(t0, 3)));
        s[b][2] = rotl16(xor3(TA(t0, 2), TB(t1, 3), cc.d2r));
        s[b][3] = xor3(TB(t0, 1), cc.d3, rotl16(TA(t1, 2)));
        w[b][0] = y[b].x; w[b][1] = y[b].y; w[b][2] = y[b].z; w[b][3] = y[b].w;
        acc[b] = make_uint4(0, 0, 0, 0);
    }
#undef TA
#undef TB
#pragma unroll
    for (int r = 2; r < NR; r++) {
        if (r > 2) {
#pragma unroll
            for (int b = 0; b < NB; b++) aes_round<AES_OFF>(lds, lb, rk, r, s[b][0], s[b][1], s[b][2], s[b][3]);
        }
        const int g = r - 2;
        if (g < 8) {
#pragma unroll
            for (int b = 0; b < NB; b++) gmul_word<PI, 2>(lds, w[b][g >> 1], g >> 1, acc[b], 2 * (g & 1));
#pragma unroll
            for (int b = 0; b < NB; b++) {
                asm volatile("" : "+v"(s[b][0]), "+v"(s[b][1]), "+v"(s[b][2]), "+v"(s[b][3]), "+v"(acc[b].x),
                             "+v"(acc[b].y), "+v"(acc[b].z), "+v"(acc[b].w));
                if (g < 2) asm volatile("" : "+v"(w[b][1]), "+v"(w[b][2]), "+v"(w[b][3]));
                else if (g < 4) asm volatile("" : "+v"(w[b][2]), "+v"(w[b][3]));
                else if (g < 6) asm volatile("" : "+v"(w[b][3]));
            }
        }
    }
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint32_t o[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t a = tlook<AES_OFF>(lds, s[b][c], lb, 0, 0);
            uint32_t bb = tlook<AES_OFF>(lds, s[b][(c + 1) & 3], lb, 1, 0);
            uint32_t d2 = tlook<AES_OFF>(lds, s[b][(c + 2) & 3], lb, 2, 0);
            uint32_t d3 = tlook<AES_OFF>(lds, s[b][(c + 3) & 3], lb, 3, 0);
            uint32_t lo = __builtin_amdgcn_perm(bb, a, 0x0C0C0501u);
            uint32_t hi = __builtin_amdgcn_perm(d3, d2, 0x06020C0Cu);
            o[c] = __builtin_amdgcn_bitop3_b32(lo, hi, rk[4 * NR + c], 0x56);
        }
        ks[b] = make_uint4(o[0], o[1], o[2], o[3]);
        prod[b] = acc[b];
    }
}

__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }

/* ---------------- GF(2^128) bitwise helpers (key setup only) ----------- */
/* big-endian (hi = bytes 0..7) representation */
struct G128 { uint64_t hi, lo; };

__device__ __forceinline__ G128 g_shr1(G128 v)
{
    /* masks, not branches: H is secret and a one-lane branch is timed by exec */
    const uint64_t lsb = 0 - (v.lo & 1);
    G128 r;
    r.lo = (v.lo >> 1) | (v.hi << 63);
    r.hi = (v.hi >> 1) ^ (lsb & 0xE100000000000000ULL);
    return r;
}

__device__ inline G128 g_mul(G128 x, G128 y)
{
    G128 z = { 0, 0 }, v = y;
    for (int i = 0; i < 128; i++) {
        const uint64_t bit = (i < 64) ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1;
        const uint64_t m = 0 - bit;
        z.hi ^= v.hi & m;
        z.lo ^= v.lo & m;
        v = g_shr1(v);
    }
    return z;
}

__device__ __forceinline__ uint4 g_to_words(G128 v)
{
    return make_uint4(bswap32((uint32_t) (v.hi >> 32)), bswap32((uint32_t) v.hi),
                      bswap32((uint32_t) (v.lo >> 32)), bswap32((uint32_t) v.lo));
}

__device__ __forceinline__ G128 g_from_words(uint4 w)
{
    G128 v;
    v.hi = ((uint64_t) bswap32(w.x) << 32) | bswap32(w.y);
    v.lo = ((uint64_t) bswap32(w.z) << 32) | bswap32(w.w);
    return v;
}

/* x * P with base[j] = P * x^j (words, tlsrec_keysetup_kernel's LDS base):
 * the XOR of the base entries of x's set bits, masked, not branched -- over
 * four lanes: lane r (= lane & 3) sums terms 32 r .. 32 r + 31, the XOR over
 * the four lanes gives the product in each of them (the four lanes of a
 * group must be active together) */
__device__ inline G128 g_mul_base_q(const uint4 *base, G128 x, int r)
{
    const uint64_t half = r < 2 ? x.hi : x.lo;
    const int top = (r & 1) ? 31 : 63;
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll 8
    for (int i = 0; i < 32; i++) {
        const uint32_t m = 0u - (uint32_t) ((half >> (top - i)) & 1);
        const uint4 b = base[32 * r + i];
        acc.x ^= b.x & m; acc.y ^= b.y & m; acc.z ^= b.z & m; acc.w ^= b.w & m;
    }
#pragma unroll
    for (int d = 1; d < 4; d <<= 1) {
        acc.x ^= (uint32_t) __shfl_xor((int) acc.x, d);
        acc.y ^= (uint32_t) __shfl_xor((int) acc.y, d);
        acc.z ^= (uint32_t) __shfl_xor((int) acc.z, d);
        acc.w ^= (uint32_t) __shfl_xor((int) acc.w, d);
    }
    return g_from_words(acc);
}


/* ---------------- ChaCha20 (RFC 8439 2.3) ------------------------------ */
#define TLSREC_QR(a, b, c, d)                                  \
    do {                                                       \
        a += b; d ^= a; d = rotl32(d, 16);                     \
        c += d; b ^= c; b = rotl32(b, 12);                     \
        a += b; d ^= a; d = rotl32(d, 8);                      \
        c += d; b ^= c; b = rotl32(b, 7);                      \
    } while (0)
/* the quarter round after its first addition (a already holds a + b) */
#define TLSREC_QR_A(a, b, c, d)                                \
    do {                                                       \
        d ^= a; d = rotl32(d, 16);                             \
        c += d; b ^= c; b = rotl32(b, 12);                     \
        a += b; d ^= a; d = rotl32(d, 8);                      \
        c += d; b ^= c; b = rotl32(b, 7);                      \
    } while (0)

/* ---- counter-independent part of the first double round ----
 * Only word 12 (the block counter) varies along a record's key stream, and in
 * the first column round it meets words 0, 4, 8 only: the quarter rounds of
 * columns 1..3 are the same for every block of the record.  chacha_cc_make()
 * runs them once per record; chacha_block_cc() starts from the 13 words:
 *   cc[0] = w0 + w4 (the column-0 round's first sum, both inputs constant)
 *   cc[1..3] = x5, x9, x13   cc[5..7] = x6, x10, x14   cc[9..11] = x7, x11, x15
 *   cc[4] = x1 + x6, cc[8] = x2 + x7 (the first sums of the diagonal quarter
 *   rounds (1,6,11,12) and (2,7,8,13), whose a and b are both cached)
 *   cc[12] = x3
 * (x = the state after the column round).  Per block: 3 of the 80 quarter
 * rounds and 3 more additions fewer, ~4 % of the block's VALU work. */
constexpr int CHACHA_CC_WORDS = 13;

__device__ __forceinline__ void chacha_cc_make(const uint32_t key[8], const uint32_t nonce[3],
                                               uint32_t cc[CHACHA_CC_WORDS])
{
    uint32_t x[16] = { 0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                       key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                       0u, nonce[0], nonce[1], nonce[2] };
    cc[0] = x[0] + x[4];
    TLSREC_QR(x[1], x[5], x[9], x[13]);
    TLSREC_QR(x[2], x[6], x[10], x[14]);
    TLSREC_QR(x[3], x[7], x[11], x[15]);
    cc[1] = x[5]; cc[2] = x[9]; cc[3] = x[13];
    cc[4] = x[1] + x[6]; cc[5] = x[6]; cc[6] = x[10]; cc[7] = x[14];
    cc[8] = x[2] + x[7]; cc[9] = x[7]; cc[10] = x[11]; cc[11] = x[15];
    cc[12] = x[3];
}

/* ChaCha20 block `counter` from the cached words (= chacha_block) */
template <typename W>
__device__ __forceinline__ void chacha_block_cc(W key, W nonce, W cc, uint32_t counter, uint32_t out[16])
{
    uint32_t x[16];
    x[0] = cc[0]; x[4] = key[0]; x[8] = key[4]; x[12] = counter;
    TLSREC_QR_A(x[0], x[4], x[8], x[12]);
    x[5] = cc[1]; x[9] = cc[2]; x[13] = cc[3];
    x[1] = cc[4]; x[6] = cc[5]; x[10] = cc[6]; x[14] = cc[7];
    x[2] = cc[8]; x[7] = cc[9]; x[11] = cc[10]; x[15] = cc[11];
    x[3] = cc[12];
    TLSREC_QR(x[0], x[5], x[10], x[15]);
    TLSREC_QR_A(x[1], x[6], x[11], x[12]);
    TLSREC_QR_A(x[2], x[7], x[8], x[13]);
    TLSREC_QR(x[3], x[4], x[9], x[14]);
#pragma unroll
    for (int i = 1; i < 10; i++) {
        TLSREC_QR(x[0], x[4], x[8], x[12]);
        TLSREC_QR(x[1], x[5], x[9], x[13]);
        TLSREC_QR(x[2], x[6], x[10], x[14]);
        TLSREC_QR(x[3], x[7], x[11], x[15]);
        TLSREC_QR(x[0], x[5], x[10], x[15]);
        TLSREC_QR(x[1], x[6], x[11], x[12]);
        TLSREC_QR(x[2], x[7], x[8], x[13]);
        TLSREC_QR(x[3], x[4], x[9], x[14]);
    }
    out[0] = x[0] + 0x61707865u; out[1] = x[1] + 0x3320646eu;
    out[2] = x[2] + 0x79622d32u; out[3] = x[3] + 0x6b206574u;
#pragma unroll
    for (int i = 0; i < 8; i++) out[4 + i] = x[4 + i] + key[i];
    out[12] = x[12] + counter;
#pragma unroll
    for (int i = 0; i < 3; i++) out[13 + i] = x[13 + i] + nonce[i];
}

__device__ __forceinline__ void chacha_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3],
                                             uint32_t out[16])
{
    const uint32_t in[16] = { 0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                              key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                              counter, nonce[0], nonce[1], nonce[2] };
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = in[i];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        TLSREC_QR(x[0], x[4], x[8], x[12]);
        TLSREC_QR(x[1], x[5], x[9], x[13]);
        TLSREC_QR(x[2], x[6], x[10], x[14]);
        TLSREC_QR(x[3], x[7], x[11], x[15]);
        TLSREC_QR(x[0], x[5], x[10], x[15]);
        TLSREC_QR(x[1], x[6], x[11], x[12]);
        TLSREC_QR(x[2], x[7], x[8], x[13]);
        TLSREC_QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}

/* Two blocks of one key stream (counters c0, c1) in lockstep: the eight
 * independent quarter-round chains of a double round interleave, twice the
 * ILP of chacha_block for the dependency-bound VALU pipeline. */
__device__ __forceinline__ void chacha_block2(const uint32_t key[8], uint32_t c0, uint32_t c1, const uint32_t nonce[3],
                                              uint32_t o0[16], uint32_t o1[16])
{
    const uint32_t in[16] = { 0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                              key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                              0u, nonce[0], nonce[1], nonce[2] };
    uint32_t x[16], y[16];
#pragma unroll
    for (int i = 0; i < 16; i++) { x[i] = in[i]; y[i] = in[i]; }
    x[12] = c0;
    y[12] = c1;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        TLSREC_QR(x[0], x[4], x[8], x[12]);  TLSREC_QR(y[0], y[4], y[8], y[12]);
        TLSREC_QR(x[1], x[5], x[9], x[13]);  TLSREC_QR(y[1], y[5], y[9], y[13]);
        TLSREC_QR(x[2], x[6], x[10], x[14]); TLSREC_QR(y[2], y[6], y[10], y[14]);
        TLSREC_QR(x[3], x[7], x[11], x[15]); TLSREC_QR(y[3], y[7], y[11], y[15]);
        TLSREC_QR(x[0], x[5], x[10], x[15]); TLSREC_QR(y[0], y[5], y[10], y[15]);
        TLSREC_QR(x[1], x[6], x[11], x[12]); TLSREC_QR(y[1], y[6], y[11], y[12]);
        TLSREC_QR(x[2], x[7], x[8], x[13]);  TLSREC_QR(y[2], y[7], y[8], y[13]);
        TLSREC_QR(x[3], x[4], x[9], x[14]);  TLSREC_QR(y[3], y[4], y[9], y[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) {
        o0[i] = x[i] + in[i];
        o1[i] = y[i] + in[i];
    }
    o0[12] += c0;
    o1[12] += c1;
}

/* ---------------- Poly1305 in 26-bit limbs ----------------------------- */
struct P5 { uint32_t v[5]; };

#define TLSREC_M26 0x3ffffffu

__device__ __forceinline__ P5 p_zero() { P5 r; for (int i = 0; i < 5; i++) r.v[i] = 0; return r; }

/* 16-byte little-endian block plus 2^128 (every AEAD block is full, RFC 8439 2.8) */
__device__ __forceinline__ P5 p_block(uint4 w)
{
    P5 r;
    r.v[0] = w.x & TLSREC_M26;
    r.v[1] = ((w.x >> 26) | (w.y << 6)) & TLSREC_M26;
    r.v[2] = ((w.y >> 20) | (w.z << 12)) & TLSREC_M26;
    r.v[3] = ((w.z >> 14) | (w.w << 18)) & TLSREC_M26;
    r.v[4] = (w.w >> 8) | (1u << 24);
    return r;
}

/* clamped r from the first 16 bytes of the one-time key */
__device__ __forceinline__ P5 p_from_r(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3)
{
    k0 &= 0x0fffffffu; k1 &= 0x0ffffffcu; k2 &= 0x0ffffffcu; k3 &= 0x0ffffffcu;
    P5 r;
    r.v[0] = k0 & TLSREC_M26;
    r.v[1] = ((k0 >> 26) | (k1 << 6)) & TLSREC_M26;
    r.v[2] = ((k1 >> 20) | (k2 << 12)) & TLSREC_M26;
    r.v[3] = ((k2 >> 14) | (k3 << 18)) & TLSREC_M26;
    r.v[4] = k3 >> 8;
    return r;
}

__device__ __forceinline__ P5 p_add(P5 a, P5 b)
{
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i];
    return r;
}

__device__ __forceinline__ P5 p_sel(bool c, P5 a, P5 b)
{
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}

/* h * r mod 2^130-5 (partially reduced).  Input limbs < 2^27, output limbs
 * < 2^26 except limb 1 < 2^26 + 2^6. */
__device__ __forceinline__ P5 p_mul(P5 h, P5 r)
{
    const uint32_t s1 = r.v[1] * 5, s2 = r.v[2] * 5, s3 = r.v[3] * 5, s4 = r.v[4] * 5;
    uint64_t d0 = (uint64_t) h.v[0] * r.v[0] + (uint64_t) h.v[1] * s4 + (uint64_t) h.v[2] * s3 +
                  (uint64_t) h.v[3] * s2 + (uint64_t) h.v[4] * s1;
    uint64_t d1 = (uint64_t) h.v[0] * r.v[1] + (uint64_t) h.v[1] * r.v[0] + (uint64_t) h.v[2] * s4 +
                  (uint64_t) h.v[3] * s3 + (uint64_t) h.v[4] * s2;
    uint64_t d2 = (uint64_t) h.v[0] * r.v[2] + (uint64_t) h.v[1] * r.v[1] + (uint64_t) h.v[2] * r.v[0] +
                  (uint64_t) h.v[3] * s4 + (uint64_t) h.v[4] * s3;
    uint64_t d3 = (uint64_t) h.v[0] * r.v[3] + (uint64_t) h.v[1] * r.v[2] + (uint64_t) h.v[2] * r.v[1] +
                  (uint64_t) h.v[3] * r.v[0] + (uint64_t) h.v[4] * s4;
    uint64_t d4 = (uint64_t) h.v[0] * r.v[4] + (uint64_t) h.v[1] * r.v[3] + (uint64_t) h.v[2] * r.v[2] +
                  (uint64_t) h.v[3] * r.v[1] + (uint64_t) h.v[4] * r.v[0];
    P5 o;
    uint64_t c;
    c = d0 >> 26; o.v[0] = (uint32_t) d0 & TLSREC_M26; d1 += c;
    c = d1 >> 26; o.v[1] = (uint32_t) d1 & TLSREC_M26; d2 += c;
    c = d2 >> 26; o.v[2] = (uint32_t) d2 & TLSREC_M26; d3 += c;
    c = d3 >> 26; o.v[3] = (uint32_t) d3 & TLSREC_M26; d4 += c;
    c = d4 >> 26; o.v[4] = (uint32_t) d4 & TLSREC_M26;
    uint64_t t = (uint64_t) o.v[0] + c * 5;
    o.v[0] = (uint32_t) t & TLSREC_M26;
    o.v[1] += (uint32_t) (t >> 26);
    return o;
}

/* full carry so that every limb < 2^26 (value < 2^130 + small) */
__device__ __forceinline__ P5 p_carry(P5 h)
{
    uint32_t c;
    c = h.v[0] >> 26; h.v[0] &= TLSREC_M26; h.v[1] += c;
    c = h.v[1] >> 26; h.v[1] &= TLSREC_M26; h.v[2] += c;
    c = h.v[2] >> 26; h.v[2] &= TLSREC_M26; h.v[3] += c;
    c = h.v[3] >> 26; h.v[3] &= TLSREC_M26; h.v[4] += c;
    c = h.v[4] >> 26; h.v[4] &= TLSREC_M26; h.v[0] += c * 5;
    c = h.v[0] >> 26; h.v[0] &= TLSREC_M26; h.v[1] += c;
    return h;
}

/* tag = (h mod p) + s mod 2^128, as 4 little-endian words */
__device__ __forceinline__ uint4 p_finish(P5 h, uint4 s)
{
    h = p_carry(h);
    h = p_carry(h);
    /* g = h + 5 - 2^130 */
    uint32_t g[5], c;
    g[0] = h.v[0] + 5; c = g[0] >> 26; g[0] &= TLSREC_M26;
    g[1] = h.v[1] + c; c = g[1] >> 26; g[1] &= TLSREC_M26;
    g[2] = h.v[2] + c; c = g[2] >> 26; g[2] &= TLSREC_M26;
    g[3] = h.v[3] + c; c = g[3] >> 26; g[3] &= TLSREC_M26;
    g[4] = h.v[4] + c - (1u << 26);
    uint32_t mask = (g[4] >> 31) - 1;   /* all ones if h >= p */
#pragma unroll
    for (int i = 0; i < 5; i++) h.v[i] = (h.v[i] & ~mask) | (g[i] & mask);
    uint32_t w0 = h.v[0] | (h.v[1] << 26);
    uint32_t w1 = (h.v[1] >> 6) | (h.v[2] << 20);
    uint32_t w2 = (h.v[2] >> 12) | (h.v[3] << 14);
    uint32_t w3 = (h.v[3] >> 18) | (h.v[4] << 8);
    uint64_t f = (uint64_t) w0 + s.x;
    uint32_t o0 = (uint32_t) f;
    f = (uint64_t) w1 + s.y + (f >> 32);
    uint32_t o1 = (uint32_t) f;
    f = (uint64_t) w2 + s.z + (f >> 32);
    uint32_t o2 = (uint32_t) f;
    f = (uint64_t) w3 + s.w + (f >> 32);
    return make_uint4(o0, o1, o2, (uint32_t) f);
}

/* compile-time log2 of a power of two (lanes per record, tree depths) */
template <int L> struct Log2;
template <> struct Log2<1> { static constexpr int v = 0; };
template <> struct Log2<2> { static constexpr int v = 1; };
template <> struct Log2<4> { static constexpr int v = 2; };
template <> struct Log2<8> { static constexpr int v = 3; };
template <> struct Log2<16> { static constexpr int v = 4; };
template <> struct Log2<32> { static constexpr int v = 5; };
template <> struct Log2<64> { static constexpr int v = 6; };

} /* namespace tlsrec */

#endif /* TLSREC_DEVICE_H */
