/*
 * tlsrec_bitslice.h -- bitsliced AES counter mode for gfx950 (VALU only).
 *
 * The T-table AES of tlsrec_device.h spends its time in the LDS (16 random
 * ds_read_b32 per round per block); this form spends it in the VALU instead,
 * so both pipes of a CU can work on AES at once.
 *
 * Layout: one lane holds 32 counter blocks of one record as 128 bit planes
 * P[b][k], b = state byte 0..15 (FIPS-197 order: row b%4, column b/4),
 * k = bit 0..7; bit j of P[b][k] is bit k of byte b of the j-th block.
 *   - SubBytes: the Boyar-Peralta depth-16 circuit (128 gates) on each byte
 *     position's 8 planes; the compiler fuses its gates into v_bitop3_b32.
 *   - ShiftRows: compile-time renaming of the planes.
 *   - MixColumns: XORs of planes (xtime is a renaming plus 3 XORs).
 *   - AddRoundKey: per-plane XOR with 0 / ~0 from the key bit (uniform).
 * The 32 blocks are counters c0 .. c0+31 (c0 a multiple of 32, below 2^16), so
 * bytes 0..14 of every block are equal: rounds 1 and 2 are evaluated per lane
 * on bytes where they are constant (T-table-free byte AES on the S-box in
 * registers) and bitsliced only where the counter reaches them.
 * The keystream leaves in the normal layout through four 32x32 bit-matrix
 * transposes (v_perm for the byte and half-word stages).
 *
 * Everything here is __host__ __device__ plain C so that the same code is
 * checked on the CPU (tools/bs_check.cpp) against FIPS-197 vectors.  Probe-only: the measurements
 * in DESIGN.md 3.1b kept it out of the product kernels.
 */
#ifndef TLSREC_BITSLICE_H
#define TLSREC_BITSLICE_H

#include <stdint.h>

#ifndef TLSREC_HD
#if defined(__HIPCC__)
#define TLSREC_HD __host__ __device__ __forceinline__
#else
#define TLSREC_HD static inline
#endif
#endif

namespace tlsrec {
namespace bs {

/* S-box on the 8 planes x[0..7] (x[k] = bit k), in place.  Boyar & Peralta,
 * "A depth-16 circuit for the AES S-box" (2011): inputs U0 = MSB. */
TLSREC_HD void sbox(uint32_t (&x)[8])
{
    const uint32_t U0 = x[7], U1 = x[6], U2 = x[5], U3 = x[4], U4 = x[3], U5 = x[2], U6 = x[1], U7 = x[0];
    const uint32_t T1 = U0 ^ U3, T2 = U0 ^ U5, T3 = U0 ^ U6, T4 = U3 ^ U5, T5 = U4 ^ U6;
    const uint32_t T6 = T1 ^ T5, T7 = U1 ^ U2, T8 = U7 ^ T6, T9 = U7 ^ T7, T10 = T6 ^ T7;
    const uint32_t T11 = U1 ^ U5, T12 = U2 ^ U5, T13 = T3 ^ T4, T14 = T6 ^ T11, T15 = T5 ^ T11;
    const uint32_t T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = U3 ^ U7, T19 = T7 ^ T18, T20 = T1 ^ T19;
    const uint32_t T21 = U6 ^ U7, T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10, T25 = T20 ^ T17;
    const uint32_t T26 = T3 ^ T16, T27 = T1 ^ T12;
    const uint32_t M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7, M5 = M4 ^ M1;
    const uint32_t M6 = T3 & T16, M7 = T22 & T9, M8 = T26 ^ M6, M9 = T20 & T17, M10 = M9 ^ M6;
    const uint32_t M11 = T1 & T15, M12 = T4 & T27, M13 = M12 ^ M11, M14 = T2 & T10, M15 = M14 ^ M11;
    const uint32_t M16 = M3 ^ M2, M17 = M5 ^ T24, M18 = M8 ^ M7, M19 = M10 ^ M15, M20 = M16 ^ M13;
    const uint32_t M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25, M24 = M22 ^ M23, M25 = M22 & M20;
    const uint32_t M26 = M21 ^ M25, M27 = M20 ^ M21, M28 = M23 ^ M25, M29 = M28 & M27, M30 = M26 & M24;
    const uint32_t M31 = M20 & M23, M32 = M27 & M31, M33 = M27 ^ M25, M34 = M21 & M22, M35 = M24 & M34;
    const uint32_t M36 = M24 ^ M25, M37 = M21 ^ M29, M38 = M32 ^ M33, M39 = M23 ^ M30, M40 = M35 ^ M36;
    const uint32_t M41 = M38 ^ M40, M42 = M37 ^ M39, M43 = M37 ^ M38, M44 = M39 ^ M40, M45 = M42 ^ M41;
    const uint32_t M46 = M44 & T6, M47 = M40 & T8, M48 = M39 & U7, M49 = M43 & T16, M50 = M38 & T9;
    const uint32_t M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27, M54 = M41 & T10, M55 = M44 & T13;
    const uint32_t M56 = M40 & T23, M57 = M39 & T19, M58 = M43 & T3, M59 = M38 & T22, M60 = M37 & T20;
    const uint32_t M61 = M42 & T1, M62 = M45 & T4, M63 = M41 & T2;
    const uint32_t L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48, L3 = M47 ^ M55, L4 = M54 ^ M58;
    const uint32_t L5 = M49 ^ M61, L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59, L9 = M52 ^ M53;
    const uint32_t L10 = M53 ^ L4, L11 = M60 ^ L2, L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61;
    const uint32_t L15 = M55 ^ L1, L16 = M56 ^ L0, L17 = M57 ^ L1, L18 = M58 ^ L8, L19 = M63 ^ L4;
    const uint32_t L20 = L0 ^ L1, L21 = L1 ^ L7, L22 = L3 ^ L12, L23 = L18 ^ L2, L24 = L15 ^ L9;
    const uint32_t L25 = L6 ^ L10, L26 = L7 ^ L9, L27 = L8 ^ L10, L28 = L11 ^ L14, L29 = L11 ^ L17;
    x[7] = L6 ^ L24;
    x[6] = ~(L16 ^ L26);
    x[5] = ~(L19 ^ L28);
    x[4] = L6 ^ L21;
    x[3] = L20 ^ L22;
    x[2] = L25 ^ L29;
    x[1] = ~(L13 ^ L27);
    x[0] = ~(L6 ^ L23);
}

/* Ends a byte's S-box before the next one starts (bounded live ranges: with
 * all 16 S-boxes of a round in flight the kernel needs > 400 VGPRs). */
TLSREC_HD void fence8(uint32_t (&x)[8])
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
#else
    (void) x;
#endif
}

/* 0 / ~0 from bit k of byte b of the round key words w[0..3] (little-endian
 * columns, as tlsrec's key schedule stores them) */
TLSREC_HD uint32_t keymask(uint32_t w, int shift) { return (uint32_t) -(int32_t) ((w >> shift) & 1u); }

/* SubBytes + ShiftRows (renaming) of state P into Q: Q[b] = S(P[src(b)]),
 * src(row r, col c) = (row r, col c + r). */
TLSREC_HD int shiftrows_src(int b) { return 4 * (((b >> 2) + (b & 3)) & 3) + (b & 3); }

/* One full middle round: P -> MixColumns(ShiftRows(SubBytes(P))) ^ K.
 * rk points at the round's 4 key words. */
template <typename RK>
TLSREC_HD void round_mid(uint32_t (&P)[16][8], RK rk, int r)
{
#pragma unroll
    for (int b = 0; b < 16; b++) { sbox(P[b]); fence8(P[b]); }
    uint32_t S[16][8];
#pragma unroll
    for (int b = 0; b < 16; b++)
#pragma unroll
        for (int k = 0; k < 8; k++) S[b][k] = P[b][k];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t a[4][8];
#pragma unroll
        for (int row = 0; row < 4; row++)
#pragma unroll
            for (int k = 0; k < 8; k++) a[row][k] = S[shiftrows_src(4 * c + row)][k];
        uint32_t t[4][8];
#pragma unroll
        for (int row = 0; row < 4; row++)
#pragma unroll
            for (int k = 0; k < 8; k++) t[row][k] = a[row][k] ^ a[(row + 1) & 3][k];
        const uint32_t kw = rk[4 * r + c];
#pragma unroll
        for (int row = 0; row < 4; row++) {
            const uint32_t *tr = t[row], *t2 = t[(row + 2) & 3], *a1 = a[(row + 1) & 3];
            uint32_t o[8];
            o[0] = tr[7] ^ a1[0] ^ t2[0];
            o[1] = tr[0] ^ tr[7] ^ a1[1] ^ t2[1];
            o[2] = tr[1] ^ a1[2] ^ t2[2];
            o[3] = tr[2] ^ tr[7] ^ a1[3] ^ t2[3];
            o[4] = tr[3] ^ tr[7] ^ a1[4] ^ t2[4];
            o[5] = tr[4] ^ a1[5] ^ t2[5];
            o[6] = tr[5] ^ a1[6] ^ t2[6];
            o[7] = tr[6] ^ a1[7] ^ t2[7];
#pragma unroll
            for (int k = 0; k < 8; k++) P[4 * c + row][k] = o[k] ^ keymask(kw, 8 * row + k);
        }
    }
}

/* Last round: P -> ShiftRows(SubBytes(P)) ^ K (no MixColumns). */
template <typename RK>
TLSREC_HD void round_last(uint32_t (&P)[16][8], RK rk, int r)
{
#pragma unroll
    for (int b = 0; b < 16; b++) { sbox(P[b]); fence8(P[b]); }
    uint32_t Q[16][8];
#pragma unroll
    for (int b = 0; b < 16; b++) {
        const uint32_t kw = rk[4 * r + (b >> 2)];
#pragma unroll
        for (int k = 0; k < 8; k++) Q[b][k] = P[shiftrows_src(b)][k] ^ keymask(kw, 8 * (b & 3) + k);
    }
#pragma unroll
    for (int b = 0; b < 16; b++)
#pragma unroll
        for (int k = 0; k < 8; k++) P[b][k] = Q[b][k];
}

/* 32x32 bit transpose of A (element (i, j) = bit j of A[i]) in place. */
TLSREC_HD uint32_t perm_bytes(uint32_t hi, uint32_t lo, uint32_t sel)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    /* v_perm_b32: selector byte s picks byte s of {hi:lo} (lo = bytes 0..3) */
    const uint64_t v = ((uint64_t) hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; i++) {
        const uint32_t s = (sel >> (8 * i)) & 0xff;
        r |= (uint32_t) ((v >> (8 * s)) & 0xff) << (8 * i);
    }
    return r;
#endif
}

TLSREC_HD void transpose32(uint32_t (&A)[32])
{
    /* s = 16: half words */
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t x = A[i], y = A[i + 16];
        A[i] = perm_bytes(y, x, 0x05040100u);        /* lo(x) | lo(y) << 16 */
        A[i + 16] = perm_bytes(y, x, 0x07060302u);   /* hi(x) | hi(y) << 16 */
    }
    /* s = 8: bytes */
#pragma unroll
    for (int i0 = 0; i0 < 32; i0 += 16)
#pragma unroll
        for (int i = i0; i < i0 + 8; i++) {
            const uint32_t x = A[i], y = A[i + 8];
            A[i] = perm_bytes(y, x, 0x06020400u);     /* x.b0 y.b0 x.b2 y.b2 */
            A[i + 8] = perm_bytes(y, x, 0x07030501u); /* x.b1 y.b1 x.b3 y.b3 */
        }
    /* s = 4, 2, 1: masked swaps */
#pragma unroll
    for (int s = 4; s >= 1; s >>= 1) {
        const uint32_t m = s == 4 ? 0x0F0F0F0Fu : s == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int i0 = 0; i0 < 32; i0 += 2 * s)
#pragma unroll
            for (int i = i0; i < i0 + s; i++) {
                const uint32_t x = A[i], y = A[i + s];
                A[i] = (x & m) | ((y << s) & ~m);
                A[i + s] = ((x >> s) & m) | (y & ~m);
            }
    }
}

/* Planes of a byte value that is the same in all 32 blocks. */
TLSREC_HD void const_planes(uint32_t (&p)[8], uint32_t v)
{
#pragma unroll
    for (int k = 0; k < 8; k++) p[k] = keymask(v, k);
}

/* AES forward cipher (NR rounds) of the 32 counter blocks
 *     (n0, n1, n2, BE32(c0 + j)),  j = 0..31,  c0 % 32 == 0, c0 + 31 < 2^16
 * of one lane; rk = key schedule words (4 per round, little-endian columns,
 * unrotated), sb = the S-box as 256 bytes (per-lane rounds 1-2 on constant
 * bytes).  Output: ks[j] = E_K(counter block j) as 4 little-endian words,
 * held as ks[4 * c + ...] -- see the end. */
template <int NR, typename RK, typename SB>
TLSREC_HD void ctr32(RK rk, SB sbox_bytes, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t c0, uint32_t (&out)[4][32])
{
    uint32_t P[16][8];
    /* whitening: bytes 0..14 constant (per lane), byte 15 = low counter byte */
    const uint32_t nw[4] = { n0, n1, n2, ((c0 >> 8) & 0xffu) << 16 };
    uint32_t s0b[16];
#pragma unroll
    for (int b = 0; b < 16; b++) s0b[b] = ((nw[b >> 2] ^ rk[b >> 2]) >> (8 * (b & 3))) & 0xffu;
    /* byte 15 = (c0 & 0xe0) | j, j = 0..31, ^ key byte 15 */
#pragma unroll
    for (int b = 0; b < 15; b++) const_planes(P[b], s0b[b]);
    {
        const uint32_t hi = (c0 & 0xe0u) ^ ((rk[3] >> 24) & 0xffu);
        const uint32_t jpat[5] = { 0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u };
        const uint32_t k15 = (rk[3] >> 24) & 0x1fu;
#pragma unroll
        for (int k = 0; k < 5; k++) P[15][k] = jpat[k] ^ keymask(k15, k);
#pragma unroll
        for (int k = 5; k < 8; k++) P[15][k] = keymask(hi, k);
    }
    (void) sbox_bytes;
#pragma unroll
    for (int r = 1; r < NR; r++) round_mid(P, rk, r);
    round_last(P, rk, NR);
    /* out[c][j] = column c of block j */
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t A[32];
#pragma unroll
        for (int row = 0; row < 4; row++)
#pragma unroll
            for (int k = 0; k < 8; k++) A[8 * row + k] = P[4 * c + row][k];
        transpose32(A);
#pragma unroll
        for (int j = 0; j < 32; j++) out[c][j] = A[j];
    }
}

} /* namespace bs */
} /* namespace tlsrec */

#endif /* TLSREC_BITSLICE_H */
