/*
 * kernels.hip -- gfx950 kernels of the TLS record engine.
 *
 *   tlsrec_keysetup_kernel   per key slot: AES key schedule, H = E_K(0),
 *                            H^(2^i) and their GHASH position tables.
 *   tlsrec_gcm_kernel        AES-128/256-GCM record protect / unprotect,
 *                            the psa_aead_encrypt/decrypt calls of
 *                            ssl_msg.c:1043 and :1412 fused with the record
 *                            framing around them.
 *   tlsrec_chachapoly_kernel ChaCha20-Poly1305 likewise.
 *
 * Work decomposition: a wavefront owns a chunk of up to 64
 * records.  A pre-pass gives each lane one record's one-off block (E_K(J0)
 * for GCM, the Poly1305 key block for ChaCha20-Poly1305).  Then L lanes
 * (L = 8 for GCM: 8 x 16 B = one 128-B line per record per step) walk one
 * record; GHASH / Poly1305 are evaluated as L interleaved Horner chains with
 * a uniform multiplier H^L / r^(4L), combined at the end by a log2(L) tree.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>
#include <type_traits>

#include "tlsrec.h"
#include "tlsrec_device.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"
#include "tlsrec_recdev.h"

namespace tlsrec {

/* ======================================================================
 * Key setup
 * ==================================================================== */
__device__ inline void aes_key_expand(const uint8_t *key, int nk, uint32_t *rk)
{
    const int nr = nk + 6, total = 4 * (nr + 1);
    for (int i = 0; i < nk; i++) {
        rk[i] = (uint32_t) key[4 * i] | ((uint32_t) key[4 * i + 1] << 8) |
                ((uint32_t) key[4 * i + 2] << 16) | ((uint32_t) key[4 * i + 3] << 24);
    }
    uint32_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = (t >> 8) | (t << 24);
            t = (uint32_t) kSbox.v[t & 0xff] | ((uint32_t) kSbox.v[(t >> 8) & 0xff] << 8) |
                ((uint32_t) kSbox.v[(t >> 16) & 0xff] << 16) | ((uint32_t) kSbox.v[t >> 24] << 24);
            t ^= rcon;
            rcon = xtime8(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t) kSbox.v[t & 0xff] | ((uint32_t) kSbox.v[(t >> 8) & 0xff] << 8) |
                ((uint32_t) kSbox.v[(t >> 16) & 0xff] << 16) | ((uint32_t) kSbox.v[t >> 24] << 24);
        }
        rk[i] = rk[i - nk] ^ t;
    }
}

/* byte-oriented AES (one lane; only used for H = E_K(0^128)) */
__device__ inline void aes_encrypt_bytes(const uint32_t *rk, int nr, uint8_t st[16])
{
    for (int i = 0; i < 16; i++) st[i] ^= (uint8_t) (rk[i / 4] >> (8 * (i % 4)));
    for (int r = 1; r <= nr; r++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++) t[4 * c + row] = kSbox.v[st[4 * ((c + row) & 3) + row]];
        if (r != nr) {
            for (int c = 0; c < 4; c++) {
                uint32_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                uint32_t all = a0 ^ a1 ^ a2 ^ a3;
                t[4 * c + 0] = (uint8_t) (a0 ^ all ^ xtime8(a0 ^ a1));
                t[4 * c + 1] = (uint8_t) (a1 ^ all ^ xtime8(a1 ^ a2));
                t[4 * c + 2] = (uint8_t) (a2 ^ all ^ xtime8(a2 ^ a3));
                t[4 * c + 3] = (uint8_t) (a3 ^ all ^ xtime8(a3 ^ a0));
            }
        }
        for (int i = 0; i < 16; i++) st[i] = t[i] ^ (uint8_t) (rk[4 * r + i / 4] >> (8 * (i % 4)));
    }
}

/* ARIA key schedule and byte-wise block (RFC 5794 2.2, 2.3), one lane:
 * only for the round keys and H = E_K(0^128) of a slot. */
__device__ inline void aria_round_bytes(uint8_t d[16], const uint8_t rk[16], bool odd, bool diffuse)
{
    uint32_t x[16], y[16];
    for (int i = 0; i < 16; i++) {
        const int t = odd ? (i & 3) : ((i & 3) ^ 2);
        x[i] = kAriaSbox.v[t][d[i] ^ rk[i]];
    }
    if (diffuse) {
        TLSREC_ARIA_A(y, x);
        for (int i = 0; i < 16; i++) d[i] = (uint8_t) y[i];
    } else {
        for (int i = 0; i < 16; i++) d[i] = (uint8_t) x[i];
    }
}

__device__ inline int aria_key_expand(const uint8_t *key, int keylen, uint8_t ek[17][16])
{
    const uint8_t C[3][16] = {
        { 0x51, 0x7c, 0xc1, 0xb7, 0x27, 0x22, 0x0a, 0x94, 0xfe, 0x13, 0xab, 0xe8, 0xfa, 0x9a, 0x6e, 0xe0 },
        { 0x6d, 0xb1, 0x4a, 0xcc, 0x9e, 0x21, 0xc8, 0x20, 0xff, 0x28, 0xb1, 0xd5, 0xef, 0x5d, 0xe2, 0xb0 },
        { 0xdb, 0x92, 0x37, 0x1d, 0x21, 0x26, 0xe9, 0x70, 0x03, 0x24, 0x97, 0x75, 0x04, 0xe8, 0xc9, 0x0e },
    };
    const int first = keylen == 16 ? 0 : keylen == 24 ? 1 : 2, nr = keylen / 4 + 8;
    uint8_t w[4][16], t[16], kr[16];
    for (int i = 0; i < 16; i++) { w[0][i] = key[i]; kr[i] = 16 + i < keylen ? key[16 + i] : 0; }
    for (int i = 0; i < 16; i++) t[i] = w[0][i];
    aria_round_bytes(t, C[first], true, true);
    for (int i = 0; i < 16; i++) w[1][i] = t[i] ^ kr[i];
    for (int i = 0; i < 16; i++) t[i] = w[1][i];
    aria_round_bytes(t, C[(first + 1) % 3], false, true);
    for (int i = 0; i < 16; i++) w[2][i] = t[i] ^ w[0][i];
    for (int i = 0; i < 16; i++) t[i] = w[2][i];
    aria_round_bytes(t, C[(first + 2) % 3], true, true);
    for (int i = 0; i < 16; i++) w[3][i] = t[i] ^ w[1][i];
    const int rot[5] = { 19, 31, 128 - 61, 128 - 31, 128 - 19 };   /* right rotations */
    for (int e = 0; e < nr + 1; e++) {
        const uint8_t *a = w[e % 4], *b = w[(e % 4 + 1) % 4];
        const int n = rot[e / 4], by = n / 8, bi = n % 8;
        for (int i = 0; i < 16; i++) {
            const uint8_t hi = b[(i - by + 16) % 16], lo = b[(i - by - 1 + 32) % 16];
            const uint8_t r = (uint8_t) (bi ? ((hi >> bi) | (lo << (8 - bi))) : hi);
            ek[e][i] = a[i] ^ r;
        }
    }
    return nr;
}

__device__ inline void aria_encrypt_bytes(const uint8_t ek[17][16], int nr, uint8_t st[16])
{
    for (int r = 1; r < nr; r++) aria_round_bytes(st, ek[r - 1], (r & 1) != 0, true);
    aria_round_bytes(st, ek[nr - 1], false, false);
    for (int i = 0; i < 16; i++) st[i] ^= ek[nr][i];
}

/* Camellia key schedule and 64-bit-word block (RFC 3713 2.2-2.4), one lane:
 * only for the subkeys and H = E_K(0^128) of a slot. */
__device__ inline uint64_t cam_f64(uint64_t x, uint64_t k)
{
    x ^= k;
    const uint32_t xh = (uint32_t) (x >> 32), xl = (uint32_t) x;
    const uint32_t u = kCamSbox.sp[0][xh >> 24] ^ kCamSbox.sp[1][(xh >> 16) & 0xff] ^
                       kCamSbox.sp[2][(xh >> 8) & 0xff] ^ kCamSbox.sp[3][xh & 0xff];
    const uint32_t v = kCamSbox.sp[1][xl >> 24] ^ kCamSbox.sp[2][(xl >> 16) & 0xff] ^
                       kCamSbox.sp[3][(xl >> 8) & 0xff] ^ kCamSbox.sp[0][xl & 0xff];
    return ((uint64_t) (u ^ v) << 32) | (u ^ ((u >> 8) | (u << 24)) ^ v);
}

__device__ inline void cam_rol128(uint64_t hi, uint64_t lo, int n, uint64_t &oh, uint64_t &ol)
{
    if (n >= 64) { const uint64_t t = hi; hi = lo; lo = t; n -= 64; }
    if (n == 0) { oh = hi; ol = lo; return; }
    oh = (hi << n) | (lo >> (64 - n));
    ol = (lo << n) | (hi >> (64 - n));
}

/* the 26 / 34 subkeys in use order (kw1 kw2 | k1..k6 | ke1 ke2 | ... | kw3 kw4) */
__device__ inline int cam_key_expand(const uint8_t *key, int keylen, uint64_t sk[34])
{
    const uint64_t SIGMA[6] = { 0xA09E667F3BCC908BULL, 0xB67AE8584CAA73B2ULL, 0xC6EF372FE94F82BEULL,
                                0x54FF53A5F1D36F1CULL, 0x10E527FADE682D1DULL, 0xB05688C2B3E6C1FDULL };
    uint64_t w[4] = { 0, 0, 0, 0 };
    for (int i = 0; i < keylen; i++) w[i / 8] = (w[i / 8] << 8) | key[i];
    if (keylen == 24) w[3] = ~w[2];
    /* src: 0 KL, 1 KR, 2 KA, 3 KB as (hi, lo) */
    uint64_t src[4][2] = { { w[0], w[1] }, { w[2], w[3] }, { 0, 0 }, { 0, 0 } };
    uint64_t d1 = w[0] ^ w[2], d2 = w[1] ^ w[3];
    d2 ^= cam_f64(d1, SIGMA[0]);
    d1 ^= cam_f64(d2, SIGMA[1]);
    d1 ^= w[0];
    d2 ^= w[1];
    d2 ^= cam_f64(d1, SIGMA[2]);
    d1 ^= cam_f64(d2, SIGMA[3]);
    src[2][0] = d1; src[2][1] = d2;
    d1 ^= w[2];
    d2 ^= w[3];
    d2 ^= cam_f64(d1, SIGMA[4]);
    d1 ^= cam_f64(d2, SIGMA[5]);
    src[3][0] = d1; src[3][1] = d2;
    /* (source, rotation, halves: 3 both, 1 high, 2 low), RFC 3713 2.2 */
    const uint8_t s128[14][3] = { { 0, 0, 3 }, { 2, 0, 3 }, { 0, 15, 3 }, { 2, 15, 3 }, { 2, 30, 3 },
                                  { 0, 45, 3 }, { 2, 45, 1 }, { 0, 60, 2 }, { 2, 60, 3 }, { 0, 77, 3 },
                                  { 0, 94, 3 }, { 2, 94, 3 }, { 0, 111, 3 }, { 2, 111, 3 } };
    const uint8_t s256[17][3] = { { 0, 0, 3 }, { 3, 0, 3 }, { 1, 15, 3 }, { 2, 15, 3 }, { 1, 30, 3 },
                                  { 3, 30, 3 }, { 0, 45, 3 }, { 2, 45, 3 }, { 0, 60, 3 }, { 1, 60, 3 },
                                  { 3, 60, 3 }, { 0, 77, 3 }, { 2, 77, 3 }, { 1, 94, 3 }, { 2, 94, 3 },
                                  { 0, 111, 3 }, { 3, 111, 3 } };
    const int rows = keylen == 16 ? 14 : 17;
    int n = 0;
    for (int i = 0; i < rows; i++) {
        const uint8_t *e = keylen == 16 ? s128[i] : s256[i];
        uint64_t h, l;
        cam_rol128(src[e[0]][0], src[e[0]][1], e[1], h, l);
        if (e[2] & 1) sk[n++] = h;
        if (e[2] & 2) sk[n++] = l;
    }
    for (int i = n; i < 34; i++) sk[i] = 0;
    return keylen == 16 ? 18 : 24;
}

__device__ inline void cam_encrypt_u64(const uint64_t sk[34], int nr, uint64_t &hi, uint64_t &lo)
{
    uint64_t d1 = hi ^ sk[0], d2 = lo ^ sk[1];
    int i = 2;
    const int groups = nr / 6;
    for (int g = 0; g < groups; g++) {
        for (int r = 0; r < 3; r++) {
            d2 ^= cam_f64(d1, sk[i++]);
            d1 ^= cam_f64(d2, sk[i++]);
        }
        if (g != groups - 1) {
            uint32_t x1 = (uint32_t) (d1 >> 32), x2 = (uint32_t) d1;
            uint32_t k1 = (uint32_t) (sk[i] >> 32), k2 = (uint32_t) sk[i];
            uint32_t t = x1 & k1;
            x2 ^= (t << 1) | (t >> 31);
            x1 ^= x2 | k2;
            d1 = ((uint64_t) x1 << 32) | x2;
            i++;
            uint32_t y1 = (uint32_t) (d2 >> 32), y2 = (uint32_t) d2;
            k1 = (uint32_t) (sk[i] >> 32); k2 = (uint32_t) sk[i];
            y1 ^= y2 | k2;
            t = y1 & k1;
            y2 ^= (t << 1) | (t >> 31);
            d2 = ((uint64_t) y1 << 32) | y2;
            i++;
        }
    }
    hi = d2 ^ sk[i];
    lo = d1 ^ sk[i + 1];
}

/* One 256-thread workgroup per slot. */
__global__ __launch_bounds__(256) void tlsrec_keysetup_kernel(SlotState *slots, uint4 *ghtab,
                                                             const tlsrec_key_material *keys,
                                                             uint32_t first, uint32_t count)
{
    __shared__ G128 pw[KEY_TABLES];
    __shared__ uint4 base[KEY_TABLES][128];
    const uint32_t slot = first + blockIdx.x;
    if (blockIdx.x >= count) return;
    SlotState *st = &slots[slot];
    const tlsrec_key_material km = keys[blockIdx.x];
    const int tid = threadIdx.x;
    /* every AES cipher gets its key schedule (GCM and CCM), GCM also H and
     * the GHASH tables */
    const bool aes = tlsrec_cipher_nr(km.cipher) != 0;
    const bool aria = tlsrec_cipher_is_aria(km.cipher);
    const bool cam = tlsrec_cipher_is_cam(km.cipher);
    const bool gcm = tlsrec_cipher_is_gcm(km.cipher) || tlsrec_cipher_is_alt_gcm(km.cipher);
    if (tid == 0) {
        st->km = km;
        st->km.reserved[0] = 0;   /* CID length mirror (tlsrec_recdev.h plan_key) */
        st->nr = 0;
        st->cid_len = 0;          /* a (re)load leaves the slot without a CID */
        if (aes) {
            const int nk = (int) tlsrec_cipher_keylen(km.cipher) / 4;
            aes_key_expand(km.key, nk, st->rk);
            st->nr = (uint32_t) (nk + 6);
            for (int i = 0; i < 4 * (nk + 7); i++) {
                const bool middle = i >= 4 && i < 4 * (nk + 6);
                st->rkr[i] = middle ? __builtin_amdgcn_alignbit(st->rk[i], st->rk[i], 16) : st->rk[i];
            }
            uint8_t h[16] = { 0 };
            aes_encrypt_bytes(st->rk, nk + 6, h);
            G128 H;
            H.hi = 0; H.lo = 0;
            for (int i = 0; i < 8; i++) { H.hi = (H.hi << 8) | h[i]; H.lo = (H.lo << 8) | h[8 + i]; }
            for (int i = 0; i < 16; i++) st->h[i] = h[i];
            pw[0] = H;
            for (int p = 1; p < KEY_TABLES; p++) pw[p] = g_mul(pw[p - 1], pw[p - 1]);
        } else if (aria) {
            uint8_t ek[17][16];
            const int nr = aria_key_expand(km.key, (int) tlsrec_cipher_keylen(km.cipher), ek);
            for (int e = 0; e < 17; e++)
                for (int c = 0; c < 4; c++)
                    st->ark[4 * e + c] = e <= nr ? ((uint32_t) ek[e][4 * c] | ((uint32_t) ek[e][4 * c + 1] << 8) |
                                                    ((uint32_t) ek[e][4 * c + 2] << 16) | ((uint32_t) ek[e][4 * c + 3] << 24))
                                                 : 0u;
            uint8_t h[16] = { 0 };
            aria_encrypt_bytes(ek, nr, h);
            G128 H;
            H.hi = 0; H.lo = 0;
            for (int i = 0; i < 8; i++) { H.hi = (H.hi << 8) | h[i]; H.lo = (H.lo << 8) | h[8 + i]; }
            for (int i = 0; i < 16; i++) st->h[i] = h[i];
            pw[0] = H;
            for (int p = 1; p < KEY_TABLES; p++) pw[p] = g_mul(pw[p - 1], pw[p - 1]);
        } else if (cam) {
            /* Camellia: the subkeys as (high, low) word pairs (tlsrec_device.h cam_encrypt) */
            uint64_t sk[34];
            const int nr = cam_key_expand(km.key, (int) tlsrec_cipher_keylen(km.cipher), sk);
            for (int i = 0; i < 34; i++) {
                st->ark[2 * i] = (uint32_t) (sk[i] >> 32);
                st->ark[2 * i + 1] = (uint32_t) sk[i];
            }
            G128 H;
            H.hi = 0; H.lo = 0;
            cam_encrypt_u64(sk, nr, H.hi, H.lo);
            for (int i = 0; i < 8; i++) { st->h[i] = (uint8_t) (H.hi >> (56 - 8 * i)); st->h[8 + i] = (uint8_t) (H.lo >> (56 - 8 * i)); }
            pw[0] = H;
            for (int p = 1; p < KEY_TABLES; p++) pw[p] = g_mul(pw[p - 1], pw[p - 1]);
        }
    }
    __syncthreads();
    if (!gcm) return;
    /* base[p][j] = H^(2^p) * x^j */
    if (tid < KEY_TABLES) {
        G128 v = pw[tid];
        for (int j = 0; j < 128; j++) {
            base[tid][j] = g_to_words(v);
            v = g_shr1(v);
        }
    }
    __syncthreads();
    uint4 *out = ghtab + (size_t) slot * KEY_TABLE_WORDS;
    for (int e = tid; e < KEY_TABLES * 32 * 16; e += 256) {
        const int p = e >> 9, k = (e >> 4) & 31, nib = e & 15;
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (int i = 0; i < 4; i++)
            if ((nib >> (3 - i)) & 1) acc = xor4(acc, base[p][4 * k + i]);
        out[e] = acc;
    }
}

/* The GCM record kernel lives in tlsrec_gcm.h (instantiated by gcm_*.hip). */

/* ======================================================================
 * Bucket pass: group the batch's records by key for the GCM kernels (a key
 * pass stages one key's GHASH tables for a whole workgroup), ChaCha records
 * after them; records without a usable slot get BAD_INPUT_DATA here.
 *   key index: AES-128-GCM -> slot, AES-256-GCM -> cap + slot, AES-192-GCM
 *   -> 2 cap + slot, AES-CCM (any size/tag) -> 3 cap + slot, ChaCha -> 4 cap,
 *   ARIA-128/192/256-GCM -> (4, 5, 6) cap + 1 + slot, ARIA-CCM -> the CCM
 *   class, none -> no index.
 * Atomics are wave-aggregated when the wave's records share one key (a
 * batch already grouped by key costs one atomic per wave).
 * ==================================================================== */
__device__ __forceinline__ uint32_t bucket_key(const BucketArgs &a, const tlsrec_batch_rec &d)
{
    if (d.slot >= a.capacity) return 0xffffffffu;
    const int c = a.slots[d.slot].km.cipher;
    switch (c) {
        case TLSREC_CIPHER_AES_128_GCM: return d.slot;
        case TLSREC_CIPHER_AES_256_GCM: return a.capacity + d.slot;
        case TLSREC_CIPHER_AES_192_GCM: return 2 * a.capacity + d.slot;
        case TLSREC_CIPHER_CHACHA20_POLY1305: return 4 * a.capacity;
        /* ARIA-GCM classes after the ChaCha counter: 4 cap + 1 + (0..2) cap + slot */
        case TLSREC_CIPHER_ARIA_128_GCM: return 4 * a.capacity + 1 + d.slot;
        case TLSREC_CIPHER_ARIA_192_GCM: return 5 * a.capacity + 1 + d.slot;
        case TLSREC_CIPHER_ARIA_256_GCM: return 6 * a.capacity + 1 + d.slot;
        /* Camellia-GCM classes after ARIA's: (7, 8, 9) cap + 1 + slot */
        case TLSREC_CIPHER_CAMELLIA_128_GCM: return 7 * a.capacity + 1 + d.slot;
        case TLSREC_CIPHER_CAMELLIA_192_GCM: return 8 * a.capacity + 1 + d.slot;
        case TLSREC_CIPHER_CAMELLIA_256_GCM: return 9 * a.capacity + 1 + d.slot;
        default:
            return (tlsrec_cipher_is_ccm(c) || tlsrec_cipher_is_alt_ccm(c)) ? 3 * a.capacity + d.slot : 0xffffffffu;
    }
}

/* One wave's claim on the counters ctr[key] for its pending lanes: lanes
 * sharing the wave's first pending key take one atomic together (rank from
 * mbcnt), the rest one atomic each.  Returns the lane's position. */
__device__ __forceinline__ uint32_t claim_group(uint32_t *ctr, uint32_t key, bool pend)
{
    const uint64_t pmask = __ballot(pend);
    if (pmask == 0) return 0;
    const int lead = __builtin_ctzll(pmask);
    const uint32_t first = __builtin_amdgcn_readlane(key, lead);
    const bool grp = pend && key == first;
    const uint64_t same = __ballot(grp);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (same >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) same, 0));
    uint32_t base = 0;
    if (grp && rank == 0) base = atomicAdd(&ctr[first], (uint32_t) __popcll(same));
    base = __builtin_amdgcn_readlane(base, lead);
    if (grp) return base + rank;
    return pend ? atomicAdd(&ctr[key], 1u) : 0u;
}

/* ChaCha records share one counter: always one atomic per wave for them;
 * GCM records: one per wave when the wave's GCM records share a key (a batch
 * grouped by key), else one per record (distinct addresses, no contention). */
__device__ __forceinline__ uint32_t bucket_claim(const BucketArgs &a, uint32_t *ctr, uint32_t key)
{
    const bool cp = key == 4 * a.capacity;
    const uint32_t pc = claim_group(ctr, key, cp);
    const uint32_t pg = claim_group(ctr, key, key != 0xffffffffu && !cp);
    return cp ? pc : pg;
}

__global__ __launch_bounds__(256) void tlsrec_bucket_count_kernel(BucketArgs a)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t key = 0xffffffffu;
    if (i < a.n) {
        const tlsrec_batch_rec d = a.recs[i];
        key = bucket_key(a, d);
        if (key == 0xffffffffu) bad_slot_result(d, &a.res[i]);
    }
    (void) bucket_claim(a, a.counts, key);
}

__global__ __launch_bounds__(256) void tlsrec_bucket_scatter_kernel(BucketArgs a)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t key = 0xffffffffu;
    if (i < a.n) key = bucket_key(a, a.recs[i]);
    const uint32_t pos = bucket_claim(a, a.cursor, key);
    if (key != 0xffffffffu) a.perm[pos] = i;
}

/* ======================================================================
 * ChaCha20-Poly1305
 * ==================================================================== */
__device__ __forceinline__ P5 p_from_words(uint4 w)
{
    P5 r;
    r.v[0] = w.x & TLSREC_M26;
    r.v[1] = ((w.x >> 26) | (w.y << 6)) & TLSREC_M26;
    r.v[2] = ((w.y >> 20) | (w.z << 12)) & TLSREC_M26;
    r.v[3] = ((w.z >> 14) | (w.w << 18)) & TLSREC_M26;
    r.v[4] = (w.w >> 8) | (1u << 24);
    return r;
}

/* Poly1305 Horner over blocks 0..3 of a CID record's AAD (block 0 = a0, in
 * limb form): A_1 r^(a-1) + ... + A_a.  Out of line, as gcm_cid_aad_fold. */
__device__ __noinline__ P5 cp_cid_aad_fold(P5 a0, const uint32_t *r1w, const tlsrec_plan &p,
                                           const tlsrec_batch_rec &d, const uint8_t *cid)
{
    P5 r1;
#pragma unroll
    for (int i = 0; i < 5; i++) r1.v[i] = r1w[i];
    P5 f = p_add(p_mul(a0, r1), p_from_words(cid_aad_block<1, 0>(p, d, cid)));
    if (p.aad_len > 32) f = p_add(p_mul(f, r1), p_from_words(cid_aad_block<2, 0>(p, d, cid)));
    if (p.aad_len > 48) f = p_add(p_mul(f, r1), p_from_words(cid_aad_block<3, 0>(p, d, cid)));
    return f;
}

template <int L>
__device__ __forceinline__ P5 shfl_p5(P5 v, int src)
{
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = __shfl(v.v[i], src);
    return r;
}

/* Per-record constants of the ChaCha20-Poly1305 kernel, one per chunk
 * position of a wave, written by the wave's pre-pass and read (L lanes per
 * record) from LDS in the record loop instead of living in VGPRs. */
struct CpRec {
    uint32_t key[8];
    uint32_t nonce[3];
    uint32_t pad0;
    uint32_t s[4];           /* Poly1305 s */
    uint32_t r1[5], r2[5], r3[5], rl[5];   /* r, r^2, r^3, r^(4L) (26-bit limbs) */
    uint32_t aadf[5];        /* DTLS 1.2 + CID: the 2..4 AAD blocks Horner-folded */
};
static_assert(sizeof(CpRec) == 164, "CpRec layout");

__device__ __forceinline__ P5 p_lds(const uint32_t *v)
{
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = v[i];
    return r;
}

/* 64-bit limb accumulator: sums of 26x28-bit limb products, reduced once */
struct D5 { uint64_t v[5]; };

__device__ __forceinline__ void p_mac(D5 &d, const P5 &h, const P5 &r)
{
    const uint32_t s1 = r.v[1] * 5, s2 = r.v[2] * 5, s3 = r.v[3] * 5, s4 = r.v[4] * 5;
    d.v[0] += (uint64_t) h.v[0] * r.v[0] + (uint64_t) h.v[1] * s4 + (uint64_t) h.v[2] * s3 +
              (uint64_t) h.v[3] * s2 + (uint64_t) h.v[4] * s1;
    d.v[1] += (uint64_t) h.v[0] * r.v[1] + (uint64_t) h.v[1] * r.v[0] + (uint64_t) h.v[2] * s4 +
              (uint64_t) h.v[3] * s3 + (uint64_t) h.v[4] * s2;
    d.v[2] += (uint64_t) h.v[0] * r.v[2] + (uint64_t) h.v[1] * r.v[1] + (uint64_t) h.v[2] * r.v[0] +
              (uint64_t) h.v[3] * s4 + (uint64_t) h.v[4] * s3;
    d.v[3] += (uint64_t) h.v[0] * r.v[3] + (uint64_t) h.v[1] * r.v[2] + (uint64_t) h.v[2] * r.v[1] +
              (uint64_t) h.v[3] * r.v[0] + (uint64_t) h.v[4] * s4;
    d.v[4] += (uint64_t) h.v[0] * r.v[4] + (uint64_t) h.v[1] * r.v[3] + (uint64_t) h.v[2] * r.v[2] +
              (uint64_t) h.v[3] * r.v[1] + (uint64_t) h.v[4] * r.v[0];
}

/* carry-propagate a D5 of up to four limb products plus a block (< 2^59 per
 * limb) into limbs < 2^26, limb 1 < 2^26 + 2^10 -- the form p_mul returns */
__device__ __forceinline__ P5 p_reduce(D5 d)
{
    P5 o;
    uint64_t c;
    c = d.v[0] >> 26; o.v[0] = (uint32_t) d.v[0] & TLSREC_M26; d.v[1] += c;
    c = d.v[1] >> 26; o.v[1] = (uint32_t) d.v[1] & TLSREC_M26; d.v[2] += c;
    c = d.v[2] >> 26; o.v[2] = (uint32_t) d.v[2] & TLSREC_M26; d.v[3] += c;
    c = d.v[3] >> 26; o.v[3] = (uint32_t) d.v[3] & TLSREC_M26; d.v[4] += c;
    c = d.v[4] >> 26; o.v[4] = (uint32_t) d.v[4] & TLSREC_M26;
    const uint64_t t = (uint64_t) o.v[0] + c * 5;
    o.v[0] = (uint32_t) t & TLSREC_M26;
    o.v[1] += (uint32_t) (t >> 26);
    return o;
}

__device__ __forceinline__ void chacha_block_kn(const uint32_t *kn, uint32_t counter, uint32_t out[16])
{
    uint32_t key[8], nw[3];
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = kn[i];
#pragma unroll
    for (int i = 0; i < 3; i++) nw[i] = kn[8 + i];
    chacha_block(key, counter, nw, out);
}

template <int L, bool DEC, bool CID = false>
__global__ __launch_bounds__(CP_THREADS) __attribute__((amdgpu_waves_per_eu(2))) void tlsrec_chachapoly_kernel(CpArgs a)
{
    constexpr int R = 64 / L;
    constexpr int LOGL = Log2<L>::v;
    __shared__ CpRec crec[CP_WAVES][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g = lane / L, q = lane % L;
    const uint32_t lo = a.perm ? *a.lo : 0u;
    const uint32_t count = a.perm ? *a.hi - lo : (uint32_t) a.n;
    const uint64_t chunk = ((uint64_t) blockIdx.x * CP_WAVES + wave) * a.rpw;

    /* ---- pre-pass: per chunk position, the record's key/nonce, the one-time
     * Poly1305 key (ChaCha20 block 0, RFC 8439 2.6) and powers of r ---- */
    bool mine = false;
    uint32_t my_rec = 0;
    {
        const uint64_t pos = chunk + (uint64_t) lane;
        CpRec &cr = crec[wave][lane];
        uint32_t key[8] = { 0 }, nw[3] = { 0, 0, 0 };
        if (lane < (int) a.rpw && pos < count) {
            my_rec = a.perm ? a.perm[lo + pos] : (uint32_t) pos;
            const tlsrec_batch_rec d = a.recs[my_rec];
            if (!a.perm && !(d.slot < a.capacity && a.slots[d.slot].km.cipher != 0))
                bad_slot_result(d, &a.res[my_rec]);
            if (d.slot < a.capacity && a.slots[d.slot].km.cipher == TLSREC_CIPHER_CHACHA20_POLY1305) {
                mine = true;
                const tlsrec_key_material km = a.slots[d.slot].km;
                tlsrec_plan p;
                make_plan<DEC, CID>(p, d, km, &a.slots[d.slot], a.in);
                nonce_words<DEC>(p, d, a.in, nw);
                for (int i = 0; i < 8; i++) key[i] = ld_u32le(km.key + 4 * i);
            }
        }
        uint32_t blk[16];
        chacha_block(key, 0, nw, blk);
        for (int i = 0; i < 8; i++) cr.key[i] = key[i];
        for (int i = 0; i < 3; i++) cr.nonce[i] = nw[i];
        for (int i = 0; i < 4; i++) cr.s[i] = blk[4 + i];
        const P5 r1 = p_from_r(blk[0], blk[1], blk[2], blk[3]);
        const P5 r2 = p_mul(r1, r1);
        const P5 r3 = p_mul(r2, r1);
        P5 rl = p_mul(r2, r2);                                  /* r^4 */
        for (int i = 0; i < LOGL; i++) rl = p_mul(rl, rl);      /* r^(4L) */
        for (int i = 0; i < 5; i++) {
            cr.r1[i] = r1.v[i];
            cr.r2[i] = r2.v[i];
            cr.r3[i] = r3.v[i];
            cr.rl[i] = rl.v[i];
        }
    }
    /* lanes read other lanes' CpRec: the wave's own LDS writes land first */

    for (uint32_t rr = 0; rr < a.rpw; rr += R) {
        const uint32_t slot_in_chunk = rr + (uint32_t) g;
        const bool owner_mine = __shfl((int) mine, (int) slot_in_chunk & 63) != 0;
        const bool active = slot_in_chunk < a.rpw && owner_mine;
        const uint64_t ridx = (uint32_t) __shfl((int) my_rec, (int) slot_in_chunk & 63);
        const CpRec &cr = crec[wave][slot_in_chunk & 63];
        tlsrec_batch_rec d;
        tlsrec_plan p;
        bool run = false;
        if (active) {
            d = a.recs[ridx];
            const tlsrec_key_material km = a.slots[d.slot].km;
            make_plan<DEC, CID>(p, d, km, &a.slots[d.slot], a.in);
            if (p.status != 0) {
                if (q == 0) finish_early(p, d, a.out, &a.res[ridx]);
            } else {
                run = true;
            }
        }
        const uint32_t aead_len = run ? p.aead_len : 0;
        const uint32_t B = (aead_len + 63) >> 6;              /* ChaCha20 chunks */
        const uint32_t M = (aead_len + 15) >> 4;              /* Poly1305 C blocks */
        const uint32_t v = B ? M - 4 * (B - 1) : 0;
        const uint32_t z = (L - B % L) % L;
        const uint32_t J = run ? (B + z) / L : 0;
        const uint32_t Jmax = wave_max(J);
        uint4 aadw = make_uint4(0, 0, 0, 0);
        bool cidaad = false;  /* AAD of 2..4 blocks, folded into cr.aadf */
        const uint8_t *src = a.in;
        uint8_t *dst = a.out;
        bool aligned = false;
        uint32_t content_len = 0;
        if (run) {
            aadw = aad_words(p);
            cidaad = CID && p.aad_len > 16;
            if (cidaad && q == 0) {   /* DTLS 1.2 + CID: one lane folds, all read */
                const P5 f = cp_cid_aad_fold(p_from_words(aadw), cr.r1, p, d, a.slots[d.slot].cid);
                uint32_t *w = const_cast<uint32_t *>(cr.aadf);
#pragma unroll
                for (int i = 0; i < 5; i++) w[i] = f.v[i];
            }
            src = a.in + d.buf_off + p.aead_pos;
            dst = a.out + d.buf_off + p.aead_pos;
            aligned = true;   /* any byte offset: see GcmJob::setup */
            content_len = DEC ? aead_len : p.content_len;
        }
        const uint8_t inner_type = run ? p.inner_type : 0;
        const bool tls13 = run && p.inner;   /* TLS 1.3 or DTLS 1.2 + CID inner plaintext */
        /* a readable 16-byte address for lanes with nothing to load */
        const uint8_t *safe = run ? src : reinterpret_cast<const uint8_t *>(a.recs);

        P5 acc = p_zero(), vf = p_zero();
        uint32_t nzpos = 0;                 /* TLS 1.3: 1 + position of the last non-zero 16-B block */

        /* general step: any chunk (front padding, AAD fold at chunk 0, the
         * final chunk with v <= 4 Poly1305 blocks, partial or unaligned data) */
        auto general = [&](uint32_t j) {
            const int32_t b = (int32_t) (L * j + q) - (int32_t) z;
            const bool live = run && j < J;
            const bool valid = live && b >= 0 && (uint32_t) b < B;
            /* all four loads first (full aligned blocks directly, the rest from
             * a safe address and redone below), a ChaCha block ahead of use */
            uint4 ct[4];
            bool fast[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint32_t pos = (uint32_t) b * 64 + 16 * t;
                fast[t] = valid && aligned && pos + 16 <= content_len;
                ct[t] = gload16(fast[t] ? src + pos : safe);
            }
            asm volatile("" ::: "memory");
            uint32_t ks[16];
            chacha_block_kn(cr.key, (uint32_t) b + 1u, ks);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint32_t pos = (uint32_t) b * 64 + 16 * t;
                const uint4 k = make_uint4(ks[4 * t], ks[4 * t + 1], ks[4 * t + 2], ks[4 * t + 3]);
                if (fast[t]) {
                    const uint4 o = xor4(ct[t], k);
                    gstore16(dst + pos, o);
                    if (!DEC) ct[t] = o;
                    if (DEC && tls13 && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                } else if (valid && pos < aead_len) {
                    const uint4 blk = load_block(src, pos, content_len, aead_len, inner_type, aligned);
                    const uint4 o = mask_block(xor4(blk, k), pos, aead_len);
                    store_block(dst, pos, aead_len, o, aligned);
                    ct[t] = DEC ? blk : o;
                    if (DEC && tls13 && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                } else {
                    ct[t] = make_uint4(0, 0, 0, 0);
                }
            }
            /* Horner over this chunk's Poly1305 blocks (AAD folded before C_0) */
            const P5 r1 = p_lds(cr.r1);
            const uint32_t vv = (valid && (uint32_t) b == B - 1) ? v : 4;
            P5 x = p_from_words(ct[0]);
            if (b == 0) x = p_add(x, p_mul(cidaad ? p_lds(cr.aadf) : p_from_words(aadw), r1));
#pragma unroll
            for (int t = 1; t < 4; t++) {
                P5 y = p_add(p_mul(x, r1), p_from_words(ct[t]));
                x = p_sel((uint32_t) t < vv, y, x);
            }
            const bool is_final = valid && (uint32_t) b == B - 1;
            if (is_final) vf = x;
            P5 an = (j == 0) ? p_zero() : p_mul(acc, p_lds(cr.rl));
            an = p_add(an, (valid && !is_final) ? x : p_zero());
            if (live && !is_final) acc = an;
        };

        /* Body chunks [1, jh): every lane of the wave holds a full, aligned,
         * non-final chunk inside its record's content (wave-uniform bound):
         * no masks, and Poly1305 as acc*r^(4L) + c0 r^3 + c1 r^2 + c2 r + c3
         * with one carry propagation per chunk. */
        uint32_t jh = 0;
        {
            const uint32_t bmax = (run && aligned && B > 0) ? min(B - 1, content_len / 64) : 0;
            const uint32_t h = wave_min(run ? (bmax + z) / L : 0);
            jh = h > 1 ? h : 0;
        }
        const uint32_t jl = jh ? 1u : Jmax;
        uint32_t j = 0;
        for (; j < jl; j++) general(j);
        /* one body chunk: load (a ChaCha20 block ahead of use), XOR, store,
         * Horner step acc*r^(4L) + c0 r^3 + c1 r^2 + c2 r + c3 */
        auto absorb = [&](uint4 (&c)[4], const uint32_t (&ks)[16], uint32_t b) {
            uint8_t *dp = dst + (size_t) b * 64;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint4 o = xor4(c[t], make_uint4(ks[4 * t], ks[4 * t + 1], ks[4 * t + 2], ks[4 * t + 3]));
                gstore16(dp + 16 * t, o);
                if (DEC && tls13 && (o.x | o.y | o.z | o.w)) nzpos = b * 64 + 16 * t + 1;
                if (!DEC) c[t] = o;
            }
            D5 dd;
            const P5 c3 = p_from_words(c[3]);
#pragma unroll
            for (int i = 0; i < 5; i++) dd.v[i] = c3.v[i];
            p_mac(dd, acc, p_lds(cr.rl));
            p_mac(dd, p_from_words(c[0]), p_lds(cr.r3));
            p_mac(dd, p_from_words(c[1]), p_lds(cr.r2));
            p_mac(dd, p_from_words(c[2]), p_lds(cr.r1));
            acc = p_reduce(dd);
        };
        /* two chunks per lane per step: two key-stream blocks in lockstep */
        for (; j + 1 < jh; j += 2) {
            const uint32_t b0 = L * j + q - z, b1 = b0 + L;
            uint4 c0[4], c1[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                c0[t] = gload16(src + (size_t) b0 * 64 + 16 * t);
                c1[t] = gload16(src + (size_t) b1 * 64 + 16 * t);
            }
            asm volatile("" ::: "memory");
            uint32_t ks0[16], ks1[16];
            {
                uint32_t key[8], nw[3];
#pragma unroll
                for (int i = 0; i < 8; i++) key[i] = cr.key[i];
#pragma unroll
                for (int i = 0; i < 3; i++) nw[i] = cr.nonce[i];
                chacha_block2(key, b0 + 1u, b1 + 1u, nw, ks0, ks1);
            }
            absorb(c0, ks0, b0);
            absorb(c1, ks1, b1);
        }
        for (; j < jh; j++) {
            const uint32_t b = L * j + q - z;
            const uint8_t *sp = src + (size_t) b * 64;
            uint4 c[4];
#pragma unroll
            for (int t = 0; t < 4; t++) c[t] = gload16(sp + 16 * t);
            /* keep the loads here, a ChaCha20 block ahead of their use: left
             * alone, the scheduler sinks each to just before its XOR and the
             * step pays four serial memory latencies */
            asm volatile("" ::: "memory");
            uint32_t ks[16];
            chacha_block_kn(cr.key, b + 1u, ks);
            absorb(c, ks, b);
        }
        for (; j < Jmax; j++) general(j);

        if (run && B == 0 && q == L - 1) vf = cidaad ? p_lds(cr.aadf) : p_from_words(aadw);
        /* rotated tree: logical ql = (q+1) % L, anchored at chunk B-2;
         * level i combines with r^(4 * 2^i) */
        const P5 r1 = p_lds(cr.r1), r2 = p_lds(cr.r2);
        const P5 r4 = p_mul(r2, r2);
        P5 rpow[LOGL + 1];
        rpow[0] = r4;
#pragma unroll
        for (int i = 1; i <= LOGL; i++) rpow[i] = p_mul(rpow[i - 1], rpow[i - 1]);
        const int ql = (q + 1) % L;
#pragma unroll
        for (int i = LOGL - 1; i >= 0; i--) {
            const int sh = 1 << i;
            const int src_lane = (lane - q) + ((ql + sh + L - 1) % L);
            P5 o = shfl_p5<L>(acc, src_lane);
            P5 t = p_add(p_mul(acc, rpow[i]), o);
            acc = p_carry(t);
        }
        /* in lane L-1: poly = r * (r * (vf + r^(4-delta) * W) + LEN) */
        const uint32_t delta = 4 - v;
        P5 rd = delta == 0 ? r4 : (delta == 1 ? p_lds(cr.r3) : (delta == 2 ? r2 : r1));
        P5 X = p_add(p_mul(acc, rd), vf);
        X = p_mul(p_carry(X), r1);
        const uint32_t alen = run ? p.aad_len : 0;
        X = p_add(X, p_from_words(make_uint4(alen, 0, aead_len, 0)));
        X = p_mul(p_carry(X), r1);
        const uint4 sw = make_uint4(cr.s[0], cr.s[1], cr.s[2], cr.s[3]);
        const uint4 tag = p_finish(X, sw);
        if (!run) continue;
        const int leader = lane - q + (L - 1);
        if (!DEC) {
            if (q == L - 1) {
                store_block(dst, aead_len, aead_len + 16, tag, false);
                tlsrec_batch_res r;
                r.status = p.post_status;
                r.data_offset = p.data_offset;
                r.data_len = p.data_len;
                r.type = p.type;
                r.cid_len = p.cid_set ? p.cid_len : 0;
                r.reserved[0] = r.reserved[1] = 0;
                a.res[ridx] = r;
            }
        } else {
            uint4 want = load_block(src, aead_len, aead_len + 16, aead_len + 16, 0, false);
            uint32_t diff = (want.x ^ tag.x) | (want.y ^ tag.y) | (want.z ^ tag.z) | (want.w ^ tag.w);
            diff = __shfl(diff, leader);
            uint32_t nzkey = 0;
            if (tls13 && nzpos) {
                const uint32_t pos = nzpos - 1;
                nzkey = last_nonzero_key(load_block(dst, pos, aead_len, aead_len, 0, false), pos);
            }
            const uint32_t key2 = group_max<L>(nzkey);
            tlsrec_batch_res r;
            r.data_offset = p.data_offset;
            r.data_len = p.data_len;
            r.type = d.type;
            r.cid_len = 0;
            r.reserved[0] = r.reserved[1] = 0;
            if (diff != 0) {
                zero_range(a.out + d.buf_off, p.aead_pos, d.buf_len, q, L);
                r.status = TLSREC_E_INVALID_MAC;
            } else if (p.inner) {
                if (key2 == 0) {
                    r.status = TLSREC_E_INVALID_RECORD;
                } else {
                    r.status = 0;
                    r.data_len = (key2 >> 8) - 1;
                    r.type = (uint8_t) (key2 & 0xff);
                }
            } else {
                r.status = 0;
            }
            if (q == L - 1) a.res[ridx] = r;
        }
    }
}


/* ======================================================================
 * Launchers
 * ==================================================================== */
template <int L, bool DEC>
static hipError_t launch_cp_t(const CpArgs &a, uint32_t grid, hipStream_t st)
{
    if (a.cid) {   /* key table with DTLS connection IDs: L = 2 */
        if constexpr (L == 2)
            hipLaunchKernelGGL((tlsrec_chachapoly_kernel<2, DEC, true>), dim3(grid), dim3(CP_THREADS), 0, st, a);
        else
            return hipErrorInvalidValue;
    } else {
        hipLaunchKernelGGL((tlsrec_chachapoly_kernel<L, DEC>), dim3(grid), dim3(CP_THREADS), 0, st, a);
    }
    return hipGetLastError();
}

} /* namespace tlsrec */

using namespace tlsrec;

/* gcm_enc.hip / gcm_dec.hip / gcm_alt_enc.hip / gcm_alt_dec.hip */
extern "C" {
hipError_t tlsrec__launch_gcm_enc(const GcmArgs *a, int lanes, int nr, int waves, uint32_t grid, hipStream_t st);
hipError_t tlsrec__launch_gcm_dec(const GcmArgs *a, int lanes, int nr, int waves, uint32_t grid, hipStream_t st);
hipError_t tlsrec__launch_gcm_alt_enc(const GcmArgs *a, int nr, int cid, uint32_t grid, hipStream_t st);
hipError_t tlsrec__launch_gcm_alt_dec(const GcmArgs *a, int nr, int cid, uint32_t grid, hipStream_t st);
}

extern "C" hipError_t tlsrec__launch_keysetup(SlotState *slots, uint4 *ghtab, const tlsrec_key_material *keys,
                                              uint32_t first, uint32_t count, hipStream_t st)
{
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(tlsrec_keysetup_kernel, dim3(count), dim3(256), 0, st, slots, ghtab, keys, first, count);
    return hipGetLastError();
}

extern "C" hipError_t tlsrec__launch_gcm_aria(const GcmArgs *a, int dec, int nr, int cid, uint32_t grid, hipStream_t st)
{
    return dec ? tlsrec__launch_gcm_alt_dec(a, nr, cid, grid, st) : tlsrec__launch_gcm_alt_enc(a, nr, cid, grid, st);
}

extern "C" hipError_t tlsrec__launch_gcm(const GcmArgs *a, int dec, int lanes, int nr, int waves, uint32_t grid,
                                         hipStream_t st)
{
    return dec ? tlsrec__launch_gcm_dec(a, lanes, nr, waves, grid, st) : tlsrec__launch_gcm_enc(a, lanes, nr, waves, grid, st);
}

extern "C" hipError_t tlsrec__launch_bucket_count(const BucketArgs *a, hipStream_t st)
{
    if (a->n == 0) return hipSuccess;
    hipLaunchKernelGGL(tlsrec_bucket_count_kernel, dim3((a->n + 255) / 256), dim3(256), 0, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t tlsrec__launch_bucket_scatter(const BucketArgs *a, hipStream_t st)
{
    if (a->n == 0) return hipSuccess;
    hipLaunchKernelGGL(tlsrec_bucket_scatter_kernel, dim3((a->n + 255) / 256), dim3(256), 0, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t tlsrec__launch_chachapoly(const CpArgs *a, int dec, int lanes, uint32_t grid, hipStream_t st)
{
    switch (lanes) {
        case 1: return dec ? launch_cp_t<1, true>(*a, grid, st) : launch_cp_t<1, false>(*a, grid, st);
        case 2: return dec ? launch_cp_t<2, true>(*a, grid, st) : launch_cp_t<2, false>(*a, grid, st);
        case 4: return dec ? launch_cp_t<4, true>(*a, grid, st) : launch_cp_t<4, false>(*a, grid, st);
        case 8: return dec ? launch_cp_t<8, true>(*a, grid, st) : launch_cp_t<8, false>(*a, grid, st);
        default: return hipErrorInvalidValue;
    }
}
