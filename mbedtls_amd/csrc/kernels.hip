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
__device__ inline void aes_key_expand(const uint8_t *sb, const uint8_t *key, int nk, uint32_t *rk)
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
            t = (uint32_t) sb[t & 0xff] | ((uint32_t) sb[(t >> 8) & 0xff] << 8) |
                ((uint32_t) sb[(t >> 16) & 0xff] << 16) | ((uint32_t) sb[t >> 24] << 24);
            t ^= rcon;
            rcon = xtime8(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t) sb[t & 0xff] | ((uint32_t) sb[(t >> 8) & 0xff] << 8) |
                ((uint32_t) sb[(t >> 16) & 0xff] << 16) | ((uint32_t) sb[t >> 24] << 24);
        }
        rk[i] = rk[i - nk] ^ t;
    }
}

/* byte-oriented AES (one lane; only used for H = E_K(0^128)) */
__device__ inline void aes_encrypt_bytes(const uint8_t *sb, const uint32_t *rk, int nr, uint8_t st[16])
{
    for (int i = 0; i < 16; i++) st[i] ^= (uint8_t) (rk[i / 4] >> (8 * (i % 4)));
    for (int r = 1; r <= nr; r++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++) t[4 * c + row] = sb[st[4 * ((c + row) & 3) + row]];
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
__device__ inline void aria_round_bytes(const uint8_t *sb, uint8_t d[16], const uint8_t rk[16], bool odd, bool diffuse)
{
    uint32_t x[16], y[16];
    for (int i = 0; i < 16; i++) {
        const int t = odd ? (i & 3) : ((i & 3) ^ 2);
        x[i] = sb[t * 256 + (d[i] ^ rk[i])];
    }
    if (diffuse) {
        TLSREC_ARIA_A(y, x);
        for (int i = 0; i < 16; i++) d[i] = (uint8_t) y[i];
    } else {
        for (int i = 0; i < 16; i++) d[i] = (uint8_t) x[i];
    }
}

__device__ inline int aria_key_expand(const uint8_t *sb, const uint8_t *key, int keylen, uint8_t ek[17][16])
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
    aria_round_bytes(sb, t, C[first], true, true);
    for (int i = 0; i < 16; i++) w[1][i] = t[i] ^ kr[i];
    for (int i = 0; i < 16; i++) t[i] = w[1][i];
    aria_round_bytes(sb, t, C[(first + 1) % 3], false, true);
    for (int i = 0; i < 16; i++) w[2][i] = t[i] ^ w[0][i];
    for (int i = 0; i < 16; i++) t[i] = w[2][i];
    aria_round_bytes(sb, t, C[(first + 2) % 3], true, true);
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

__device__ inline void aria_encrypt_bytes(const uint8_t *sb, const uint8_t ek[17][16], int nr, uint8_t st[16])
{
    for (int r = 1; r < nr; r++) aria_round_bytes(sb, st, ek[r - 1], (r & 1) != 0, true);
    aria_round_bytes(sb, st, ek[nr - 1], false, false);
    for (int i = 0; i < 16; i++) st[i] ^= ek[nr][i];
}

/* Camellia key schedule and 64-bit-word block (RFC 3713 2.2-2.4), one lane:
 * only for the subkeys and H = E_K(0^128) of a slot. */
__device__ inline uint64_t cam_f64(const uint8_t *sb, uint64_t x, uint64_t k)
{
    x ^= k;
    const uint32_t xh = (uint32_t) (x >> 32), xl = (uint32_t) x;
    const uint32_t A = ((uint32_t) sb[0 * 256 + (xh >> 24)] << 24) | ((uint32_t) sb[1 * 256 + ((xh >> 16) & 0xff)] << 16) |
                       ((uint32_t) sb[2 * 256 + ((xh >> 8) & 0xff)] << 8) | sb[3 * 256 + (xh & 0xff)];
    const uint32_t B = ((uint32_t) sb[1 * 256 + (xl >> 24)] << 24) | ((uint32_t) sb[2 * 256 + ((xl >> 16) & 0xff)] << 16) |
                       ((uint32_t) sb[3 * 256 + ((xl >> 8) & 0xff)] << 8) | sb[0 * 256 + (xl & 0xff)];
    /* P-layer as in cam_f (tlsrec_device.h) */
    const uint32_t U = A ^ ((B << 8) | (B >> 24));
    const uint32_t V = B ^ ((U << 16) | (U >> 16));
    const uint32_t U2 = U ^ ((V >> 8) | (V << 24));
    return ((uint64_t) (V ^ ((U2 >> 8) | (U2 << 24))) << 32) | U2;
}

__device__ inline void cam_rol128(uint64_t hi, uint64_t lo, int n, uint64_t &oh, uint64_t &ol)
{
    if (n >= 64) { const uint64_t t = hi; hi = lo; lo = t; n -= 64; }
    if (n == 0) { oh = hi; ol = lo; return; }
    oh = (hi << n) | (lo >> (64 - n));
    ol = (lo << n) | (hi >> (64 - n));
}

/* the 26 / 34 subkeys in use order (kw1 kw2 | k1..k6 | ke1 ke2 | ... | kw3 kw4) */
__device__ inline int cam_key_expand(const uint8_t *sb, const uint8_t *key, int keylen, uint64_t sk[34])
{
    const uint64_t SIGMA[6] = { 0xA09E667F3BCC908BULL, 0xB67AE8584CAA73B2ULL, 0xC6EF372FE94F82BEULL,
                                0x54FF53A5F1D36F1CULL, 0x10E527FADE682D1DULL, 0xB05688C2B3E6C1FDULL };
    uint64_t w[4] = { 0, 0, 0, 0 };
    for (int i = 0; i < keylen; i++) w[i / 8] = (w[i / 8] << 8) | key[i];
    if (keylen == 24) w[3] = ~w[2];
    /* src: 0 KL, 1 KR, 2 KA, 3 KB as (hi, lo) */
    uint64_t src[4][2] = { { w[0], w[1] }, { w[2], w[3] }, { 0, 0 }, { 0, 0 } };
    uint64_t d1 = w[0] ^ w[2], d2 = w[1] ^ w[3];
    d2 ^= cam_f64(sb, d1, SIGMA[0]);
    d1 ^= cam_f64(sb, d2, SIGMA[1]);
    d1 ^= w[0];
    d2 ^= w[1];
    d2 ^= cam_f64(sb, d1, SIGMA[2]);
    d1 ^= cam_f64(sb, d2, SIGMA[3]);
    src[2][0] = d1; src[2][1] = d2;
    d1 ^= w[2];
    d2 ^= w[3];
    d2 ^= cam_f64(sb, d1, SIGMA[4]);
    d1 ^= cam_f64(sb, d2, SIGMA[5]);
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

__device__ inline void cam_encrypt_u64(const uint8_t *sb, const uint64_t sk[34], int nr, uint64_t &hi, uint64_t &lo)
{
    uint64_t d1 = hi ^ sk[0], d2 = lo ^ sk[1];
    int i = 2;
    const int groups = nr / 6;
    for (int g = 0; g < groups; g++) {
        for (int r = 0; r < 3; r++) {
            d2 ^= cam_f64(sb, d1, sk[i++]);
            d1 ^= cam_f64(sb, d2, sk[i++]);
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
/* 8 waves per SIMD (64 VGPRs, 24 spilled): one workgroup per slot runs long
 * dependent chains (key expansion, the squarings of H, the power ladder), so
 * resident workgroups are the throughput.  The H^1..H^64 values of r04 had
 * taken it to 102 VGPRs and 4 waves (keysched 14.3 -> 11.5 M connections/s);
 * same box, profiles/r04w: 4 waves 11.6 M, 6 waves 14.4 M, 8 waves 16.0 M. */
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void tlsrec_keysetup_kernel(SlotState *slots, uint4 *ghtab, uint8_t *cipher_of,
                                                             const tlsrec_key_material *keys,
                                                             uint32_t first, uint32_t count)
{
    __shared__ G128 pw[KEY_TABLES];
    __shared__ G128 hp[KEY_HPOW_N];     /* H^1 .. H^64 */
    __shared__ uint4 base[KEY_TABLES][128];
    /* the key schedule is built in LDS, not in the slot: the single lane
     * that expands it and encrypts H reads it back word by word, and each
     * of those reads from global memory was a full round trip (64 K AES-256
     * slots: 5.6 ms with the schedule in the slot) */
    __shared__ uint64_t ksched[34];
    /* the cipher's S-boxes for that lane, from LDS (a constant-memory lookup
     * per S-box byte is a memory round trip on its dependent chain) */
    __shared__ uint8_t sb[4 * 256];
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
    for (int i = tid; i < 4 * 256; i += 256)
        sb[i] = aria ? kAriaSbox.v[i >> 8][i & 255] : (cam ? kCamSbox.v[i >> 8][i & 255] : kSbox.v[i & 255]);
    __syncthreads();
    if (tid == 0) {
        st->km = km;
        cipher_of[slot] = km.cipher;
        st->km.reserved[0] = 0;   /* CID length mirror (tlsrec_recdev.h plan_key) */
        st->nr = 0;
        st->cid_len = 0;          /* a (re)load leaves the slot without a CID */
        if (aes) {
            const int nk = (int) tlsrec_cipher_keylen(km.cipher) / 4;
            uint32_t *rk = reinterpret_cast<uint32_t *>(ksched);
            aes_key_expand(sb, km.key, nk, rk);
            st->nr = (uint32_t) (nk + 6);
            for (int i = 0; i < 4 * (nk + 7); i++) {
                const bool middle = i >= 4 && i < 4 * (nk + 6);
                st->rk[i] = rk[i];
                st->rkr[i] = middle ? __builtin_amdgcn_alignbit(rk[i], rk[i], 16) : rk[i];
            }
            uint8_t h[16] = { 0 };
            aes_encrypt_bytes(sb, rk, nk + 6, h);
            G128 H;
            H.hi = 0; H.lo = 0;
            for (int i = 0; i < 8; i++) { H.hi = (H.hi << 8) | h[i]; H.lo = (H.lo << 8) | h[8 + i]; }
            for (int i = 0; i < 16; i++) st->h[i] = h[i];
            pw[0] = H;
            for (int p = 1; p < KEY_TABLES; p++) pw[p] = g_mul(pw[p - 1], pw[p - 1]);
        } else if (aria) {
            uint8_t (*ek)[16] = reinterpret_cast<uint8_t (*)[16]>(ksched);
            const int nr = aria_key_expand(sb, km.key, (int) tlsrec_cipher_keylen(km.cipher), ek);
            for (int e = 0; e < 17; e++)
                for (int c = 0; c < 4; c++)
                    st->ark[4 * e + c] = e <= nr ? ((uint32_t) ek[e][4 * c] | ((uint32_t) ek[e][4 * c + 1] << 8) |
                                                    ((uint32_t) ek[e][4 * c + 2] << 16) | ((uint32_t) ek[e][4 * c + 3] << 24))
                                                 : 0u;
            uint8_t h[16] = { 0 };
            aria_encrypt_bytes(sb, ek, nr, h);
            G128 H;
            H.hi = 0; H.lo = 0;
            for (int i = 0; i < 8; i++) { H.hi = (H.hi << 8) | h[i]; H.lo = (H.lo << 8) | h[8 + i]; }
            for (int i = 0; i < 16; i++) st->h[i] = h[i];
            pw[0] = H;
            for (int p = 1; p < KEY_TABLES; p++) pw[p] = g_mul(pw[p - 1], pw[p - 1]);
        } else if (cam) {
            /* Camellia: the subkeys as (high, low) word pairs (tlsrec_device.h cam_encrypt) */
            uint64_t *sk = ksched;
            const int nr = cam_key_expand(sb, km.key, (int) tlsrec_cipher_keylen(km.cipher), sk);
            for (int i = 0; i < 34; i++) {
                st->ark[2 * i] = (uint32_t) (sk[i] >> 32);
                st->ark[2 * i + 1] = (uint32_t) sk[i];
            }
            G128 H;
            H.hi = 0; H.lo = 0;
            cam_encrypt_u64(sb, sk, nr, H.hi, H.lo);
            for (int i = 0; i < 8; i++) { st->h[i] = (uint8_t) (H.hi >> (56 - 8 * i)); st->h[8 + i] = (uint8_t) (H.lo >> (56 - 8 * i)); }
            pw[0] = H;
            for (int p = 1; p < KEY_TABLES; p++) pw[p] = g_mul(pw[p - 1], pw[p - 1]);
        }
    }
    __syncthreads();
    if (!gcm) return;
    if (tid < 4) {                      /* H^2, H^4, H^8, H^16 for the table-free lane tree */
        const uint4 w = g_to_words(pw[tid + 1]);
        st->hpow[tid][0] = w.x; st->hpow[tid][1] = w.y; st->hpow[tid][2] = w.z; st->hpow[tid][3] = w.w;
    }
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
    /* H^1 .. H^64 as values, by a ladder: level k makes H^(2^k + j) =
     * H^(2^k) * H^j for j = 1 .. 2^k - 1 (57 products over five levels, one
     * each, four lanes per product -- g_mul_base_q).  Per lane t + 1 as a
     * product of the powers H^(2^b) of its set bits, the up-to-five chained
     * 128-term multiplies of the busiest lanes held the whole wave: the slot
     * setup took 4.6 instead of 3.8 ms per 64 K keys. */
    if (tid < KEY_TABLES) hp[(1 << tid) - 1] = pw[tid];       /* H^1, H^2, H^4, .., H^64 */
    __syncthreads();
    for (int k = 1; k < KEY_TABLES - 1; k++) {
        const int m = (1 << k) - 1;
        if (tid < 4 * m) {
            const int j = (tid >> 2) + 1;
            const G128 x = g_mul_base_q(base[k], hp[j - 1], tid & 3);
            if ((tid & 3) == 0) hp[(1 << k) + j - 1] = x;
        }
        __syncthreads();
    }
    if (tid < KEY_HPOW_N) out[KEY_HPOW_OFF + tid] = g_to_words(hp[tid]);
    for (int e = tid; e < KEY_TABLES * 32 * 16; e += 256) {
        const int p = e >> 9, k = (e >> 4) & 31, nib = e & 15;
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (int i = 0; i < 4; i++)
            if ((nib >> (3 - i)) & 1) acc = xor4(acc, base[p][4 * k + i]);
        out[e] = acc;
    }
    /* H^8 again as G5 tables (tlsrec_device.h gmul5): window k, entry n =
     * sum of P x^j over the set bits of n, j = the GCM bit index of the word
     * bit the index bit comes from; lo halves then hi halves */
    uint2 *g5 = reinterpret_cast<uint2 *>(out + KEY_G5_OFF);
    for (int e = tid; e < KEY_G5_WORDS; e += 256) {
        const int k = e >> 5, n = e & 31;
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (int i = 0; i < g5_bits(k); i++)
            if ((n >> i) & 1) {
                const int t = g5_bit(k, i);
                const int j = 8 * (4 * g5_word(k, i) + t / 8) + (7 - t % 8);
                acc = xor4(acc, base[KEY_G5_POWER][j]);
            }
        g5[k * 32 + n] = make_uint2(acc.x, acc.y);                 /* lo halves at k * 256 B */
        g5[G5_HI / 8 + k * 32 + n] = make_uint2(acc.z, acc.w);    /* hi halves at G5_HI + k * 256 B */
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
/* (r06: the per-slot counters transposed 32 x 32 within aligned 1 024-slot
 * blocks, so that a wave's 32 consecutive slots fall on 32 lines, measured
 * neutral on c4s -- 881 / 881 GiB/s same box, profiles/r06/ab -- and left) */
__device__ __forceinline__ uint32_t bucket_key(const BucketArgs &a, const tlsrec_batch_rec &d, uint32_t i)
{
    if (d.slot >= a.capacity) return 0xffffffffu;
    const int c = a.cipher_of[d.slot];
    constexpr uint32_t S = CP_SPREAD;
    const uint32_t slot = d.slot;
    switch (c) {
        case TLSREC_CIPHER_AES_128_GCM: return slot;
        case TLSREC_CIPHER_AES_256_GCM: return a.capacity + slot;
        case TLSREC_CIPHER_AES_192_GCM: return 2 * a.capacity + slot;
        case TLSREC_CIPHER_CHACHA20_POLY1305:   /* the wave's counter, one per line */
            return 4 * a.capacity + ((i >> 6) & (CP_COUNTERS - 1)) * CP_STRIDE;
        /* ARIA-GCM classes after the ChaCha counters: 4 cap + S + (0..2) cap + slot */
        case TLSREC_CIPHER_ARIA_128_GCM: return 4 * a.capacity + S + slot;
        case TLSREC_CIPHER_ARIA_192_GCM: return 5 * a.capacity + S + slot;
        case TLSREC_CIPHER_ARIA_256_GCM: return 6 * a.capacity + S + slot;
        /* Camellia-GCM classes after ARIA's: (7, 8, 9) cap + S + slot */
        case TLSREC_CIPHER_CAMELLIA_128_GCM: return 7 * a.capacity + S + slot;
        case TLSREC_CIPHER_CAMELLIA_192_GCM: return 8 * a.capacity + S + slot;
        case TLSREC_CIPHER_CAMELLIA_256_GCM: return 9 * a.capacity + S + slot;
        default:
            return (tlsrec_cipher_is_ccm(c) || tlsrec_cipher_is_alt_ccm(c)) ? 3 * a.capacity + slot : 0xffffffffu;
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
    const bool cp = key >= 4 * a.capacity && key < 4 * a.capacity + CP_SPREAD;
    const uint32_t pc = claim_group(ctr, key, cp);
    const uint32_t pg = claim_group(ctr, key, key != 0xffffffffu && !cp);
    return cp ? pc : pg;
}

/* counts to zero: a kernel on the batch's stream rather than
 * hipMemsetAsync / a device-to-device copy, so the whole bucket pass is
 * kernels in stream order on any HIP runtime (a C host on the system HIP
 * 7.2 runtime saw a scatter read cursors that an offsets copy had not yet
 * written, leaving stale perm entries) */
__global__ __launch_bounds__(256) void tlsrec_bucket_zero_kernel(BucketArgs a)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < a.nk) a.counts[i] = 0;
}

/* Fail closed, as the reference's `auth_done != 1 -> INTERNAL_ERROR` check
 * (ssl_msg.c:1260 encrypt, :1804 decrypt): before any AEAD kernel of a batch
 * runs, every record's result reads INTERNAL_ERROR, and only the kernel that
 * protects (or rejects) the record overwrites it.  A record no kernel reaches
 * can never read as success, whatever the caller left in `res`.  The bucket
 * count kernel writes the same sentinel for the records it groups; this one
 * covers identity order. */
__device__ __forceinline__ void unreached_result(tlsrec_batch_res *res)
{
    tlsrec_batch_res r;
    r.status = TLSREC_ERR_SSL_INTERNAL_ERROR;
    r.data_offset = 0;
    r.data_len = 0;
    r.type = 0;
    r.cid_len = 0;
    r.reserved[0] = r.reserved[1] = 0;
    *res = r;
}

__global__ __launch_bounds__(256) void tlsrec_res_guard_kernel(tlsrec_batch_res *res, uint32_t n)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) unreached_result(&res[i]);
}

__global__ __launch_bounds__(256) void tlsrec_bucket_count_kernel(BucketArgs a)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t key = 0xffffffffu;
    if (i < a.n) {
        const tlsrec_batch_rec d = a.recs[i];
        key = bucket_key(a, d, i);
        if (key == 0xffffffffu)
            bad_slot_result(d, &a.res[i]);
        else
            unreached_result(&a.res[i]);    /* the record's AEAD kernel overwrites it */
    }
    /* the count's old value is the record's rank within its key: the
     * scatter then needs no second round of atomics (with keys round-robin,
     * one per record: half the bucket pass, 14 % of a c4s step) */
    const uint32_t rank = bucket_claim(a, a.counts, key);
    if (i < a.n) a.keyrank[i] = make_uint2(key, rank);
}

__global__ __launch_bounds__(256) void tlsrec_bucket_scatter_kernel(BucketArgs a)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const uint2 kr = a.keyrank[i];
    if (kr.x != 0xffffffffu) {
        const uint32_t p = a.offs[kr.x] + kr.y;
        a.perm[p] = i;
        /* the GCM classes' descriptors in perm order (not CCM, 3 cap.., or
         * ChaCha, 4 cap..4 cap + CP_SPREAD: their kernels read recs[]) */
        if (a.srecs && (kr.x < 3 * a.capacity || kr.x >= 4 * a.capacity + CP_SPREAD)) a.srecs[p] = a.recs[i];
    }
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
    uint32_t s[4];                          /* Poly1305 s */
    uint32_t r1[5];                         /* r (26-bit limbs) */
    uint32_t rl[4][5];                      /* r^L, r^2L, r^3L, r^4L */
};
static_assert(sizeof(CpRec) == 164, "CpRec layout");
static_assert(sizeof(tlsrec_batch_rec) == 40 && sizeof(tlsrec_key_material) == 64, "descriptor words");

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

/* carry-propagate a D5 of up to four limb products plus a block (< 2^61 per
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

/* Keystream exchange slot of (chunk lane c, 16-B group g) in a wave's 4 KiB
 * LDS row: the group rotates with c >> 1 so that the eight lanes of a
 * ds_write_b128 lane group hit 32 distinct banks. */
__device__ __forceinline__ uint32_t ks_slot(uint32_t c, uint32_t g)
{
    return 4u * c + ((g + (c >> 1)) & 3u);
}

/* the half-size exchange row (two slots per lane): lanes c .. c+7 of a
 * ds_write_b128 group land on 8 distinct 16-byte bank quads */
__device__ __forceinline__ uint32_t ks_half(uint32_t c, uint32_t g)
{
    return 2u * c + ((g + (c >> 2)) & 1u);
}

/*
 * ChaCha20-Poly1305 record kernel (RFC 8439 2.8 around the framing plan).
 *
 * Slot layout.  L lanes serve one record; a step covers L ChaCha20 blocks =
 * 4L 16-byte slots of the record, and in load / store t (0..3) lane q touches
 * slot L*t + q -- the record's L lanes move L*16 contiguous bytes per
 * instruction, whole 128-B lines at L = 8 and 32-B runs at L = 2, instead of
 * each lane walking its own 64-byte block (which held the kernel to ~4 TB/s of
 * HBM).  Lane q still computes ChaCha20 block L*j - z + q of the record (z =
 * front padding in blocks, so that every record ends in its last step); the
 * 64-byte keystream goes through the wave's LDS row (4 x ds_write_b128,
 * 4 x ds_read_b128) to the lanes that hold its slots.
 *
 * Poly1305.  Lane q owns the slots = q (mod L), in order, as a Horner chain
 * with multiplier r^L: per step acc*r^(4L) + X_0 r^(3L) + X_1 r^(2L) + X_2 r^L
 * + X_3, front-padding slots X = 0, slots past the record's last block
 * skipped.  A lane's chain then ends at one of the record's last L blocks, d
 * blocks before the end, and the record's sum is  sum_q acc_q r^(d_q)  (a
 * shuffle-add over the L lanes), then the length block and s.
 */
/* 3 waves per SIMD (the L = 2 kernels; L >= 4 and CID are held to 2 by their
 * LDS): the per-record first-column-round words take the VGPRs to 172-176,
 * and at 2 waves the c3 shape lost what the 3 saved quarter rounds gain;
 * capped at 168 the compiler spills 6-12 registers outside the step loop
 * (same box: c3 1 224 -> 1 220, c3d 1 195 -> 1 204, 16 KiB 1 637 -> 1 677 GiB/s) */
/* SRC (r05, encrypt): the contents at a.in + a.src_off[i] (the stream / DTLS
 * send path, tlsrec__batch_src), partial blocks read byte-wise; a template
 * flag, not a run-time test: as one, it cost c3 1.5 % (same box) */
template <int L, bool DEC, bool CID = false, bool SRC = false>
__global__ __launch_bounds__(CP_THREADS) __attribute__((amdgpu_waves_per_eu(3))) void tlsrec_chachapoly_kernel(CpArgs a)
{
    constexpr int R = 64 / L;
    constexpr int LOGL = Log2<L>::v;
    __shared__ CpRec crec[CP_WAVES][64];
    /* keystream exchange: 4 KiB per wave, or (L <= 2) 2 KiB in two phases --
     * a lane's reads then need only half its block's slots at a time, and the
     * workgroup's 50 KiB of LDS let three workgroups (12 waves, the VGPR bound)
     * share a CU instead of two */
    constexpr bool SPLIT = L <= 2;
    __shared__ uint4 kst[CP_WAVES][SPLIT ? 128 : 256];
    __shared__ uint32_t cidf[CP_WAVES][CID ? 64 : 1][5];   /* CID: AAD blocks Horner-folded */
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g = lane / L, q = lane % L;
    const uint32_t lo = a.perm ? *a.lo : 0u;
    const uint32_t count = a.perm ? *a.hi - lo : (uint32_t) a.n;
    const uint64_t chunk = ((uint64_t) blockIdx.x * CP_WAVES + wave) * a.rpw;

    /* ---- pre-pass: per chunk position, the record's key/nonce, the one-time
     * Poly1305 key (ChaCha20 block 0, RFC 8439 2.6) and powers of r ---- */
    bool mine = false;
    uint32_t my_rec = 0;
    /* the chunk position's descriptor and key material, kept for the record
     * rounds (shuffled to the record's lanes: no second trip to memory) */
    uint32_t dm[10] = { 0 }, kmm[8] = { 0 };
    {
        const uint64_t pos = chunk + (uint64_t) lane;
        CpRec &cr = crec[wave][lane];
        uint32_t key[8] = { 0 }, nw[3] = { 0, 0, 0 };
        if (lane < (int) a.rpw && pos < count) {
            my_rec = a.perm ? a.perm[lo + pos] : (uint32_t) pos;
            const tlsrec_batch_rec d = a.recs[my_rec];
            const bool reach = !TLSREC_HOOK_SKIP(my_rec, a.skip);   /* test hook: the guard's INTERNAL_ERROR stays */
            if (reach && !a.perm && !(d.slot < a.capacity && a.slots[d.slot].km.cipher != 0))
                bad_slot_result(d, &a.res[my_rec]);
            if (reach && d.slot < a.capacity && a.slots[d.slot].km.cipher == TLSREC_CIPHER_CHACHA20_POLY1305) {
                mine = true;
                const tlsrec_key_material km = a.slots[d.slot].km;
                __builtin_memcpy(dm, &d, sizeof(dm));
                __builtin_memcpy(kmm, &km, sizeof(kmm));    /* all but the key: the plan's inputs */
                tlsrec_plan p;
                make_plan<DEC, CID>(p, d, km, &a.slots[d.slot], a.in);
                nonce_words<DEC>(p, d, km, a.in, nw);
                for (int i = 0; i < 8; i++) key[i] = ld_u32le(km.key + 4 * i);
            }
        }
        uint32_t blk[16];
        chacha_block(key, 0, nw, blk);
        for (int i = 0; i < 8; i++) cr.key[i] = key[i];
        for (int i = 0; i < 3; i++) cr.nonce[i] = nw[i];
        for (int i = 0; i < 4; i++) cr.s[i] = blk[4 + i];
        const P5 r1 = p_from_r(blk[0], blk[1], blk[2], blk[3]);
        P5 rL = r1;
        for (int i = 0; i < LOGL; i++) rL = p_mul(rL, rL);     /* r^L */
        const P5 r2L = p_mul(rL, rL);
        const P5 r3L = p_mul(r2L, rL);
        const P5 r4L = p_mul(r2L, r2L);
        for (int i = 0; i < 5; i++) {
            cr.r1[i] = r1.v[i];
            cr.rl[0][i] = rL.v[i];
            cr.rl[1][i] = r2L.v[i];
            cr.rl[2][i] = r3L.v[i];
            cr.rl[3][i] = r4L.v[i];
        }
    }
    /* lanes read other lanes' CpRec: the wave's own LDS writes land first */

    /* this lane's keystream exchange slots: writes (own block, group t) and
     * reads (slot L*t + q of its record) */
    uint4 *const krow = kst[wave];
    uint32_t kw[4], kr[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const uint32_t u = (uint32_t) (L * t + q);
        if constexpr (SPLIT) {
            /* slot t of a lane's block goes out in phase t >> 1; the slot a
             * lane reads for t, u % 4 of lane (lane - q + u / 4), comes in
             * phase (u % 4) >> 1: t even / odd at L = 2, t < 2 / >= 2 at L = 1 */
            kw[t] = ks_half((uint32_t) lane, (uint32_t) t & 1u);
            kr[t] = ks_half((uint32_t) (lane - q) + u / 4, (u % 4) & 1u);
        } else {
            kw[t] = ks_slot((uint32_t) lane, (uint32_t) t);
            kr[t] = ks_slot((uint32_t) (lane - q) + u / 4, u % 4);
        }
    }

    for (uint32_t rr = 0; rr < a.rpw; rr += R) {
        const uint32_t slot_in_chunk = rr + (uint32_t) g;
        const bool owner_mine = __shfl((int) mine, (int) slot_in_chunk & 63) != 0;
        const bool active = slot_in_chunk < a.rpw && owner_mine;
        const uint64_t ridx = (uint32_t) __shfl((int) my_rec, (int) slot_in_chunk & 63);
        const CpRec &cr = crec[wave][slot_in_chunk & 63];
        const uint32_t *aadf = cidf[wave][CID ? (slot_in_chunk & 63) : 0];
        tlsrec_batch_rec d;
        tlsrec_plan p;
        bool run = false;
        {
            uint32_t w[10], k[16] = { 0 };
#pragma unroll
            for (int i = 0; i < 10; i++) w[i] = (uint32_t) __shfl((int) dm[i], (int) slot_in_chunk & 63);
#pragma unroll
            for (int i = 0; i < 8; i++) k[i] = (uint32_t) __shfl((int) kmm[i], (int) slot_in_chunk & 63);
            __builtin_memcpy(&d, w, sizeof(w));
            if (active) {
                tlsrec_key_material km;
                __builtin_memcpy(&km, k, sizeof(km));
                make_plan<DEC, CID>(p, d, km, &a.slots[d.slot], a.in);
                if (p.status != 0) {
                    if (q == 0) finish_early(p, d, a.out, &a.res[ridx]);
                } else {
                    run = true;
                }
            }
        }
        /* the record's key stream: first column round, once per record (chacha_cc_make) */
        uint32_t kcc[CHACHA_CC_WORDS];
        {
            uint32_t key[8], nw[3];
#pragma unroll
            for (int i = 0; i < 8; i++) key[i] = cr.key[i];
#pragma unroll
            for (int i = 0; i < 3; i++) nw[i] = cr.nonce[i];
            chacha_cc_make(key, nw, kcc);
        }
        const uint32_t aead_len = run ? p.aead_len : 0;
        const uint32_t B = (aead_len + 63) >> 6;              /* ChaCha20 blocks (64 B) */
        const uint32_t M = (aead_len + 15) >> 4;              /* Poly1305 C blocks (16 B) */
        const uint32_t z = (L - B % L) % L;                   /* front padding, in 64-B blocks */
        const uint32_t J = run ? (B + z) / L : 0;
        const uint32_t Jmax = wave_max(J);
        uint4 aadw = make_uint4(0, 0, 0, 0);
        bool cidaad = false;  /* AAD of 2..4 blocks, folded into aadf */
        const uint8_t *src = a.in;
        uint8_t *dst = a.out;
        uint32_t content_len = 0;
        if (run) {
            aadw = aad_words(p);
            cidaad = CID && p.aad_len > 16;
            if (cidaad && q == 0) {   /* DTLS 1.2 + CID: one lane folds, all read */
                const P5 f = cp_cid_aad_fold(p_from_words(aadw), cr.r1, p, d, a.slots[d.slot].cid);
                uint32_t *w = const_cast<uint32_t *>(aadf);
#pragma unroll
                for (int i = 0; i < 5; i++) w[i] = f.v[i];
            }
            src = a.in + d.buf_off + p.aead_pos;
            dst = a.out + d.buf_off + p.aead_pos;
            content_len = DEC ? aead_len : p.content_len;
            if constexpr (SRC) src = a.in + a.src_off[ridx];   /* the content in the caller's buffer */
        }
        /* partial blocks 16 B wide (in place), or byte-wise from a caller's buffer */
        constexpr bool wide = !SRC;
        const uint8_t inner_type = run ? p.inner_type : 0;
        const bool tls13 = run && p.inner;   /* TLS 1.3 or DTLS 1.2 + CID inner plaintext */
        /* a readable 16-byte address for slots with nothing to load, in a
         * line the step's other lanes read anyway: the record start for the
         * front padding of step 0, its last content bytes for the tail (the
         * start would be a second HBM trip by then) */
        const uint8_t *safe0 = run ? (wide ? src : dst) : reinterpret_cast<const uint8_t *>(a.recs);
        const uint8_t *safe = run && wide ? src + (content_len >= 16 ? (content_len - 16) & ~15u : 0u) : safe0;
        /* slot (L*t + q) of step j is record block 4(L j - z) + L t + q */
        const int32_t base0 = (int32_t) q - 4 * (int32_t) z;

        P5 acc = p_zero();
        uint32_t nzpos = 0;                 /* TLS 1.3: 1 + position of the last non-zero 16-B block */
        /* decrypt: the received tag (after the AEAD data in the record
         * buffer), loaded now and compared after the loop */
        const uint4 want = (DEC && run) ? gload16(src + aead_len) : make_uint4(0, 0, 0, 0);

        /* this lane's keystream block of step j, exchanged: K[t] = the
         * keystream of slot L*t + q */
        auto keystream = [&](uint32_t j, uint4 (&K)[4]) {
            uint32_t ks[16];
            chacha_block_cc<const uint32_t *>(cr.key, cr.nonce, kcc, L * j - z + (uint32_t) q + 1u, ks);
            asm volatile("" ::: "memory");   /* after the previous step's reads */
            if constexpr (SPLIT) {
#pragma unroll
                for (int ph = 0; ph < 2; ph++) {
#pragma unroll
                    for (int t = 2 * ph; t < 2 * ph + 2; t++)
                        krow[kw[t]] = make_uint4(ks[4 * t], ks[4 * t + 1], ks[4 * t + 2], ks[4 * t + 3]);
                    asm volatile("" ::: "memory");
#pragma unroll
                    for (int t = 0; t < 4; t++)
                        if ((L == 1 ? t >> 1 : t & 1) == ph) K[t] = krow[kr[t]];   /* ((L t + q) % 4) >> 1 */
                    asm volatile("" ::: "memory");   /* phase 1 writes after phase 0 reads (in-order queue) */
                }
            } else {
#pragma unroll
                for (int t = 0; t < 4; t++)
                    krow[kw[t]] = make_uint4(ks[4 * t], ks[4 * t + 1], ks[4 * t + 2], ks[4 * t + 3]);
                /* other lanes' writes: same wave, in-order LDS queue */
                asm volatile("" ::: "memory");
#pragma unroll
                for (int t = 0; t < 4; t++) K[t] = krow[kr[t]];
            }
        };

        /* general step: any step (front padding, the AAD fold at block 0,
         * partial or ragged blocks, the record's end) */
        auto general = [&](uint32_t j) {
            const bool live = run && j < J;
            uint4 ct[4];
            bool fast[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int32_t i = (int32_t) (4 * L * j) + base0 + L * t;
                const uint32_t pos = (uint32_t) i * 16;
                fast[t] = live && i >= 0 && pos + 16 <= content_len;
                ct[t] = gload16(fast[t] ? src + pos : (j == 0 ? safe0 : safe));
            }
            uint4 K[4];
            keystream(j, K);
            const P5 r1 = p_lds(cr.r1), rL = p_lds(cr.rl[0]);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int32_t i = (int32_t) (4 * L * j) + base0 + L * t;
                const uint32_t pos = (uint32_t) i * 16;
                const bool valid = live && i >= 0 && (uint32_t) i < M;
                P5 x = p_zero();
                if (fast[t]) {
                    const uint4 o = xor4(ct[t], K[t]);
                    gstore16(dst + pos, o);
                    if (DEC && tls13 && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                    x = p_from_words(DEC ? ct[t] : o);
                } else if (valid) {
                    const uint4 blk = load_block(src, pos, content_len, aead_len, inner_type, wide);
                    const uint4 o = mask_block(xor4(blk, K[t]), pos, aead_len);
                    store_block(dst, pos, aead_len, o, true);
                    if (DEC && tls13 && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                    x = p_from_words(DEC ? blk : o);
                }
                /* the AAD block(s) enter as A*r folded into C_0 */
                if (valid && i == 0) x = p_add(x, p_mul(cidaad ? p_lds(aadf) : p_from_words(aadw), r1));
                /* Horner link of this lane's chain: slots past the record's
                 * last block leave it where it ended */
                const P5 y = p_add(p_mul(acc, rL), x);
                if (live && i < (int32_t) M) acc = y;
            }
        };

        /* Body steps [1, jh): every slot of every lane of the wave is a full
         * 16-byte block inside its record's content (wave-uniform bound): no
         * masks, Poly1305 as acc*r^(4L) + X_0 r^(3L) + X_1 r^(2L) + X_2 r^L + X_3
         * with one carry propagation per step. */
        uint32_t jh = 0;
        {
            const uint32_t cfull = run ? content_len / 64 : 0;      /* full 64-B blocks of content */
            const uint32_t h = wave_min(run ? (cfull + z) / L : 0);
            jh = h > 1 ? h : 0;
        }
        auto body = [&](uint32_t j, bool fold) {
            const uint32_t pos0 = (uint32_t) ((int32_t) (4 * L * j) + base0) * 16;
            uint4 c[4];
#pragma unroll
            for (int t = 0; t < 4; t++) c[t] = gload16(src + pos0 + 16 * L * t);
            uint4 K[4];
            keystream(j, K);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint32_t pos = pos0 + 16 * L * t;
                const uint4 o = xor4(c[t], K[t]);
                gstore16(dst + pos, o);
                if (DEC && tls13 && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                if (!DEC) c[t] = o;
            }
            D5 dd;
            const P5 x3 = p_from_words(c[3]);
#pragma unroll
            for (int i = 0; i < 5; i++) dd.v[i] = x3.v[i];
            P5 x0 = p_from_words(c[0]);
            /* step 0 without front padding: slot 0 (lane q = 0, t = 0) is C_0,
             * which takes the AAD as A*r (limbs stay < 2^27: the D5 sum holds) */
            if (fold && q == 0) x0 = p_add(x0, p_mul(p_from_words(aadw), p_lds(cr.r1)));
            p_mac(dd, acc, p_lds(cr.rl[3]));
            p_mac(dd, x0, p_lds(cr.rl[2]));
            p_mac(dd, p_from_words(c[1]), p_lds(cr.rl[1]));
            p_mac(dd, p_from_words(c[2]), p_lds(cr.rl[0]));
            acc = p_reduce(dd);
        };
        /* step 0 takes the body when no record of the wave has front padding
         * (whole steps, e.g. 1 408-B TLS 1.3 records at L = 2) and the AAD is
         * one block; otherwise the general step */
        const bool body0 = jh != 0 && !CID && wave_max(z) == 0;
        const uint32_t jl = jh ? 1u : Jmax;
        uint32_t j = 0;
        if (body0) {
            body(0, true);
            j = 1;
        }
        for (; j < jl; j++) general(j);
        for (; j < jh; j++) body(j, false);
        for (; j < Jmax; j++) general(j);

        /* sum_q acc_q r^(d_q), d_q = blocks from the end of lane q's chain to
         * the record's last block (K = slot of that block) */
        const P5 r1 = p_lds(cr.r1);
        {
            const uint32_t K = 4 * z + M - 1;                     /* M >= 1 where it matters */
            const uint32_t dq = (K - (uint32_t) q) % L;
            P5 rp = r1;
#pragma unroll
            for (int i = 0; i < LOGL; i++) {
                acc = p_sel((dq >> i) & 1, p_mul(acc, rp), acc);
                if (i + 1 < LOGL) rp = p_mul(rp, rp);
            }
            /* the L lanes' sum by DPP butterfly steps (VALU, not the LDS pipe) */
            auto step = [&](auto sc) {
                constexpr int S = decltype(sc)::value;
                if constexpr (S < L) {
                    P5 w;
#pragma unroll
                    for (int i = 0; i < 5; i++) w.v[i] = partner<S>(acc.v[i], lane);
                    acc = p_add(acc, w);
                }
            };
            step(std::integral_constant<int, 1>());
            step(std::integral_constant<int, 2>());
            step(std::integral_constant<int, 4>());
        }
        /* H1 = A r^M + sum_i C_i r^(M-1-i); tag = (H1 r + LEN) r + s */
        P5 X = M ? p_carry(acc) : (cidaad ? p_lds(aadf) : p_from_words(aadw));
        X = p_mul(X, r1);
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
            uint32_t diff = (want.x ^ tag.x) | (want.y ^ tag.y) | (want.z ^ tag.z) | (want.w ^ tag.w);
            diff = group_or<L>(lane == leader ? diff : 0u);       /* the leader's verdict, to all */
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
    } else if (!DEC && a.src_off) {   /* stream / DTLS send (tlsrec__batch_src) */
        hipLaunchKernelGGL((tlsrec_chachapoly_kernel<L, false, false, true>), dim3(grid), dim3(CP_THREADS), 0, st, a);
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

extern "C" hipError_t tlsrec__launch_keysetup(SlotState *slots, uint4 *ghtab, uint8_t *cipher_of,
                                              const tlsrec_key_material *keys, uint32_t first, uint32_t count,
                                              hipStream_t st)
{
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(tlsrec_keysetup_kernel, dim3(count), dim3(256), 0, st, slots, ghtab, cipher_of, keys, first,
                       count);
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

extern "C" hipError_t tlsrec__launch_bucket_zero(const BucketArgs *a, hipStream_t st)
{
    hipLaunchKernelGGL(tlsrec_bucket_zero_kernel, dim3((a->nk + 255) / 256), dim3(256), 0, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t tlsrec__launch_bucket_count(const BucketArgs *a, hipStream_t st)
{
    if (a->n == 0) return hipSuccess;
    hipLaunchKernelGGL(tlsrec_bucket_count_kernel, dim3((a->n + 255) / 256), dim3(256), 0, st, *a);
    return hipGetLastError();
}

/* ======================================================================
 * Exclusive scan of uint32 counts (the bucket pass's per-key offsets, the
 * stream / DTLS layers' per-connection record offsets): reduce-then-scan in
 * two launches.  Block b owns SCAN_CHUNK consecutive counts; the reduce
 * kernel writes each block's sum, the apply kernel re-sums the sums of the
 * blocks before it (at most a few hundred: 64 K keys x 10 classes is 161
 * blocks) and scans its chunk.  No library call, no host sync; scratch =
 * one word per block.
 * ==================================================================== */
constexpr uint32_t SCAN_THREADS = 256, SCAN_PER_THREAD = 16, SCAN_CHUNK = SCAN_THREADS * SCAN_PER_THREAD;

/* exclusive scan over the block's 256 thread values (LDS, Hillis-Steele) */
__device__ __forceinline__ uint32_t block_exclusive(uint32_t v, uint32_t *sh)
{
    const uint32_t t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
#pragma unroll
    for (uint32_t o = 1; o < SCAN_THREADS; o <<= 1) {
        const uint32_t add = t >= o ? sh[t - o] : 0u;
        __syncthreads();
        sh[t] += add;
        __syncthreads();
    }
    const uint32_t incl = sh[t];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(SCAN_THREADS) void tlsrec_scan_reduce_kernel(const uint32_t *in, uint32_t n,
                                                                        uint32_t *bsum)
{
    __shared__ uint32_t sh[SCAN_THREADS];
    const uint64_t base = (uint64_t) blockIdx.x * SCAN_CHUNK;
    uint32_t v = 0;
    for (uint32_t k = threadIdx.x; k < SCAN_CHUNK; k += SCAN_THREADS)
        if (base + k < n) v += in[base + k];
    const uint32_t ex = block_exclusive(v, sh);
    if (threadIdx.x == SCAN_THREADS - 1) bsum[blockIdx.x] = ex + v;
}

__global__ __launch_bounds__(SCAN_THREADS) void tlsrec_scan_apply_kernel(const uint32_t *in, uint32_t n,
                                                                       const uint32_t *bsum, uint32_t *out)
{
    __shared__ uint32_t sh[SCAN_THREADS];
    /* the sums of the blocks before this one */
    uint32_t pre = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += SCAN_THREADS) pre += bsum[b];
    const uint32_t prex = block_exclusive(pre, sh);
    if (threadIdx.x == SCAN_THREADS - 1) sh[0] = prex + pre;    /* after block_exclusive's last barrier */
    __syncthreads();
    const uint32_t block_base = sh[0];
    __syncthreads();
    /* thread t scans its SCAN_PER_THREAD consecutive counts */
    const uint64_t first = (uint64_t) blockIdx.x * SCAN_CHUNK + (uint64_t) threadIdx.x * SCAN_PER_THREAD;
    uint32_t v[SCAN_PER_THREAD], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER_THREAD; k++) {
        v[k] = first + k < n ? in[first + k] : 0u;
        sum += v[k];
    }
    uint32_t run = block_base + block_exclusive(sum, sh);
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER_THREAD; k++) {
        if (first + k < n) out[first + k] = run;
        run += v[k];
    }
}

#ifdef TLSREC_TEST_HOOKS
/* Self-test of the cross-lane helpers (tlsrec_recdev.h) for
 * tests/test_lane_ops_gpu.py: one wave, lane i holds v_i = (i * 37 + 11) & 63
 * plus 100 * i; rows of 64 words:
 *   0-5 partner<1, 2, 4, 8, 16, 32>, 6-11 from_up<1, 2, 4, 8, 16, 32>,
 *   12 wave_max, 13 wave_min, 14 group_max<8>, 15 group_or<4> of 1 << (i % 32),
 *   16 group sum<8> by the Poly1305 butterfly steps */
__global__ __launch_bounds__(64) void tlsrec_lane_ops_kernel(uint32_t *out)
{
    const int lane = threadIdx.x;
    const uint32_t v = (uint32_t) ((lane * 37 + 11) & 63) + 100u * (uint32_t) lane;
    out[0 * 64 + lane] = partner<1>(v, lane);
    out[1 * 64 + lane] = partner<2>(v, lane);
    out[2 * 64 + lane] = partner<4>(v, lane);
    out[3 * 64 + lane] = partner<8>(v, lane);
    out[4 * 64 + lane] = partner<16>(v, lane);
    out[5 * 64 + lane] = partner<32>(v, lane);
    out[6 * 64 + lane] = from_up<1>(v, lane);
    out[7 * 64 + lane] = from_up<2>(v, lane);
    out[8 * 64 + lane] = from_up<4>(v, lane);
    out[9 * 64 + lane] = from_up<8>(v, lane);
    out[10 * 64 + lane] = from_up<16>(v, lane);
    out[11 * 64 + lane] = from_up<32>(v, lane);
    out[12 * 64 + lane] = wave_max(v);
    out[13 * 64 + lane] = wave_min(v);
    out[14 * 64 + lane] = group_max<8>(v);
    out[15 * 64 + lane] = group_or<4>(1u << (lane & 31));
    uint32_t sum = v;
    sum += partner<1>(sum, lane);
    sum += partner<2>(sum, lane);
    sum += partner<4>(sum, lane);
    out[16 * 64 + lane] = sum;
}

extern "C" int tlsrec__test_lane_ops(uint32_t *host_out /* 17 x 64 words */)
{
    uint32_t *d = nullptr;
    if (hipMalloc((void **) &d, 17 * 64 * 4) != hipSuccess) return -1;
    hipLaunchKernelGGL(tlsrec_lane_ops_kernel, dim3(1), dim3(64), 0, 0, d);
    const hipError_t e = hipMemcpy(host_out, d, 17 * 64 * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    return e == hipSuccess ? 0 : -1;
}
#endif /* TLSREC_TEST_HOOKS */

extern "C" size_t tlsrec__scan_scratch_bytes(uint32_t n)
{
    return ((size_t) n + SCAN_CHUNK - 1) / SCAN_CHUNK * 4 + 4;
}

extern "C" hipError_t tlsrec__exclusive_scan(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t *scratch,
                                             hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const uint32_t nb = (n + SCAN_CHUNK - 1) / SCAN_CHUNK;
    hipLaunchKernelGGL(tlsrec_scan_reduce_kernel, dim3(nb), dim3(SCAN_THREADS), 0, st, in, n, scratch);
    hipLaunchKernelGGL(tlsrec_scan_apply_kernel, dim3(nb), dim3(SCAN_THREADS), 0, st, in, n, scratch, out);
    return hipGetLastError();
}

#ifdef TLSREC_TEST_HOOKS
/* tests/test_scan_gpu.py: the scan over host arrays (copies in, scans, copies out) */
extern "C" int tlsrec__test_scan(const uint32_t *host_in, uint32_t n, uint32_t *host_out)
{
    uint32_t *d = nullptr;
    const size_t sb = tlsrec__scan_scratch_bytes(n);
    if (hipMalloc((void **) &d, (size_t) n * 8 + sb + 16) != hipSuccess) return -1;
    hipError_t e = hipMemcpy(d, host_in, (size_t) n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = tlsrec__exclusive_scan(d, d + n, n, d + 2 * (size_t) n, 0);
    if (e == hipSuccess) e = hipMemcpy(host_out, d + n, (size_t) n * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    return e == hipSuccess ? 0 : -1;
}
#endif /* TLSREC_TEST_HOOKS */

extern "C" hipError_t tlsrec__launch_res_guard(tlsrec_batch_res *res, uint32_t n, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(tlsrec_res_guard_kernel, dim3((n + 255) / 256), dim3(256), 0, st, res, n);
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
