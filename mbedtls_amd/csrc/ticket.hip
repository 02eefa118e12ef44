/*
 * ticket.hip -- session-ticket protection on the GPU.
 *
 * mbedtls_ssl_ticket_write / mbedtls_ssl_ticket_parse (library/ssl_ticket.c
 * :210-306, :334-412) for a batch of tickets: the same layout
 *     key_name[4] || iv[12] || len16 || state || tag[16]     (ssl_ticket.c:44-55)
 * the same AEAD call (nonce = iv, AAD = the 18 header bytes, :271-279 /
 * :384-391), the same checks and error codes (CHK_BUF_PTR, length, key
 * selection by name -> SESSION_TICKET_EXPIRED, INVALID_MAC), with the ticket
 * key's AEAD: GCM or CCM (16-byte tag) over AES, ARIA or Camellia, or
 * ChaCha20-Poly1305 -- every AEAD key type mbedtls_ssl_ticket_setup accepts
 * (ssl_ticket.c:188-209).
 *
 * Tickets are short (a serialized session, ~100-300 B) and use at most two
 * keys, so each lane owns one ticket and runs its AEAD sequentially; a wave
 * serves its tickets in key passes (wave-min over the lanes' slots: round
 * keys in SGPRs, the key's GHASH H-table staged into the wave's own 8 KiB of
 * LDS).  AES T-tables and the ARIA / Camellia S-box images as in
 * tlsrec_device.h, staged only for the key families the two ticket keys use
 * (template mask IMG, picked on the host).  The caller supplies the IVs
 * (the reference draws them with psa_generate_random, :255) and the
 * serialized state (mbedtls_ssl_session_save / _load stay on the host).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "tlsrec.h"
#include "tlsrec_device.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"
#include "tlsrec_recdev.h"

namespace tlsrec {

constexpr int TK_WAVES = 4;
constexpr int TK_THREADS = TK_WAVES * 64;
constexpr uint32_t TK_AAD = 18, TK_MIN = 34, TK_TAG = 16;

struct TicketArgs {
    const SlotState *slots;
    const uint4 *ghtab;
    uint32_t capacity;
    uint32_t kslot[2];
    uint32_t kname[2];        /* key names as little-endian words */
    uint32_t active;
    const tlsrec_ticket *t;
    uint32_t n;
    uint8_t *arena;
    tlsrec_ticket_res *res;
};

TLSREC_HD int tk_cipher_ok(int c)
{
    return tlsrec_cipher_is_gcm(c) || (tlsrec_cipher_is_ccm(c) && tlsrec_cipher_taglen(c) == 16) ||
           tlsrec_cipher_is_alt_gcm(c) || tlsrec_cipher_is_alt_ccm(c) || c == TLSREC_CIPHER_CHACHA20_POLY1305;
}

/* LDS images of the kernel instantiation IMG (1 AES T-tables, 2 ARIA S-box
 * image, 4 Camellia S-box image): AES at 0, then the waves' H tables, then
 * the images present */
template <int IMG>
struct TkLds {
    static constexpr int AES = 0;
    static constexpr int HT = (IMG & 1) ? 65536 : 0;
    static constexpr int ARIA = HT + TK_WAVES * 8192;
    static constexpr int CAM = ARIA + ((IMG & 2) ? 32768 : 0);
    static constexpr int BYTES = CAM + ((IMG & 4) ? 32768 : 0);
};

/* the ticket key's block cipher: AES (BC 0) from the T-tables at OFF, ARIA /
 * Camellia (NR 12..16 / 18, 24) from the S-box image at OFF */
template <int NR, int BC, int OFF>
__device__ __forceinline__ uint4 tk_block(const uint8_t *lds, uint32_t lb, const kconst_u32 *rk, uint4 in)
{
    if constexpr (BC == 0)
        return aes_encrypt<NR, OFF>(lds, lb, rk, in);
    else
        return alt_encrypt<NR, OFF>(lds, lb, rk, in);
}

/* byte-granular block access (tickets are short; any alignment) */
__device__ __forceinline__ uint4 tk_load(const uint8_t *p, uint32_t pos, uint32_t len)
{
    return load_block(p, pos, len, len, 0, false);
}

/* GCM over one ticket: J0 = iv || 1, AAD = two GHASH blocks */
template <int NR, bool DEC, int BC = 0, int OFF = 0>
__device__ bool tk_gcm(const uint8_t *lds, const uint8_t *ht, uint32_t lb, const kconst_u32 *rk, uint8_t *buf,
                       uint32_t len)
{
    const uint32_t n0 = ld_u32le(buf + 4), n1 = ld_u32le(buf + 8), n2 = ld_u32le(buf + 12);
    const uint4 ej0 = tk_block<NR, BC, OFF>(lds, lb, rk, make_uint4(n0, n1, n2, bswap32(1u)));
    uint4 z = gmul<0>(ht, tk_load(buf, 0, TK_AAD));
    z = gmul<0>(ht, xor4(z, tk_load(buf, 16, TK_AAD)));
    uint8_t *p = buf + TK_AAD;
    for (uint32_t pos = 0; pos < len; pos += 16) {
        const uint4 ks = tk_block<NR, BC, OFF>(lds, lb, rk, make_uint4(n0, n1, n2, bswap32(pos / 16 + 2)));
        const uint4 in = tk_load(p, pos, len);
        const uint4 out = mask_block(xor4(in, ks), pos, len);
        store_block(p, pos, len, out, false);
        z = gmul<0>(ht, xor4(z, DEC ? in : out));
    }
    z = gmul<0>(ht, xor4(z, make_uint4(0, bswap32(TK_AAD * 8), 0, bswap32(len * 8))));
    const uint4 tag = xor4(z, ej0);
    if (!DEC) {
        store_block(p, len, len + TK_TAG, tag, false);
        return true;
    }
    const uint4 want = tk_load(p, len, len + TK_TAG);
    return ((want.x ^ tag.x) | (want.y ^ tag.y) | (want.z ^ tag.z) | (want.w ^ tag.w)) == 0;
}

/* CCM (16-byte tag) over one ticket: A = len16(18) || AAD in two blocks */
template <int NR, bool DEC, int BC = 0, int OFF = 0>
__device__ bool tk_ccm(const uint8_t *lds, uint32_t lb, const kconst_u32 *rk, uint8_t *buf, uint32_t len)
{
    const uint32_t n0 = ld_u32le(buf + 4), n1 = ld_u32le(buf + 8), n2 = ld_u32le(buf + 12);
    const uint32_t m0 = n0 << 8, m1 = __builtin_amdgcn_alignbyte(n1, n0, 3),
                   m2 = __builtin_amdgcn_alignbyte(n2, n1, 3), m3 = n2 >> 24;
    const uint32_t flags = 0x40u | (((TK_TAG - 2) / 2) << 3) | 2u;
    uint4 x = tk_block<NR, BC, OFF>(lds, lb, rk,
                                 make_uint4(m0 | flags, m1, m2,
                                            m3 | (((len >> 16) & 0xff) << 8) | (((len >> 8) & 0xff) << 16) |
                                                ((len & 0xff) << 24)));
    /* 0x00 0x12 aad[0..13] | aad[14..17] 0... */
    const uint4 a0 = tk_load(buf, 0, TK_AAD), a1 = tk_load(buf, 16, TK_AAD);
    const uint4 b1 = make_uint4((TK_AAD << 8) | (a0.x << 16), __builtin_amdgcn_alignbyte(a0.y, a0.x, 2),
                                __builtin_amdgcn_alignbyte(a0.z, a0.y, 2), __builtin_amdgcn_alignbyte(a0.w, a0.z, 2));
    const uint4 b2 = make_uint4(__builtin_amdgcn_alignbyte(a1.x, a0.w, 2), a1.x >> 16, 0, 0);
    x = tk_block<NR, BC, OFF>(lds, lb, rk, xor4(x, b1));
    x = tk_block<NR, BC, OFF>(lds, lb, rk, xor4(x, b2));
    uint8_t *p = buf + TK_AAD;
    const uint32_t c0 = m0 | 2u;
    for (uint32_t pos = 0; pos < len; pos += 16) {
        const uint32_t ctr = pos / 16 + 1;
        const uint4 ks = tk_block<NR, BC, OFF>(lds, lb, rk,
                                            make_uint4(c0, m1, m2,
                                                       m3 | (((ctr >> 16) & 0xff) << 8) | (((ctr >> 8) & 0xff) << 16) |
                                                           ((ctr & 0xff) << 24)));
        const uint4 in = tk_load(p, pos, len);
        const uint4 out = mask_block(xor4(in, ks), pos, len);
        store_block(p, pos, len, out, false);
        x = tk_block<NR, BC, OFF>(lds, lb, rk, xor4(x, DEC ? out : in));
    }
    const uint4 tag = xor4(x, tk_block<NR, BC, OFF>(lds, lb, rk, make_uint4(c0, m1, m2, m3)));
    if (!DEC) {
        store_block(p, len, len + TK_TAG, tag, false);
        return true;
    }
    const uint4 want = tk_load(p, len, len + TK_TAG);
    return ((want.x ^ tag.x) | (want.y ^ tag.y) | (want.z ^ tag.z) | (want.w ^ tag.w)) == 0;
}

/* ChaCha20-Poly1305 (RFC 8439 2.8) over one ticket */
template <bool DEC>
__device__ bool tk_chachapoly(const tlsrec_key_material &km, uint8_t *buf, uint32_t len)
{
    uint32_t key[8], nw[3], blk[16];
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = ld_u32le(km.key + 4 * i);
    nw[0] = ld_u32le(buf + 4);
    nw[1] = ld_u32le(buf + 8);
    nw[2] = ld_u32le(buf + 12);
    chacha_block(key, 0, nw, blk);
    const P5 r = p_from_r(blk[0], blk[1], blk[2], blk[3]);
    const uint4 s = make_uint4(blk[4], blk[5], blk[6], blk[7]);
    P5 h = p_zero();
    /* AAD: 18 bytes padded to 32 */
    h = p_carry(p_mul(p_add(h, p_block(tk_load(buf, 0, TK_AAD))), r));
    h = p_carry(p_mul(p_add(h, p_block(tk_load(buf, 16, TK_AAD))), r));
    uint8_t *p = buf + TK_AAD;
    for (uint32_t pos = 0; pos < len; pos += 64) {
        uint32_t ks[16];
        chacha_block(key, pos / 64 + 1, nw, ks);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t bp = pos + 16 * t;
            if (bp < len) {
                const uint4 in = tk_load(p, bp, len);
                const uint4 out = mask_block(xor4(in, make_uint4(ks[4 * t], ks[4 * t + 1], ks[4 * t + 2],
                                                                 ks[4 * t + 3])),
                                             bp, len);
                store_block(p, bp, len, out, false);
                h = p_carry(p_mul(p_add(h, p_block(DEC ? in : out)), r));
            }
        }
    }
    h = p_carry(p_mul(p_add(h, p_block(make_uint4(TK_AAD, 0, len, 0))), r));
    const uint4 tag = p_finish(h, s);
    if (!DEC) {
        store_block(p, len, len + TK_TAG, tag, false);
        return true;
    }
    const uint4 want = tk_load(p, len, len + TK_TAG);
    return ((want.x ^ tag.x) | (want.y ^ tag.y) | (want.z ^ tag.z) | (want.w ^ tag.w)) == 0;
}

template <bool DEC, int IMG>
__global__ __launch_bounds__(TK_THREADS) void tlsrec_ticket_kernel(TicketArgs a)
{
    using LY = TkLds<IMG>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LY::BYTES];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t lb = (uint32_t) (lane & 31) << 2;
    if constexpr ((IMG & 1) != 0) aes_fill_tables(lds + LY::AES, tid, TK_THREADS);
    if constexpr ((IMG & 2) != 0) aria_fill_tables(lds + LY::ARIA, tid, TK_THREADS);
    if constexpr ((IMG & 4) != 0) cam_fill_tables(lds + LY::CAM, tid, TK_THREADS);
    __syncthreads();
    uint8_t *ht = lds + LY::HT + wave * 8192;
    const uint32_t i = blockIdx.x * TK_THREADS + tid;

    /* framing checks of ssl_ticket.c; my_slot = the key to run the AEAD with */
    uint32_t my_slot = 0xffffffffu, len = 0, tlen = 0;
    int32_t st = 0;
    uint8_t *buf = nullptr;
    if (i < a.n) {
        const tlsrec_ticket t = a.t[i];
        buf = a.arena + t.off;
        if (!DEC) {
            const uint32_t space = t.len, clear = t.clear_len, k = a.active & 1;
            const uint32_t s = a.kslot[k];
            const bool usable = s < a.capacity && tk_cipher_ok(a.slots[s].km.cipher);
            if (space < TK_MIN) {
                st = TLSREC_ERR_SSL_BUFFER_TOO_SMALL;                      /* CHK_BUF_PTR, :236 */
            } else if (!usable) {
                st = TLSREC_ERR_SSL_BAD_INPUT_DATA;
            } else {
                const uint32_t name = a.kname[k];
                for (int b = 0; b < 4; b++) buf[b] = (uint8_t) (name >> (8 * b));   /* :253 */
                if (clear > space - TK_AAD) {
                    st = TLSREC_ERR_SSL_BUFFER_TOO_SMALL;                  /* session_save, :259-261 */
                } else if (clear > 65535) {
                    st = 0;                                                /* :262-266 returns 0, no tlen */
                } else {
                    buf[16] = (uint8_t) (clear >> 8);                      /* :268 */
                    buf[17] = (uint8_t) clear;
                    if (clear + TK_TAG > space - TK_AAD) {
                        st = TLSREC_ERR_SSL_BUFFER_TOO_SMALL;              /* PSA output buffer */
                    } else {
                        my_slot = s;
                        len = clear;
                        tlen = TK_MIN + clear;                             /* :305 */
                    }
                }
            }
        } else {
            const uint32_t tl = t.len;
            if (tl < TK_MIN) {
                st = TLSREC_ERR_SSL_BAD_INPUT_DATA;                        /* :356-358 */
            } else {
                const uint32_t enc = ((uint32_t) buf[16] << 8) | buf[17];
                if (tl != TK_MIN + enc) {
                    st = TLSREC_ERR_SSL_BAD_INPUT_DATA;                    /* :372-375 */
                } else {
                    const uint32_t name = ld_u32le(buf);
                    const int k = name == a.kname[0] ? 0 : (name == a.kname[1] ? 1 : -1);
                    if (k < 0) {
                        st = TLSREC_ERR_SSL_SESSION_TICKET_EXPIRED;        /* :378-381 */
                    } else {
                        const uint32_t s = a.kslot[k];
                        if (s >= a.capacity || !tk_cipher_ok(a.slots[s].km.cipher)) {
                            st = TLSREC_ERR_SSL_BAD_INPUT_DATA;
                        } else {
                            my_slot = s;
                            len = enc;
                            tlen = enc;
                        }
                    }
                }
            }
        }
    }

    for (;;) {
        const uint32_t s = __builtin_amdgcn_readfirstlane(wave_min(my_slot));
        if (s == 0xffffffffu) break;
        const tlsrec_key_material km = a.slots[s].km;
        const int c = km.cipher;
        if (tlsrec_cipher_is_gcm(c) || tlsrec_cipher_is_alt_gcm(c)) {
            /* stage this key's H table into the wave's LDS (in-order LDS queue:
             * the wave's writes land before its reads) */
            const uint4 *src = a.ghtab + (size_t) s * KEY_TABLE_WORDS;
            for (int e = lane; e < 512; e += 64) reinterpret_cast<uint4 *>(ht)[e] = src[e];
        }
        const bool mine = my_slot == s;
        my_slot = mine ? 0xffffffffu : my_slot;
        if (!mine) continue;
        const bool alt = tlsrec_cipher_is_alt_gcm(c) || tlsrec_cipher_is_alt_ccm(c);
        const kconst_u32 *rk = (const kconst_u32 *) (uintptr_t) (alt ? a.slots[s].ark : a.slots[s].rkr);
        const uint32_t nr = alt ? tlsrec_cipher_alt_nr(c) : tlsrec_cipher_nr(c);
        bool ok = false;
        if (tlsrec_cipher_is_gcm(c)) {
            if constexpr ((IMG & 1) != 0)
                ok = nr == 10 ? tk_gcm<10, DEC>(lds, ht, lb, rk, buf, len)
                   : nr == 12 ? tk_gcm<12, DEC>(lds, ht, lb, rk, buf, len) : tk_gcm<14, DEC>(lds, ht, lb, rk, buf, len);
        } else if (tlsrec_cipher_is_ccm(c)) {
            if constexpr ((IMG & 1) != 0)
                ok = nr == 10 ? tk_ccm<10, DEC>(lds, lb, rk, buf, len)
                   : nr == 12 ? tk_ccm<12, DEC>(lds, lb, rk, buf, len) : tk_ccm<14, DEC>(lds, lb, rk, buf, len);
        } else if (tlsrec_cipher_is_alt_gcm(c)) {
            if (nr < 18) {
                if constexpr ((IMG & 2) != 0)
                    ok = nr == 12 ? tk_gcm<12, DEC, 1, LY::ARIA>(lds, ht, lb, rk, buf, len)
                       : nr == 14 ? tk_gcm<14, DEC, 1, LY::ARIA>(lds, ht, lb, rk, buf, len)
                                  : tk_gcm<16, DEC, 1, LY::ARIA>(lds, ht, lb, rk, buf, len);
            } else {
                if constexpr ((IMG & 4) != 0)
                    ok = nr == 18 ? tk_gcm<18, DEC, 2, LY::CAM>(lds, ht, lb, rk, buf, len)
                                  : tk_gcm<24, DEC, 2, LY::CAM>(lds, ht, lb, rk, buf, len);
            }
        } else if (tlsrec_cipher_is_alt_ccm(c)) {
            if (nr < 18) {
                if constexpr ((IMG & 2) != 0)
                    ok = nr == 12 ? tk_ccm<12, DEC, 1, LY::ARIA>(lds, lb, rk, buf, len)
                       : nr == 14 ? tk_ccm<14, DEC, 1, LY::ARIA>(lds, lb, rk, buf, len)
                                  : tk_ccm<16, DEC, 1, LY::ARIA>(lds, lb, rk, buf, len);
            } else {
                if constexpr ((IMG & 4) != 0)
                    ok = nr == 18 ? tk_ccm<18, DEC, 2, LY::CAM>(lds, lb, rk, buf, len)
                                  : tk_ccm<24, DEC, 2, LY::CAM>(lds, lb, rk, buf, len);
            }
        } else {
            ok = tk_chachapoly<DEC>(km, buf, len);
        }
        if (DEC && !ok) {
            for (uint32_t b = 0; b < len; b++) buf[TK_AAD + b] = 0;       /* PSA clears its output */
            st = TLSREC_ERR_SSL_INVALID_MAC;
            tlen = 0;
        }
    }
    if (i < a.n) {
        tlsrec_ticket_res r;
        r.status = st;
        r.tlen = st == 0 ? tlen : 0;
        r.reserved[0] = r.reserved[1] = 0;
        a.res[i] = r;
    }
}

} /* namespace tlsrec */

using namespace tlsrec;

/* engine.hip */
extern "C" const SlotState *tlsrec__keytab_slots(const tlsrec_keytab *kt);
extern "C" const uint4 *tlsrec__keytab_ghtab(const tlsrec_keytab *kt);
extern "C" int tlsrec__keytab_cipher(const tlsrec_keytab *kt, uint32_t slot);

static int ticket_batch(const tlsrec_keytab *kt, const tlsrec_ticket_keys *keys, const tlsrec_ticket *t, uint32_t n,
                        uint8_t *arena, tlsrec_ticket_res *res, void *stream, bool dec)
{
    if (!kt || !keys || (n && (!t || !arena || !res))) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (n == 0) return 0;
    TicketArgs a;
    a.slots = tlsrec__keytab_slots(kt);
    a.ghtab = tlsrec__keytab_ghtab(kt);
    a.capacity = tlsrec_keytab_capacity(kt);
    for (int k = 0; k < 2; k++) {
        a.kslot[k] = keys->slot[k];
        a.kname[k] = (uint32_t) keys->name[k][0] | ((uint32_t) keys->name[k][1] << 8) |
                     ((uint32_t) keys->name[k][2] << 16) | ((uint32_t) keys->name[k][3] << 24);
    }
    a.active = keys->active;
    a.t = t;
    a.n = n;
    a.arena = arena;
    a.res = res;
    const uint32_t grid = (n + TK_THREADS - 1) / TK_THREADS;
    hipStream_t st = (hipStream_t) stream;
    /* LDS images for the two keys' block ciphers (host mirror of the slots) */
    int img = 0;
    for (int k = 0; k < 2; k++) {
        const int c = keys->slot[k] < a.capacity ? tlsrec__keytab_cipher(kt, keys->slot[k]) : 0;
        if (!tk_cipher_ok(c) || c == TLSREC_CIPHER_CHACHA20_POLY1305) continue;
        img |= tlsrec_cipher_is_alt_gcm(c) || tlsrec_cipher_is_alt_ccm(c) ? (tlsrec_cipher_cam_nr(c) ? 4 : 2) : 1;
    }
    if (img == 0) img = 1;
    switch (img) {
#define TK_LAUNCH(I)                                                                                      \
    case I:                                                                                               \
        if (dec) hipLaunchKernelGGL((tlsrec_ticket_kernel<true, I>), dim3(grid), dim3(TK_THREADS), 0, st, a); \
        else hipLaunchKernelGGL((tlsrec_ticket_kernel<false, I>), dim3(grid), dim3(TK_THREADS), 0, st, a);  \
        break;
        TK_LAUNCH(1) TK_LAUNCH(2) TK_LAUNCH(3) TK_LAUNCH(4) TK_LAUNCH(5) TK_LAUNCH(6) TK_LAUNCH(7)
#undef TK_LAUNCH
    }
    return hipGetLastError() == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
}

extern "C" int tlsrec_ticket_write(const tlsrec_keytab *kt, const tlsrec_ticket_keys *keys, const tlsrec_ticket *t,
                                   uint32_t n, uint8_t *arena, tlsrec_ticket_res *res, void *stream)
{
    return ticket_batch(kt, keys, t, n, arena, res, stream, false);
}

extern "C" int tlsrec_ticket_parse(const tlsrec_keytab *kt, const tlsrec_ticket_keys *keys, const tlsrec_ticket *t,
                                   uint32_t n, uint8_t *arena, tlsrec_ticket_res *res, void *stream)
{
    return ticket_batch(kt, keys, t, n, arena, res, stream, true);
}
