/*
 * ccm.hip -- AES-CCM / CCM_8 record protection.
 *
 * The psa_aead_encrypt/decrypt calls of ssl_msg.c:1043 / :1412 for the CCM
 * suites of mbedtls_ssl_cipher_to_psa (ssl_tls.c:2185-2235: PSA_ALG_CCM, or
 * its 8-byte shortened-tag form for the CCM_8 suites), fused with the same
 * record framing the GCM / ChaCha20-Poly1305 kernels apply (tlsrec_frame.h).
 *
 * CCM (NIST SP 800-38C) with the TLS 12-byte nonce (q = 3):
 *   B0 = flags || N || len24, A1 = len16(AAD) || AAD || 0  (AAD <= 13 B)
 *   X_0 = E(B0), X_1 = E(X_0 ^ A1), X_(i+1) = E(X_i ^ P_i)   (CBC-MAC)
 *   C_i = P_i ^ E(ctr_i), ctr_i = 2 || N || i24, tag = MSB_t(X_last ^ E(ctr_0))
 *
 * The CBC-MAC is one dependent chain per record, so a record belongs to ONE
 * lane, which runs the MAC chain and the counter-mode chain side by side (two
 * independent AES per block).  Parallelism comes from records: a 512-thread
 * workgroup holds 512 records; a wave serves its records in key passes (the
 * records of one slot at a time, round keys in SGPRs through the constant
 * address space) -- the bucket pass has sorted them by slot already.  AES is
 * the T-table form of tlsrec_device.h (tables in LDS, conflict-free), so the
 * kernel is LDS-bound at ~2 x 224 lookups per 16-byte block.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tlsrec.h"
#include "tlsrec_device.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"
#include "tlsrec_recdev.h"

namespace tlsrec {

constexpr int CCM_WAVES = 8;
constexpr int CCM_THREADS = CCM_WAVES * 64;

/* little-endian words of a 16-byte block given as bytes b0..b15 */
__device__ __forceinline__ uint32_t w4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3)
{
    return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}

/* ARIA: ARIA-CCM / Camellia-CCM (NR = 12/14/16 / 18/24; the S-box image,
 * round keys SlotState::ark) -- the CCM construction around it unchanged */
template <int NR, bool ARIA, typename RK>
__device__ __forceinline__ uint4 blk_encrypt(const uint8_t *lds, uint32_t lb, RK rk, uint4 in)
{
    if constexpr (ARIA)
        return alt_encrypt<NR, 0>(lds, lb, rk, in);
    else
        return aes_encrypt<NR, 0>(lds, lb, rk, in);
}

template <int NR, bool DEC, bool CID = false, bool ARIA = false>
__global__ __launch_bounds__(CCM_THREADS) void tlsrec_ccm_kernel(CcmArgs a)
{
    /* T0/T1 x 32 copies (64 KiB), or the ARIA / Camellia S-box image (32 KiB) */
    __shared__ __attribute__((aligned(16))) uint8_t lds[ARIA ? 32768 : 65536];
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t lanebase = (uint32_t) (lane & 31) << 2;   /* T-table / S-box image copy */
    const uint32_t lo = a.perm ? *a.lo : 0u;
    const uint32_t count = a.perm ? *a.hi - lo : (uint32_t) a.n;
    const uint64_t wg_base = (uint64_t) blockIdx.x * CCM_THREADS;
    if (wg_base >= count) return;                              /* uniform, before the barrier */
    if constexpr (ARIA)
        alt_fill_tables<NR>(lds, tid, CCM_THREADS);
    else
        aes_fill_tables(lds, tid, CCM_THREADS);
    __syncthreads();

    /* this lane's record */
    uint32_t my_slot = 0xffffffffu, my_rec = 0;
    {
        const uint64_t pos = wg_base + (uint64_t) tid;
        if (pos < count) {
            my_rec = a.perm ? a.perm[lo + pos] : (uint32_t) pos;
            const uint32_t s = a.recs[my_rec].slot;
            const bool usable = s < a.capacity && a.slots[s].km.cipher != 0;
            const int c = usable ? a.slots[s].km.cipher : 0;   /* no read past the table */
            if (TLSREC_HOOK_SKIP(my_rec, a.skip)) {
                /* test hook: an unreached record keeps the guard's INTERNAL_ERROR */
            } else if (usable && (ARIA ? tlsrec_cipher_is_alt_ccm(c) && tlsrec_cipher_alt_nr(c) == NR
                                : tlsrec_cipher_is_ccm(c) && tlsrec_cipher_nr(c) == NR))
                my_slot = s;
            else if (!a.perm && !usable && a.flag_nr == (ARIA ? 100u + NR : (uint32_t) NR))
                bad_slot_result(a.recs[my_rec], &a.res[my_rec]);   /* identity order: flagged by one launch */
        }
    }

    for (;;) {
        const uint32_t s = __builtin_amdgcn_readfirstlane(wave_min(my_slot));
        if (s == 0xffffffffu) break;
        const bool mine = my_slot == s;
        my_slot = mine ? 0xffffffffu : my_slot;
        if (!mine) continue;
        const kconst_u32 *rk = (const kconst_u32 *) (uintptr_t) (ARIA ? a.slots[s].ark : a.slots[s].rkr);
        const tlsrec_key_material km = a.slots[s].km;
        const tlsrec_batch_rec d = a.recs[my_rec];
        tlsrec_plan p;
        make_plan<DEC, CID>(p, d, km, &a.slots[s], a.in);
        if (p.status != 0) {
            finish_early(p, d, a.out, &a.res[my_rec]);
            continue;
        }
        const uint32_t taglen = km.taglen;
        uint32_t nw[3];
        nonce_words<DEC>(p, d, km, a.in, nw);
        const uint32_t n0 = nw[0], n1 = nw[1], n2 = nw[2];
        const uint8_t *src = a.in + d.buf_off + p.aead_pos;
        uint8_t *dst = a.out + d.buf_off + p.aead_pos;
        const uint32_t aead_len = p.aead_len;
        const uint32_t content_len = DEC ? aead_len : p.content_len;
        /* nonce bytes N0..N11 sit in block bytes 1..12: shift the nonce words by one byte */
        const uint32_t m0 = n0 << 8, m1 = __builtin_amdgcn_alignbyte(n1, n0, 3),
                       m2 = __builtin_amdgcn_alignbyte(n2, n1, 3), m3 = n2 >> 24;
        /* B0: flags = Adata | M' = (t-2)/2 | L' = q-1 = 2 */
        const uint32_t flags = 0x40u | (((taglen - 2) / 2) << 3) | 2u;
        uint4 x = blk_encrypt<NR, ARIA>(lds, lanebase, rk,
                                     make_uint4(m0 | flags, m1, m2,
                                                m3 | w4(0, (aead_len >> 16) & 0xff, (aead_len >> 8) & 0xff,
                                                        aead_len & 0xff)));
        /* A1 = len16(aad) || aad || zeros (the record AAD is 5 or 13 bytes;
         * with a DTLS 1.2 CID 23..55, continued below) */
        {
            uint8_t ab[16];
#pragma unroll
            for (int i = 0; i < 16; i++) ab[i] = 0;
            ab[0] = 0;
            ab[1] = p.aad_len;
#pragma unroll
            for (int i = 0; i < 14; i++)
                if (i < (int) p.aad_len) ab[2 + i] = p.aad[i];
            const uint4 a1 = make_uint4(w4(ab[0], ab[1], ab[2], ab[3]), w4(ab[4], ab[5], ab[6], ab[7]),
                                        w4(ab[8], ab[9], ab[10], ab[11]), w4(ab[12], ab[13], ab[14], ab[15]));
            x = blk_encrypt<NR, ARIA>(lds, lanebase, rk, xor4(x, a1));
            if (CID && p.aad_len > 14) {   /* DTLS 1.2 + CID: 23..55 AAD bytes after len16 */
                const uint8_t *cid = a.slots[s].cid;
                x = blk_encrypt<NR, ARIA>(lds, lanebase, rk, xor4(x, cid_aad_block<1, 2>(p, d, cid)));
                if (p.aad_len > 30) x = blk_encrypt<NR, ARIA>(lds, lanebase, rk, xor4(x, cid_aad_block<2, 2>(p, d, cid)));
                if (p.aad_len > 46) x = blk_encrypt<NR, ARIA>(lds, lanebase, rk, xor4(x, cid_aad_block<3, 2>(p, d, cid)));
            }
        }
        /* counter blocks: 2 || N || i24 */
        const uint32_t c0 = m0 | 2u;
        uint32_t nzpos = 0;
        const uint32_t nblk = (aead_len + 15) / 16;
        for (uint32_t i = 0; i < nblk; i++) {
            const uint32_t pos = 16 * i, ctr = i + 1;
            const uint4 cb = make_uint4(c0, m1, m2, m3 | w4(0, (ctr >> 16) & 0xff, (ctr >> 8) & 0xff, ctr & 0xff));
            /* a 16-byte read stays inside the record while the tag (room)
             * covers it; the CCM_8 tail block takes the byte path */
            const bool wide = pos + 16 <= aead_len + taglen;
            const uint4 in = load_block(src, pos, content_len, aead_len, p.inner_type, wide);
            if (DEC) {
                const uint4 ks = blk_encrypt<NR, ARIA>(lds, lanebase, rk, cb);
                const uint4 pt = mask_block(xor4(in, ks), pos, aead_len);
                store_block(dst, pos, aead_len, pt, true);
                if (p.inner && (pt.x | pt.y | pt.z | pt.w)) nzpos = pos + 1;
                x = blk_encrypt<NR, ARIA>(lds, lanebase, rk, xor4(x, pt));
            } else {
                /* MAC and keystream are independent: two AES chains interleave */
                const uint4 ks = blk_encrypt<NR, ARIA>(lds, lanebase, rk, cb);
                x = blk_encrypt<NR, ARIA>(lds, lanebase, rk, xor4(x, in));
                store_block(dst, pos, aead_len, mask_block(xor4(in, ks), pos, aead_len), true);
            }
        }
        const uint4 s0 = blk_encrypt<NR, ARIA>(lds, lanebase, rk, make_uint4(c0, m1, m2, m3));
        const uint4 tag = xor4(x, s0);
        tlsrec_batch_res r;
        r.cid_len = 0;
        r.reserved[0] = r.reserved[1] = 0;
        if (!DEC) {
            store_block(dst, aead_len, aead_len + taglen, tag, false);
            if (p.explicit_iv && p.post_status == 0) {
                uint8_t *e = a.out + d.buf_off + p.data_offset;
                for (int i = 0; i < 8; i++) e[i] = d.ctr[i];
            }
            r.status = p.post_status;
            r.data_offset = p.data_offset;
            r.data_len = p.data_len;
            r.type = p.type;
            r.cid_len = p.cid_set ? p.cid_len : 0;
        } else {
            const uint4 want = load_block(src, aead_len, aead_len + taglen, aead_len + taglen, 0, false);
            const uint4 got = mask_block(tag, 0, taglen);
            const uint32_t diff = (want.x ^ got.x) | (want.y ^ got.y) | (want.z ^ got.z) | (want.w ^ got.w);
            r.data_offset = p.data_offset;
            r.data_len = p.data_len;
            r.type = d.type;
            if (diff != 0) {
                /* PSA wipes the whole output buffer on a bad tag */
                zero_range(a.out + d.buf_off, p.aead_pos, d.buf_len, 0, 1);
                r.status = TLSREC_E_INVALID_MAC;
            } else if (p.inner) {                              /* ssl_msg.c:1809-1829 */
                const uint32_t key = nzpos ? last_nonzero_key(load_block(dst, nzpos - 1, aead_len, aead_len, 0, false),
                                                              nzpos - 1)
                                           : 0u;
                if (key == 0) {
                    r.status = TLSREC_E_INVALID_RECORD;
                } else {
                    r.status = 0;
                    r.data_len = (key >> 8) - 1;
                    r.type = (uint8_t) (key & 0xff);
                }
            } else {
                r.status = 0;
            }
        }
        a.res[my_rec] = r;
    }
}

} /* namespace tlsrec */

using namespace tlsrec;

extern "C" hipError_t tlsrec__launch_ccm(const CcmArgs *a, int dec, uint32_t nr_mask, hipStream_t st)
{
    /* one workgroup per CCM_THREADS positions; with a permutation the record
     * count is on the device, so the grid covers all n and surplus
     * workgroups exit at once.  One launch per AES key size present. */
    const uint32_t g = (uint32_t) ((a->n + CCM_THREADS - 1) / CCM_THREADS);
    if (g == 0) return hipSuccess;
    CcmArgs b = *a;
    /* nr_mask: AES rounds at bit NR, ARIA / Camellia rounds at bit NR + 4; the
     * first variant present flags unusable slots in identity order (ARIA and
     * Camellia: 100 + NR) */
    b.flag_nr = (nr_mask & (1u << 10)) ? 10 : (nr_mask & (1u << 12)) ? 12 : (nr_mask & (1u << 14)) ? 14
              : (nr_mask & (1u << 16)) ? 112 : (nr_mask & (1u << 18)) ? 114 : (nr_mask & (1u << 20)) ? 116
              : (nr_mask & (1u << 22)) ? 118 : 124;
    hipError_t e = hipSuccess;
#define TLSREC_CCM_LAUNCH(NR, ARIA, BIT)                                                                      \
    if (e == hipSuccess && (nr_mask & (1u << (BIT)))) {                                                       \
        if (b.cid) {                                                                                          \
            if (dec) hipLaunchKernelGGL((tlsrec_ccm_kernel<NR, true, true, ARIA>), dim3(g), dim3(CCM_THREADS), 0, st, b); \
            else hipLaunchKernelGGL((tlsrec_ccm_kernel<NR, false, true, ARIA>), dim3(g), dim3(CCM_THREADS), 0, st, b); \
        } else if (dec) hipLaunchKernelGGL((tlsrec_ccm_kernel<NR, true, false, ARIA>), dim3(g), dim3(CCM_THREADS), 0, st, b); \
        else hipLaunchKernelGGL((tlsrec_ccm_kernel<NR, false, false, ARIA>), dim3(g), dim3(CCM_THREADS), 0, st, b); \
        e = hipGetLastError();                                                                                \
    }
    TLSREC_CCM_LAUNCH(10, false, 10)
    TLSREC_CCM_LAUNCH(12, false, 12)
    TLSREC_CCM_LAUNCH(14, false, 14)
    TLSREC_CCM_LAUNCH(12, true, 16)
    TLSREC_CCM_LAUNCH(14, true, 18)
    TLSREC_CCM_LAUNCH(16, true, 20)
    TLSREC_CCM_LAUNCH(18, true, 22)     /* Camellia-128 */
    TLSREC_CCM_LAUNCH(24, true, 28)     /* Camellia-192 / -256 */
#undef TLSREC_CCM_LAUNCH
    return e;
}
