/*
 * tlsrec_recdev.h -- per-record device helpers shared by the AEAD kernels
 * (kernels.hip: AES-GCM, ChaCha20-Poly1305; ccm.hip: AES-CCM): the framing
 * plan applied to a batch descriptor, block loads/stores with the TLS 1.3
 * inner plaintext spliced in, early-exit results, nonce / AAD words.
 */
#ifndef TLSREC_RECDEV_H
#define TLSREC_RECDEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tlsrec.h"
#include "tlsrec_device.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"

namespace tlsrec {

/* ======================================================================
 * Shared record helpers
 * ==================================================================== */
__device__ __forceinline__ uint32_t ld_u32le(const uint8_t *p)
{
    return (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16) | ((uint32_t) p[3] << 24);
}

/* zero the bytes of a block at or beyond `len` */
__device__ __forceinline__ uint4 mask_block(uint4 v, uint32_t pos, uint32_t len)
{
    if (pos + 16 <= len) return v;
    uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int32_t valid = (int32_t) len - (int32_t) (pos + 4 * i);
        uint32_t m = valid >= 4 ? 0xffffffffu : (valid <= 0 ? 0u : (0xffffffffu >> (8 * (4 - valid))));
        w[i] &= m;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

/* Load one 16-byte block of the AEAD input.  `pos` is the block offset within
 * the AEAD region [0, aead_len); bytes at [content_len, aead_len) are the
 * TLS 1.3 inner type byte followed by zero padding (ssl_msg.c:466-491), bytes
 * >= aead_len are zero.  With a 16-B aligned region the full 16-byte read is
 * always inside the record buffer: the tag (decrypt) or the tag room checked
 * at ssl_msg.c:995-998 (encrypt) follows the AEAD data. */
__device__ __forceinline__ uint4 load_block(const uint8_t *src, uint32_t pos, uint32_t content_len,
                                            uint32_t aead_len, uint8_t inner_type, bool aligned)
{
    uint4 v;
    if (aligned) {
        v = gload16(src + pos);
        if (pos + 16 <= content_len) return v;
        v = mask_block(v, pos, content_len);
    } else {
        uint32_t w[4] = { 0, 0, 0, 0 };
#pragma unroll 1
        for (uint32_t i = 0; i < 16; i++) {
            if (pos + i < content_len) w[i >> 2] |= (uint32_t) src[pos + i] << (8 * (i & 3));
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    if (content_len >= pos && content_len < pos + 16 && content_len < aead_len) {
        const uint32_t e = content_len - pos, sh = 8 * (e & 3), t = (uint32_t) inner_type << sh;
        if ((e >> 2) == 0) v.x |= t;
        else if ((e >> 2) == 1) v.y |= t;
        else if ((e >> 2) == 2) v.z |= t;
        else v.w |= t;
    }
    return v;
}

__device__ __forceinline__ void store_block(uint8_t *dst, uint32_t pos, uint32_t len, uint4 v, bool aligned)
{
    if (aligned && pos + 16 <= len) {
        gstore16(dst + pos, v);
        return;
    }
    const uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll 1
    for (uint32_t i = 0; i < 16; i++) {
        if (pos + i < len) {
            const uint32_t d = i >> 2;
            const uint32_t wd = d == 0 ? w[0] : (d == 1 ? w[1] : (d == 2 ? w[2] : w[3]));
            dst[pos + i] = (uint8_t) (wd >> (8 * (i & 3)));
        }
    }
}

/* (index+1) << 8 | value of the last non-zero byte of a block, or 0 */
__device__ __forceinline__ uint32_t last_nonzero_key(uint4 v, uint32_t pos)
{
    const uint32_t w[4] = { v.x, v.y, v.z, v.w };
    uint32_t key = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        if (w[d] != 0) {
            uint32_t e = (31 - __builtin_clz(w[d])) >> 3;
            key = ((pos + 4 * d + e + 1) << 8) | ((w[d] >> (8 * e)) & 0xff);
        }
    }
    return key;
}

__device__ __forceinline__ uint4 shfl4(uint4 v, int src)
{
    return make_uint4(__shfl(v.x, src), __shfl(v.y, src), __shfl(v.z, src), __shfl(v.w, src));
}

/* ----------------------------------------------------------------------
 * Cross-lane moves on the VALU (DPP, v_permlane16/32_swap) instead of
 * ds_bpermute, which is an LDS-pipe instruction -- the pipe the table
 * kernels are bound by.  gfx950 DPP controls: quad_perm
 * 0x00-0xFF, row_shl:n 0x100+n, row_ror:n 0x120+n, row_mirror 0x140,
 * row_half_mirror 0x141 (a row = 16 lanes).
 * -------------------------------------------------------------------- */
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v)
{
    return (uint32_t) __builtin_amdgcn_update_dpp((int) v, (int) v, CTRL, 0xF, 0xF, false);
}

/* lane i gets lane i ^ 16 (v_permlane16_swap: odd rows <-> even rows) */
__device__ __forceinline__ uint32_t xor16(uint32_t v, int lane)
{
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((lane >> 4) & 1) ? r[0] : r[1];
}

/* lane i gets lane i ^ 32 (v_permlane32_swap: upper half <-> lower half) */
__device__ __forceinline__ uint32_t xor32(uint32_t v, int lane)
{
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane >> 5) ? r[0] : r[1];
}

/* Butterfly partner of step S (1, 2, 4, 8, 16, 32) for a reduction over
 * aligned groups of 2S lanes: after the steps 1 .. S every lane holds the
 * reduction of its group.  Steps 4 and 8 are mirrors (i <-> 7 - i, i <-> 15 - i
 * within the row), not xors: they pair each lane with one of the other half,
 * which already holds that half's reduction. */
template <int S>
__device__ __forceinline__ uint32_t partner(uint32_t v, int lane)
{
    static_assert(S == 1 || S == 2 || S == 4 || S == 8 || S == 16 || S == 32, "butterfly step");
    if constexpr (S == 1) return dpp<0xB1>(v);          /* quad_perm [1,0,3,2] */
    else if constexpr (S == 2) return dpp<0x4E>(v);     /* quad_perm [2,3,0,1] */
    else if constexpr (S == 4) return dpp<0x141>(v);    /* row_half_mirror */
    else if constexpr (S == 8) return dpp<0x140>(v);    /* row_mirror */
    else if constexpr (S == 16) return xor16(v, lane);
    else return xor32(v, lane);
}

/* lane i gets lane i + SH, for the lanes q < SH of aligned groups of 2 SH or
 * more lanes (the GHASH lane tree); other lanes get unspecified values */
template <int SH>
__device__ __forceinline__ uint32_t from_up(uint32_t v, int lane)
{
    if constexpr (SH < 16) return dpp<0x100 + SH>(v);    /* row_shl:SH */
    else if constexpr (SH == 16) return xor16(v, lane);
    else return xor32(v, lane);
}

template <int SH>
__device__ __forceinline__ uint4 from_up4(uint4 v, int lane)
{
    return make_uint4(from_up<SH>(v.x, lane), from_up<SH>(v.y, lane), from_up<SH>(v.z, lane), from_up<SH>(v.w, lane));
}

/* For a symmetric op the 16- and 32-lane steps need no lane select: after
 * v_permlane16/32_swap(v, v) the two results hold, in every lane, its own
 * value and its partner's (in some order), and op(own, partner) is the same
 * either way. */
template <int G, typename F>
__device__ __forceinline__ uint32_t group_reduce(uint32_t v, F op)
{
    if constexpr (G >= 2) v = op(v, dpp<0xB1>(v));
    if constexpr (G >= 4) v = op(v, dpp<0x4E>(v));
    if constexpr (G >= 8) v = op(v, dpp<0x141>(v));
    if constexpr (G >= 16) v = op(v, dpp<0x140>(v));
    if constexpr (G >= 32) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = op(r[0], r[1]);
    }
    if constexpr (G >= 64) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        v = op(r[0], r[1]);
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
    return group_reduce<64>(v, [](uint32_t a, uint32_t b) { return max(a, b); });
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
    return group_reduce<64>(v, [](uint32_t a, uint32_t b) { return min(a, b); });
}

template <int L>
__device__ __forceinline__ uint32_t group_max(uint32_t v)
{
    return group_reduce<L>(v, [](uint32_t a, uint32_t b) { return max(a, b); });
}

template <int L>
__device__ __forceinline__ uint32_t group_or(uint32_t v)
{
    return group_reduce<L>(v, [](uint32_t a, uint32_t b) { return a | b; });
}

template <int L>
__device__ __forceinline__ uint32_t group_xor(uint32_t v)
{
    return group_reduce<L>(v, [](uint32_t a, uint32_t b) { return a ^ b; });
}

/* every lane of an aligned group of L lanes gets the XOR of the group's values */
template <int L>
__device__ __forceinline__ uint4 group_xor4(uint4 v)
{
    return make_uint4(group_xor<L>(v.x), group_xor<L>(v.y), group_xor<L>(v.z), group_xor<L>(v.w));
}

__device__ __forceinline__ void zero_range(uint8_t *dst, uint32_t from, uint32_t to, int q, int L)
{
    for (uint32_t i = from + (uint32_t) q; i < to; i += (uint32_t) L) dst[i] = 0;
}

__device__ __forceinline__ tlsrec_plan_key plan_key(const tlsrec_key_material &km, const SlotState *st)
{
    tlsrec_plan_key k;
    k.tls13 = km.tls_minor == 4;
    k.fixed_ivlen = km.fixed_ivlen;
    k.taglen = km.taglen;
    k.iv = km.iv;
    /* km.reserved[0] mirrors st->cid_len (tlsrec_keytab_set_cid): the plan
     * needs no load beyond the key material the kernel already holds */
    k.cid_len = km.reserved[0];
    k.cid = st->cid;
    return k;
}

/* The plan of batch record d under slot st (km = st->km, already loaded);
 * `in` is the input arena (decrypt reads the record's CID bytes there).
 * CID = false: the kernel instantiation for key tables without connection IDs
 * (every slot's CID is empty), in which all CID code folds away; a record
 * that carries a CID there gets UNEXPECTED_CID (ssl_msg.c:1313-1320). */
template <bool DEC, bool CID = false>
__device__ __forceinline__ void make_plan(tlsrec_plan &p, const tlsrec_batch_rec &d, const tlsrec_key_material &km,
                                          const SlotState *st, const uint8_t *in)
{
    tlsrec_plan_key k = plan_key(km, st);
    if (!CID) {
        k.cid_len = 0;
        k.cid = nullptr;
    }
    if (DEC) {
        if (CID) {
            const uint32_t off = (uint32_t) d.cid_off[0] | ((uint32_t) d.cid_off[1] << 8) |
                                 ((uint32_t) d.cid_off[2] << 16) | ((uint32_t) d.cid_off[3] << 24);
            tlsrec_plan_decrypt(&p, &k, d.ctr, d.type, d.ver, d.buf_len, d.data_offset, d.data_len,
                                in + d.buf_off + off, d.cid_len);
        } else {
            tlsrec_plan_decrypt(&p, &k, d.ctr, d.type, d.ver, d.buf_len, d.data_offset, d.data_len, nullptr, 0);
            if (d.cid_len != 0 && p.status != TLSREC_E_INTERNAL_ERROR) {   /* after :1301-1307 */
                p.status = TLSREC_E_UNEXPECTED_CID;
                p.data_offset = d.data_offset;
                p.data_len = d.data_len;
                p.type = d.type;
            }
        }
    } else {
        tlsrec_plan_encrypt(&p, &k, d.ctr, d.type, d.ver, d.buf_len, d.data_offset, d.data_len,
                            km.granularity ? km.granularity : TLSREC_PADDING_GRANULARITY);
    }
}

/* Block I >= 1 of the RFC 9146 AAD of a CID record (block 0 is p.aad), the
 * byte stream shifted right by SHIFT bytes (CCM's len16 prefix, SHIFT = 2).
 * cid = the slot's CID (for decrypt the plan checked it equals the record's). */
template <int I, int SHIFT>
__device__ __forceinline__ uint4 cid_aad_block(const tlsrec_plan &p, const tlsrec_batch_rec &d, const uint8_t *cid)
{
    uint32_t w[4] = { 0, 0, 0, 0 };
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int k = 16 * I + j - SHIFT;
        const uint32_t b = k < 0 ? 0u : tlsrec_cid_aad_byte((uint32_t) k, p.type, d.ver, d.ctr, cid, p.cid_len, p.aead_len);
        w[j >> 2] |= b << (8 * (j & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

/* Record naming no usable key slot (out of range or never loaded). */
__device__ inline void bad_slot_result(const tlsrec_batch_rec &d, tlsrec_batch_res *res)
{
    tlsrec_batch_res r;
    r.status = TLSREC_ERR_SSL_BAD_INPUT_DATA;
    r.data_offset = d.data_offset;
    r.data_len = d.data_len;
    r.type = d.type;
    r.cid_len = 0;
        r.reserved[0] = r.reserved[1] = 0;
    *res = r;
}

/* Record whose plan stopped before the AEAD: status + pre-AEAD side effects. */
__device__ inline void finish_early(const tlsrec_plan &p, const tlsrec_batch_rec &d, uint8_t *out,
                                    tlsrec_batch_res *res)
{
    if (p.side_type) {
        uint8_t *b = out + d.buf_off + p.side_pos;
        b[0] = d.type;
        for (uint32_t i = 0; i < p.side_zeros; i++) b[1 + i] = 0;
    }
    tlsrec_batch_res r;
    r.status = p.status;
    r.data_offset = p.data_offset;
    r.data_len = p.data_len;
    r.type = p.type;
    r.cid_len = p.cid_set ? p.cid_len : 0;
        r.reserved[0] = r.reserved[1] = 0;
    *res = r;
}

/* The record nonce as three little-endian words, ssl_build_record_nonce
 * (ssl_msg.c:768-781): the fixed IV (12 bytes, or 4 for the TLS 1.2 GCM /
 * CCM suites) XOR the sequence number in bytes 4..11 -- or, decrypting a
 * record with an explicit nonce, the record's 8 bytes at data_offset
 * (ssl_msg.c:1352-1365).  Built from the key material's words: the plan's
 * byte form (tlsrec_frame.h tlsrec__nonce, through a pointer into km) kept
 * the key material and the nonce bytes in scratch memory, 13 byte stores per
 * call in the GCM kernels. */
template <bool DEC>
__device__ __forceinline__ void nonce_words(const tlsrec_plan &p, const tlsrec_batch_rec &d,
                                            const tlsrec_key_material &km, const uint8_t *in, uint32_t nw[3])
{
    uint32_t iv[3], ctr[2];
    __builtin_memcpy(iv, km.iv, 12);
    __builtin_memcpy(ctr, d.ctr, 8);
    const bool full = km.fixed_ivlen == 12;
    nw[0] = iv[0];
    nw[1] = (full ? iv[1] : 0u) ^ ctr[0];
    nw[2] = (full ? iv[2] : 0u) ^ ctr[1];
    if (DEC && p.explicit_iv) {   /* encrypt uses rec->ctr (ssl_msg.c:1012-1019) */
        const uint8_t *e = in + d.buf_off + d.data_offset;   /* ssl_msg.c:1360 dynamic_iv = data */
        nw[1] = ld_u32le(e);
        nw[2] = ld_u32le(e + 4);
    }
}

__device__ __forceinline__ uint4 aad_words(const tlsrec_plan &p)
{
    uint32_t w[4];
    for (int i = 0; i < 4; i++) w[i] = ld_u32le(p.aad + 4 * i);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

} /* namespace tlsrec */

#endif /* TLSREC_RECDEV_H */
