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

__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t) __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t) __shfl_xor(v, o));
    return v;
}

template <int L>
__device__ __forceinline__ uint32_t group_max(uint32_t v)
{
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) v = max(v, (uint32_t) __shfl_xor(v, o));
    return v;
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

template <bool DEC>
__device__ __forceinline__ void nonce_words(const tlsrec_plan &p, const tlsrec_batch_rec &d, const uint8_t *in,
                                            uint32_t nw[3])
{
    uint8_t nonce[12];
    for (int i = 0; i < 12; i++) nonce[i] = p.nonce[i];
    if (DEC && p.explicit_iv) {   /* encrypt uses rec->ctr (ssl_msg.c:1012-1019) */
        const uint8_t *e = in + d.buf_off + d.data_offset;   /* ssl_msg.c:1360 dynamic_iv = data */
        for (int i = 0; i < 8; i++) nonce[4 + i] = e[i];
    }
    nw[0] = ld_u32le(nonce);
    nw[1] = ld_u32le(nonce + 4);
    nw[2] = ld_u32le(nonce + 8);
}

__device__ __forceinline__ uint4 aad_words(const tlsrec_plan &p)
{
    uint32_t w[4];
    for (int i = 0; i < 4; i++) w[i] = ld_u32le(p.aad + 4 * i);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

} /* namespace tlsrec */

#endif /* TLSREC_RECDEV_H */
