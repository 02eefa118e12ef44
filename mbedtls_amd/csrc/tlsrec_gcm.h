/*
 * tlsrec_gcm.h -- the GCM record kernel (AES, and ARIA / Camellia through the
 * LDS-table cipher slot) and its launch dispatch.  Included by the per-
 * direction translation units gcm_enc.hip / gcm_dec.hip / gcm_alt_enc.hip /
 * gcm_alt_dec.hip, which instantiate it (the instantiations dominate the
 * build; one unit per direction lets them compile in parallel).
 */
#ifndef TLSREC_GCM_H
#define TLSREC_GCM_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>

#include "tlsrec.h"
#include "tlsrec_clmul.h"
#include "tlsrec_device.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"
#include "tlsrec_recdev.h"

#ifndef TLSREC_GCM_LINE_GROUPS
#define TLSREC_GCM_LINE_GROUPS 1
#endif

/* Ablation builds (tools/build_variant.sh, never the product library): what
 * a per-round piece of the paired small-record passes costs, by leaving it
 * out -- bit 0 the lane-power multiply (tags wrong), bit 1 the per-key H^L
 * table build (the previous key's table is used: tags wrong).  0 = off. */
#ifndef TLSREC_ABLATE
#define TLSREC_ABLATE 0
#endif
/* paired passes: the tag stage's plan fields kept in LDS from the setup
 * (r06; bit 0 decrypt, bit 1 encrypt) */
#ifndef TLSREC_PLAN_STASH
#define TLSREC_PLAN_STASH 0      /* measured: no gain, the spills move */
#endif

namespace tlsrec {

/* ======================================================================
 * AES-GCM
 * ==================================================================== */
/* WP (wave passes): each wave keeps only its current key's H^L table in its
 * own 8 KiB of LDS; the once-per-record multiplies (AAD fold, tree, final)
 * read the key's tables in global memory -- except the 16-lane tree, which
 * multiplies by H^8 .. H^1 held as values (gtree_v, GcmArgs::tm). */
/* G5: the Horner table H^L is the 13 KiB 5-bit form (gmul5) after the tree's
 * 4-bit tables H^1 .. H^(L/2). */
/* PAIR (paired wave passes): 16 waves, the two waves of a pair share one
 * H^L table (8 pairs x 8 KiB), so small records of many keys run at the
 * 16-wave occupancy of the single-key kernel; the AAD-fold slots shrink to
 * one per record of a round (64 / L per wave) to fit. */
template <int L, int W, bool WP = false, bool G5 = false, bool PAIR = false>
struct GcmLds {
    static constexpr int NT = PAIR ? W / 2 : (WP ? W : Log2<L>::v + (G5 ? 0 : 1));  /* 4-bit GHASH tables */
    /* The wave-pass kernels hold 64 KiB of per-wave (per-pair) tables: the
     * T-tables go first there, so that every lookup address (< 64 KiB) folds
     * into the 16-bit ds_read offset; behind 64 KiB of tables each of the 202
     * lookups of a step cost one more v_or for its address.  The per-wave
     * tables are addressed from a register base anyway. */
    static constexpr int GH = WP ? 65536 : 0;
    static constexpr int HG5 = GH + NT * 8192;          /* G5 Horner table */
    static constexpr int AES = WP ? 0 : HG5 + (G5 ? KEY_G5_WORDS * 16 : 0);   /* T0/T1 x 32 copies */
    static constexpr int EJ0 = WP ? HG5 : AES + 65536;  /* W waves x 64 x 16 B */
    static constexpr int FOLDN = PAIR ? 64 / L : 64;    /* AAD-fold slots per wave */
    static constexpr int FOLD = EJ0 + W * 64 * 16;      /* W waves x FOLDN x 16 B: AAD fold */
    static constexpr int CTL = FOLD + W * FOLDN * 16;
    static constexpr int BYTES = CTL + (PAIR ? 128 : 16);
    static_assert(BYTES <= 160 * 1024, "LDS budget");
};

/* Barrier of the two waves of a pair (PAIR): a monotonic LDS counter that
 * both waves bump once per barrier; every wave of a pair passes the same
 * number of barriers (both see the same key sequence), so the spin always
 * ends. The fences order the table writes before the bump and the reads
 * after it. */
__device__ __forceinline__ void pair_sync(uint32_t *cnt, uint32_t &phase, int lane)
{
    phase += 2;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (v >= phase) break;
        __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

/* Half ph of the pair builds windows 16 ph .. 16 ph + 15 of the 4-bit
 * position table of P (tlsrec_clmul.h) at tab: lane (k, q) makes entries
 * 4q .. 4q + 3 of window 16 ph + k (tlsrec_gtab4_quad: the window's base and
 * its three multiples by X, then XORs -- r06; r05's lane (k0, n) made one
 * entry of four windows, each entry from four general shifts, ~4x the VALU
 * work).  Out of line: the record kernel's registers are full, and inlined
 * the build moved its spills into the per-record code. */
#ifndef TLSREC_GTAB_QUAD
#define TLSREC_GTAB_QUAD 1
#endif
__device__ __noinline__ void gtab4_build_half(uint8_t *tab, const uint4 *pp, int lane, int ph)
{
    const uint4 pv = *pp;
    const uint32_t pw[4] = { pv.x, pv.y, pv.z, pv.w };
#if TLSREC_GTAB_QUAD
    const uint32_t k = 16u * (uint32_t) ph + ((uint32_t) lane >> 2), q = (uint32_t) lane & 3u;
    uint32_t w[4][4];
    tlsrec_gtab4_quad(pw, k, q, w);
    uint4 *dst = reinterpret_cast<uint4 *>(tab + k * 256 + q * 64);
#pragma unroll
    for (int t = 0; t < 4; t++) dst[t] = make_uint4(w[t][0], w[t][1], w[t][2], w[t][3]);
#else
    const uint32_t n = (uint32_t) lane & 15u, k0 = 16u * (uint32_t) ph + ((uint32_t) lane >> 4);
    uint64_t bh, bl;
    tlsrec_gtab4_base(pw, k0, &bh, &bl);
    uint4 *dst = reinterpret_cast<uint4 *>(tab + k0 * 256 + n * 16);
#pragma unroll
    for (int t = 0; t < 4; t++) {
        uint64_t eh, el;
        uint32_t w[4];
        tlsrec_gtab4_entry(bh, bl, n, &eh, &el);
        tlsrec_g_to_words(eh, el, w);
        dst[t * 64] = make_uint4(w[0], w[1], w[2], w[3]);    /* window k0 + 4 t */
        if (t < 3) tlsrec_gf128_shr(&bh, &bl, 16);
    }
#endif
}

/* Per-record state that the AEAD loop reads (kept small: it lives in
 * VGPRs across the loop). */
struct GcmJob {
    bool run, aligned, inner;   /* inner: TLS 1.3 / DTLS 1.2 + CID inner plaintext */
    bool wide_tail;             /* partial blocks read 16 B wide (in place); false: byte-wise (GcmArgs::src_off) */
    uint8_t inner_type;
    uint32_t aead_len, content_len, aad_len;
    uint32_t nw0, nw1, nw2;
    uint4 aadw;
    const uint8_t *src;
    uint8_t *dst;

    template <bool DEC>
    __device__ __forceinline__ void setup(const tlsrec_plan &p, const tlsrec_batch_rec &d,
                                          const tlsrec_key_material &km, const uint8_t *in, uint8_t *out)
    {
        uint32_t nw[3];
        nonce_words<DEC>(p, d, km, in, nw);
        nw0 = nw[0]; nw1 = nw[1]; nw2 = nw[2];
        aadw = aad_words(p);
        aad_len = p.aad_len;
        aead_len = p.aead_len;
        content_len = DEC ? p.aead_len : p.content_len;
        inner_type = p.inner_type;
        inner = p.inner;
        src = in + d.buf_off + p.aead_pos;
        dst = out + d.buf_off + p.aead_pos;
        /* 16-byte global accesses need no 16-byte alignment on gfx950: the
         * HSA target runs in unaligned-access mode (hipcc emits
         * global_load_dwordx4 for a byte-aligned 16-byte memcpy), so records
         * at any byte offset -- the stream path's records follow 5-byte
         * headers -- take the wide path; the wide read of a block never
         * leaves the record buffer (tag / tag room follows the AEAD data) */
        aligned = true;
        wide_tail = true;
        run = true;
    }
};

/* GHASH Horner over blocks 0..3 of a CID record's AAD (block 0 = a0), leaving
 * the last block un-multiplied (the kernel's AAD fold applies that H).  Out
 * of line: CID records are rare, the record kernel's registers are not. */
__device__ __noinline__ uint4 gcm_cid_aad_fold(const uint8_t *gp, uint4 a0, const tlsrec_plan &p,
                                               const tlsrec_batch_rec &d, const uint8_t *cid)
{
    uint4 f = xor4(gmul<0>(gp, a0), cid_aad_block<1, 0>(p, d, cid));
    if (p.aad_len > 32) f = xor4(gmul<0>(gp, f), cid_aad_block<2, 0>(p, d, cid));
    if (p.aad_len > 48) f = xor4(gmul<0>(gp, f), cid_aad_block<3, 0>(p, d, cid));
    return f;
}

/* The lane tree with table-free multiplies (tlsrec_clmul.h) by the powers
 * P[k] = H^(2^k) held as values (k <= 4: L <= 32): for the wave passes, whose
 * per-record tables otherwise come from HBM (a key's H^8, H^4, H^2 tables, 24
 * KiB, for 4 records of 16 KiB at L = 16). */
/* Out of line (r05): inlined, its ~600 instructions shifted the register
 * allocation and schedule of the record loop around it (a faster multiply
 * cost k4 1.2 % through a 5-instruction longer step loop, same box). */
__device__ __forceinline__ uint4 gf_mul_i(uint4 x, uint4 p)
{
    const uint32_t a[4] = { x.x, x.y, x.z, x.w }, b[4] = { p.x, p.y, p.z, p.w };
    uint32_t r[4];
    tlsrec_gf128_mul(a, b, r);
    return make_uint4(r[0], r[1], r[2], r[3]);
}
__device__ __noinline__ uint4 gf_mul_v(uint4 x, uint4 p) { return gf_mul_i(x, p); }

template <int SH>
__device__ __forceinline__ uint4 gtree_v(const uint4 (&P)[5], uint4 Y, int lane, int q)
{
    if constexpr (SH >= 1) {
        uint4 o = from_up4<SH>(Y, lane);
        if (q < SH) Y = xor4(gf_mul_v(Y, P[Log2<SH>::v]), o);
        return gtree_v<SH / 2>(P, Y, lane, q);
    } else {
        return Y;
    }
}

/* lanes q < SH: Y_q = Y_q * H^SH ^ Y_(q+SH); leaves sum_q Y_q H^(2SH-1-q) in q = 0.
 * Only lanes q < SH multiply (the others' values are never read again), so a
 * level's table reads shrink with it: L - 1 lane-multiplies per record instead
 * of L log2 L (the shuffle runs on every lane: its sources must be active). */
template <int SH>
__device__ __forceinline__ uint4 gtree(const uint8_t *lds, uint4 Y, int lane, int q)
{
    if constexpr (SH >= 1) {
        uint4 o = from_up4<SH>(Y, lane);
        if (q < SH) Y = xor4(gmul<Log2<SH>::v>(lds, Y), o);
        return gtree<SH / 2>(lds, Y, lane, q);
    } else {
        return Y;
    }
}

/* ARIA: the block cipher is ARIA (NR = 12/14/16 rounds, S-box tables in the
 * T-table LDS region, round keys SlotState::ark) -- GCM around it unchanged */
template <int L, int NR, bool DEC, int W, int B, bool WP = false, bool CID = false, bool ARIA = false,
          bool G5 = false, bool PAIR = false>
__global__ __launch_bounds__(W * 64) void tlsrec_gcm_kernel(GcmArgs a)
{
    static_assert(!G5 || (L == 1 << KEY_G5_POWER && !WP && !CID && !ARIA && B == 1), "G5: the 8-lane 16-wave kernel");
    static_assert(!PAIR || (WP && W == 16 && B == 1 && !CID && !ARIA && !G5), "PAIR: 16-wave paired wave passes");
    using LY = GcmLds<L, W, WP, G5, PAIR>;
    constexpr int NTHR = W * 64;
    constexpr int LOGL = Log2<L>::v;
    constexpr int R = 64 / L;
    /* the kernel's only LDS object, so it starts at LDS address 0 and every
     * table offset folds into the ds_read immediate */
    __shared__ __attribute__((aligned(16))) uint8_t lds[LY::BYTES];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g = lane / L, q = lane % L;
    const uint32_t lanebase = (uint32_t) (lane & 31) << 2;   /* T-table / S-box image copy */
    uint32_t *ctl = reinterpret_cast<uint32_t *>(lds + LY::CTL);

    /* This workgroup's positions: wave w owns positions base + k*W + w,
     * k < rpw (interleaved, so a key's run of records in perm spreads over
     * all waves of the workgroup within one key pass). */
    const uint32_t lo = a.perm ? *a.lo : 0u;
    const uint32_t count = a.perm ? *a.hi - lo : (uint32_t) a.n;
    const uint64_t wg_base = (uint64_t) blockIdx.x * W * a.rpw;
    if (wg_base >= count) return;                      /* uniform: before any barrier */

    if constexpr (ARIA)
        alt_fill_tables<NR>(lds + LY::AES, tid, NTHR);
    else
        aes_fill_tables(lds + LY::AES, tid, NTHR);

    /* PAIR: wave w is half ph of pair pr; the pair owns 2 rpw contiguous
     * positions and its halves take them alternately, so both see the same
     * key runs */
    const int pr = wave & (W / 2 - 1), ph = wave / (W / 2);
    /* pass membership: lane l tracks the record at chunk position k = l
     * (PAIR: of the pair's 2 rpw positions from cb); its descriptor is
     * dsrc[my_d] -- the key-ordered copy the bucket pass wrote (a.srecs,
     * contiguous per key), or recs[] itself.  (r05: membership and the key
     * passes as two inlined lambdas; the G5 kernel then allocates with 20
     * instead of 22 spilled VGPRs, 100 instead of 104 B of scratch) */
    const tlsrec_batch_rec *const dsrc = (a.perm && a.srecs) ? a.srecs + lo : a.recs;
    auto membership = [&](uint64_t cb, uint64_t pend, uint32_t &my_slot, uint32_t &my_rec,
                          uint32_t &my_d) __attribute__((always_inline)) {
        {
            /* WP: a wave's positions are contiguous (its key runs stay together) */
            const uint64_t pos = PAIR ? cb + 2 * (uint64_t) lane + (uint64_t) ph
                                 : WP ? wg_base + (uint64_t) wave * a.rpw + lane : wg_base + (uint64_t) lane * W + wave;
            if (lane < (int) a.rpw && pos < pend) {
                my_rec = a.perm ? a.perm[lo + pos] : (uint32_t) pos;
                my_d = (a.perm && a.srecs) ? (uint32_t) pos : my_rec;
                const uint32_t s = dsrc[my_d].slot;
                if (TLSREC_HOOK_SKIP(my_rec, a.skip)) {
                    /* test hook: an unreached record keeps the guard's INTERNAL_ERROR */
                } else if (s < a.capacity && a.slots[s].km.cipher == a.cipher) {
                    my_slot = s;
                } else if (!a.perm && !(s < a.capacity && a.slots[s].km.cipher != 0)) {
                    /* identity order: this kernel is the only one that sees the record */
                    bad_slot_result(a.recs[my_rec], &a.res[my_rec]);
                }
            }
        }
    };
    /* the key passes over the lanes' positions */
    /* Horner multiplier table H^L (hor) and the per-record tables H^1..H^(L/2) (gp) */
    constexpr int HPI = WP ? 0 : LOGL;                   /* H^L table index from hor */
    const uint8_t *hor = WP ? lds + LY::GH + (PAIR ? pr : wave) * 8192 : (G5 ? lds + LY::HG5 : lds + LY::GH);
    /* E_K(J0) once per lane before the passes (r05) -- every AES kernel but
     * the single-key G5 one, whose one pass covers all its lanes anyway (in
     * the 16-wave key passes: c4 +0.6 %, and the ARIA / Camellia kernels
     * 0 / -1.2 % same box, so those keep the per-pass AES) */
    constexpr bool EJ0_ONCE = WP || (!G5 && !ARIA);
    uint32_t phase = 0;                                  /* PAIR barrier count */
    auto passes = [&](uint32_t my_slot, uint32_t my_rec, uint32_t my_d) __attribute__((always_inline)) {
        if constexpr (EJ0_ONCE) {
            /* E_K(J0) of the lane's own record under its own key, once, before
             * the passes (r05): per key pass it cost a whole SIMD AES for the
             * few lanes of that key -- with 16 records per key, one AES per
             * round of 8 records.  The lane reads its slot's round keys as
             * vectors; the LDS slot keeps the value across the passes. */
            uint4 ej0 = make_uint4(0, 0, 0, 0);
            if (my_slot != 0xffffffffu) {
                const SlotState *ss = &a.slots[my_slot];
                const tlsrec_key_material km = ss->km;
                const tlsrec_batch_rec d = dsrc[my_d];
                tlsrec_plan p;
                make_plan<DEC, CID>(p, d, km, ss, a.in);
                uint32_t nw[3];
                nonce_words<DEC>(p, d, km, a.in, nw);
                if constexpr (ARIA)
                    ej0 = alt_encrypt<NR, LY::AES>(lds, lanebase, (const uint32_t *) ss->ark,
                                                   make_uint4(nw[0], nw[1], nw[2], bswap32(1u)));
                else
                    ej0 = aes_encrypt<NR, LY::AES>(lds, lanebase, (const uint32_t *) ss->rkr,
                                                   make_uint4(nw[0], nw[1], nw[2], bswap32(1u)));
            }
            reinterpret_cast<uint4 *>(lds + LY::EJ0)[wave * 64 + lane] = ej0;
        }
        for (int iter = 0;; iter++) {
            uint32_t s;
            if constexpr (PAIR) {
                /* the pair's smallest pending slot: both halves agree on it, stage
                 * half of its H^L table each, and meet before the table is used
                 * (the first barrier also tells the pair the previous table is no
                 * longer read) */
                uint32_t *pmin = ctl + 4 + 2 * pr;
                uint32_t *pcnt = ctl + 20 + pr;
                const uint32_t m = __builtin_amdgcn_readfirstlane(wave_min(my_slot));
                if (lane == 0) pmin[ph] = m;
                pair_sync(pcnt, phase, lane);
                s = __builtin_amdgcn_readfirstlane(min(pmin[0], pmin[1]));
                if (s == 0xffffffffu) break;
                if ((TLSREC_ABLATE & 2) != 0) {
                    /* ablation: no table build */
                } else if (a.tm & 16u) {
                    /* built from H^L itself (tm bit 4, r05): one 16-byte read of
                     * the key's powers instead of 8 KiB of table per key pass */
                    gtab4_build_half(const_cast<uint8_t *>(hor), a.ghtab + (size_t) s * KEY_TABLE_WORDS + KEY_HPOW_OFF + (L - 1),
                                     lane, ph);
                } else {
                    const uint4 *src = a.ghtab + (size_t) s * KEY_TABLE_WORDS + LOGL * 512;
                    uint4 *dst = reinterpret_cast<uint4 *>(const_cast<uint8_t *>(hor));
                    for (int i = lane + ph * 256; i < (ph + 1) * 256; i += 64) dst[i] = src[i];
                }
                pair_sync(pcnt, phase, lane);
            } else if constexpr (WP) {
                /* wave pass: the wave's smallest pending slot; stage its H^L table
                 * into the wave's LDS (in-order LDS queue: the wave's writes land
                 * before its reads; the asm keeps the compiler from hoisting) */
                s = __builtin_amdgcn_readfirstlane(wave_min(my_slot));
                if (s == 0xffffffffu) break;
                const uint4 *src = a.ghtab + (size_t) s * KEY_TABLE_WORDS + LOGL * 512;
                uint4 *dst = reinterpret_cast<uint4 *>(const_cast<uint8_t *>(hor));
                for (int i = lane; i < 512; i += 64) dst[i] = src[i];
                asm volatile("" ::: "memory");
            } else {
                uint32_t *cur = &ctl[iter & 1];
                if (my_slot != 0xffffffffu) atomicMin(cur, my_slot);
                __syncthreads();
                s = __builtin_amdgcn_readfirstlane(*cur);
                if (s == 0xffffffffu) break;
                if (tid == 0) ctl[(iter + 1) & 1] = 0xffffffffu;
                /* stage the slot's GHASH tables and round keys -- with lane powers
                 * (tm bit 3) only the Horner multiplier's: the tree tables H^1 ..
                 * H^(L/2) are not read (G5: its 13 KiB table alone; 4-bit: H^L) */
                {
                    const uint4 *src = a.ghtab + (size_t) s * KEY_TABLE_WORDS;
                    uint4 *dst = reinterpret_cast<uint4 *>(lds + LY::GH);
                    const int t0 = (WP && !CID && (a.tm & 8u)) ? (G5 ? LY::NT : LY::NT - 1) : 0;
                    for (int i = tid + t0 * 512; i < LY::NT * 512; i += NTHR) dst[i] = src[i];
                    if constexpr (G5) {
                        uint4 *d5 = reinterpret_cast<uint4 *>(lds + LY::HG5);
                        for (int i = tid; i < KEY_G5_WORDS; i += NTHR) d5[i] = src[KEY_G5_OFF + i];
                    }
                }
                __syncthreads();
            }
            const uint8_t *gp = WP ? reinterpret_cast<const uint8_t *>(a.ghtab + (size_t) s * KEY_TABLE_WORDS) : lds + LY::GH;
            /* H as a value (wave passes, tm bit 2): the AAD fold and the final multiplies */
            uint4 h1v = make_uint4(0, 0, 0, 0);
            if constexpr (WP)
                if (a.tm & 4u) __builtin_memcpy(&h1v, a.slots[s].h, 16);
            /* Round keys through the constant address space: scalar loads.  (Read
             * through a.slots they compile to vector loads + vmcnt(0) waits in
             * every round, since the kernel's own stores might alias the table.) */
            const kconst_u32 *rk = (const kconst_u32 *) (uintptr_t) (ARIA ? a.slots[s].ark : a.slots[s].rkr);
            const tlsrec_key_material km = a.slots[s].km;

            /* ---- pre-pass: E_K(J0) for each record of this wave's chunk ---- */
            if constexpr (!EJ0_ONCE) {
                uint4 ej0 = make_uint4(0, 0, 0, 0);
                bool mine = my_slot == s;
                uint32_t nw[3] = { 0, 0, 0 };
                if (mine) {
                    const tlsrec_batch_rec d = dsrc[my_d];
                    tlsrec_plan p;
                    make_plan<DEC, CID>(p, d, km, &a.slots[s], a.in);
                    nonce_words<DEC>(p, d, km, a.in, nw);
                    /* only this pass's records: with many keys of few records
                     * each, most of a wave's 64 positions belong to other passes
                     * (masked lanes issue no table reads) */
                    if constexpr (ARIA)
                        ej0 = alt_encrypt<NR, LY::AES>(lds, lanebase, rk, make_uint4(nw[0], nw[1], nw[2], bswap32(1u)));
                    else
                        ej0 = aes_encrypt<NR, LY::AES>(lds, lanebase, rk, make_uint4(nw[0], nw[1], nw[2], bswap32(1u)));
                }
                reinterpret_cast<uint4 *>(lds + LY::EJ0)[wave * 64 + lane] = ej0;
            }
            /* lanes of this wave read other lanes' E(J0): the wave's own LDS
             * writes complete before its later reads (in-order LDS queue). */

            /* ---- record rounds: L lanes per record, R records per wave ----
             * The pass's records hold a contiguous run [k0, k1] of this wave's
             * chunk positions (positions are in key order); the rounds start at
             * its first one (r05), so a key whose run does not begin on a multiple
             * of R takes ceil(run / R) rounds instead of one more, half empty --
             * with 16 KiB records, 23 per key: 3 rounds of 4 per half instead of 4 */
            const uint64_t runm = __ballot(my_slot == s);
            const uint32_t k0 = runm ? (uint32_t) __builtin_ctzll(runm) : 0u;
            const uint32_t k1 = runm ? 64u - (uint32_t) __builtin_clzll(runm) : 0u;   /* one past the last */
            for (uint32_t rr = k0; rr < k1; rr += R) {
                const uint32_t slot_in_chunk = rr + (uint32_t) g;
                const uint32_t owner_slot = __shfl(my_slot, (int) slot_in_chunk & 63);
                const bool active = slot_in_chunk < a.rpw && owner_slot == s;
                /* a key's records sit in a contiguous run of each wave's chunk
                 * positions: rounds holding none of them are skipped (wave-uniform,
                 * no barrier inside the round) -- with many keys of few records
                 * each, the pass would otherwise walk all rpw positions */
                if (__ballot(active) == 0) continue;
                const uint64_t ridx = (uint32_t) __shfl((int) my_rec, (int) slot_in_chunk & 63);
                const uint64_t didx = (uint32_t) __shfl((int) my_d, (int) slot_in_chunk & 63);
                /* Only what the AEAD loop needs stays live across it; the plan is
                 * re-derived from the (cached) descriptor afterwards. */
                GcmJob jb;
                jb.run = false;
                if (active) {
                    const tlsrec_batch_rec d = dsrc[didx];
                    tlsrec_plan p;
                    make_plan<DEC, CID>(p, d, km, &a.slots[s], a.in);
                    if (p.status != 0) {
                        if (q == 0) finish_early(p, d, a.out, &a.res[ridx]);
                    } else {
                        jb.setup<DEC>(p, d, km, a.in, a.out);
                        if constexpr (PAIR && (TLSREC_PLAN_STASH & (DEC ? 1 : 2)) != 0) {
                            /* (r06) what the tag stage needs of the plan, in the
                             * record's fold slot (unused with lane powers): the
                             * stage no longer reloads the descriptor and re-derives
                             * the plan (only a failed tag does, for the wipe) */
                            if (q == 0)
                                reinterpret_cast<uint4 *>(lds + LY::FOLD)[wave * LY::FOLDN + g] =
                                    make_uint4(p.data_offset, p.data_len, (uint32_t) p.post_status,
                                               (uint32_t) p.type | ((uint32_t) d.type << 8));
                            if constexpr (!DEC)
                                if (q == 0 && p.explicit_iv && p.post_status == 0) {
                                    /* the explicit nonce now, not after the AEAD: the
                                     * AEAD never reads these 8 bytes of head room */
                                    uint8_t *e = a.out + d.buf_off + p.data_offset;
                                    for (int i = 0; i < 8; i++) e[i] = d.ctr[i];
                                }
                        }
                        if constexpr (!DEC)
                            if (a.src_off) {           /* the content in the caller's buffer (stream send) */
                                jb.src = a.in + a.src_off[ridx];
                                jb.wide_tail = false;
                            }
                        /* DTLS 1.2 + CID: AAD of 2..4 blocks, Horner-folded
                         * into the block the AAD fold multiplies by H below */
                        if (CID && p.aad_len > 16) jb.aadw = gcm_cid_aad_fold(gp, jb.aadw, p, d, a.slots[s].cid);
                    }
                }
                const uint32_t m = jb.run ? (jb.aead_len + 15) >> 4 : 0;   /* GHASH C blocks */
                const uint32_t mm = m ? m : 1;
                constexpr uint32_t BL = (uint32_t) (B * L);
                /* Lane powers (tm bit 3; not with CIDs): the whole GHASH input A, C_1 ..
                 * C_m, LEN in the lane layout -- C_1 at position 0 (line-aligned, no
                 * front padding), LEN at position m, and A at position -1, i.e. the
                 * block lane L-1's chain holds before its first one (its Xp starts
                 * as A: no step, no multiply).  A lane's chain stops at the record's
                 * end, so lane q's Horner sum needs one multiply, by H^(d+1) with d
                 * = (m - q) mod L its last block's distance to LEN (the key's powers
                 * as values, KEY_HPOW_OFF), and an XOR over the record's lanes gives
                 * GHASH: no AAD fold, no lane tree, no final multiplies (8 sequential
                 * multiplies per record at L = 32 before, 4 at L = 2). */
                /* (m a multiple of BL: LEN would open a step of its own; lane 0
                 * takes it at the tail instead, Y_0 = Y_0 H^L + LEN, one multiply) */
                /* wave passes only: as a run-time flag in the 16-wave key-pass
                 * kernels it cost c2 5 % with the flag off (the hot loop carries
                 * the LEN position test and its registers; same box, r04p/q:
                 * 737 -> 700 GiB/s), and on it was no faster (r04e) */
                /* the paired passes are compiled for lane powers only (r06): with
                 * the fold and the two final multiplies by H as a value in them too,
                 * their out-of-line calls cost 28 spilled VGPRs whose stores ran in
                 * every round (engine.hip picks the 8-wave passes for the other
                 * TREEMUL modes) */
                const bool lp = PAIR || (WP && !CID && (a.tm & 8u));
                const bool lenx = lp && m % BL == 0;
                const uint32_t z = lp ? 0u : (BL - mm % BL) % BL;           /* front padding: position of C_1 */
                const uint32_t J = jb.run ? (lp ? (lenx ? m / BL : (m + BL) / BL) : (mm + z) / BL) : 0;
                const uint32_t Jmax = wave_max(J);
                /* AAD folded into the first ciphertext block: X(C_0) ^= AAD*H (or
                 * X = AAD when there is no ciphertext); kept in LDS, not VGPRs --
                 * only the step with cc == 0 reads it. */
                uint4 *fold = reinterpret_cast<uint4 *>(lds + LY::FOLD) + (PAIR ? wave * LY::FOLDN + g : wave * 64 + lane);
                /* the lane that holds block 0 (cc == 0) */
                if (!lp && jb.run && (uint32_t) q == z % L) {
                    uint4 f = jb.aadw;
                    if (m) {
                        if constexpr (WP)   /* tm bit 2: by H as a value -- the key's H^1 table is 8 KiB of
                                             * global memory, and a multiply touches 32 lines of it */
                            f = (a.tm & 4u) ? gf_mul_v(f, h1v) : gmul<0>(gp, f);
                        else
                            f = gmul<0>(gp, f);
                    }
                    *fold = f;
                }
                /* Pipelined Horner: step j computes Z = (Z ^ X_(j-1)) * H^L, which
                 * does not depend on step j's keystream, so its table reads share
                 * the AES rounds' phases (aes_ghash); after the loop Y = Z ^ X_last. */
                uint4 Z = make_uint4(0, 0, 0, 0), Xp = make_uint4(0, 0, 0, 0);
                if (lp && jb.run && q == L - 1) Xp = jb.aadw;              /* A: position -1, lane L-1's chain */
                /* TLS 1.3 inner type: position + 1 of the last non-zero output block */
                uint32_t nzpos = 0;
                /* a readable 16-byte address for lanes with nothing to load */
                const uint8_t *safe = jb.run ? (jb.wide_tail ? jb.src : jb.dst) : reinterpret_cast<const uint8_t *>(a.recs);
                /* Body steps [1, jh): every lane of the wave holds a full, aligned
                 * block inside its record's content (wave-uniform bound), so they run
                 * without masks or branches.  Step 0 (AAD fold, front padding) and
                 * the tail (partial blocks, ragged lengths) take the general step. */
                uint32_t jh = 0;
                {
                    const uint32_t mfast = (jb.run && jb.aligned) ? jb.content_len / 16 : 0;
                    if constexpr (WP && DEC) {
                        /* (r05) a round whose wave holds idle lanes -- a key run
                         * that does not fill it -- still takes the body over the
                         * running lanes' full blocks: the idle lanes load and
                         * store a dummy buffer (GcmArgs::dummy) and their
                         * results are never used; the bound keeps their
                         * addresses inside it.  Decrypt only: compiled into the
                         * encrypt kernels it cost the DTLS / stream send rows
                         * 3-4 % (same box), whose rounds are full anyway. */
                        uint32_t h = jb.run ? (mfast + z) / BL : 0xffffffffu;
                        h = wave_min(h);
                        if (__ballot(!jb.run)) {
                            constexpr uint32_t hmax = GCM_DUMMY_BYTES / (16 * BL) - 4;
                            h = a.dummy ? (h < hmax ? h : hmax) : 0;
                            if (!jb.run) {
                                jb.src = a.dummy;
                                jb.dst = a.dummy;
                                jb.nw0 = jb.nw1 = jb.nw2 = 0;
                                jb.inner = false;
                            }
                        }
                        jh = h > 1 ? h : 0;
                    } else {
                        uint32_t h = jb.run ? (mfast + z) / BL : 0;
                        h = wave_min(h);
                        jh = h > 1 ? h : 0;
                    }
                }
                /* with lane powers step 0 holds no AAD fold and no front
                 * padding (C_1 at position 0): when it is full it joins the
                 * body (r05; decrypt -- in the encrypt kernels it cost the
                 * DTLS / stream send rows 3 %) */
                const uint32_t jl = jh ? ((DEC && lp) ? 0u : 1u) : Jmax;
                auto steps = [&](auto cached) {
                    constexpr bool CACHED = decltype(cached)::value;
                    CtrCache ccache;
                    if constexpr (CACHED) ccache = ctr_cache<LY::AES>(lds, lanebase, rk, jb.nw0, jb.nw1, jb.nw2);
                    auto crypt = [&](int32_t cc, uint4 y, uint4 &ks, uint4 &Zn) {
                        const uint32_t ctrw = bswap32((uint32_t) cc + 2u);
                        if constexpr (CACHED) {
                            aes_ghash<NR, LY::AES, HPI, 2, 1, G5>(lds, hor, lanebase, rk, ccache, ctrw, y, ks, Zn);
                        } else {
                            if constexpr (ARIA)
                                ks = alt_encrypt<NR, LY::AES>(lds, lanebase, rk, make_uint4(jb.nw0, jb.nw1, jb.nw2, ctrw));
                            else
                                ks = aes_encrypt<NR, LY::AES>(lds, lanebase, rk, make_uint4(jb.nw0, jb.nw1, jb.nw2, ctrw));
                            if constexpr (G5)
                                Zn = gmul5(hor, y);
                            else
                                Zn = gmul<HPI>(hor, y);
                        }
                    };
                    auto general = [&](uint32_t j) {
                        const bool live = jb.run && j < J;
    #pragma unroll
                        for (int b = 0; b < B; b++) {
                            const int32_t cc = (int32_t) (BL * j + L * b + q) - (int32_t) z;
                            const bool valid = live && cc >= 0 && (uint32_t) cc < m;
                            const uint32_t pos = (uint32_t) cc * 16;
                            /* full, aligned interior block: plain 16-byte load/store */
                            const bool fast = valid && jb.aligned && pos + 16 <= jb.content_len;
                            uint4 blk = gload16(fast ? jb.src + pos : safe);
                            uint4 ks, Zn;
                            crypt(cc, xor4(Z, Xp), ks, Zn);
                            uint4 X = make_uint4(0, 0, 0, 0);
                            if (fast) {
                                const uint4 o = xor4(blk, ks);
                                gstore16(jb.dst + pos, o);
                                X = DEC ? blk : o;
                                if (DEC && jb.inner && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                            } else if (valid) {
                                blk = load_block(jb.src, pos, jb.content_len, jb.aead_len, jb.inner_type,
                                                 jb.aligned && jb.wide_tail);
                                const uint4 o = mask_block(xor4(blk, ks), pos, jb.aead_len);
                                store_block(jb.dst, pos, jb.aead_len, o, jb.aligned);
                                X = DEC ? blk : o;
                                if (DEC && jb.inner && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                            }
                            if (lp) {
                                if (cc == (int32_t) m)
                                    X = make_uint4(0, bswap32(jb.aad_len * 8), 0, bswap32(jb.aead_len * 8));
                                if (live && cc <= (int32_t) m) { Z = Zn; Xp = X; }    /* the chain ends at LEN */
                            } else {
                                if (live && cc == 0) X = xor4(X, *fold);
                                if (live) { Z = Zn; Xp = X; }
                            }
                        }
                    };
                    uint32_t j = 0;
                    for (; j < jl; j++) general(j);
                    {
                        const uint8_t *sp = jb.src + (size_t) (BL * j + q - z) * 16;
                        uint8_t *dp = jb.dst + (size_t) (BL * j + q - z) * 16;
                        /* 2 / 4 lanes per record (the paired passes over small
                         * records): a record's 128-byte line spans G = 128 / (16 L)
                         * steps, and 32 records per wave keep 4 MiB of such lines
                         * live per XCD -- the L2's size -- so lines were fetched
                         * and written back part-used.  Load G steps' blocks
                         * together and store them together: each line is touched
                         * once per direction. */
                        if constexpr ((PAIR || (TLSREC_GCM_LINE_GROUPS & 2)) && L <= 4 && B == 1 &&
                                      (TLSREC_GCM_LINE_GROUPS & 1)) {
                            constexpr int G = 128 / (16 * L);
                            /* single steps up to a group boundary: groups then
                             * start on a line for records without front padding
                             * (z = 0: whole-block AEAD lengths, 128-byte slots) */
                            for (; j < jh && j % G != 0; j++) {
                                const int32_t cc = (int32_t) (BL * j + q) - (int32_t) z;
                                const uint4 blk = gload16(sp);
                                uint4 ks, Zn;
                                crypt(cc, xor4(Z, Xp), ks, Zn);
                                const uint4 o = xor4(blk, ks);
                                gstore16(dp, o);
                                if (DEC && jb.inner && (o.x | o.y | o.z | o.w)) nzpos = (uint32_t) cc * 16 + 1;
                                Z = Zn;
                                Xp = DEC ? blk : o;
                                sp += 16 * BL;
                                dp += 16 * BL;
                            }
                            for (; j + G <= jh; j += G) {
                                uint4 blk[G], out[G];
    #pragma unroll
                                for (int t = 0; t < G; t++) blk[t] = gload16(sp + 16 * BL * t);
    #pragma unroll
                                for (int t = 0; t < G; t++) {
                                    const int32_t cc = (int32_t) (BL * (j + t) + q) - (int32_t) z;
                                    uint4 ks, Zn;
                                    crypt(cc, xor4(Z, Xp), ks, Zn);
                                    out[t] = xor4(blk[t], ks);
                                    if (DEC && jb.inner && (out[t].x | out[t].y | out[t].z | out[t].w))
                                        nzpos = (uint32_t) cc * 16 + 1;
                                    Z = Zn;
                                    Xp = DEC ? blk[t] : out[t];
                                }
    #pragma unroll
                                for (int t = 0; t < G; t++) gstore16(dp + 16 * BL * t, out[t]);
                                sp += 16 * BL * G;
                                dp += 16 * BL * G;
                            }
                        }
                        for (; j < jh; j++) {
    #pragma unroll
                            for (int b = 0; b < B; b++) {
                                const int32_t cc = (int32_t) (BL * j + L * b + q) - (int32_t) z;
                                const uint4 blk = gload16(sp + 16 * L * b);
                                uint4 ks, Zn;
                                crypt(cc, xor4(Z, Xp), ks, Zn);
                                const uint4 o = xor4(blk, ks);
                                gstore16(dp + 16 * L * b, o);
                                if (DEC && jb.inner && (o.x | o.y | o.z | o.w)) nzpos = (uint32_t) cc * 16 + 1;
                                Z = Zn;
                                Xp = DEC ? blk : o;
                            }
                            sp += 16 * BL;
                            dp += 16 * BL;
                        }
                    }
                    for (; j < Jmax; j++) general(j);
                };
                /* counters stay below 2^16 (any TLS record): cached rounds 1-2 */
                if constexpr (ARIA) {
                    steps(std::integral_constant<bool, false>());   /* no cached rounds for ARIA */
                } else {
                    if (wave_max(m) + 2 < 65536u)
                        steps(std::integral_constant<bool, true>());
                    else
                        steps(std::integral_constant<bool, false>());
                }
                uint4 Y = xor4(Z, Xp);
                /* lane powers: this lane's H^(L - q), read while the tail runs */
                uint4 hq = make_uint4(0, 0, 0, 0);
                if (lp) hq = a.ghtab[(size_t) s * KEY_TABLE_WORDS + KEY_HPOW_OFF + (m + (uint32_t) (L - q)) % L];
                uint32_t nzkey = 0;
                if (DEC && jb.inner && nzpos) {
                    /* the lane's last non-zero plaintext block, as written above */
                    const uint32_t pos = nzpos - 1;
                    nzkey = last_nonzero_key(load_block(jb.dst, pos, jb.aead_len, jb.aead_len, 0, false), pos);
                }
                /* tree: sum_q Y_q H^(L-q) */
                /* L = 8 and 32 (the paired passes of DTLS / stream records, 16 per
                 * key, and of k4) too: their tree read the key's H^1 .. H^16 tables
                 * from HBM, 8 KiB each, for a handful of records per key */
                if (lp) {
                    /* LEN after a whole last step: one more Horner step, by the
                     * H^L table the pass holds in LDS (r05; a table-free multiply
                     * by the value H^L before: ~1 000 VALU instructions per
                     * round, for every 16 KiB record of k4 / DTLS) */
                    if (__ballot(lenx && q == 0))
                        if (lenx && q == 0)
                            Y = xor4(gmul<HPI>(hor, Y), make_uint4(0, bswap32(jb.aad_len * 8), 0, bswap32(jb.aead_len * 8)));
                    if constexpr ((TLSREC_ABLATE & 1) != 0)
                        Y = group_xor4<L>(xor4(Y, hq));                  /* ablation: no multiply */
                    else
                        Y = group_xor4<L>(PAIR ? gf_mul_i(Y, hq) : gf_mul_v(Y, hq));   /* GHASH, in every lane of the record */
                } else if constexpr (WP && L >= 2 && L <= 32) {
                    if (a.tm & (L == 16 ? 1u : 2u)) {
                        const SlotState &ss = a.slots[s];
                        uint4 h1;
                        __builtin_memcpy(&h1, ss.h, 16);                 /* H: bytes at a 4-byte-aligned offset */
                        const uint4 P[5] = { h1,
                                             make_uint4(ss.hpow[0][0], ss.hpow[0][1], ss.hpow[0][2], ss.hpow[0][3]),
                                             make_uint4(ss.hpow[1][0], ss.hpow[1][1], ss.hpow[1][2], ss.hpow[1][3]),
                                             make_uint4(ss.hpow[2][0], ss.hpow[2][1], ss.hpow[2][2], ss.hpow[2][3]),
                                             make_uint4(ss.hpow[3][0], ss.hpow[3][1], ss.hpow[3][2], ss.hpow[3][3]) };
                        Y = gtree_v<L / 2>(P, Y, lane, q);
                    } else {
                        Y = gtree<L / 2>(gp, Y, lane, q);
                    }
                } else {
                    Y = gtree<L / 2>(gp, Y, lane, q);
                }
                if (!lp && q == 0) {                                     /* the group leader's sum */
                    uint4 lenw = make_uint4(0, bswap32(jb.aad_len * 8), 0, bswap32(jb.aead_len * 8));
                    if (WP && (a.tm & 4u)) {
                        Y = gf_mul_v(Y, h1v);                            /* T */
                        Y = gf_mul_v(xor4(Y, lenw), h1v);                /* GHASH */
                    } else {
                        Y = gmul<0>(gp, Y);                              /* T */
                        Y = gmul<0>(gp, xor4(Y, lenw));                  /* GHASH */
                    }
                }
                if (!jb.run) continue;
                const uint4 ej0 = reinterpret_cast<const uint4 *>(lds + LY::EJ0)[wave * 64 + (slot_in_chunk & 63)];
                const uint4 tag = xor4(Y, ej0);
                if constexpr (PAIR && (TLSREC_PLAN_STASH & (DEC ? 1 : 2)) != 0) {
                    const uint4 ps = reinterpret_cast<const uint4 *>(lds + LY::FOLD)[wave * LY::FOLDN + g];
                    tlsrec_batch_res r;
                    r.data_offset = ps.x;
                    r.data_len = ps.y;
                    r.cid_len = 0;
                    r.reserved[0] = r.reserved[1] = 0;
                    if (!DEC) {
                        if (q == 0) {
                            store_block(jb.dst, jb.aead_len, jb.aead_len + 16, tag, false);
                            r.status = (int32_t) ps.z;
                            r.type = (uint8_t) ps.w;
                            a.res[ridx] = r;
                        }
                    } else {
                        uint4 want = load_block(jb.src, jb.aead_len, jb.aead_len + 16, jb.aead_len + 16, 0, false);
                        uint32_t diff = (want.x ^ tag.x) | (want.y ^ tag.y) | (want.z ^ tag.z) | (want.w ^ tag.w);
                        diff = group_or<L>(q == 0 ? diff : 0u);               /* the group leader's verdict, to all */
                        uint32_t key = group_max<L>(nzkey);
                        r.type = (uint8_t) (ps.w >> 8);                       /* d.type */
                        if (diff != 0) {
                            /* PSA wipes the whole output buffer on a bad tag (the
                             * plan's AEAD position from the descriptor again) */
                            const tlsrec_batch_rec d = dsrc[didx];
                            tlsrec_plan p;
                            make_plan<DEC, CID>(p, d, km, &a.slots[s], a.in);
                            zero_range(a.out + d.buf_off, p.aead_pos, d.buf_len, q, L);
                            r.status = TLSREC_E_INVALID_MAC;
                        } else if (jb.inner) {                               /* ssl_msg.c:1809-1829 */
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
                        if (q == 0) a.res[ridx] = r;
                    }
                    continue;
                }
                const tlsrec_batch_rec d = dsrc[didx];
                tlsrec_plan p;
                make_plan<DEC, CID>(p, d, km, &a.slots[s], a.in);
                if (!DEC) {
                    if (q == 0) {
                        store_block(jb.dst, jb.aead_len, jb.aead_len + 16, tag, false);
                        if (p.explicit_iv && p.post_status == 0) {
                            uint8_t *e = a.out + d.buf_off + p.data_offset;
                            for (int i = 0; i < 8; i++) e[i] = d.ctr[i];
                        }
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
                    uint4 want = load_block(jb.src, jb.aead_len, jb.aead_len + 16, jb.aead_len + 16, 0, false);
                    uint32_t diff = (want.x ^ tag.x) | (want.y ^ tag.y) | (want.z ^ tag.z) | (want.w ^ tag.w);
                    diff = group_or<L>(q == 0 ? diff : 0u);               /* the group leader's verdict, to all */
                    uint32_t key = group_max<L>(nzkey);
                    tlsrec_batch_res r;
                    r.data_offset = p.data_offset;
                    r.data_len = p.data_len;
                    r.type = d.type;
                    r.cid_len = 0;
                    r.reserved[0] = r.reserved[1] = 0;
                    if (diff != 0) {
                        /* PSA wipes the whole output buffer on a bad tag */
                        zero_range(a.out + d.buf_off, p.aead_pos, d.buf_len, q, L);
                        r.status = TLSREC_E_INVALID_MAC;
                    } else if (p.inner) {                                /* ssl_msg.c:1809-1829 */
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
                    if (q == 0) a.res[ridx] = r;
                }
            }
            my_slot = (my_slot == s) ? 0xffffffffu : my_slot;
        }
    };
    uint32_t my_slot = 0xffffffffu, my_rec = 0, my_d = 0;
    membership(PAIR ? wg_base + (uint64_t) pr * 2 * a.rpw : 0, count, my_slot, my_rec, my_d);
    if (tid == 0) { ctl[0] = 0xffffffffu; ctl[1] = 0xffffffffu; }
    if (PAIR && tid >= 4 && tid < 32) ctl[tid] = 0;     /* pair minima [4, 20), barrier counters [20, 28) */
    __syncthreads();
    passes(my_slot, my_rec, my_d);
}

/* ======================================================================
 * Launchers
 * ==================================================================== */
template <int L, int NR, bool DEC>
static hipError_t launch_gcm_pair(const GcmArgs &a, uint32_t grid, hipStream_t st)
{
    /* paired wave passes: 16 waves x 1 block per lane, a pair per H^L table */
    hipLaunchKernelGGL((tlsrec_gcm_kernel<L, NR, DEC, 16, 1, true, false, false, false, true>), dim3(grid),
                       dim3(16 * 64), 0, st, a);
    return hipGetLastError();
}

template <int L, int NR, bool DEC>
static hipError_t launch_gcm_wp(const GcmArgs &a, uint32_t grid, hipStream_t st)
{
    /* wave passes: 8 waves x 2 blocks per lane (LDS: 8 x 8 KiB H^L + 64 KiB T-tables) */
    hipLaunchKernelGGL((tlsrec_gcm_kernel<L, NR, DEC, 8, 2, true>), dim3(grid), dim3(8 * 64), 0, st, a);
    return hipGetLastError();
}

/* ARIA-GCM: one configuration (8 lanes, ARIA_GCM_WAVES = 16 waves), with or
 * without CIDs.  The ARIA round spills ~50 VGPRs at this budget; the 8-wave
 * variant (no spills) measured 291 vs 357 GiB/s: occupancy wins. */
template <int NR, bool DEC>
static hipError_t launch_gcm_aria(const GcmArgs &a, uint32_t grid, hipStream_t st, bool cid)
{
    static_assert(ARIA_GCM_WAVES == 16, "ARIA-GCM launch shape");
    if (cid)
        hipLaunchKernelGGL((tlsrec_gcm_kernel<8, NR, DEC, 16, 1, false, true, true>), dim3(grid), dim3(16 * 64), 0, st, a);
    else
        hipLaunchKernelGGL((tlsrec_gcm_kernel<8, NR, DEC, 16, 1, false, false, true>), dim3(grid), dim3(16 * 64), 0, st, a);
    return hipGetLastError();
}

/* key tables with DTLS connection IDs: one configuration (8 lanes, 16 waves) */
template <int NR, bool DEC>
static hipError_t launch_gcm_cid(const GcmArgs &a, uint32_t grid, hipStream_t st)
{
    hipLaunchKernelGGL((tlsrec_gcm_kernel<8, NR, DEC, 16, 1, false, true>), dim3(grid), dim3(16 * 64), 0, st, a);
    return hipGetLastError();
}

template <int L, int NR, bool DEC, int W>
static hipError_t launch_gcm_t(const GcmArgs &a, uint32_t grid, hipStream_t st)
{
    /* 16 waves x 1 block per lane, or 8 waves x 2 independent blocks per lane */
    if constexpr (W == 8) {
        hipLaunchKernelGGL((tlsrec_gcm_kernel<L, NR, DEC, 8, 2>), dim3(grid), dim3(8 * 64), 0, st, a);
    } else if constexpr (L == 1 << KEY_G5_POWER) {
        /* 8 lanes: the Horner multiplier H^8 from the 5-bit (G5) table */
        if (a.g5)
            hipLaunchKernelGGL((tlsrec_gcm_kernel<L, NR, DEC, 16, 1, false, false, false, true>), dim3(grid),
                               dim3(16 * 64), 0, st, a);
        else
            hipLaunchKernelGGL((tlsrec_gcm_kernel<L, NR, DEC, 16, 1>), dim3(grid), dim3(16 * 64), 0, st, a);
    } else {
        hipLaunchKernelGGL((tlsrec_gcm_kernel<L, NR, DEC, 16, 1>), dim3(grid), dim3(16 * 64), 0, st, a);
    }
    return hipGetLastError();
}

template <int L, bool DEC>
static hipError_t launch_gcm_nr(const GcmArgs &a, int nr, int waves, uint32_t grid, hipStream_t st)
{
    if (waves == -16) {  /* CID variant (engine: the key table holds connection IDs; L = 8) */
        if constexpr (L == 8) {
            if (nr == 10) return launch_gcm_cid<10, DEC>(a, grid, st);
            if (nr == 12) return launch_gcm_cid<12, DEC>(a, grid, st);
            if (nr == 14) return launch_gcm_cid<14, DEC>(a, grid, st);
        }
        return hipErrorInvalidValue;
    }
    if (waves == -32) {  /* paired wave passes (engine: many keys, small records) */
        if constexpr (L == 4 || L == 8 || L == 16) {
            if (nr == 10) return launch_gcm_pair<L, 10, DEC>(a, grid, st);
            if (nr == 14) return launch_gcm_pair<L, 14, DEC>(a, grid, st);
        }
        return hipErrorInvalidValue;
    }
    if (waves == -8) {   /* wave-pass variant (engine: many keys, few records each) */
        if constexpr (L == 4 || L == 16 || L == 64) {
            if (nr == 10) return launch_gcm_wp<L, 10, DEC>(a, grid, st);
            if (nr == 14) return launch_gcm_wp<L, 14, DEC>(a, grid, st);
        }
        return hipErrorInvalidValue;
    }
    if (nr == 12) return launch_gcm_t<L, 12, DEC, 16>(a, grid, st);   /* AES-192: 16-wave variant only */
    if (waves == 8)
        return nr == 10 ? launch_gcm_t<L, 10, DEC, 8>(a, grid, st) : launch_gcm_t<L, 14, DEC, 8>(a, grid, st);
    return nr == 10 ? launch_gcm_t<L, 10, DEC, 16>(a, grid, st) : launch_gcm_t<L, 14, DEC, 16>(a, grid, st);
}

template <bool DEC>
hipError_t gcm_dispatch(const GcmArgs &a, int lanes, int nr, int waves, uint32_t grid, hipStream_t st)
{
    switch (lanes) {
        case 2:   /* wave passes only */
            if (waves == -32) {
                if (nr == 10) return launch_gcm_pair<2, 10, DEC>(a, grid, st);
                if (nr == 14) return launch_gcm_pair<2, 14, DEC>(a, grid, st);
                return hipErrorInvalidValue;
            }
            if (waves != -8) return hipErrorInvalidValue;
            if (nr == 10) return launch_gcm_wp<2, 10, DEC>(a, grid, st);
            if (nr == 14) return launch_gcm_wp<2, 14, DEC>(a, grid, st);
            return hipErrorInvalidValue;
        case 4: return launch_gcm_nr<4, DEC>(a, nr, waves, grid, st);
        case 8: return launch_gcm_nr<8, DEC>(a, nr, waves, grid, st);
        case 16: return launch_gcm_nr<16, DEC>(a, nr, waves, grid, st);
        case 32:  /* paired wave passes only (a wave holds 2 records of a key) */
            if (waves != -32) return hipErrorInvalidValue;
            if (nr == 10) return launch_gcm_pair<32, 10, DEC>(a, grid, st);
            if (nr == 14) return launch_gcm_pair<32, 14, DEC>(a, grid, st);
            return hipErrorInvalidValue;
        case 64: return launch_gcm_nr<64, DEC>(a, nr, waves, grid, st);
        default: return hipErrorInvalidValue;
    }
}

/* ARIA (12/14/16 rounds) and Camellia (18/24) through the LDS-table cipher slot */
template <bool DEC>
hipError_t gcm_alt_dispatch(const GcmArgs &a, int nr, int cid, uint32_t grid, hipStream_t st)
{
    switch (nr) {
        case 12: return launch_gcm_aria<12, DEC>(a, grid, st, cid);
        case 14: return launch_gcm_aria<14, DEC>(a, grid, st, cid);
        case 16: return launch_gcm_aria<16, DEC>(a, grid, st, cid);
        case 18: return launch_gcm_aria<18, DEC>(a, grid, st, cid);
        case 24: return launch_gcm_aria<24, DEC>(a, grid, st, cid);
        default: return hipErrorInvalidValue;
    }
}

} /* namespace tlsrec */

#endif /* TLSREC_GCM_H */
