/*
 * server.hip -- the record server: a resident kernel that serves the
 * single-record entry points (tlsrec_encrypt_buf / tlsrec_decrypt_buf, the
 * drop-in for mbedtls_ssl_encrypt_buf / _decrypt_buf at ssl_msg.c:2697 and
 * :3835) without a kernel launch, a copy-engine transfer or a stream sync
 * per record.
 *
 * A call through the launch path costs ~10 us of launch + sync, ~12 us per
 * copy-engine transfer and the kernel's own table staging:
 * 33-41 us for a lone 1.4 KiB record.  Here each wave of a resident grid owns
 * one request slot in pinned, host-mapped memory and polls it:
 *
 *   host thread                          server wave (slot i)
 *   -----------                          --------------------
 *   copy record into slot i, desc  ->
 *   store hdr = (bytes, seq)       ->    sees hdr.seq != served (system-scope acquire)
 *                                        one burst: descriptor + record -> LDS
 *                                        AEAD in LDS (AES T-tables resident)
 *                                        record + result -> slot i (posted writes)
 *   spin on done == seq            <-    done = seq (system-scope release)
 *   copy record out
 *
 * AES-128/192/256-GCM and ChaCha20-Poly1305 without connection IDs, records up
 * to SRV_BUF bytes; everything else (CCM, ARIA, Camellia, CID transforms) stays
 * on the coalescing launch path in engine.hip, which is also the fallback
 * whenever the server cannot take a request.
 *
 * A record is served by one wave, 64 lanes, with the same framing plan and
 * the same results as the batch kernels (tlsrec_recdev.h):
 *   GCM: lane q takes the blocks j = q (mod 64) of the GHASH input A, C_1 ..
 *        C_m, LEN (j = 0 the AAD, whose counter block J0 gives E_K(J0)), each
 *        C block's keystream from the T-tables, a Horner chain per lane with
 *        H^64 (the key's 4-bit table staged to LDS), then Y_q * H^(n - j_last)
 *        (H^1 .. H^64 precomputed per key slot by the key setup, KEY_HPOW_OFF) and an
 *        XOR over the 64 lanes by DPP / permlane.
 *   ChaCha20-Poly1305: lane q makes ChaCha20 block q (+ 64 k), block 0 being
 *        the one-time Poly1305 key; Poly1305 runs the same lane-Horner form
 *        with r^64 and r^1 .. r^64 built in LDS by doubling.
 *
 * Termination: a server grid lives `life` ticks of the device wall clock
 * (TLSREC_SERVER_MS, default 20 ms) and at most `max_iter` polls, and leaves
 * early on the set's stop word (process exit, or batch work arriving: below)
 * or when no request of the set was claimed for `idle` ticks
 * (TLSREC_SERVER_IDLE_MS, default 1 ms), so a hipDeviceSynchronize after the
 * last single-record call waits about that long, not a whole window.  The
 * host submits to a grid only inside its window minus a margin and launches
 * the next grid on the other slot set when the window closes.
 *
 * The idle exit is ordered against host submits (r05, r06): before it posts
 * a request the host bumps the set's `activity` word and then reads `closing`
 * (both in host-mapped memory, a full fence between); the idle exit is
 * workgroup 0's alone: it writes `closing` = 1, fences, and re-reads
 * `activity` -- changed, it clears `closing` and stays.  Whichever of the two
 * stores comes first, one side sees the other's (Dekker), and a host that
 * read 1 does not post at all and launches the next grid on the other set.
 * A host that read `closing` = 0 posts its request and only then bumps
 * `settled` (a host that read 1 bumps it without posting): workgroup 0
 * commits the exit (the device-memory `quit` word, which the other
 * workgroups poll) only when `settled` has caught up with `activity`, so a
 * claim whose post is still in flight -- the host thread descheduled between
 * claim and post -- keeps the grid.  A workgroup that sees `quit` or `stop`
 * polls its slot once more before it leaves: a request posted before the
 * commit is served, never stranded.  `closing` stays 1 after a commit, so a
 * grid that left while no call came is found the same way.  A request a grid
 * never took (its kernel ended: a stop word racing a post) is withdrawn and
 * runs on the launch path.
 *
 * Yielding to batch work (r04): the grid holds 64 CUs (89 KiB of LDS each,
 * so no 128 KiB batch workgroup fits beside it).  Every batch launch outside
 * the single-record engine (tlsrec_batch_*, the stream / DTLS layers, the
 * host pipeline) calls tlsrec__server_yield before its kernels -- the live
 * grids get their stop word -- and tlsrec__server_note_batch after them,
 * which records an event on the batch's stream.  No grid is launched while
 * that event is pending; single-record calls meanwhile take the coalescing
 * launch path, whose kernels queue with the batch like any other work.
 */
#include <hip/hip_runtime.h>
#include <atomic>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "tlsrec.h"
#include "tlsrec_clmul.h"
#include "tlsrec_device.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"
#include "tlsrec_recdev.h"

using namespace tlsrec;

namespace {

constexpr int SRV_WAVES = 2;                        /* waves per workgroup: both serve its one request slot */
constexpr int SRV_GROUPS = 64;
constexpr int SRV_SLOTS = SRV_GROUPS;               /* 64 slots per set */
constexpr int SRV_LANES = SRV_WAVES * 64;           /* lanes per record */
constexpr uint32_t SRV_BUF = 17408;                 /* staged bytes per request (16 KiB record + room) */
constexpr int SRV_TAB_OFF = 65536;                  /* H^64 table (GCM, 8 KiB) / r^1..r^128 (ChaCha, 2.5 KiB) */
constexpr int SRV_STAGE_OFF = SRV_TAB_OFF + 8192;   /* the record */
constexpr int SRV_XCH_OFF = SRV_STAGE_OFF + (int) SRV_BUF;   /* wave 1 -> wave 0 partial sums, poll decisions */
constexpr int SRV_LDS = SRV_XCH_OFF + 256;
static_assert(SRV_LDS <= 160 * 1024, "server LDS budget");
static_assert(SRV_STAGE_OFF % 16 == 0 && SRV_XCH_OFF % 16 == 0, "16-byte aligned staging");

/* Request descriptor (lanes 0..8 read it as 16-byte chunks): the record's
 * batch descriptor and the framing plan the host computed for it with the
 * same code (tlsrec_frame.h; the explicit nonce of a TLS 1.2 GCM record
 * filled in from the record), so the device goes straight to the AEAD. */
struct SrvDesc {
    tlsrec_batch_rec d;       /* buf_off = alignment prefix, slot unused */
    uint32_t pad[4];
    tlsrec_plan p;
    uint8_t pad2[144 - 56 - sizeof(tlsrec_plan)];
};
static_assert(sizeof(SrvDesc) == 144, "SrvDesc layout");

/* What one poll reads (four 8-byte loads in flight together):
 *   w[0] = seq | staged bytes << 32 | cipher << 48 | dec << 56 | nr << 57 | skip << 62
 *          (skip: the test hook tlsrec__test_skip_record -- the request is
 *          answered with its INTERNAL_ERROR result and nothing else)
 *   w[1] = the slot's SlotState, w[2] its GHASH tables, w[3] its H^1 .. H^64
 *          (device addresses < 2^48), each | (seq & 0xffff) << 48
 * The host writes w[1..3] before w[0] (release); a poll that sees a new seq
 * in w[0] but an older one in w[1..3] read a request half-posted and polls
 * again.  So the wave knows the key slot at once and its key loads go out
 * with the record's. */
constexpr uint64_t SRV_PTR_MASK = (1ull << 48) - 1;

/* One request slot in pinned host memory mapped into the device. */
struct SrvReq {
    uint64_t w[4];
    uint8_t pad0[32];
    uint32_t done;            /* seq of the last request served (device writes) */
    uint8_t pad1[60];
    SrvDesc desc;
    tlsrec_batch_res res;
    uint64_t trace[10];       /* TLSREC_SERVER_TRACE: device wall-clock stamps of the request's phases */
    uint8_t pad3[16];
    uint8_t buf[SRV_BUF];
};
static_assert(offsetof(SrvReq, done) == 64 && offsetof(SrvReq, desc) == 128 && offsetof(SrvReq, res) == 272 &&
                  offsetof(SrvReq, buf) == 384 && sizeof(SrvReq) % 64 == 0,
              "SrvReq layout");

/* A set's control words in pinned host memory mapped into the device, one
 * cache line each (the idle-exit handshake above). */
struct SrvCtl {
    uint32_t stop;            /* host: leave now (process exit, batch work) */
    uint8_t pad0[60];
    uint32_t activity;        /* host: bumped before every post to this grid */
    uint8_t pad1[60];
    uint32_t closing;         /* workgroup 0: deciding to leave idle (1), or left */
    uint8_t pad2[60];
    uint32_t settled;         /* host: bumped after each claim's post (or after a claim that found closing = 1) */
    uint8_t pad3[60];
};
static_assert(offsetof(SrvCtl, activity) == 64 && offsetof(SrvCtl, closing) == 128 && offsetof(SrvCtl, settled) == 192 &&
                  sizeof(SrvCtl) == 256,
              "SrvCtl layout");

/* ---------------- LDS record access (16-byte aligned AEAD region) -------- */
__device__ __forceinline__ uint4 lds16(const uint8_t *p) { return *reinterpret_cast<const uint4 *>(p); }
__device__ __forceinline__ void sts16(uint8_t *p, uint4 v) { *reinterpret_cast<uint4 *>(p) = v; }

/* load_block (tlsrec_recdev.h) on the staged record */
__device__ __forceinline__ uint4 srv_load_block(const uint8_t *src, uint32_t pos, uint32_t content_len,
                                                uint32_t aead_len, uint8_t inner_type)
{
    uint4 v = lds16(src + pos);
    if (pos + 16 <= content_len) return v;
    v = mask_block(v, pos, content_len);
    if (content_len >= pos && content_len < pos + 16 && content_len < aead_len) {
        const uint32_t e = content_len - pos, sh = 8 * (e & 3), t = (uint32_t) inner_type << sh;
        if ((e >> 2) == 0) v.x |= t;
        else if ((e >> 2) == 1) v.y |= t;
        else if ((e >> 2) == 2) v.z |= t;
        else v.w |= t;
    }
    return v;
}

__device__ __forceinline__ void srv_store_block(uint8_t *dst, uint32_t pos, uint32_t len, uint4 v)
{
    if (pos + 16 <= len) {
        sts16(dst + pos, v);
        return;
    }
    const uint32_t w[4] = { v.x, v.y, v.z, v.w };
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        if (pos + i < len) dst[pos + i] = (uint8_t) (w[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t i)
{
    const uint32_t w = (i >> 2) == 0 ? v.x : ((i >> 2) == 1 ? v.y : ((i >> 2) == 2 ? v.z : v.w));
    return (w >> (8 * (i & 3))) & 0xffu;
}

__device__ __forceinline__ uint4 xor_all(uint4 v)
{
    auto x = [](uint32_t a, uint32_t b) { return a ^ b; };
    return make_uint4(group_reduce<64>(v.x, x), group_reduce<64>(v.y, x), group_reduce<64>(v.z, x),
                      group_reduce<64>(v.w, x));
}

/* x * y in GF(2^128) without tables (tlsrec_clmul.h) */
__device__ __forceinline__ uint4 srv_gfmul(uint4 x, uint4 y)
{
    const uint32_t a[4] = { x.x, x.y, x.z, x.w }, b[4] = { y.x, y.y, y.z, y.w };
    uint32_t r[4];
    tlsrec_gf128_mul(a, b, r);
    return make_uint4(r[0], r[1], r[2], r[3]);
}

/* ---------------- compact AES / ChaCha20 for the server ------------------ *
 * A served record is one wave on a SIMD with nothing else to run, so its
 * time is latency: a wave keeps at most 15 LDS requests in flight (lgkmcnt),
 * and on the box an AES-256 block took 2.3 us for one block per lane and 6.7
 * us for four interleaved (TLSREC_SERVER_TRACE) -- the LDS request rate of
 * one wave, not VALU issue.  So the rounds are a loop (a smaller request
 * path: same-box A/B against the batch kernels' unrolled AES, 1.4 KiB p50
 * 11.4-11.9 vs 12.0-13.2 us, 16 threads 387-406 K vs 282-335 K round trips/s,
 * profiles/r03m_server/ab_rolled_vs_unrolled.txt), each round's lookups all
 * issue before one wait, and the round keys sit one word per lane (lane i =
 * word i of the rotated schedule), four v_readlane per round. */
struct LaneKeys {
    uint32_t v;
    __device__ __forceinline__ uint32_t operator[](int i) const { return (uint32_t) __builtin_amdgcn_readlane(v, i); }
};

/* All 16 T-table lookups of a round for every block, then one wait: with a
 * single wave per SIMD nothing else hides the LDS latency, and left alone
 * the compiler interleaves each lookup's XOR right behind it (a wait per
 * couple of lookups).  The asm takes the lookups as operands, so every XOR
 * comes after it, and its memory clobber keeps every read before it. */
#define SRV_PIN16(t)                                                                                              \
    asm volatile("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]),       \
                      "+v"(t[7]), "+v"(t[8]), "+v"(t[9]), "+v"(t[10]), "+v"(t[11]), "+v"(t[12]), "+v"(t[13]),    \
                      "+v"(t[14]), "+v"(t[15]) : : "memory")

template <int NB>
__device__ __forceinline__ void srv_lookups(const uint8_t *lds, uint32_t lb, const uint32_t (&s)[NB][4], int last,
                                            uint32_t (&t)[NB][16])
{
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            /* middle rounds: T0 / T1 alternating; last round: T0 only (S-box bytes) */
            t[b][4 * c + 0] = tlook<0>(lds, s[b][c], lb, 0, 0);
            t[b][4 * c + 1] = tlook<0>(lds, s[b][(c + 1) & 3], lb, 1, last ? 0 : 1);
            t[b][4 * c + 2] = tlook<0>(lds, s[b][(c + 2) & 3], lb, 2, 0);
            t[b][4 * c + 3] = tlook<0>(lds, s[b][(c + 3) & 3], lb, 3, last ? 0 : 1);
        }
#pragma unroll
    for (int b = 0; b < NB; b++) SRV_PIN16(t[b]);
}

template <int NR, int NB>
__device__ __forceinline__ void srv_aes(const uint8_t *lds, uint32_t lb, LaneKeys rk, const uint4 (&in)[NB],
                                        uint4 (&out)[NB])
{
    uint32_t s[NB][4], t[NB][16];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        s[b][0] = in[b].x ^ rk[0];
        s[b][1] = in[b].y ^ rk[1];
        s[b][2] = in[b].z ^ rk[2];
        s[b][3] = in[b].w ^ rk[3];
    }
#pragma unroll 1
    for (int r = 1; r < NR; r++) {
        const uint32_t k[4] = { rk[4 * r], rk[4 * r + 1], rk[4 * r + 2], rk[4 * r + 3] };
        srv_lookups<NB>(lds, lb, s, 0, t);
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int c = 0; c < 4; c++)     /* rotated round keys: see aes_encrypt */
                s[b][c] = xor3(t[b][4 * c], t[b][4 * c + 1], rotl16(xor3(t[b][4 * c + 2], t[b][4 * c + 3], k[c])));
    }
    srv_lookups<NB>(lds, lb, s, 1, t);
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint32_t o[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {          /* last round: S[x] is byte 1 (and byte 2) of T0[x] */
            const uint32_t lo = __builtin_amdgcn_perm(t[b][4 * c + 1], t[b][4 * c], 0x0C0C0501u);
            const uint32_t hi = __builtin_amdgcn_perm(t[b][4 * c + 3], t[b][4 * c + 2], 0x06020C0Cu);
            o[c] = __builtin_amdgcn_bitop3_b32(lo, hi, rk[4 * NR + c], 0x56);
        }
        out[b] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

/* chacha_block (tlsrec_device.h) with the double rounds as a loop */
__device__ __forceinline__ void srv_chacha_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3],
                                                 uint32_t out[16])
{
    const uint32_t in[16] = { 0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                              key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                              counter, nonce[0], nonce[1], nonce[2] };
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = in[i];
#pragma unroll 1
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

/* Everything a served record needs, uniform over the wave (the AEAD's own
 * per-lane inputs -- H^64 table, closing power, round keys -- are passed
 * beside it). */
struct SrvJob {
    tlsrec_batch_rec d;
    tlsrec_plan p;
    uint8_t *rec;             /* the record's first byte in LDS (staging + d.buf_off) */
};

/* Tag handling shared by both AEADs: encrypt writes the tag and the explicit
 * nonce, decrypt compares, wipes on a mismatch (PSA zeroes the output) and
 * takes the TLS 1.3 inner type / length from the last non-zero byte. */
template <bool DEC>
__device__ __forceinline__ tlsrec_batch_res srv_finish(const SrvJob &J, uint4 tag, uint32_t nzkey, int lane)
{
    const tlsrec_plan &p = J.p;
    uint8_t *base = J.rec + p.aead_pos;
    tlsrec_batch_res r;
    r.data_offset = p.data_offset;
    r.data_len = p.data_len;
    r.cid_len = 0;
    r.reserved[0] = r.reserved[1] = 0;
    if (!DEC) {
        if (lane < 16) base[p.aead_len + lane] = (uint8_t) byte_of(tag, (uint32_t) lane);
        if (p.explicit_iv && p.post_status == 0 && lane < 8) {
            uint32_t c[2];
            __builtin_memcpy(c, J.d.ctr, 8);
            J.rec[p.data_offset + lane] = (uint8_t) (c[lane >> 2] >> (8 * (lane & 3)));
        }
        r.status = p.post_status;
        r.type = p.type;
        r.cid_len = p.cid_set ? p.cid_len : 0;
        return r;
    }
    uint32_t diff = lane < 16 ? (base[p.aead_len + lane] ^ byte_of(tag, (uint32_t) lane)) : 0u;
    diff = group_or<64>(diff);
    const uint32_t key = group_max<64>(nzkey);
    r.status = 0;
    r.type = J.d.type;
    if (diff != 0) {
        for (uint32_t i = p.aead_pos + (uint32_t) lane; i < J.d.buf_len; i += 64) J.rec[i] = 0;
        r.status = TLSREC_E_INVALID_MAC;
    } else if (p.inner) {                                  /* ssl_msg.c:1809-1829 */
        if (key == 0) {
            r.status = TLSREC_E_INVALID_RECORD;
        } else {
            r.data_len = (key >> 8) - 1;
            r.type = (uint8_t) (key & 0xff);
        }
    }
    return r;
}

__device__ __forceinline__ void nonce_of(const tlsrec_plan &p, uint32_t nw[3])
{
    nw[0] = ld_u32le(p.nonce);
    nw[1] = ld_u32le(p.nonce + 4);
    nw[2] = ld_u32le(p.nonce + 8);
}

/* ---------------- AES-GCM, one record per workgroup (2 waves) -------------- */
/* Lane g = 64 wave + lane of the workgroup takes the blocks j = g (mod 128)
 * of A, C_1 .. C_m, LEN.  tab: the key's H^64 table in LDS (the Horner
 * multiplier H^128 is two multiplies by it); hq: lane i of each wave holds
 * H^(i+1); rk: the round keys (rotated form); xch: wave 1's partial sums. */
template <int NR, bool DEC>
__device__ __forceinline__ tlsrec_batch_res srv_gcm(const SrvJob &J, const uint8_t *lds, const uint8_t *tab, uint4 hq,
                                                    LaneKeys rk, int wave, int lane, uint8_t *xch, uint64_t *tst)
{
    const tlsrec_plan &p = J.p;
    const uint32_t g = (uint32_t) (wave * 64 + lane);
    uint32_t nw[3];
    nonce_of(p, nw);
    const uint32_t m = (p.aead_len + 15) >> 4;         /* C blocks */
    const uint32_t n = m + 2;                          /* A, C_1 .. C_m, LEN */
    const uint32_t K = (n + SRV_LANES - 1) / SRV_LANES;
    const uint32_t content_len = DEC ? p.aead_len : p.content_len;
    uint8_t *base = J.rec + p.aead_pos;
    /* this lane's chain ends at j_last; it closes with H^d, d = n - j_last in
     * 1 .. 128: H^d = H^(d-64) * H^64 above 64 */
    const uint32_t kq = g < n ? (n - 1 - g) / SRV_LANES + 1 : 0;
    const uint32_t d = kq ? n - (g + SRV_LANES * (kq - 1)) : 1;
    const uint32_t dl = d > 64 ? d - 64 : d;
    const uint4 hd = make_uint4(__shfl(hq.x, (int) dl - 1), __shfl(hq.y, (int) dl - 1), __shfl(hq.z, (int) dl - 1),
                                __shfl(hq.w, (int) dl - 1));
    const uint32_t lanebase = (uint32_t) (lane & 31) << 2;
    const uint4 aadw = aad_words(p);
    const uint4 lenw = make_uint4(0, bswap32((uint32_t) p.aad_len * 8), 0, bswap32(p.aead_len * 8));
    uint4 Y = make_uint4(0, 0, 0, 0), ej0 = make_uint4(0, 0, 0, 0);
    uint32_t nzpos = 0;
    auto block = [&](uint32_t k, uint4 ks) {
        const uint32_t j = g + SRV_LANES * k;
        uint4 X = make_uint4(0, 0, 0, 0);
        if (j == 0) {
            ej0 = ks;
            X = aadw;
        } else if (j <= m) {
            const uint32_t pos = (j - 1) * 16;
            const uint4 blk = srv_load_block(base, pos, content_len, p.aead_len, p.inner_type);
            const uint4 o = mask_block(xor4(blk, ks), pos, p.aead_len);
            srv_store_block(base, pos, p.aead_len, o);
            X = DEC ? blk : o;
            if (DEC && p.inner && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
        } else if (j == m + 1) {
            X = lenw;
        }
        /* Horner by H^128 (one wait per table multiply) */
        if (j < n) Y = k ? xor4(gmul<0, 1>(tab, gmul<0, 1>(tab, Y)), X) : X;
    };
    /* four / two steps' counter blocks at a time: independent AES chains
     * interleave (a lane's AES is a dependent LDS round trip per round) */
    auto ctrb = [&](uint32_t c) { return make_uint4(nw[0], nw[1], nw[2], bswap32(c)); };
    uint32_t k = 0;
#pragma unroll 1
    for (; k + 3 < K; k += 4) {
        const uint32_t j = g + SRV_LANES * k;
        const uint4 x[4] = { ctrb(j + 1), ctrb(j + 1 + SRV_LANES), ctrb(j + 1 + 2 * SRV_LANES),
                             ctrb(j + 1 + 3 * SRV_LANES) };
        uint4 ks[4];
        srv_aes<NR, 4>(lds, lanebase, rk, x, ks);
        block(k, ks[0]);
        block(k + 1, ks[1]);
        block(k + 2, ks[2]);
        block(k + 3, ks[3]);
    }
    if (k + 1 < K) {
        const uint32_t j = g + SRV_LANES * k;
        const uint4 x[2] = { ctrb(j + 1), ctrb(j + 1 + SRV_LANES) };
        uint4 ks[2];
        srv_aes<NR, 2>(lds, lanebase, rk, x, ks);
        block(k, ks[0]);
        block(k + 1, ks[1]);
        k += 2;
    }
    if (k < K) {
        const uint4 x[1] = { ctrb(g + SRV_LANES * k + 1) };
        uint4 ks[1];
        srv_aes<NR, 1>(lds, lanebase, rk, x, ks);
        if (tst && k == 0) tst[2] = __builtin_amdgcn_readfirstlane((uint32_t) (ks[0].x ^ ks[0].y)) == 0x5bd1e995u
                                        ? 0 : wall_clock64();
        block(k, ks[0]);
    }
    if (tst) tst[0] = __builtin_amdgcn_readfirstlane((uint32_t) (Y.x ^ Y.y)) == 0x5bd1e995u ? 0 : wall_clock64();
    if (kq) {
        Y = srv_gfmul(Y, hd);
        if (d > 64) Y = gmul<0, 1>(tab, Y);
    }
    if (tst) tst[1] = __builtin_amdgcn_readfirstlane((uint32_t) (Y.x ^ Y.y)) == 0x5bd1e995u ? 0 : wall_clock64();
    uint4 S = xor_all(Y);
    uint32_t nzkey = 0;
    if (DEC && p.inner && nzpos)
        nzkey = last_nonzero_key(mask_block(lds16(base + nzpos - 1), nzpos - 1, p.aead_len), nzpos - 1);
    nzkey = group_max<64>(nzkey);
    uint32_t *x = reinterpret_cast<uint32_t *>(xch);
    if (wave == 1 && lane == 0) {
        x[0] = S.x; x[1] = S.y; x[2] = S.z; x[3] = S.w;
        x[4] = nzkey;
    }
    __syncthreads();
    tlsrec_batch_res r = {};
    if (wave == 0) {
        S = xor4(S, make_uint4(x[0], x[1], x[2], x[3]));
        nzkey = max(nzkey, x[4]);
        const uint4 e0 = make_uint4(__builtin_amdgcn_readlane(ej0.x, 0), __builtin_amdgcn_readlane(ej0.y, 0),
                                    __builtin_amdgcn_readlane(ej0.z, 0), __builtin_amdgcn_readlane(ej0.w, 0));
        r = srv_finish<DEC>(J, xor4(S, e0), nzkey, lane);
    }
    __syncthreads();                                   /* wave 0's tag / wipe land before the copy-out */
    return r;
}

/* ---------------- ChaCha20-Poly1305, one record per workgroup --------------- */
__device__ __forceinline__ P5 p_rd(const uint32_t *t) { P5 r; for (int i = 0; i < 5; i++) r.v[i] = t[i]; return r; }
__device__ __forceinline__ void p_wr(uint32_t *t, const P5 &v) { for (int i = 0; i < 5; i++) t[i] = v.v[i]; }

__device__ __forceinline__ P5 p_sum_all(P5 v, int lane)
{
    auto lvl = [&](auto sc) {
        constexpr int S = decltype(sc)::value;
        P5 w;
#pragma unroll
        for (int i = 0; i < 5; i++) w.v[i] = partner<S>(v.v[i], lane);
        v = p_add(v, w);
    };
    lvl(std::integral_constant<int, 1>());
    lvl(std::integral_constant<int, 2>());
    lvl(std::integral_constant<int, 4>());
    v = p_carry(v);                    /* 8 terms: limbs < 2^29 */
    lvl(std::integral_constant<int, 8>());
    lvl(std::integral_constant<int, 16>());
    lvl(std::integral_constant<int, 32>());
    return p_carry(v);
}

/* Poly1305 of A, C_1 .. C_M, LEN over the record's ciphertext in LDS:
 * sum_j X_j r^(n - j), lane g taking j = g (mod 128); this wave's part */
__device__ __forceinline__ P5 srv_poly(const uint8_t *base, const tlsrec_plan &p, const uint32_t *rpow, uint32_t g,
                                       int lane)
{
    const uint32_t M = (p.aead_len + 15) >> 4;
    const uint32_t n = M + 2;
    const uint32_t K = (n + SRV_LANES - 1) / SRV_LANES;
    const P5 r128 = p_rd(rpow + 5 * (SRV_LANES - 1));
    const uint4 aadw = aad_words(p);
    P5 Y = p_zero();
    for (uint32_t k = 0; k < K; k++) {
        const uint32_t j = g + SRV_LANES * k;
        if (j >= n) break;
        uint4 w;
        if (j == 0) w = aadw;
        else if (j <= M) w = mask_block(lds16(base + (j - 1) * 16), (j - 1) * 16, p.aead_len);
        else w = make_uint4(p.aad_len, 0, p.aead_len, 0);
        const P5 x = p_block(w);
        Y = k ? p_add(p_mul(Y, r128), x) : x;
    }
    const uint32_t kq = g < n ? (n - 1 - g) / SRV_LANES + 1 : 0;
    if (kq) Y = p_mul(Y, p_rd(rpow + 5 * (n - (g + SRV_LANES * (kq - 1)) - 1)));
    else Y = p_zero();
    return p_sum_all(Y, lane);
}

template <bool DEC>
__device__ __forceinline__ tlsrec_batch_res srv_chachapoly(const SrvJob &J, const uint32_t *key, uint8_t *tab,
                                                           int wave, int lane, uint8_t *xch)
{
    const tlsrec_plan &p = J.p;
    const uint32_t g = (uint32_t) (wave * 64 + lane);
    uint32_t nw[3];
    nonce_of(p, nw);
    const uint32_t B = (p.aead_len + 63) >> 6;         /* ChaCha20 blocks of data; counters 0 .. B */
    const uint32_t KC = (B + 1 + SRV_LANES - 1) / SRV_LANES;
    const uint32_t content_len = DEC ? p.aead_len : p.content_len;
    uint8_t *base = J.rec + p.aead_pos;
    uint32_t *x = reinterpret_cast<uint32_t *>(xch);

    /* step 0's keystream: lane g makes block g, g = 0 the one-time key */
    uint32_t ks0[16];
    srv_chacha_block(key, g, nw, ks0);
    /* r^1 .. r^128 in LDS: wave 0 doubles up to r^64, wave 1 multiplies by r^64 */
    uint32_t *rpow = reinterpret_cast<uint32_t *>(tab);
    if (wave == 0) {
        uint32_t r0[8];
#pragma unroll
        for (int i = 0; i < 8; i++) r0[i] = __builtin_amdgcn_readlane(ks0[i], 0);
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < 8; i++) x[8 + i] = r0[i];
        P5 rq = p_from_r(r0[0], r0[1], r0[2], r0[3]);
        if (lane == 0) p_wr(rpow, rq);
#pragma unroll
        for (int t = 0; t < 6; t++) {
            const int s = 1 << t;
            if (lane >= s && lane < 2 * s) {
                rq = p_mul(p_rd(rpow + 5 * (lane - s)), p_rd(rpow + 5 * (s - 1)));
                p_wr(rpow + 5 * lane, rq);
            }
            asm volatile("" ::: "memory");
        }
    }
    __syncthreads();
    if (wave == 1) p_wr(rpow + 5 * g, p_mul(p_rd(rpow + 5 * lane), p_rd(rpow + 5 * 63)));   /* r^(g+1) */
    __syncthreads();
    P5 h = p_zero();
    if (DEC) {
        h = srv_poly(base, p, rpow, g, lane);          /* over the ciphertext, before it is replaced */
        __syncthreads();
    }
    uint32_t nzpos = 0;
    for (uint32_t k = 0; k < KC; k++) {
        const uint32_t c = g + SRV_LANES * k;
        uint32_t ks[16];
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 16; i++) ks[i] = ks0[i];
        } else if (c <= B) {
            srv_chacha_block(key, c, nw, ks);
        }
        if (c >= 1 && c <= B) {
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const uint32_t pos = (c - 1) * 64 + 16 * t;
                if (pos < p.aead_len) {
                    const uint4 blk = srv_load_block(base, pos, content_len, p.aead_len, p.inner_type);
                    const uint4 o = mask_block(
                        xor4(blk, make_uint4(ks[4 * t], ks[4 * t + 1], ks[4 * t + 2], ks[4 * t + 3])), pos, p.aead_len);
                    srv_store_block(base, pos, p.aead_len, o);
                    if (DEC && p.inner && (o.x | o.y | o.z | o.w)) nzpos = pos + 1;
                }
            }
        }
    }
    if (!DEC) {
        __syncthreads();                               /* the whole ciphertext in LDS */
        h = srv_poly(base, p, rpow, g, lane);
    }
    uint32_t nzkey = 0;
    if (DEC && p.inner && nzpos)
        nzkey = last_nonzero_key(mask_block(lds16(base + nzpos - 1), nzpos - 1, p.aead_len), nzpos - 1);
    nzkey = group_max<64>(nzkey);
    if (wave == 1 && lane == 0) {
        p_wr(x, h);
        x[5] = nzkey;
    }
    __syncthreads();
    tlsrec_batch_res r = {};
    if (wave == 0) {
        h = p_carry(p_add(h, p_rd(x)));
        nzkey = max(nzkey, x[5]);
        const uint4 s = make_uint4(x[12], x[13], x[14], x[15]);
        r = srv_finish<DEC>(J, p_finish(h, s), nzkey, lane);
    }
    __syncthreads();                                   /* wave 0's tag / wipe land before the copy-out */
    return r;
}

__device__ __forceinline__ uint64_t ld_sys64(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t ld_sys32(const uint32_t *p)
{
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

__device__ __forceinline__ uint32_t comp(uint4 v, int i)
{
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

/* One request, both waves: the record, its descriptor and the key slot's data
 * in one burst of loads (record and descriptor over PCIe, key data from HBM),
 * the AEAD in LDS, the record and result back to the slot.  Called by both
 * waves with the same arguments: every branch around a barrier is uniform. */
__device__ __forceinline__ void srv_serve(SrvReq *rq, uint64_t w0, const SlotState *st, const uint4 *ghtab,
                                          const uint4 *hpw, const uint8_t *lds, int wave, int lane, uint32_t flags)
{
    const uint32_t trace = flags & 1u;
    const uint64_t ts0 = trace ? wall_clock64() : 0;
    const uint64_t cy0 = trace ? __builtin_readcyclecounter() : 0;
    uint64_t tsx[4] = { 0, 0, 0, 0 };
    uint64_t *tst = (trace && wave == 0) ? tsx : nullptr;
    uint8_t *L = const_cast<uint8_t *>(lds);
    uint8_t *tab = L + SRV_TAB_OFF, *stage = L + SRV_STAGE_OFF, *xch = L + SRV_XCH_OFF;
    const uint32_t g = (uint32_t) (wave * 64 + lane);
    const uint32_t bytes = (uint32_t) (w0 >> 32) & 0xffffu;
    const uint32_t cipher = (uint32_t) (w0 >> 48) & 0xffu;
    const bool dec = (w0 >> 56) & 1u;
    const uint32_t nr = (uint32_t) (w0 >> 57) & 0x1fu;
    const bool skip = TLSREC_HOOK_SKIP(1u, (uint32_t) (w0 >> 62) & 1u);
    const bool gcm = cipher != TLSREC_CIPHER_CHACHA20_POLY1305;
    const uint32_t n16 = bytes > SRV_BUF ? 0u : (bytes + 15) / 16;
    /* descriptor chunks (lanes 0..8) and key material (lanes 0..3) in each
     * wave; the rotated round keys one word per lane, this lane's H^(lane+1),
     * half of the H^64 table per wave (GCM); every 16-byte chunk of the
     * record, split over the two waves */
    const uint4 dc = lane < 9 ? gload16(reinterpret_cast<const uint8_t *>(&rq->desc) + 16 * lane) : make_uint4(0, 0, 0, 0);
    const uint8_t *sp = reinterpret_cast<const uint8_t *>(st);
    const uint4 sc = lane < 4 ? gload16(sp + 16 * lane) : make_uint4(0, 0, 0, 0);
    LaneKeys rk;
    rk.v = (gcm && lane < 60) ? st->rkr[lane] : 0u;
    uint4 hq = make_uint4(0, 0, 0, 0), ht[4];
    if (gcm) {
        hq = hpw[lane];
#pragma unroll
        for (int i = 0; i < 4; i++) ht[i] = ghtab[6 * 512 + g + SRV_LANES * i];
    }
    constexpr int NCH = (int) (SRV_BUF / 16 + SRV_LANES - 1) / SRV_LANES;
    uint4 r[NCH];
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        const uint32_t i = g + (uint32_t) SRV_LANES * k;
        if (i < n16) r[k] = gload16(rq->buf + 16 * i);
    }
#pragma unroll
    for (int k = 0; k < NCH; k++) {
        const uint32_t i = g + (uint32_t) SRV_LANES * k;
        if (i < n16) sts16(stage + 16 * i, r[k]);
    }
    if (gcm) {
#pragma unroll
        for (int i = 0; i < 4; i++) sts16(tab + 16 * (g + SRV_LANES * i), ht[i]);
    }
    uint32_t w[36];
#pragma unroll
    for (int i = 0; i < 36; i++) w[i] = __builtin_amdgcn_readlane(comp(dc, i & 3), i >> 2);
    SrvJob J;
    __builtin_memcpy(&J.d, w, sizeof(J.d));
    __builtin_memcpy(&J.p, w + 14, sizeof(J.p));
    J.rec = stage + J.d.buf_off;
    uint32_t kw[16];
#pragma unroll
    for (int i = 0; i < 16; i++) kw[i] = __builtin_amdgcn_readlane(comp(sc, i & 3), i >> 2);
    const uint32_t km_cipher = kw[0] & 0xffu, km_cid = (kw[1] >> 8) & 0xffu;
    tlsrec_batch_res res;
    res.status = TLSREC_ERR_SSL_INTERNAL_ERROR;
    res.data_offset = res.data_len = 0;
    res.type = res.cid_len = 0;
    res.reserved[0] = res.reserved[1] = 0;
    /* the host checked these; a request outside them is refused, not served.
     * Wave 0's verdict goes to both waves through LDS: the AEAD below has
     * barriers, so the branch must be the same in both */
    uint32_t *x = reinterpret_cast<uint32_t *>(xch);
    if (wave == 0 && lane == 0)
        x[20] = (!skip && n16 != 0 && (uint64_t) J.d.buf_off + J.d.buf_len + 32 <= SRV_BUF && J.d.cid_len == 0 &&
                 km_cipher == cipher && km_cid == 0 && J.p.status == 0 && J.p.cid_len == 0 &&
                 (uint64_t) J.p.aead_pos + J.p.aead_len + 16 <= J.d.buf_len &&
                 ((J.d.buf_off + J.p.aead_pos) & 15) == 0) ? 1u : 0u;
    if (trace) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   /* tracing: every load landed */
    const uint64_t ts1 = trace ? wall_clock64() : 0;
    __syncthreads();                                   /* the staged record and table, both halves; the verdict */
    const bool ok = __builtin_amdgcn_readfirstlane(x[20]) != 0;
    if (ok) {
        if (!gcm) {
            const uint32_t *key = kw + 8;              /* tlsrec_key_material.key at byte 32 */
            res = dec ? srv_chachapoly<true>(J, key, tab, wave, lane, xch)
                      : srv_chachapoly<false>(J, key, tab, wave, lane, xch);
        } else if (nr == 10 && cipher == TLSREC_CIPHER_AES_128_GCM) {
            res = dec ? srv_gcm<10, true>(J, lds, tab, hq, rk, wave, lane, xch, tst)
                      : srv_gcm<10, false>(J, lds, tab, hq, rk, wave, lane, xch, tst);
        } else if (nr == 14 && cipher == TLSREC_CIPHER_AES_256_GCM) {
            res = dec ? srv_gcm<14, true>(J, lds, tab, hq, rk, wave, lane, xch, tst)
                      : srv_gcm<14, false>(J, lds, tab, hq, rk, wave, lane, xch, tst);
        } else if (nr == 12 && cipher == TLSREC_CIPHER_AES_192_GCM) {
            res = dec ? srv_gcm<12, true>(J, lds, tab, hq, rk, wave, lane, xch, tst)
                      : srv_gcm<12, false>(J, lds, tab, hq, rk, wave, lane, xch, tst);
        }
    }
    const uint64_t ts2 = trace ? wall_clock64() : 0;
    const uint64_t cy2 = trace ? __builtin_readcyclecounter() : 0;
    if (trace && wave == 0 && lane == 0) {
        rq->trace[0] = ts0;
        rq->trace[1] = ts1;
        rq->trace[2] = ts2;
        rq->trace[4] = tsx[0];
        rq->trace[5] = tsx[1];
        rq->trace[6] = cy2 - cy0;
        rq->trace[7] = tsx[2] ? tsx[2] - ts1 : 0;
        rq->trace[8] = 0;
    }
    /* the record (whole staged range, both halves) and the result back to the slot */
    if (ok)
        for (uint32_t i = g; i < n16; i += SRV_LANES) gstore16(rq->buf + 16 * i, lds16(stage + 16 * i));
    if (wave == 0 && lane == 0) {
        uint4 rv;
        __builtin_memcpy(&rv, &res, sizeof(rv));
        gstore16(reinterpret_cast<uint8_t *>(&rq->res), rv);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      /* this wave's record stores, system scope */
    __syncthreads();                                   /* ... and the other wave's */
}

} /* namespace */

/* The resident grid: workgroup b (two waves, one per SIMD pair) owns request
 * slot b.  Wave 0 polls; every poll's verdict goes to wave 1 through LDS
 * (double-buffered by poll parity) behind one barrier, so both waves leave
 * the loop together.  At most one wave per SIMD (the LDS holds one workgroup
 * per CU): the compiler is told to schedule for one wave per EU -- all
 * lookups of an AES round in flight together. */
__global__ __launch_bounds__(SRV_WAVES * 64) __attribute__((amdgpu_waves_per_eu(1, 1))) void tlsrec_server_kernel(
    SrvReq *reqs, SrvCtl *sc, uint64_t life_ticks, uint32_t max_iter, uint32_t flags, uint32_t *quit,
    uint64_t idle_ticks)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[SRV_LDS];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    aes_fill_tables(lds, tid, SRV_WAVES * 64);
    SrvReq *rq = reqs + blockIdx.x;
    uint32_t *ctl = reinterpret_cast<uint32_t *>(lds + SRV_XCH_OFF + 128);   /* [2][10] poll verdicts */
    __syncthreads();
    const uint64_t t0 = wall_clock64();
    uint32_t served = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&rq->done, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_SYSTEM));
    uint32_t idle = 0;
    /* workgroup 0's idle clock: the activity word as last seen, and when it changed */
    uint32_t a_seen = blockIdx.x == 0 ? ld_sys32(&sc->activity) : 0u;
    uint64_t t_seen = t0;
    for (uint32_t it = 0;; it++) {
        uint32_t *c = ctl + (it & 1) * 10;
        if (wave == 0) {
            /* verdict: 0 idle, 1 serve, 2 leave, 3 poll again at once */
            uint32_t v = 2;
            uint64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
            if (it < max_iter) {
                h0 = ld_sys64(&rq->w[0]);
                h1 = ld_sys64(&rq->w[1]);
                h2 = ld_sys64(&rq->w[2]);
                h3 = ld_sys64(&rq->w[3]);
                const uint32_t seq = __builtin_amdgcn_readfirstlane((uint32_t) h0);
                if (seq != served) {
                    const uint64_t tagw = (uint64_t) (seq & 0xffffu) << 48;
                    v = (((h1 ^ tagw) | (h2 ^ tagw) | (h3 ^ tagw)) >> 48) ? 3u : 1u;   /* half-posted: again */
                    v = __builtin_amdgcn_readfirstlane(v);
                } else if ((it & 15) == 0 &&
                           (ld_sys32(&sc->stop) != 0 ||
                            __builtin_amdgcn_readfirstlane(
                                __hip_atomic_load(quit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) != 0)) {
                    v = 2;
                } else {
                    const uint64_t now = wall_clock64();
                    v = (uint64_t) (now - t0) > life_ticks ? 2u : 0u;
                    if (blockIdx.x == 0 && (it & 15) == 8 && v == 0) {
                        /* the idle exit (workgroup 0 for the grid): no claim
                         * seen for idle_ticks -> closing = 1, fence, re-read */
                        const uint32_t a = ld_sys32(&sc->activity);
                        if (a != a_seen) {
                            a_seen = a;
                            t_seen = now;
                        } else if (now - t_seen > idle_ticks) {
                            __hip_atomic_store(&sc->closing, 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                            const uint32_t a2 = __builtin_amdgcn_readfirstlane(
                                __hip_atomic_load(&sc->activity, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM));
                            const uint32_t s2 = __builtin_amdgcn_readfirstlane(
                                __hip_atomic_load(&sc->settled, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM));
                            if (a2 == a_seen && s2 == a2) {
                                /* committed: every claim so far has posted (or backed off); the
                                 * other workgroups leave at their next stop check, after one
                                 * more poll of their slot */
                                __hip_atomic_store(quit, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                                v = 2u;
                            } else {
                                /* a claim landed, or one is still posting: stay (a host that
                                 * claims now reads closing = 0) */
                                __hip_atomic_store(&sc->closing, 0u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
                                a_seen = a2;
                                t_seen = now;
                            }
                        }
                    }
                }
                if (v == 2u && seq == served) {
                    /* leaving (stop, quit, window or idle exit): poll the slot once more,
                     * after the decision -- a request posted before the commit is served */
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                    h0 = ld_sys64(&rq->w[0]);
                    h1 = ld_sys64(&rq->w[1]);
                    h2 = ld_sys64(&rq->w[2]);
                    h3 = ld_sys64(&rq->w[3]);
                    const uint32_t s2 = __builtin_amdgcn_readfirstlane((uint32_t) h0);
                    if (s2 != served) {
                        const uint64_t tagw = (uint64_t) (s2 & 0xffffu) << 48;
                        /* half-posted: poll again (the host's w[0] follows w[1..3]) */
                        v = __builtin_amdgcn_readfirstlane((((h1 ^ tagw) | (h2 ^ tagw) | (h3 ^ tagw)) >> 48) ? 3u : 1u);
                    }
                }
            }
            if (lane == 0) {
                c[0] = v;
                c[1] = (uint32_t) h0; c[2] = (uint32_t) (h0 >> 32);
                c[3] = (uint32_t) h1; c[4] = (uint32_t) (h1 >> 32);
                c[5] = (uint32_t) h2; c[6] = (uint32_t) (h2 >> 32);
                c[7] = (uint32_t) h3; c[8] = (uint32_t) (h3 >> 32);
            }
        }
        __syncthreads();
        const uint32_t v = __builtin_amdgcn_readfirstlane(c[0]);
        if (v == 2) break;
        if (v == 1) {
            /* (readfirstlane returns int: widen through uint32_t, never sign-extend) */
            auto u64 = [&](int i) {
                return (uint64_t) (uint32_t) __builtin_amdgcn_readfirstlane(c[i]) |
                       (uint64_t) (uint32_t) __builtin_amdgcn_readfirstlane(c[i + 1]) << 32;
            };
            const uint64_t a0 = u64(1);
            /* synchronizes with the host's release of w[0]: the record and
             * descriptor it wrote before are visible to the loads below */
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            srv_serve(rq, a0, reinterpret_cast<const SlotState *>(u64(3) & SRV_PTR_MASK),
                      reinterpret_cast<const uint4 *>(u64(5) & SRV_PTR_MASK),
                      reinterpret_cast<const uint4 *>(u64(7) & SRV_PTR_MASK), lds, wave, lane, flags);
            const uint32_t seq = (uint32_t) a0;
            if (wave == 0 && lane == 0) {
                if (flags & 1u) {
                    rq->trace[3] = wall_clock64();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                }
                __hip_atomic_store(&rq->done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            served = seq;
            idle = 0;
        } else if (v == 0 && wave == 0) {
            /* a slot idle for ~1 ms polls every few us instead of every ~2 us
             * (the host hands out the lowest free slot, so busy slots stay hot) */
            if (++idle > 512) __builtin_amdgcn_s_sleep(127);
            else __builtin_amdgcn_s_sleep(8);
        }
    }
}

/* ======================================================================
 * Host side
 * ==================================================================== */
namespace {

struct SrvSet {
    SrvReq *h = nullptr, *d = nullptr;
    SrvCtl *ctl_h = nullptr, *ctl_d = nullptr;
    uint32_t *quit = nullptr;         /* device: workgroup 0 committed to the idle exit */
    uint32_t activity = 0;            /* host copy of ctl_h->activity */
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    bool launched = false;
    uint64_t t_launch = 0;
    uint32_t seq[SRV_SLOTS] = {};
    uint8_t busy[SRV_SLOTS] = {};
    uint32_t nbusy = 0;
};

pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
SrvSet g_set[2];
int g_cur = 0;
int g_state = 0;                  /* 0 not yet set up, 1 ready, -1 unavailable */
std::atomic<int> g_enabled{1};
int g_debug = 0;                  /* TLSREC_SERVER_DEBUG=1: one line per request on stderr */
int g_trace = 0;                  /* TLSREC_SERVER_TRACE=1: device phase times, summed, printed at exit */
uint64_t g_tr_n = 0, g_tr_sum[3] = { 0, 0, 0 }, g_tr_aes = 0, g_tr_mul = 0, g_tr_gcm = 0, g_tr_cyc = 0, g_tr_a1 = 0,
         g_tr_b1 = 0;
double g_tick_ns = 10.0;
uint64_t g_submit_ns = 0, g_life_ticks = 0, g_idle_ticks = 0;
/* A waiting host thread spins while the waiting threads fit the process's
 * CPUs and yields its CPU between polls once they do not (r06): with 32
 * calling threads on the box's 16 CPUs pure spinning kept descheduled
 * threads -- whose requests were done, or not yet posted -- off the CPUs
 * for milliseconds, and 7-9 of 128 K calls went to the launch path (a set
 * switch waiting on an unanswered slot, a grid ending before a late post);
 * yielding had none.  At 16 threads spinning stays ahead (same box, 3 reps,
 * profiles/r06/ab/threads_*.jsonl).  TLSREC_SERVER_SPIN_US: < 0 spin
 * always, >= 0 yield after that long always.  Parking on a futex behind a
 * poller thread measured slower than both (a parked call waits for its
 * wake-up). */
int64_t g_spin_ns = -2;                   /* -2: adaptive (above) */
std::atomic<uint32_t> g_waiting{0};
uint32_t g_ncpu = 1;
/* batch work (tlsrec__server_yield / _note_batch): no grid while any is
 * queued or pending.  Batches may run on several streams at once: each
 * records its own event in a small ring, and the batches between their yield
 * and their note (kernels still being queued) are counted. */
int g_yield = 1;                  /* TLSREC_SERVER_YIELD=0: the server ignores batch work */
constexpr int BATCH_EVS = 16;
hipEvent_t g_batch_ev[BATCH_EVS] = {};
uint32_t g_batch_pending = 0;     /* bit k: event k recorded, not yet seen complete */
uint32_t g_batch_next = 0;
uint32_t g_batch_queueing = 0;    /* batches between tlsrec__server_yield and _note_batch */
std::atomic<uint64_t> g_yields{0};
/* why a call took the launch path: batch work pending, the other set not
 * drained, the grid gone before it took the request (tlsrec__server_why);
 * claims that found a grid closing (and moved to the other set) */
uint64_t g_why_batch = 0, g_why_drain = 0, g_why_withdrawn = 0, g_why_noslot = 0, g_closing = 0;
uint32_t g_max_iter = 0;
#ifdef TLSREC_TEST_HOOKS
/* TLSREC_TEST_SERVER_POST_DELAY_US (test-hooks build only): a host thread
 * that has claimed a slot waits this long before it posts -- the descheduled
 * host thread of the idle-exit handshake, made deterministic */
uint64_t g_test_post_delay_ns = 0;
#endif
std::atomic<uint64_t> g_served{0}, g_fallback{0}, g_launches{0};

uint64_t now_ns()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t) t.tv_sec * 1000000000ull + (uint64_t) t.tv_nsec;
}

void srv_shutdown()
{
    pthread_mutex_lock(&g_mu);
    for (auto &S : g_set) {
        if (S.launched) {
            __atomic_store_n(&S.ctl_h->stop, 1u, __ATOMIC_RELEASE);
            const hipError_t e = hipEventSynchronize(S.ev);
            if (g_debug) fprintf(stderr, "tlsrec server: shutdown, grid drained: %s\n", hipGetErrorString(e));
            S.launched = false;
        }
        if (S.quit) (void) hipFree(S.quit);
        S.quit = nullptr;
    }
    for (auto &e : g_batch_ev)
        if (e) {
            (void) hipEventSynchronize(e);
            (void) hipEventDestroy(e);
            e = nullptr;
        }
    g_state = -1;
    if (g_trace && g_tr_n)
        fprintf(stderr, "{\"server_trace\": {\"requests\": %llu, \"load_us\": %.2f, \"aead_us\": %.2f, "
                        "\"writeback_us\": %.2f}}\n",
                (unsigned long long) g_tr_n, g_tr_sum[0] * g_tick_ns / 1e3 / g_tr_n,
                g_tr_sum[1] * g_tick_ns / 1e3 / g_tr_n, g_tr_sum[2] * g_tick_ns / 1e3 / g_tr_n);
    if (g_trace && g_tr_n)
        fprintf(stderr, "{\"server_trace_detail\": {\"gcm_to_horner_end_us\": %.2f, \"gcm_final_mul_us\": %.2f, "
                        "\"first_aes_call_us\": %.2f, \"first_blocks_us\": %.2f, \"clock_ghz\": %.3f}}\n",
                g_tr_gcm ? g_tr_aes * g_tick_ns / 1e3 / g_tr_gcm : 0.0, g_tr_gcm ? g_tr_mul * g_tick_ns / 1e3 / g_tr_gcm : 0.0,
                g_tr_gcm ? g_tr_a1 * g_tick_ns / 1e3 / g_tr_gcm : 0.0, g_tr_gcm ? g_tr_b1 * g_tick_ns / 1e3 / g_tr_gcm : 0.0,
                (double) g_tr_cyc / ((double) (g_tr_sum[0] + g_tr_sum[1]) * g_tick_ns));
    pthread_mutex_unlock(&g_mu);
}

int srv_setup_locked()
{
    if (g_state) return g_state;
    g_state = -1;
    g_debug = getenv("TLSREC_SERVER_DEBUG") != nullptr;
    g_trace = getenv("TLSREC_SERVER_TRACE") != nullptr;
    const char *e = getenv("TLSREC_SERVER");
    if (e && strcmp(e, "0") == 0) return g_state;
    double ms = 20.0;
    if (const char *m = getenv("TLSREC_SERVER_MS")) ms = atof(m);
    if (!(ms >= 1.0)) ms = 1.0;
    if (ms > 200.0) ms = 200.0;
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        return g_state;
    g_life_ticks = (uint64_t) (ms * khz);
    double idle_ms = 1.0;
    if (const char *m = getenv("TLSREC_SERVER_IDLE_MS")) idle_ms = atof(m);
    if (!(idle_ms >= 0.05)) idle_ms = 0.05;
    if (idle_ms > ms) idle_ms = ms;
    g_idle_ticks = (uint64_t) (idle_ms * khz);
    if (const char *y = getenv("TLSREC_SERVER_YIELD")) g_yield = strcmp(y, "0") != 0;
    if (const char *sp = getenv("TLSREC_SERVER_SPIN_US")) g_spin_ns = (int64_t) (atof(sp) * 1e3);
    {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        const int nc = sched_getaffinity(0, sizeof(cs), &cs) == 0 ? CPU_COUNT(&cs) : 1;
        g_ncpu = nc > 0 ? (uint32_t) nc : 1u;
        /* a cgroup CPU quota caps it (a container sees every CPU of the host) */
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = { 0 };
            unsigned long long per = 0;
            if (fscanf(f, "%31s %llu", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
                const unsigned long long c = (strtoull(q, nullptr, 10) + per - 1) / per;
                if (c > 0 && c < g_ncpu) g_ncpu = (uint32_t) c;
            }
            fclose(f);
        }
    }
#ifdef TLSREC_TEST_HOOKS
    if (const char *d = getenv("TLSREC_TEST_SERVER_POST_DELAY_US")) g_test_post_delay_ns = (uint64_t) (atof(d) * 1e3);
#endif
    g_tick_ns = 1e6 / khz;
    g_max_iter = (uint32_t) (ms * 10000.0);          /* backstop: a poll (a PCIe read + s_sleep) is > 0.1 us */
    const double margin = ms * 0.1 > 1.0 ? ms * 0.1 : 1.0;
    g_submit_ns = (uint64_t) ((ms - margin) * 1e6);
    for (auto &S : g_set) {
        void *hd = nullptr, *sd = nullptr;
        if (hipHostMalloc((void **) &S.h, sizeof(SrvReq) * SRV_SLOTS, hipHostMallocMapped | hipHostMallocCoherent) !=
                hipSuccess ||
            hipHostGetDevicePointer(&hd, S.h, 0) != hipSuccess ||
            hipHostMalloc((void **) &S.ctl_h, sizeof(SrvCtl), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer(&sd, S.ctl_h, 0) != hipSuccess ||
            hipStreamCreateWithFlags(&S.st, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&S.ev, hipEventDisableTiming) != hipSuccess ||
            hipMalloc((void **) &S.quit, 64) != hipSuccess || hipMemset(S.quit, 0, 64) != hipSuccess)
            return g_state;
        memset(S.h, 0, sizeof(SrvReq) * SRV_SLOTS);
        memset(S.ctl_h, 0, sizeof(SrvCtl));
        S.d = (SrvReq *) hd;
        S.ctl_d = (SrvCtl *) sd;
    }
    for (auto &e : g_batch_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return g_state;
    atexit(srv_shutdown);
    g_state = 1;
    return g_state;
}

bool kernel_done(SrvSet &S) { return !S.launched || hipEventQuery(S.ev) != hipErrorNotReady; }

/* every slot of S that a host thread holds has its request answered (done ==
 * the posted sequence number); an unanswered one is about to be withdrawn by
 * its thread, and a new grid must not serve it behind that thread's back */
bool held_slots_served(SrvSet &S)
{
    if (S.nbusy == 0) return true;
    for (int k = 0; k < SRV_SLOTS; k++)
        if (S.busy[k] && __atomic_load_n(&S.h[k].done, __ATOMIC_ACQUIRE) != S.seq[k]) return false;
    return true;
}

/* Under g_mu: the set to submit to, launching the next grid when the current
 * one's window has closed; NULL = not now (the caller takes the launch path). */
SrvSet *srv_current_locked(uint64_t now)
{
    SrvSet *S = &g_set[g_cur];
    /* inside its window (an idle exit is found by the caller's claim) */
    if (S->launched && S->t_launch != 0 && now - S->t_launch < g_submit_ns) return S;
    /* batch work queued or pending on the device: the launch path, no grid beside it */
    if (g_batch_queueing) {
        g_why_batch++;
        return nullptr;
    }
    for (uint32_t m = g_batch_pending; m; m &= m - 1) {
        const int k = __builtin_ctz(m);
        if (hipEventQuery(g_batch_ev[k]) == hipErrorNotReady) {
            g_why_batch++;
            return nullptr;
        }
        g_batch_pending &= ~(1u << k);
    }
    SrvSet *N = &g_set[g_cur ^ 1];
    /* the other set must be drained: its grid ended, and every slot a host
     * thread still holds was served -- its thread, descheduled past the
     * window (more calling threads than CPUs), only reads its result back,
     * which the next grid never touches: it serves a slot only when a new
     * sequence number is posted there (r06: waiting for those threads to run
     * sent 30-90 of 128 K calls at 32 threads to the launch path) */
    if (!kernel_done(*N) || !held_slots_served(*N)) {
        g_why_drain++;
        return nullptr;
    }
    __atomic_store_n(&N->ctl_h->stop, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(&N->ctl_h->closing, 0u, __ATOMIC_SEQ_CST);
    (void) hipGetLastError();         /* an earlier call's status (hipEventQuery's NotReady) is not the launch's */
    /* quit = 0 in stream order ahead of the grid (the previous grid may have set it) */
    hipError_t le = hipMemsetAsync(N->quit, 0, sizeof(uint32_t), N->st);
    if (le == hipSuccess) {
        hipLaunchKernelGGL(tlsrec_server_kernel, dim3(SRV_GROUPS), dim3(SRV_WAVES * 64), 0, N->st, N->d, N->ctl_d,
                           g_life_ticks, g_max_iter, (uint32_t) g_trace, N->quit, g_idle_ticks);
        le = hipGetLastError();
    }
    if (le != hipSuccess || hipEventRecord(N->ev, N->st) != hipSuccess) {
        if (g_debug) fprintf(stderr, "tlsrec server: launch failed: %s\n", hipGetErrorString(le));
        g_state = -1;
        return nullptr;
    }
    N->launched = true;
    N->t_launch = now;
    g_cur ^= 1;
    g_launches++;
    return N;
}

} /* namespace */

/* Serve one record.  `plan` is the record's framing plan (tlsrec_frame.h, as
 * tlsrec_encrypt_buf / _decrypt_buf computed it; status 0).  Returns 0 with
 * *out and buf filled in, 1 when the server did not take the request (the
 * caller runs the launch path), or an error. */
extern "C" int tlsrec__server_run(int dec, uint32_t cipher, uint32_t nr, const tlsrec_batch_rec *rec,
                                  const void *slot_state, const void *ghtab, const void *hpw, unsigned char *buf,
                                  size_t buf_len, const void *plan, int skip, tlsrec_batch_res *out)
{
    if (!g_enabled.load(std::memory_order_relaxed) || g_state < 0 || plan == nullptr) return 1;
    const tlsrec_plan *pl = (const tlsrec_plan *) plan;
    if (pl->status != 0 || pl->cid_len != 0) return 1;
    const uint32_t pre = (16u - (pl->aead_pos & 15u)) & 15u;
    if ((uint64_t) pre + buf_len + 32 > SRV_BUF) return 1;
    pthread_mutex_lock(&g_mu);
    if (srv_setup_locked() != 1) {
        pthread_mutex_unlock(&g_mu);
        return 1;
    }
    SrvSet *S = nullptr;
    int i = -1;
    /* at most two sets: a claim that finds the current grid closing moves to
     * the other set (launching its grid) */
    for (int attempt = 0; attempt < 2 && i < 0; attempt++) {
        S = srv_current_locked(now_ns());
        if (!S) break;
        for (int k = 0; k < SRV_SLOTS; k++)
            if (!S->busy[k]) { i = k; break; }
        if (i < 0) {
            g_why_noslot++;
            break;
        }
        /* the claim: activity, full fence, closing (workgroup 0 does the
         * mirror image before it leaves idle) */
        __atomic_store_n(&S->ctl_h->activity, ++S->activity, __ATOMIC_SEQ_CST);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        if (__atomic_load_n(&S->ctl_h->closing, __ATOMIC_SEQ_CST) != 0) {
            __atomic_fetch_add(&S->ctl_h->settled, 1u, __ATOMIC_SEQ_CST);   /* backed off: settled, no post */
            S->t_launch = 0;          /* leaving or left: never submit to it again */
            g_closing++;
            i = -1;
            S = nullptr;
        }
    }
    if (i < 0) {
        pthread_mutex_unlock(&g_mu);
        g_fallback++;
        return 1;
    }
    S->busy[i] = 1;
    S->nbusy++;
    const uint32_t seq = ++S->seq[i];
    pthread_mutex_unlock(&g_mu);
#ifdef TLSREC_TEST_HOOKS
    if (g_test_post_delay_ns) {
        const uint64_t until = now_ns() + g_test_post_delay_ns;
        while (now_ns() < until) __builtin_ia32_pause();
    }
#endif

    SrvReq *rq = &S->h[i];
    if (buf_len) memcpy(rq->buf + pre, buf, buf_len);
    SrvDesc &D = rq->desc;
    D.d = *rec;
    D.d.buf_off = pre;
    D.d.slot = 0;
    D.p = *pl;
    /* TLS 1.2 GCM decrypt: nonce bytes 4..11 are the record's explicit IV
     * (ssl_msg.c:1352-1365, the kernels' nonce_words) */
    if (dec && pl->explicit_iv) memcpy(D.p.nonce + 4, buf + rec->data_offset, 8);
    const uint64_t tag = (uint64_t) (seq & 0xffffu) << 48;
    if (g_debug)
        fprintf(stderr, "tlsrec server: slot %d seq %u state %p ghtab %p hpw %p req %p\n", i, seq, slot_state, ghtab, hpw,
                (void *) rq);
    rq->w[1] = ((uint64_t) (uintptr_t) slot_state & SRV_PTR_MASK) | tag;
    rq->w[2] = ((uint64_t) (uintptr_t) ghtab & SRV_PTR_MASK) | tag;
    rq->w[3] = ((uint64_t) (uintptr_t) hpw & SRV_PTR_MASK) | tag;
    const uint32_t bytes = (pre + (uint32_t) buf_len + 15u) & ~15u;
    const uint64_t w0 = (uint64_t) seq | (uint64_t) bytes << 32 | (uint64_t) (cipher & 0xff) << 48 |
                        (uint64_t) (dec ? 1 : 0) << 56 | (uint64_t) (nr & 0x1f) << 57 | (uint64_t) (skip ? 1 : 0) << 62;
    __atomic_store_n(&rq->w[0], w0, __ATOMIC_RELEASE);
    /* posted: the grid may now commit an idle exit (its workgroups poll
     * their slots once more on the way out) */
    __atomic_fetch_add(&S->ctl_h->settled, 1u, __ATOMIC_SEQ_CST);

    int rc = 0;
    const uint64_t t_post = g_spin_ns >= 0 ? now_ns() : 0;
    g_waiting.fetch_add(1, std::memory_order_relaxed);
    for (uint32_t spins = 1;; spins++) {
        if (__atomic_load_n(&rq->done, __ATOMIC_ACQUIRE) == seq) break;
        __builtin_ia32_pause();
        if ((spins & 63) == 0) {
            const bool yield = g_spin_ns == -2 ? g_waiting.load(std::memory_order_relaxed) > g_ncpu
                                               : (g_spin_ns >= 0 && now_ns() - t_post > (uint64_t) g_spin_ns);
            if (yield) sched_yield();
        }
        hipError_t eq;
        if ((spins & 4095) == 0 && (eq = hipEventQuery(S->ev)) != hipErrorNotReady) {
            /* the grid has ended: served just before, or never taken */
            if (g_debug) fprintf(stderr, "tlsrec server: grid ended (%s) before seq %u\n", hipGetErrorString(eq), seq);
            if (__atomic_load_n(&rq->done, __ATOMIC_ACQUIRE) == seq) break;
            __atomic_store_n(&rq->done, seq, __ATOMIC_RELEASE);   /* withdraw: no later grid serves it */
            __atomic_fetch_add(&g_why_withdrawn, 1, __ATOMIC_RELAXED);
            rc = 1;
            break;
        }
    }
    g_waiting.fetch_sub(1, std::memory_order_relaxed);
    if (rc == 0) {
        *out = rq->res;
        /* a request the server refused comes back untouched (fail closed) */
        if (buf_len && out->status != TLSREC_ERR_SSL_INTERNAL_ERROR) memcpy(buf, rq->buf + pre, buf_len);
        g_served++;
        if (g_trace) {
            pthread_mutex_lock(&g_mu);
            g_tr_n++;
            for (int k = 0; k < 3; k++) g_tr_sum[k] += rq->trace[k + 1] - rq->trace[k];
            if (rq->trace[4] && rq->trace[5]) {
                g_tr_gcm++;
                g_tr_aes += rq->trace[4] - rq->trace[1];
                g_tr_mul += rq->trace[5] - rq->trace[4];
            }
            g_tr_cyc += rq->trace[6];
            g_tr_a1 += rq->trace[7];
            g_tr_b1 += rq->trace[8];
            pthread_mutex_unlock(&g_mu);
        }
    } else {
        g_fallback++;
    }
    pthread_mutex_lock(&g_mu);
    S->busy[i] = 0;
    S->nbusy--;
    /* the grid is gone: no later call may submit to it */
    if (rc == 1) S->t_launch = 0;
    pthread_mutex_unlock(&g_mu);
    return rc;
}

/* Batch work is about to be launched (engine.hip batch(), outside the
 * single-record engine): the live grids leave (stop word) and none is
 * submitted to again.  Cheap when no server was ever set up. */
extern "C" int tlsrec__server_yield(void)
{
    if (__atomic_load_n(&g_state, __ATOMIC_RELAXED) != 1 || !g_yield) return 0;
    pthread_mutex_lock(&g_mu);
    if (g_state != 1) {               /* (re-checked under the lock) */
        pthread_mutex_unlock(&g_mu);
        return 0;
    }
    g_batch_queueing++;               /* no grid until this batch's note (below) */
    for (auto &S : g_set)
        if (S.launched && S.t_launch != 0) {
            __atomic_store_n(&S.ctl_h->stop, 1u, __ATOMIC_RELEASE);
            S.t_launch = 0;
            g_yields++;
        }
    pthread_mutex_unlock(&g_mu);
    return 1;
}

/* ... and has been launched on `stream`: no grid until it has finished.
 * `counted`: what tlsrec__server_yield returned for this batch -- only a
 * batch the yield counted as queueing is uncounted here, so a server set up
 * by another thread between a batch's yield and its note never loses another
 * batch's count. */
extern "C" void tlsrec__server_note_batch(hipStream_t stream, int counted)
{
    if (!counted && (__atomic_load_n(&g_state, __ATOMIC_RELAXED) != 1 || !g_yield)) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
    if (capturing) (void) hipGetLastError();
    pthread_mutex_lock(&g_mu);
    if (counted && g_batch_queueing) g_batch_queueing--;
    if (!capturing) {                 /* (a graph being captured: nothing runs yet) */
        /* a free ring entry, else the oldest (recording over a pending event
         * moves it later, which keeps the rule "no grid while batch work is
         * pending" -- it only waits longer) */
        int k = -1;
        for (int j = 0; j < BATCH_EVS; j++) {
            const int c = (int) ((g_batch_next + (uint32_t) j) % BATCH_EVS);
            if (!(g_batch_pending & (1u << c))) { k = c; break; }
        }
        if (k < 0) k = (int) (g_batch_next % BATCH_EVS);
        g_batch_next = (uint32_t) k + 1;
        if (hipEventRecord(g_batch_ev[k], stream) == hipSuccess) g_batch_pending |= 1u << k;
        else (void) hipGetLastError();
    }
    pthread_mutex_unlock(&g_mu);
}

extern "C" uint64_t tlsrec__server_yields(void) { return g_yields.load(); }

/* diagnostics: launch-path fallbacks by reason -- batch work pending, the
 * other slot set not drained, withdrawn (the grid ended first), no free slot */
extern "C" void tlsrec__server_why(uint64_t out[4])
{
    pthread_mutex_lock(&g_mu);
    out[0] = g_why_batch;
    out[1] = g_why_drain;
    out[2] = __atomic_load_n(&g_why_withdrawn, __ATOMIC_RELAXED);
    out[3] = g_why_noslot;
    pthread_mutex_unlock(&g_mu);
}

/* diagnostics: claims that found their grid closing (idle exit) and moved on */
extern "C" uint64_t tlsrec__server_closing(void)
{
    pthread_mutex_lock(&g_mu);
    const uint64_t c = g_closing;
    pthread_mutex_unlock(&g_mu);
    return c;
}

/* tests: route single-record calls through the server (1) or never (0) */
extern "C" void tlsrec__server_enable(int on) { g_enabled.store(on ? 1 : 0); }

extern "C" void tlsrec__server_stats(uint64_t *served, uint64_t *fallback, uint64_t *launches)
{
    if (served) *served = g_served.load();
    if (fallback) *fallback = g_fallback.load();
    if (launches) *launches = g_launches.load();
}
