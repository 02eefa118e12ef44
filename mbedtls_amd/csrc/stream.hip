/*
 * stream.hip -- the TLS record layer over whole connections.
 *
 * Receive: each connection's received bytes (a TLS byte stream starting at a
 * record header) are split at their 5-byte headers and checked as
 * ssl_parse_record_header does (library/ssl_msg.c:3561-3776, TLS branch, with
 * the mbedtls_ssl_fetch_input size limit); every complete record becomes a
 * batch descriptor (implicit sequence number = in_ctr + records before it,
 * TLS 1.3 ChangeCipherSpec passed through undecrypted as at :3819-3825); the
 * batch is decrypted in place by the AEAD kernels; a per-connection pass then
 * applies ssl_prepare_record_content's post-decrypt rules in record order
 * (:3870-3917 zero-length records, :3930-3963 in_ctr increment and
 * COUNTER_WRAPPING, :4011-4014 IN_CONTENT_LEN) and stops at the first error.
 *
 * Send: each connection's application data is cut into records of at most
 * max_frag bytes (one mbedtls_ssl_write call each), laid out back to back in
 * the output stream with their headers (mbedtls_ssl_write_record
 * :2648-2793: TLS 1.3 records carry version 0x0303, the length field is the
 * protected length), and encrypted in place by the AEAD kernels.
 *
 * Header walking is one lane per connection (each header names the next);
 * connections walk in parallel.  Bulk bytes move only in the AEAD kernels
 * (receive: in place, nothing copied) and, on send, in one copy of the
 * plaintext into its record slot (one wave per record).
 */
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>

#include "tlsrec.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"

using tlsrec::SlotState;

/* engine.hip */
extern "C" const SlotState *tlsrec__keytab_slots(const tlsrec_keytab *kt);

namespace tlsst {

constexpr uint32_t NO_SLOT = 0xFFFFFFFFu;
constexpr int MAX_VERSION = 0x0304;          /* conf->max_tls_version (TLS 1.3 build) */

__device__ __forceinline__ uint64_t be64(const uint8_t c[8])
{
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) v = (v << 8) | c[i];
    return v;
}

__device__ __forceinline__ void put_be64(uint8_t c[8], uint64_t v)
{
#pragma unroll
    for (int i = 7; i >= 0; i--) {
        c[i] = (uint8_t) v;
        v >>= 8;
    }
}

/* 16 bytes at any byte address through the global address space (gfx950
 * runs unaligned-access mode; generic pointers would load through flat) */
typedef unsigned int st_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) st_u32x4 st_glob_u32x4;
__device__ __forceinline__ uint4 load16(const uint8_t *p)
{
    const st_u32x4 v = *(const st_glob_u32x4 *) (uintptr_t) p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

/* the fail-closed result the receive emit kernels write beside each
 * descriptor (the batch guard kernel's, ssl_msg.c:1260 / :1804): the batch
 * then skips its guard launch */
__device__ __forceinline__ void guard_result(tlsrec_batch_res *res)
{
    tlsrec_batch_res r;
    memset(&r, 0, sizeof(r));
    r.status = TLSREC_ERR_SSL_INTERNAL_ERROR;
    *res = r;
}

/* TLS minor version of a loaded slot (3 or 4), 0 if the slot is unusable */
__device__ __forceinline__ uint32_t slot_minor(const SlotState *slots, uint32_t cap, uint32_t slot)
{
    if (slot >= cap) return 0;
    const tlsrec_key_material &k = slots[slot].km;
    return k.cipher ? k.tls_minor : 0;
}

/* add v to the batch's byte count: a wave-wide sum, one atomic per wave, on
 * one of BYTES_SPREAD counters a 128-byte line apart (by workgroup).  (r06:
 * on a single counter the atomics of every wave queued on one L2 line -- a
 * lane-group count kernel of 64 K waves spent 0.8 ms there, the r05 one-lane
 * kernels ~40 us of their 50.) */
constexpr int BYTES_SPREAD = 64;
constexpr int BYTES_STRIDE = 16;       /* u64 words: one 128-byte line per counter */
__device__ __forceinline__ void wave_add_bytes(unsigned long long *sum, unsigned long long v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(sum + (blockIdx.x % BYTES_SPREAD) * BYTES_STRIDE, v);
}

/* the host-mapped mailbox of the batch totals (totals_kernel, r06) */
struct TotMbox {
    uint64_t total, bytes, seq, pad;
};

/* ---------------- receive ---------------------------------------------- */
struct HdrStop {
    int32_t status;           /* header error that stopped the walk, 0 = out of bytes */
    uint32_t pos;
};

/* Walk one connection's headers (ssl_parse_record_header + fetch_input);
 * f(k, pos, type, ver, dlen) for each complete record. */
template <typename F>
__device__ HdrStop walk_in(const uint8_t *base, uint32_t len, F f)
{
    uint32_t pos = 0, k = 0;
    HdrStop st = { 0, 0 };
    while (len - pos >= 5) {
        const uint8_t *h = base + pos;
        const uint32_t type = h[0], ver = ((uint32_t) h[1] << 8) | h[2], dlen = ((uint32_t) h[3] << 8) | h[4];
        if (type < 20 || type > 23) { st.status = TLSREC_ERR_SSL_INVALID_RECORD; break; }   /* :3529-3539 */
        if (ver > (uint32_t) MAX_VERSION) { st.status = TLSREC_ERR_SSL_INVALID_RECORD; break; }
        if (dlen == 0) { st.status = TLSREC_ERR_SSL_INVALID_RECORD; break; }                /* :3723-3726 */
        if (5 + dlen > TLSREC_MAX_IN_RECORD) { st.status = TLSREC_ERR_SSL_BAD_INPUT_DATA; break; }
        if (len - pos < 5 + dlen) break;                                                     /* wait */
        f(k, pos, type, h[1], h[2], dlen);
        k++;
        pos += 5 + dlen;
    }
    st.pos = pos;
    return st;
}

__global__ void in_count_kernel(const tlsrec_stream_in *s, uint32_t n, const uint8_t *arena, uint32_t *counts,
                                HdrStop *stops, unsigned long long *bytes)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long b = 0;
    if (i < n) {
        uint32_t c = 0;
        const HdrStop st = walk_in(arena + s[i].off, s[i].len,
                                   [&](uint32_t, uint32_t, uint32_t, uint8_t, uint8_t, uint32_t dlen) { c++; b += dlen; });
        counts[i] = c;
        stops[i] = st;
    } else if (i == n) {                /* scan sentinel: offs[n] = total */
        counts[n] = 0;
    }
    wave_add_bytes(bytes, b);
}

__global__ void in_emit_kernel(const tlsrec_stream_in *s, uint32_t n, const uint8_t *arena, const uint32_t *offs,
                               const SlotState *slots, uint32_t cap, tlsrec_batch_rec *recs, uint32_t max_records,
                               tlsrec_batch_res *res)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tlsrec_stream_in si = s[i];
    const bool tls13 = slot_minor(slots, cap, si.slot) == 4;
    uint64_t seq = be64(si.in_ctr);
    tlsrec_batch_rec *out = recs + offs[i];
    walk_in(arena + si.off, si.len, [&](uint32_t k, uint32_t pos, uint32_t type, uint8_t v0, uint8_t v1, uint32_t dlen) {
        tlsrec_batch_rec d;
        memset(&d, 0, sizeof(d));
        d.buf_off = si.off + pos;                 /* rec->buf = header (:3715-3716) */
        d.buf_len = 5 + dlen;
        d.data_offset = 5;
        d.data_len = dlen;
        const bool ccs = tls13 && type == 20;      /* TLS 1.3 CCS: not decrypted, no in_ctr step */
        d.slot = ccs ? NO_SLOT : si.slot;
        put_be64(d.ctr, seq);
        d.type = (uint8_t) type;
        d.ver[0] = v0;
        d.ver[1] = v1;
        if (!ccs) seq++;
        if (offs[i] + k < max_records) {                /* (launched before the host has checked the total) */
            out[k] = d;
            guard_result(&res[offs[i] + k]);
        }
    });
}

__global__ void in_finish_kernel(const tlsrec_stream_in *s, uint32_t n, const uint32_t *offs, const uint32_t *counts,
                                 const HdrStop *stops, const SlotState *slots, uint32_t cap,
                                 const tlsrec_batch_rec *recs, tlsrec_batch_res *res, tlsrec_stream_in_res *sres)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tlsrec_stream_in si = s[i];
    const uint32_t minor = slot_minor(slots, cap, si.slot);
    uint64_t ctr = be64(si.in_ctr);
    uint32_t nbz = si.nb_zero, nrec = 0, consumed = 0;
    int32_t st = 0;
    const uint32_t first = offs[i], cnt = counts[i];
    /* records in chunks of FK: the chunk's descriptors and results are loaded
     * before the in-order rules run over them (r06: one record's loads at a
     * time left the lane waiting on memory once per record) */
#ifndef TLSREC_STREAM_FK
#define TLSREC_STREAM_FK 4
#endif
    constexpr uint32_t FK = TLSREC_STREAM_FK;
    bool broke = false;
    for (uint32_t k0 = 0; k0 < cnt && !broke; k0 += FK) {
        tlsrec_batch_res rr[FK];
        uint64_t doff[FK];
        uint32_t dslot[FK], dlen[FK], dblen[FK];
        uint8_t dtype[FK];
#pragma unroll
        for (uint32_t t = 0; t < FK; t++) {
            if (k0 + t < cnt) {
                const tlsrec_batch_rec &d = recs[first + k0 + t];
                rr[t] = res[first + k0 + t];
                doff[t] = d.buf_off;
                dslot[t] = d.slot;
                dlen[t] = d.data_len;
                dblen[t] = d.buf_len;
                dtype[t] = d.type;
            }
        }
#pragma unroll
        for (uint32_t t = 0; t < FK; t++) {
            if (broke || k0 + t >= cnt) break;
            tlsrec_batch_res r = rr[t];
            if (dslot[t] == NO_SLOT) {            /* TLS 1.3 CCS passes as received */
                r.status = 0;
                r.data_offset = 5;
                r.data_len = dlen[t];
                r.type = dtype[t];
                res[first + k0 + t] = r;
            } else {
                if (r.status) { st = r.status; broke = true; break; }
                if (r.type < 20 || r.type > 23) { st = TLSREC_ERR_SSL_INVALID_RECORD; broke = true; break; }   /* type re-check :3914-3917 */
                if (r.data_len == 0) {            /* :3888-3906 */
                    if (minor == 3 && r.type != TLSREC_MSG_APPLICATION_DATA) { st = TLSREC_ERR_SSL_INVALID_RECORD; broke = true; break; }
                    if (++nbz > 3) { st = TLSREC_ERR_SSL_INVALID_MAC; broke = true; break; }
                } else {
                    nbz = 0;
                }
                if (++ctr == 0) { st = TLSREC_ERR_SSL_COUNTER_WRAPPING; broke = true; break; }   /* :3954-3963 */
            }
            if (r.data_len > 16384) { st = TLSREC_ERR_SSL_INVALID_RECORD; broke = true; break; } /* IN_CONTENT_LEN, :4011-4014 */
            nrec++;
            consumed = (uint32_t) (doff[t] - si.off) + dblen[t];
        }
    }
    const uint32_t k = broke ? 0u : cnt;
    if (st == 0 && k == cnt) st = stops[i].status;
    tlsrec_stream_in_res o;
    memset(&o, 0, sizeof(o));
    o.status = st;
    o.first = first;
    o.nrec = nrec;
    o.consumed = consumed;
    put_be64(o.in_ctr, ctr);
    o.nb_zero = (uint8_t) nbz;
    o.nparsed = cnt;
    sres[i] = o;
}

/* ---------------- receive, lane-group framing (r06) ---------------------
 * in_count_kernel / in_emit_kernel with RG lanes per connection (a group)
 * instead of one: the header walk of walk_in, speculatively parallel -- from
 * position p the group's lanes j read the header a run of equal-length
 * records would put at p + j (5 + dlen0), dlen0 the length of the header at
 * p; the leading lanes whose headers pass walk_in's checks with that length
 * are records (each one's predecessor is a record of length dlen0), the
 * first that does not is where the next round starts.  The same records and
 * the same stop as the serial walk; a stream of full-size records takes
 * ceil(records / RG) rounds of two dependent loads, where one lane per
 * connection took a serial chain of one dependent load per record (1 M
 * headers of 64 K connections: 16 loads in a row per lane, 4 waves per CU).
 * (A single-pass form with a decoupled look-back over 16-connection tiles
 * measured 7 ms for 256 K connections: thread 0's serial look-back over
 * tiles that had published only their aggregates; not kept) */
constexpr int RG = 16;                         /* lanes per connection */
constexpr int RX_THREADS = 256;
constexpr int RX_CONNS = RX_THREADS / RG;      /* connections per workgroup */

/* the group's G bits of a wave ballot (group-uniform control flow) */
template <int G = RG>
__device__ __forceinline__ uint32_t group_ballot(bool b, int lane)
{
    return (uint32_t) (__ballot(b) >> (lane & ~(G - 1))) & (uint32_t) ((1ull << G) - 1ull);
}

struct RxHdr {
    bool ok;                  /* a record of the run */
    uint32_t pos, type, dlen;
    uint8_t v0, v1;
};

/* the header at q checked as walk_in does, and of length want */
__device__ __forceinline__ RxHdr rx_header(const uint8_t *base, uint32_t len, uint64_t q, uint32_t want, int32_t *err)
{
    RxHdr h = { false, (uint32_t) q, 0, 0, 0, 0 };
    *err = 0;
    if (q + 5 > len) return h;                                         /* out of bytes: wait */
    const uint8_t *p = base + q;
    h.type = p[0];
    h.v0 = p[1];
    h.v1 = p[2];
    h.dlen = ((uint32_t) p[3] << 8) | p[4];
    const uint32_t ver = ((uint32_t) h.v0 << 8) | h.v1;
    if (h.type < 20 || h.type > 23 || ver > (uint32_t) MAX_VERSION || h.dlen == 0)
        *err = TLSREC_ERR_SSL_INVALID_RECORD;                          /* :3529-3539, :3723-3726 */
    else if (5 + h.dlen > TLSREC_MAX_IN_RECORD)
        *err = TLSREC_ERR_SSL_BAD_INPUT_DATA;
    else
        h.ok = (uint64_t) len - q >= 5 + h.dlen && h.dlen == want;
    return h;
}

/* walk_in with the group: f(k, h, ccs_before) on the lane holding record k,
 * ccs_before = the TLS 1.3 CCS records before it (tls13 only: they take no
 * sequence number).  Returns the stop and the record count (group-uniform). */
template <int G = RG, typename F>
__device__ HdrStop group_walk(const uint8_t *base, uint32_t len, int lane, bool tls13, uint32_t *count, F f)
{
    const int q = lane & (G - 1);
    uint32_t p = 0, k = 0, nccs = 0;
    HdrStop st = { 0, 0 };
    while (len - p >= 5) {
        const uint32_t dlen0 = ((uint32_t) base[p + 3] << 8) | base[p + 4];
        const uint64_t at = (uint64_t) p + (uint64_t) q * (5 + dlen0);
        int32_t err;
        const RxHdr h = rx_header(base, len, at, dlen0, &err);
        const uint32_t okm = group_ballot<G>(h.ok, lane);
        const uint32_t m = (uint32_t) __builtin_ctz(~okm);                 /* leading records */
        if (m == 0) {                                                      /* the header at p itself */
            st.status = __shfl(err, lane & ~(G - 1));
            break;
        }
        const uint32_t ccsm = group_ballot<G>(h.ok && tls13 && h.type == 20, lane) & ((1u << m) - 1u);
        if ((uint32_t) q < m) f(k + q, h, nccs + (uint32_t) __builtin_popcount(ccsm & ((1u << q) - 1u)));
        nccs += (uint32_t) __builtin_popcount(ccsm);
        k += m;
        p += m * (5 + dlen0);
    }
    st.pos = p;
    *count = k;
    return st;
}

/* G lanes per connection: 16, or 4 / 8 when the caller's max_records says
 * connections hold that few records (r06: a 4-record stream left 12 of 16
 * lanes idle, four times the waves the walk needed) */
template <int G>
__global__ __launch_bounds__(RX_THREADS) void in_count_group_kernel(const tlsrec_stream_in *s, uint32_t n,
                                                                    const uint8_t *arena, uint32_t *counts,
                                                                    HdrStop *stops, unsigned long long *bytes)
{
    const int tid = threadIdx.x, lane = tid & 63, q = tid & (G - 1);
    const uint32_t i = blockIdx.x * (RX_THREADS / G) + (uint32_t) (tid / G);
    unsigned long long b = 0;
    if (i < n) {
        const tlsrec_stream_in si = s[i];
        uint32_t cnt = 0;
        const HdrStop st = group_walk<G>(arena + si.off, si.len, lane, false, &cnt,
                                      [&](uint32_t, const RxHdr &h, uint32_t) { b += h.dlen; });
        if (q == 0) {
            counts[i] = cnt;
            stops[i] = st;
        }
    } else if (i == n && q == 0) {      /* scan sentinel: offs[n] = total */
        counts[n] = 0;
    }
    wave_add_bytes(bytes, b);
}

template <int G>
__global__ __launch_bounds__(RX_THREADS) void in_emit_group_kernel(const tlsrec_stream_in *s, uint32_t n,
                                                                   const uint8_t *arena, const uint32_t *offs,
                                                                   const SlotState *slots, uint32_t cap,
                                                                   tlsrec_batch_rec *recs, uint32_t max_records,
                                                                   tlsrec_batch_res *res)
{
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t i = blockIdx.x * (RX_THREADS / G) + (uint32_t) (tid / G);
    if (i >= n) return;
    const tlsrec_stream_in si = s[i];
    const bool tls13 = slot_minor(slots, cap, si.slot) == 4;
    const uint64_t seq0 = be64(si.in_ctr);
    tlsrec_batch_rec *out = recs + offs[i];
    uint32_t cnt;
    group_walk<G>(arena + si.off, si.len, lane, tls13, &cnt, [&](uint32_t k, const RxHdr &h, uint32_t ccs_before) {
        tlsrec_batch_rec d;
        memset(&d, 0, sizeof(d));
        d.buf_off = si.off + h.pos;                     /* rec->buf = header (:3715-3716) */
        d.buf_len = 5 + h.dlen;
        d.data_offset = 5;
        d.data_len = h.dlen;
        const bool ccs = tls13 && h.type == 20;         /* TLS 1.3 CCS: not decrypted, no in_ctr step */
        d.slot = ccs ? NO_SLOT : si.slot;
        put_be64(d.ctr, seq0 + (k - ccs_before));       /* in_ctr + the records before that took a number */
        d.type = (uint8_t) h.type;
        d.ver[0] = h.v0;
        d.ver[1] = h.v1;
        if (offs[i] + k < max_records) {                /* (launched before the host has checked the total) */
            out[k] = d;
            guard_result(&res[offs[i] + k]);
        }
    });
}

/* ---------------- receive, one framing pass (r06, second form) ----------
 * count -> scan -> emit as one kernel: a workgroup takes the next tile of
 * connections (an atomic tile counter, so every tile it waits on is already
 * running), counts their records, publishes the tile's aggregate, finds its
 * exclusive prefix by a decoupled look-back, publishes the inclusive prefix
 * and walks its connections' headers again -- now L2-hot -- to write the
 * descriptors.  The look-back runs on a whole wave: lane j reads the status
 * of the tile j + 1 places back, so one round covers 64 predecessors; a tile
 * adds the aggregates up to the nearest inclusive prefix.  (The first single-
 * pass form, r06, looked back with one thread, one predecessor at a time, and
 * measured 7 ms: DESIGN §10.)  Tile status word: bits 62-63 the flag, bits
 * 0-31 the value. */
constexpr uint64_t TS_AGG = 1ull << 62, TS_INC = 2ull << 62;

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

/* workgroup-wide (every thread calls it, NT threads): publish the tile's
 * aggregate agg, return the sum of every earlier tile's records (the tile's
 * exclusive prefix).  Thread j reads the status of the tile j + 1 places back,
 * so one round covers NT predecessors: with all tiles of a generation done
 * counting at about the same time, the front of inclusive prefixes moves NT
 * tiles per round trip (64 per round, one wave, measured 234 us for 16 K
 * tiles of a 1 M-record stream batch). */
template <int NT>
__device__ uint32_t tile_lookback(unsigned long long *status, uint32_t tile, uint32_t agg, uint32_t aux = 0,
                                  uint32_t *aux_excl = nullptr)
{
    /* status word: flag (bits 62-63) | records (bits 32-61) | aux (bits 0-31,
     * the DTLS kernel's bytes in 64-B units): both prefix sums travel in one
     * atomic word, so no fence orders them with other memory */
    __shared__ uint32_t sh_fp[NT / 64], sh_sum[NT / 64], sh_aux[NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0)
        __hip_atomic_store(status + tile, (tile == 0 ? TS_INC : TS_AGG) | ((unsigned long long) agg << 32) | aux,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t excl = 0, xaux = 0;
    int64_t base = (int64_t) tile - 1;
    for (; tile != 0;) {
        const int64_t t = base - tid;
        const unsigned long long v = t >= 0 ? __hip_atomic_load(status + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                            : TS_INC;   /* before tile 0: an inclusive prefix of 0 */
        const uint32_t flag = (uint32_t) (v >> 62);
        const uint64_t pm = __ballot(flag == 2);
        if (lane == 0) sh_fp[wave] = pm ? (uint32_t) (wave * 64) + (uint32_t) __builtin_ctzll(pm) : (uint32_t) NT;
        __syncthreads();
        uint32_t fp = sh_fp[0];                          /* nearest inclusive prefix */
#pragma unroll
        for (int w = 1; w < NT / 64; w++) fp = min(fp, sh_fp[w]);
        if (__syncthreads_or(flag == 0 && (uint32_t) tid <= fp)) {   /* a predecessor still counting */
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        const bool in = (uint32_t) tid <= fp;
        const uint32_t ws = wave_sum_u32(in ? (uint32_t) (v >> 32) & 0x3fffffffu : 0u);
        const uint32_t wa = wave_sum_u32(in ? (uint32_t) v : 0u);
        if (lane == 0) {
            sh_sum[wave] = ws;
            sh_aux[wave] = wa;
        }
        __syncthreads();
#pragma unroll
        for (int w = 0; w < NT / 64; w++) {
            excl += sh_sum[w];
            xaux += sh_aux[w];
        }
        __syncthreads();                                 /* sh_fp / sh_sum reused next round */
        if (fp < (uint32_t) NT) break;
        base -= NT;
    }
    if (tid == 0 && tile != 0)
        __hip_atomic_store(status + tile, TS_INC | ((unsigned long long) (excl + agg) << 32) | (uint32_t) (xaux + aux),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (aux_excl) *aux_excl = xaux;
    return excl;
}

/* the workgroup's tile id (first thread claims it) */
__device__ __forceinline__ uint32_t claim_tile(uint32_t *ctr, uint32_t *sh)
{
    if (threadIdx.x == 0) *sh = atomicAdd(ctr, 1u);
    __syncthreads();
    return *sh;
}

/* Stream receive framing in one pass: RG lanes per connection as
 * in_count_group_kernel / in_emit_group_kernel; a tile is RX_CH chunks of
 * RX_CONNS connections (chunk c's group g takes connection c RX_CONNS + g of
 * the tile), so 1 M records of 4-record streams make 2 K tiles, not 16 K.
 * Writes counts, stops, offs (offs[n] = the batch's record count) and the
 * descriptors (at most max_records of them). */
/* G lanes per connection (as in_count_group_kernel), CH chunks per tile, NT
 * threads per workgroup */
#ifndef TLSREC_RX_FRAME_NT
#define TLSREC_RX_FRAME_NT 512
#endif
template <int G, int CH, int NT>
__global__ __launch_bounds__(NT) void in_frame_kernel(const tlsrec_stream_in *s, uint32_t n,
                                                              const uint8_t *arena, const SlotState *slots,
                                                              uint32_t cap, uint32_t *counts, uint32_t *offs,
                                                              HdrStop *stops, unsigned long long *bytes,
                                                              unsigned long long *tstat, uint32_t *tctr,
                                                              tlsrec_batch_rec *recs, uint32_t max_records,
                                                              tlsrec_batch_res *res)
{
    constexpr int RX_CH = CH, RX_CONNS_G = NT / G, RX_TILE = RX_CH * RX_CONNS_G;
    static_assert(RX_TILE <= NT && RX_TILE <= 128 * 2, "tile scan");
    __shared__ uint32_t sh_tile, sh_cnt[RX_TILE], sh_off[RX_TILE];
    const int tid = threadIdx.x, lane = tid & 63, q = tid & (G - 1), g = tid / G;
    const uint32_t tile = claim_tile(tctr, &sh_tile);
    const uint32_t i0 = tile * RX_TILE;
    unsigned long long b = 0;
    for (int c = 0; c < RX_CH; c++) {
        const uint32_t i = i0 + (uint32_t) (c * RX_CONNS_G + g);
        uint32_t cnt = 0;
        if (i < n) {
            const tlsrec_stream_in si = s[i];
            const HdrStop st = group_walk<G>(arena + si.off, si.len, lane, false, &cnt,
                                          [&](uint32_t, const RxHdr &h, uint32_t) { b += h.dlen; });
            if (q == 0) {
                counts[i] = cnt;
                stops[i] = st;
            }
        }
        if (q == 0) sh_cnt[c * RX_CONNS_G + g] = cnt;
    }
    wave_add_bytes(bytes, b);
    __syncthreads();
    /* the tile's exclusive scan over its RX_TILE connections (threads < RX_TILE, RX_TW waves) */
    constexpr int RX_TW = (RX_TILE + 63) / 64;
    uint32_t incl = 0, agg = 0;
    if (tid < RX_TW * 64) {
        incl = tid < RX_TILE ? sh_cnt[tid] : 0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
    }
    __syncthreads();                                      /* sh_cnt read: sh_off may take the wave totals */
    if (tid < RX_TW * 64 && lane == 63) sh_off[tid >> 6] = incl;   /* wave totals (sh_off reused below) */
    __syncthreads();
#pragma unroll
    for (int w = 0; w < RX_TW; w++) agg += sh_off[w];
    uint32_t wpre = 0;
    for (int w = 0; w < (tid >> 6) && w < RX_TW; w++) wpre += sh_off[w];
    const uint32_t excl = tile_lookback<NT>(tstat, tile, agg);
    __syncthreads();                                      /* every thread has read the wave totals */
    if (tid < RX_TILE) sh_off[tid] = excl + wpre + incl - sh_cnt[tid];
    __syncthreads();
    if (tid < RX_TILE) {
        const uint32_t i = i0 + (uint32_t) tid;
        if (i < n) offs[i] = sh_off[tid];
        if (i + 1 == n) offs[n] = sh_off[tid] + sh_cnt[tid];     /* the scan's sentinel: the batch total */
    }
    if (!recs) return;
    for (int c = 0; c < RX_CH; c++) {
        const uint32_t i = i0 + (uint32_t) (c * RX_CONNS_G + g);
        const uint32_t cnt = sh_cnt[c * RX_CONNS_G + g], off = sh_off[c * RX_CONNS_G + g];
        if (i >= n || !cnt) continue;                     /* group-uniform */
        const tlsrec_stream_in si = s[i];
        const bool tls13 = slot_minor(slots, cap, si.slot) == 4;
        const uint64_t seq0 = be64(si.in_ctr);
        tlsrec_batch_rec *out = recs + off;
        uint32_t c2;
        group_walk<G>(arena + si.off, si.len, lane, tls13, &c2, [&](uint32_t k, const RxHdr &h, uint32_t ccs_before) {
            if (off + k >= max_records) return;
            tlsrec_batch_rec d;
            memset(&d, 0, sizeof(d));
            d.buf_off = si.off + h.pos;                     /* rec->buf = header (:3715-3716) */
            d.buf_len = 5 + h.dlen;
            d.data_offset = 5;
            d.data_len = h.dlen;
            const bool ccs = tls13 && h.type == 20;         /* TLS 1.3 CCS: not decrypted, no in_ctr step */
            d.slot = ccs ? NO_SLOT : si.slot;
            put_be64(d.ctr, seq0 + (k - ccs_before));
            d.type = (uint8_t) h.type;
            d.ver[0] = h.v0;
            d.ver[1] = h.v1;
            out[k] = d;
            guard_result(&res[off + k]);
        });
    }
}

/* ---------------- send ------------------------------------------------- */
struct OutShape {
    uint32_t ok;              /* slot usable */
    uint32_t head;            /* explicit-IV room before the content (8 for TLS 1.2 GCM / CCM) */
    uint32_t tls13, gran, tag;
};

__device__ __forceinline__ OutShape out_shape(const SlotState *slots, uint32_t cap, uint32_t slot)
{
    OutShape o = { 0, 0, 0, 16, 16 };
    if (slot >= cap) return o;
    const tlsrec_key_material &k = slots[slot].km;
    if (!k.cipher) return o;
    o.ok = 1;
    o.tls13 = k.tls_minor == 4;
    o.head = (!o.tls13 && k.fixed_ivlen == 4) ? 8u : 0u;
    o.gran = k.granularity ? k.granularity : 16;
    o.tag = k.taglen;
    return o;
}

/* protected length of an n-byte record (ssl_msg.c:853-868, :1066-1075) */
__device__ __forceinline__ uint32_t out_body(const OutShape &o, uint32_t n)
{
    if (o.tls13) {
        const uint32_t inner = n + 1;
        return inner + (o.gran - inner % o.gran) % o.gran + o.tag;
    }
    return o.head + n + o.tag;
}

__device__ __forceinline__ uint32_t frag_of(const tlsrec_stream_out &s) { return s.max_frag ? s.max_frag : 16384u; }

__global__ void out_count_kernel(const tlsrec_stream_out *s, uint32_t n, const SlotState *slots, uint32_t cap,
                                 uint32_t *counts, unsigned long long *bytes)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long b = 0;
    if (i < n) {
        const uint32_t f = frag_of(s[i]);
        const bool ok = out_shape(slots, cap, s[i].slot).ok;
        counts[i] = ok ? (uint32_t) (((uint64_t) s[i].in_len + f - 1) / f) : 0u;
        b = ok ? s[i].in_len : 0;
    } else if (i == n) {
        counts[n] = 0;
    }
    wave_add_bytes(bytes, b);
}

/* records of connection i are [offs[i], offs[i] + counts[i]): park i in
 * their descriptors' slot field for the frame kernels (one load per record
 * instead of a binary search over offs) */
__global__ void __launch_bounds__(256) out_map_kernel(uint32_t n, const uint32_t *offs, const uint32_t *counts,
                                                      tlsrec_batch_rec *recs)
{
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);   /* one wave per connection */
    if (i >= n) return;
    const uint32_t f = offs[i], c = counts[i];
    for (uint32_t k = threadIdx.x & 63; k < c; k += 64) recs[f + k].slot = i;
}

/* One wave per record (4 per workgroup): header, descriptor, and the
 * plaintext copied into the record's slot of the output stream with 16-byte
 * accesses at any byte alignment (unaligned-access mode, see kernels.hip). */
/* srcoff (r05): instead of copying the application data into the output
 * stream, record j's content offset in `in` goes to srcoff[j] and the AEAD
 * kernels read it there (tlsrec__batch_src) -- one pass over the data instead
 * of a copy and an in-place pass.  With nothing to copy, a record needs one
 * thread, not a wave (LPR = 1: 64 records per wave; as one wave per record
 * this kernel took 0.36-0.43 ms of a 2 ms send of 1 M records). */
/* record k (= j - offs[i]) of connection i: header, descriptor, and the
 * content (srcoff: its offset for the AEAD to read in place; else copied
 * into the record's slot by the LPR lanes) */
template <int LPR>
__device__ __forceinline__ void out_frame_one(const tlsrec_stream_out &si, uint32_t k, uint32_t j, uint32_t lane,
                                              const SlotState *slots, uint32_t cap, const uint8_t *in, uint8_t *out,
                                              tlsrec_batch_rec *recs, uint64_t *srcoff)
{
    const uint32_t f = frag_of(si);
    const OutShape sh = out_shape(slots, cap, si.slot);
    const uint64_t src_off = (uint64_t) k * f;
    const uint64_t left = (uint64_t) si.in_len - src_off;
    const uint32_t len = left < f ? (uint32_t) left : f;
    const uint64_t pos = si.out_off + (uint64_t) k * (5 + out_body(sh, f));
    /* a record whose sequence number would come after the counter wrapped is
     * never protected: the reference stops with COUNTER_WRAPPING after the
     * record that wraps it (:2749-2756), before encrypting anything under a
     * reused sequence number (= a reused nonce).  No slot, no bytes. */
    if ((uint64_t) k > ~be64(si.out_ctr)) {
        if (lane == 0) {
            tlsrec_batch_rec d;
            memset(&d, 0, sizeof(d));
            d.slot = NO_SLOT;
            recs[j] = d;
        }
        return;
    }
    if (srcoff) {
        if (lane == 0) srcoff[j] = si.in_off + src_off;
    } else {
        const uint8_t *src = in + si.in_off + src_off;
        uint8_t *dst = out + pos + 5 + sh.head;
        const uint32_t nv = len / 16;
        for (uint32_t v = lane; v < nv; v += LPR) {
            uint4 w;
            __builtin_memcpy(&w, src + 16 * v, 16);
            __builtin_memcpy(dst + 16 * v, &w, 16);
        }
        for (uint32_t b = nv * 16 + lane; b < len; b += LPR) dst[b] = src[b];
    }
    if (lane == 0) {
        const uint32_t body = out_body(sh, len);
        uint8_t *h = out + pos;
        h[0] = sh.tls13 ? (uint8_t) TLSREC_MSG_APPLICATION_DATA : si.type;   /* final out_msgtype */
        h[1] = 3;                                  /* mbedtls_ssl_write_version(TLS 1.2 for 1.3), :2669-2674 */
        h[2] = 3;
        h[3] = (uint8_t) (body >> 8);
        h[4] = (uint8_t) body;
        tlsrec_batch_rec d;
        memset(&d, 0, sizeof(d));
        d.buf_off = pos + 5;                       /* rec.buf = out_iv */
        d.buf_len = TLSREC_OUT_BUF_SPACE;
        d.data_offset = sh.head;                   /* out_msg - out_iv */
        d.data_len = len;
        d.slot = si.slot;
        put_be64(d.ctr, be64(si.out_ctr) + k);
        d.type = si.type;
        d.ver[0] = 3;
        d.ver[1] = 3;
        recs[j] = d;
    }
}

template <int LPR>
__global__ void __launch_bounds__(256) out_frame_kernel(const tlsrec_stream_out *s, uint32_t n, const uint32_t *offs,
                                                        uint32_t total, const SlotState *slots, uint32_t cap,
                                                        const uint8_t *in, uint8_t *out, tlsrec_batch_rec *recs,
                                                        uint64_t *srcoff)
{
    const uint32_t j = blockIdx.x * (256 / LPR) + threadIdx.x / LPR, lane = threadIdx.x % LPR;
    if (j >= total) return;
    const uint32_t i = recs[j].slot;              /* connection of record j (out_map_kernel) */
    out_frame_one<LPR>(s[i], j - offs[i], j, lane, slots, cap, in, out, recs, srcoff);
}

__global__ void out_finish_kernel(const tlsrec_stream_out *s, uint32_t n, const uint32_t *offs, const uint32_t *counts,
                                  const SlotState *slots, uint32_t cap, const tlsrec_batch_res *res,
                                  tlsrec_stream_out_res *sres)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tlsrec_stream_out si = s[i];
    uint64_t ctr = be64(si.out_ctr);
    int32_t st = out_shape(slots, cap, si.slot).ok || si.in_len == 0 ? 0 : TLSREC_ERR_SSL_BAD_INPUT_DATA;
    uint32_t nrec = 0, olen = 0;
    const uint32_t first = offs[i], cnt = counts[i];
    for (uint32_t k = 0; k < cnt && st == 0; k++) {
        const tlsrec_batch_res &r = res[first + k];
        if (r.status) { st = r.status; break; }
        if (r.data_offset != 0) { st = TLSREC_ERR_SSL_INTERNAL_ERROR; break; }   /* :2704-2707 */
        olen += 5 + r.data_len;
        nrec++;
        if (++ctr == 0) st = TLSREC_ERR_SSL_COUNTER_WRAPPING;                      /* :2749-2756 */
    }
    tlsrec_stream_out_res o;
    memset(&o, 0, sizeof(o));
    o.status = st;
    o.first = first;
    o.nrec = nrec;
    o.out_len = olen;
    put_be64(o.out_ctr, ctr);
    o.nparsed = cnt;
    sres[i] = o;
}

/* ---------------- read (ssl_read_application_data) -------------------- */
/* One workgroup per connection: every thread walks the (few) records to the
 * same copy plan; the copies move 16 bytes per thread at any alignment. */
__global__ void __launch_bounds__(256) read_kernel(const tlsrec_stream_in_res *sres, uint32_t n,
                                                   const tlsrec_batch_rec *recs, const tlsrec_batch_res *res,
                                                   uint8_t *arena, const tlsrec_stream_read_req *req, uint8_t *out,
                                                   tlsrec_stream_read_res *rres)
{
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const uint32_t first = sres[i].first, nrec = sres[i].nrec, cap = req[i].out_cap;
    uint8_t *dst0 = out + req[i].out_off;
    uint32_t done = 0, full = 0, rest = 0;
    for (uint32_t k = 0; k < nrec; k++) {
        const tlsrec_batch_res r = res[first + k];
        if (r.type != TLSREC_MSG_APPLICATION_DATA) {
            full++;
            continue;
        }
        uint8_t *src = arena + recs[first + k].buf_off + r.data_offset;
        const uint32_t m = r.data_len < cap - done ? r.data_len : cap - done;
        uint8_t *dst = dst0 + done;
        const uint32_t nv = m / 16;
        for (uint32_t v = threadIdx.x; v < nv; v += blockDim.x) {
            uint4 w;
            __builtin_memcpy(&w, src + 16 * v, 16);
            __builtin_memcpy(dst + 16 * v, &w, 16);
            const uint4 z = make_uint4(0, 0, 0, 0);
            __builtin_memcpy(src + 16 * v, &z, 16);          /* mbedtls_platform_zeroize(in_offt, n) */
        }
        for (uint32_t b = nv * 16 + threadIdx.x; b < m; b += blockDim.x) {
            dst[b] = src[b];
            src[b] = 0;
        }
        done += m;
        if (m < r.data_len) {
            rest = r.data_len - m;
            break;
        }
        full++;
    }
    if (threadIdx.x == 0) {
        tlsrec_stream_read_res o;
        o.copied = done;
        o.records = full;
        o.left = rest;
        o.reserved = 0;
        rres[i] = o;
    }
}

/* ---------------- DTLS 1.2 (datagram transport) ------------------------ */
/* How a datagram's header walk ended (ssl_get_next_record / fetch_input). */
enum DgStop : int32_t {
    DG_END = 0,        /* every byte belongs to a record */
    DG_INVALID = 1,    /* a header error: INVALID_RECORD, rest of the datagram dropped (:4790-4797) */
    DG_TRAILING = 2,   /* 1..12 bytes after a record: fetch_input's INTERNAL_ERROR (:1921-1926) */
    DG_EOF = 3         /* an empty datagram: f_recv returned 0, CONN_EOF (:1968-1970) */
};

struct DtlsHdr {
    uint32_t pos, data_offset, data_len, cid_len;
};

/* mbedtls_ssl_read_version, datagram transport (ssl_msg.c:6215-6228) */
__device__ __forceinline__ uint32_t read_version_dtls(uint32_t a, uint32_t b)
{
    const uint32_t w = (a << 8) | b;
    return (uint16_t) ~(w - (w == 0xfeffu ? 0x0202u : 0x0201u));
}

__device__ __forceinline__ uint32_t dgram_len(const tlsrec_dgram &d)
{
    return d.len < TLSREC_DTLS_MAX_DATAGRAM ? d.len : (uint32_t) TLSREC_DTLS_MAX_DATAGRAM;   /* f_recv truncates */
}

/* The records of one datagram, walked with the header checks of
 * ssl_parse_record_header that decide where a record ends (:3591-3753; type
 * :3529-3539 or a tls12_cid header of conf->cid_len bytes :3616-3649, version
 * <= TLS 1.2, data_len != 0, the datagram holds the record); f(h, header) per
 * record. */
template <typename F>
__device__ __forceinline__ int32_t dtls_walk(const uint8_t *b, uint32_t len, uint32_t cid_conf, F f)
{
    if (len == 0) return DG_EOF;
    uint32_t pos = 0;
    while (pos < len) {
        const uint32_t rem = len - pos;
        if (rem < 13) return pos == 0 ? DG_INVALID : DG_TRAILING;
        const uint8_t *h = b + pos;
        const uint32_t type = h[0];
        uint32_t lo = 11, cid = 0;
        if (cid_conf != 0 && type == TLSREC_MSG_CID) {
            lo += cid_conf;
            if (rem < lo + 2) return DG_INVALID;
            cid = cid_conf;
        } else if (type < 20 || type > 23) {
            return DG_INVALID;
        }
        if (read_version_dtls(h[1], h[2]) > 0x0303u) return DG_INVALID;     /* max_tls_version, ssl_tls.c:5514-5517 */
        const uint32_t dlen = ((uint32_t) h[lo] << 8) | h[lo + 1];
        if (dlen == 0) return DG_INVALID;
        if (rem < lo + 2 + dlen) return DG_INVALID;
        const DtlsHdr d = { pos, lo + 2, dlen, cid };
        f(d, h);
        pos += lo + 2 + dlen;
    }
    return DG_END;
}

/* dtls_walk with the datagram's first 16 bytes already loaded (have16):
 * a datagram that is exactly one plain record -- the common case -- is
 * decided from registers, f gets a pointer to the loaded bytes; anything
 * else (several records, a CID header, an error) walks from memory as
 * dtls_walk does, f not having been called yet.  Same records, same stop. */
template <typename F>
__device__ __forceinline__ int32_t dtls_walk_pre(const uint8_t *b, uint32_t len, uint4 h16, bool have16,
                                                 uint32_t cid_conf, F f)
{
    if (have16) {
        uint8_t h[16];
        __builtin_memcpy(h, &h16, 16);
        const uint32_t type = h[0], dlen = ((uint32_t) h[11] << 8) | h[12];
        if (!(cid_conf != 0 && type == TLSREC_MSG_CID) && type >= 20 && type <= 23 &&
            read_version_dtls(h[1], h[2]) <= 0x0303u && dlen != 0 && len == 13 + dlen) {
            const DtlsHdr d = { 0, 13, dlen, 0 };
            f(d, (const uint8_t *) h);
            return DG_END;
        }
    }
    return dtls_walk(b, len, cid_conf, f);
}

/* A connection's datagrams d0 .. d1 - 1 in arrival order, U at a time: their
 * descriptors, then their first 16 bytes, are loaded before any is walked, so
 * one lane's walk waits on memory once per U datagrams rather than twice per
 * datagram (r06: with 16 datagrams per connection, one lane each, the count /
 * emit / finish kernels were chains of 32 dependent loads).  fr(off, hdr, p)
 * per record, fd(stop) per datagram. */
template <int U, typename FR, typename FD, typename FC>
__device__ __forceinline__ void dtls_conn_walk(uint32_t d0, uint32_t d1, const tlsrec_dgram *dg, const uint8_t *arena,
                                               uint32_t cid_conf, FR fr, FD fd, FC fc)
{
    for (uint32_t d = d0; d < d1; d += U) {
        fc();                                   /* the caller's own loads for the next U datagrams */
        uint64_t off[U];
        uint32_t len[U];
        uint4 h[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            off[u] = 0;
            len[u] = 0;
            if (d + u < d1) {
                const tlsrec_dgram g = dg[d + u];
                off[u] = g.off;
                len[u] = dgram_len(g);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) h[u] = len[u] >= 16 ? load16(arena + off[u]) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (d + u >= d1) break;
            const uint64_t o = off[u];
            fd(dtls_walk_pre(arena + o, len[u], h[u], len[u] >= 16, cid_conf,
                             [&](const DtlsHdr &hd, const uint8_t *p) { fr(o, hd, p); }));
        }
    }
}
#ifndef TLSREC_DG_U
#define TLSREC_DG_U 4
#endif
constexpr int DG_U = TLSREC_DG_U;
#ifndef TLSREC_DGF_U
#define TLSREC_DGF_U TLSREC_DG_U
#endif
constexpr int DGF_U = TLSREC_DGF_U;      /* the in-order finish's datagrams per load batch */

/* the anti-replay window (mbedtls_ssl_dtls_replay_check / _update, ssl_msg.c:3248-3306) */
struct ReplayWindow {
    uint64_t top, bits;
    bool on;

    __device__ __forceinline__ static uint64_t seq48(const uint8_t *ctr)
    {
        uint64_t v = 0;
#pragma unroll
        for (int k = 2; k < 8; k++) v = (v << 8) | ctr[k];
        return v;
    }
    __device__ __forceinline__ bool fresh(const uint8_t *ctr) const { return fresh_s(seq48(ctr)); }
    __device__ __forceinline__ void update(const uint8_t *ctr) { update_s(seq48(ctr)); }
    __device__ __forceinline__ bool fresh_s(uint64_t s) const
    {
        if (!on || s > top) return true;
        const uint64_t bit = top - s;
        return bit < 64 && !((bits >> bit) & 1);
    }
    __device__ __forceinline__ void update_s(uint64_t s)
    {
        if (!on) return;
        if (s > top) {
            const uint64_t shift = s - top;
            bits = shift >= 64 ? 1 : ((bits << shift) | 1);
            top = s;
        } else if (top - s < 64) {
            bits |= (uint64_t) 1 << (top - s);
        }
    }
};

__device__ __forceinline__ bool dtls_conn_ok(const tlsrec_dtls_in &c, uint32_t ndg, const SlotState *slots,
                                             uint32_t cap)
{
    return slot_minor(slots, cap, c.slot) == 3 && c.first_dgram <= ndg && c.ndgram <= ndg - c.first_dgram &&
           c.cid_len <= TLSREC_CID_LEN_MAX;
}

__global__ void dtls_count_kernel(const tlsrec_dtls_in *c, uint32_t n, const tlsrec_dgram *dg, uint32_t ndg,
                                  const uint8_t *arena, const SlotState *slots, uint32_t cap, uint32_t *counts,
                                  unsigned long long *bytes)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long b = 0;
    if (i < n) {
        const tlsrec_dtls_in ci = c[i];
        uint32_t cnt = 0;
        if (dtls_conn_ok(ci, ndg, slots, cap))
            for (uint32_t d = ci.first_dgram; d < ci.first_dgram + ci.ndgram; d++)
                dtls_walk(arena + dg[d].off, dgram_len(dg[d]), ci.cid_len, [&](const DtlsHdr &h, const uint8_t *) {
                    cnt++;
                    b += h.data_len;
                });
        counts[i] = cnt;
    } else if (i == n) {
        counts[n] = 0;
    }
    wave_add_bytes(bytes, b);
}

/* One descriptor per record.  A record is decrypted when its epoch matches
 * and the window the connection arrived with does not reject it: the window
 * only ever gains records, so every record the in-order pass will accept is
 * among them (replayed copies of a record that then fails its MAC included). */
__global__ void dtls_emit_kernel(const tlsrec_dtls_in *c, uint32_t n, const tlsrec_dgram *dg, uint32_t ndg,
                                 const uint8_t *arena, const uint32_t *offs, const SlotState *slots, uint32_t cap,
                                 tlsrec_batch_rec *recs, uint32_t max_records, tlsrec_batch_res *res)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tlsrec_dtls_in ci = c[i];
    if (!dtls_conn_ok(ci, ndg, slots, cap)) return;
    const ReplayWindow w0 = { ci.window_top, ci.window, (ci.flags & TLSREC_DTLS_ANTI_REPLAY) != 0 };
    uint32_t k = offs[i];
    for (uint32_t d = ci.first_dgram; d < ci.first_dgram + ci.ndgram; d++) {
        const uint64_t base = dg[d].off;
        dtls_walk(arena + base, dgram_len(dg[d]), ci.cid_len, [&](const DtlsHdr &h, const uint8_t *p) {
            tlsrec_batch_rec r;
            memset(&r, 0, sizeof(r));
            r.buf_off = base + h.pos;                  /* rec->buf = the header (:3715-3716) */
            r.buf_len = h.data_offset + h.data_len;
            r.data_offset = h.data_offset;
            r.data_len = h.data_len;
            memcpy(r.ctr, p + 3, 8);                   /* explicit epoch + sequence number (:3683-3687) */
            r.type = p[0];
            r.ver[0] = p[1];
            r.ver[1] = p[2];
            r.cid_len = (uint8_t) h.cid_len;
            r.cid_off[0] = 11;                         /* the CID follows the sequence number */
            const uint32_t epoch = ((uint32_t) p[3] << 8) | p[4];
            r.slot = (epoch == ci.in_epoch && w0.fresh(p + 3)) ? ci.slot : NO_SLOT;
            if (k < max_records) {                     /* (launched before the host has checked the total) */
                recs[k] = r;
                guard_result(&res[k]);
            }
            k++;
        });
    }
}

/* dtls_count_kernel + scan + dtls_emit_kernel in one pass (in_frame_kernel's
 * tile look-back), one lane per connection, DG_THREADS connections per tile,
 * datagrams walked DG_U at a time.  Descriptors beyond max_records are not
 * written.  S > 0: the count walk keeps each lane's first S records' header
 * fields in LDS (24 B each) and the emit builds those descriptors from there,
 * without a second walk over the header lines (r06; a connection with more
 * records walks again). */
constexpr int DG_THREADS = 256;
template <int S>
__global__ __launch_bounds__(DG_THREADS) void dtls_frame_kernel(const tlsrec_dtls_in *c, uint32_t n,
                                                                const tlsrec_dgram *dg, uint32_t ndg,
                                                                const uint8_t *arena, const SlotState *slots,
                                                                uint32_t cap, uint32_t *counts, uint32_t *offs,
                                                                unsigned long long *bytes, unsigned long long *tstat,
                                                                uint32_t *tctr, tlsrec_batch_rec *recs,
                                                                uint32_t max_records, tlsrec_batch_res *res,
                                                                TotMbox *mb, uint64_t mseq, uint32_t *dgst)
{
    __shared__ uint32_t sh_tile, sh_wsum[DG_THREADS / 64];
    constexpr int SS = S > 0 ? S : 1;
    __shared__ uint2 st_off[SS][DG_THREADS], st_ctr[SS][DG_THREADS], st_meta[SS][DG_THREADS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t tile = claim_tile(tctr, &sh_tile);
    const uint32_t i = tile * DG_THREADS + (uint32_t) tid;
    unsigned long long b = 0;
    uint32_t cnt = 0;
    tlsrec_dtls_in ci;
    bool ok = false;
    if (i < n) {
        ci = c[i];
        ok = dtls_conn_ok(ci, ndg, slots, cap);
        if (ok) {
            uint32_t d = ci.first_dgram, kd = 0;
            dtls_conn_walk<DG_U>(ci.first_dgram, ci.first_dgram + ci.ndgram, dg, arena, ci.cid_len,
                                 [&](uint64_t base, const DtlsHdr &h, const uint8_t *p) {
                                     if (S > 0 && cnt < (uint32_t) S) {
                                         const uint64_t bo = base + h.pos;
                                         st_off[cnt][tid] = make_uint2((uint32_t) bo, (uint32_t) (bo >> 32));
                                         st_ctr[cnt][tid] = make_uint2(
                                             p[3] | (uint32_t) p[4] << 8 | (uint32_t) p[5] << 16 | (uint32_t) p[6] << 24,
                                             p[7] | (uint32_t) p[8] << 8 | (uint32_t) p[9] << 16 | (uint32_t) p[10] << 24);
                                         st_meta[cnt][tid] = make_uint2(h.data_len | h.data_offset << 16,
                                                                        p[0] | (uint32_t) p[1] << 8 | (uint32_t) p[2] << 16 |
                                                                            h.cid_len << 24);
                                     }
                                     cnt++;
                                     b += h.data_len;
                                 },
                                 [&](int32_t stop) {         /* S > 0: the datagram summaries here */
                                     if (S > 0 && dgst) dgst[d] = (cnt - kd) | ((uint32_t) stop << 24);
                                     d++;
                                     kd = cnt;
                                 },
                                 [] {});
        }
        counts[i] = cnt;
    }
    wave_add_bytes(bytes, b);
    /* the tile's bytes (64-B units) ride in the look-back's status word */
    __shared__ unsigned long long sh_b[DG_THREADS / 64];
    {
        unsigned long long wb = b;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) wb += __shfl_xor(wb, o);
        if (lane == 0) sh_b[wave] = wb;
    }
    /* the tile's exclusive scan: within waves by shuffles, across waves in LDS */
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) sh_wsum[wave] = incl;
    __syncthreads();
    const uint32_t agg = sh_wsum[0] + sh_wsum[1] + sh_wsum[2] + sh_wsum[3];
    const uint32_t aux = (uint32_t) ((sh_b[0] + sh_b[1] + sh_b[2] + sh_b[3]) >> 6);
    uint32_t aux_excl = 0;
    const uint32_t excl = tile_lookback<DG_THREADS>(tstat, tile, agg, aux, &aux_excl);
    uint32_t off = excl + incl - cnt;
    for (int w = 0; w < wave; w++) off += sh_wsum[w];
    if (i < n) offs[i] = off;
    if (i + 1 == n) offs[n] = off + cnt;                  /* the scan's sentinel: the batch total */
    /* the last tile's prefix covers every tile: it hands the totals to the
     * host now, while the other tiles still emit (r06; the byte total in
     * 64-B units per tile, exact enough for the mean record size that steers
     * the AEAD launch; mb = null: the host reads the totals afterwards) */
    if (mb && tile == gridDim.x - 1 && tid == 0) {
        mb->total = excl + agg;
        mb->bytes = (unsigned long long) (aux_excl + aux) << 6;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(&mb->seq, mseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!ok) return;
    /* the emit walk also leaves each datagram's summary for the in-order
     * finish -- its records and how its walk stopped (dgst[d] = records |
     * stop << 24) -- so the finish reads 4 B per datagram and the records'
     * descriptors instead of the datagrams' header lines again (r06) */
    const ReplayWindow w0 = { ci.window_top, ci.window, (ci.flags & TLSREC_DTLS_ANTI_REPLAY) != 0 };
    if (S > 0 && cnt <= (uint32_t) S) {             /* every record's fields are in LDS (this lane's own) */
        if (!recs) return;
        for (uint32_t j = 0; j < cnt && off + j < max_records; j++) {
            const uint2 o = st_off[j][tid], cc = st_ctr[j][tid], m = st_meta[j][tid];
            tlsrec_batch_rec r;
            memset(&r, 0, sizeof(r));
            r.buf_off = o.x | (uint64_t) o.y << 32;             /* rec->buf = the header (:3715-3716) */
            r.data_len = m.x & 0xffffu;
            r.data_offset = m.x >> 16;
            r.buf_len = r.data_offset + r.data_len;
            memcpy(r.ctr, &cc, 8);                              /* explicit epoch + sequence number (:3683-3687) */
            r.type = (uint8_t) m.y;
            r.ver[0] = (uint8_t) (m.y >> 8);
            r.ver[1] = (uint8_t) (m.y >> 16);
            r.cid_len = (uint8_t) (m.y >> 24);
            r.cid_off[0] = 11;                                  /* the CID follows the sequence number */
            const uint32_t epoch = (cc.x & 0xffu) << 8 | ((cc.x >> 8) & 0xffu);
            const uint64_t s48 = (uint64_t) ((cc.x >> 16) & 0xffu) << 40 | (uint64_t) (cc.x >> 24) << 32 |
                                 (uint64_t) (cc.y & 0xffu) << 24 | ((cc.y >> 8) & 0xffu) << 16 |
                                 ((cc.y >> 16) & 0xffu) << 8 | (cc.y >> 24);
            r.slot = (epoch == ci.in_epoch && w0.fresh_s(s48)) ? ci.slot : NO_SLOT;
            recs[off + j] = r;
            guard_result(&res[off + j]);
        }
        return;
    }
    uint32_t k = off, d = ci.first_dgram, kd = off;
    dtls_conn_walk<DG_U>(ci.first_dgram, ci.first_dgram + ci.ndgram, dg, arena, ci.cid_len,
                         [&](uint64_t base, const DtlsHdr &h, const uint8_t *p) {
                             if (recs && k < max_records) {
                                 tlsrec_batch_rec r;
                                 memset(&r, 0, sizeof(r));
                                 r.buf_off = base + h.pos;                  /* rec->buf = the header (:3715-3716) */
                                 r.buf_len = h.data_offset + h.data_len;
                                 r.data_offset = h.data_offset;
                                 r.data_len = h.data_len;
                                 memcpy(r.ctr, p + 3, 8);                   /* explicit epoch + sequence number (:3683-3687) */
                                 r.type = p[0];
                                 r.ver[0] = p[1];
                                 r.ver[1] = p[2];
                                 r.cid_len = (uint8_t) h.cid_len;
                                 r.cid_off[0] = 11;                         /* the CID follows the sequence number */
                                 const uint32_t epoch = ((uint32_t) p[3] << 8) | p[4];
                                 r.slot = (epoch == ci.in_epoch && w0.fresh(p + 3)) ? ci.slot : NO_SLOT;
                                 recs[k] = r;
                                 guard_result(&res[k]);
                             }
                             k++;
                         },
                         [&](int32_t stop) {
                             if (S == 0 && dgst) dgst[d] = (k - kd) | ((uint32_t) stop << 24);
                             d++;
                             kd = k;
                         },
                         [] {});
}

/* ssl_get_next_record over each connection's datagrams in arrival order, on
 * the decrypt results (one lane per connection). */
/* A record the speculative pass decrypted but the in-order pass does not
 * reach (after a fatal error, in the rest of a datagram dropped for a bad
 * MAC, or a replay inside the batch): the reference never decrypts it, so its
 * plaintext must not stay in the arena -- its content bytes are zeroed. */
__device__ __forceinline__ void dtls_unreach_wipe(uint8_t *arena, const tlsrec_batch_rec *recs,
                                                  const tlsrec_batch_res *res, const SlotState *slots, uint32_t kk)
{
    const tlsrec_batch_rec &d = recs[kk];
    if (d.slot == NO_SLOT || res[kk].status != 0) return;
    /* the whole decrypted AEAD region: content, and with a CID the inner type
     * byte and padding (res.data_offset is past the explicit IV) */
    const uint32_t end = d.data_offset + d.data_len - slots[d.slot].km.taglen;
    uint8_t *b = arena + d.buf_off;
    for (uint32_t x = res[kk].data_offset; x < end; x++) b[x] = 0;
}

/* ssl_get_next_record over connection i's datagrams in arrival order, on
 * the decrypt results (one lane).  PRE: the datagrams DG_U at a time
 * (dtls_conn_walk), the records' results and descriptor slots loaded with
 * them. */
template <bool PRE>
__device__ void dtls_finish_one(uint32_t i, const tlsrec_dtls_in *c, const tlsrec_dgram *dg, uint32_t ndg,
                                uint8_t *arena, const uint32_t *offs, const uint32_t *counts,
                                const SlotState *slots, uint32_t cap, const tlsrec_batch_rec *recs,
                                const tlsrec_batch_res *res, int32_t *disp, tlsrec_dtls_in_res *cres,
                                const uint32_t *dgst)
{
    const tlsrec_dtls_in ci = c[i];
    ReplayWindow w = { ci.window_top, ci.window, (ci.flags & TLSREC_DTLS_ANTI_REPLAY) != 0 };
    const bool ignore_cid = (ci.flags & TLSREC_DTLS_IGNORE_UNEXPECTED_CID) != 0;
    uint32_t nbz = ci.nb_zero, bms = ci.badmac_seen, nacc = 0, done = 0, inval = 0;
    const uint32_t first = offs[i], nrec = counts[i];
    uint32_t k = first;
    int32_t st = 0;
    bool dropped = false;
    /* PRE: the next DGF_U records' results and slots (record kb + u) */
    uint32_t kb = 0;
    tlsrec_batch_res pr[DGF_U];
    uint32_t ps[DGF_U];
    auto prefetch = [&]() __attribute__((always_inline)) {
        kb = k;
#pragma unroll
        for (int u = 0; u < DGF_U; u++) {
            if (k + u < first + nrec) {
                pr[u] = res[k + u];
                ps[u] = recs[k + u].slot;
            }
        }
    };
    auto onrec = [&](uint32_t epoch, uint64_t seq) __attribute__((always_inline)) {
        const uint32_t kk = k++;
        /* PRE: records come in order, so the prefetched ones leave from the
         * head of a register queue -- shifted for every record, never indexed
         * (an indexed array would live in scratch memory) */
        bool have = false;
        uint32_t qslot = 0;
        tlsrec_batch_res qr;
        if constexpr (PRE) {
            if (kk - kb < (uint32_t) DGF_U) {
                have = true;
                qslot = ps[0];
                qr = pr[0];
#pragma unroll
                for (int u = 0; u + 1 < DGF_U; u++) {
                    ps[u] = ps[u + 1];
                    pr[u] = pr[u + 1];
                }
            }
        }
        if (st) { disp[kk] = TLSREC_DTLS_NOT_REACHED; dtls_unreach_wipe(arena, recs, res, slots, kk); return; }
        if (dropped) { disp[kk] = TLSREC_DTLS_DROPPED; dtls_unreach_wipe(arena, recs, res, slots, kk); return; }
        if (epoch != ci.in_epoch) {            /* :3755-3768, skipped after the handshake (:4727-4800) */
            disp[kk] = epoch == (uint32_t) ci.in_epoch + 1 ? TLSREC_ERR_SSL_EARLY_MESSAGE
                                                           : TLSREC_ERR_SSL_UNEXPECTED_RECORD;
            return;
        }
        if (!w.fresh_s(seq)) {                 /* :3769-3776 */
            disp[kk] = TLSREC_ERR_SSL_UNEXPECTED_RECORD;
            dtls_unreach_wipe(arena, recs, res, slots, kk);
            return;
        }
        uint32_t rslot;
        tlsrec_batch_res r;
        if constexpr (PRE) {
            if (have) {
                rslot = qslot;
                r = qr;
            } else {                            /* a datagram of several records ran past the prefetch */
                rslot = recs[kk].slot;
                r = res[kk];
            }
        } else {
            rslot = recs[kk].slot;
            r = res[kk];
        }
        if (rslot == NO_SLOT) {                /* not decrypted: impossible, the window only grows */
            st = TLSREC_ERR_SSL_INTERNAL_ERROR;
            disp[kk] = st;
            return;
        }
        int32_t e = r.status;                  /* ssl_prepare_record_content (:3810-4017) */
        if (e == TLSREC_ERR_SSL_UNEXPECTED_CID && ignore_cid) { disp[kk] = e; return; }   /* :3872-3879 */
        if (e == 0) {
            if (r.type < 20 || r.type > 23) {  /* :3914-3917 */
                e = TLSREC_ERR_SSL_INVALID_RECORD;
            } else if (r.data_len == 0) {      /* :3920-3941 */
                if (r.type != TLSREC_MSG_APPLICATION_DATA) e = TLSREC_ERR_SSL_INVALID_RECORD;
                else if (++nbz > 3) e = TLSREC_ERR_SSL_INVALID_MAC;
            } else {
                nbz = 0;
            }
        }
        if (e == 0) {
            w.update_s(seq);                   /* mbedtls_ssl_dtls_replay_update (:4003-4007) */
            if (r.data_len > 16384) e = TLSREC_ERR_SSL_INVALID_RECORD;   /* :4011-4014 */
        }
        disp[kk] = e;
        if (e == TLSREC_ERR_SSL_INVALID_MAC) { /* :4837-4873 */
            if (ci.badmac_limit != 0 && ++bms >= ci.badmac_limit) st = e;
            else dropped = true;
        } else if (e) {
            st = e;
        } else {
            nacc++;
        }
    };
    /* the header's epoch and 48-bit sequence number (:3683-3687) */
    auto hdr_rec = [&](const uint8_t *p) __attribute__((always_inline)) { onrec(((uint32_t) p[3] << 8) | p[4], ReplayWindow::seq48(p + 3)); };
    /* after each datagram */
    auto ondgram = [&](int32_t stop) __attribute__((always_inline)) {
        if (!st && !dropped) {
            if (stop == DG_INVALID) inval++;
            else if (stop == DG_TRAILING) st = TLSREC_ERR_SSL_INTERNAL_ERROR;
            else if (stop == DG_EOF) st = TLSREC_ERR_SSL_CONN_EOF;
        }
        if (!st) done++;
        dropped = false;
    };
    if (!dtls_conn_ok(ci, ndg, slots, cap)) {
        st = TLSREC_ERR_SSL_BAD_INPUT_DATA;
    } else if (PRE && dgst) {
        /* the frame kernel's datagram summaries; each record's epoch and
         * sequence number from its descriptor (ctr, :3683-3687), loaded with
         * its slot and result DGF_U records at a time into the queue */
        uint32_t kq = first;
        uint64_t qc[DGF_U];
        auto refill = [&]() __attribute__((always_inline)) {
            kb = kq;
#pragma unroll
            for (int u = 0; u < DGF_U; u++) {
                if (kq + u < first + nrec) {
                    const uint4 a = load16(reinterpret_cast<const uint8_t *>(recs + kq + u) + 16);   /* data_len, slot, ctr */
                    ps[u] = a.y;
                    qc[u] = (uint64_t) a.z | ((uint64_t) a.w << 32);
                    pr[u] = res[kq + u];
                }
            }
            kq += DGF_U;
        };
        for (uint32_t d = ci.first_dgram; d < ci.first_dgram + ci.ndgram; d++) {
            const uint32_t u = dgst[d];
            for (uint32_t r = 0; r < (u & 0xffffffu); r++) {
                if (k - kb >= (uint32_t) DGF_U || k == first) refill();
                const uint64_t c8 = qc[0];       /* ctr bytes 0..7, little-endian */
#pragma unroll
                for (int v = 0; v + 1 < DGF_U; v++) qc[v] = qc[v + 1];
                const uint32_t epoch = ((uint32_t) (c8 & 0xff) << 8) | (uint32_t) ((c8 >> 8) & 0xff);
                uint64_t seq = 0;
#pragma unroll
                for (int b = 2; b < 8; b++) seq = (seq << 8) | ((c8 >> (8 * b)) & 0xff);
                onrec(epoch, seq);
            }
            ondgram((int32_t) (u >> 24));
        }
    } else if constexpr (PRE) {
        dtls_conn_walk<DGF_U>(ci.first_dgram, ci.first_dgram + ci.ndgram, dg, arena, ci.cid_len,
                             [&](uint64_t, const DtlsHdr &, const uint8_t *p) { hdr_rec(p); }, ondgram, prefetch);
    } else {
        for (uint32_t d = ci.first_dgram; d < ci.first_dgram + ci.ndgram; d++)
            ondgram(dtls_walk(arena + dg[d].off, dgram_len(dg[d]), ci.cid_len,
                              [&](const DtlsHdr &, const uint8_t *p) { hdr_rec(p); }));
    }
    tlsrec_dtls_in_res o;
    memset(&o, 0, sizeof(o));
    o.window_top = w.top;
    o.window = w.bits;
    o.status = st;
    o.first = first;
    o.nrec = nrec;
    o.naccepted = nacc;
    o.dgrams_done = done;
    o.invalid_dgrams = inval;
    o.badmac_seen = bms;
    o.nb_zero = (uint8_t) nbz;
    cres[i] = o;
}

template <bool PRE>
__global__ void dtls_finish_kernel(const tlsrec_dtls_in *c, uint32_t n, const tlsrec_dgram *dg, uint32_t ndg,
                                   uint8_t *arena, const uint32_t *offs, const uint32_t *counts,
                                   const SlotState *slots, uint32_t cap, const tlsrec_batch_rec *recs,
                                   const tlsrec_batch_res *res, int32_t *disp, tlsrec_dtls_in_res *cres,
                                   const uint32_t *dgst)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dtls_finish_one<PRE>(i, c, dg, ndg, arena, offs, counts, slots, cap, recs, res, disp, cres, dgst);
}

/* send: one record per datagram */
__device__ __forceinline__ uint32_t dtls_cid_of(const SlotState *slots, uint32_t slot) { return slots[slot].cid_len; }

/* protected length of an n-byte record under a TLS 1.2 key (DTLSInnerPlaintext with a CID, :874-897) */
__device__ __forceinline__ uint32_t dtls_body(const OutShape &o, uint32_t cid, uint32_t n)
{
    if (cid) {
        const uint32_t inner = n + 1;
        return o.head + inner + (o.gran - inner % o.gran) % o.gran + o.tag;
    }
    return o.head + n + o.tag;
}

__global__ void dtls_out_count_kernel(const tlsrec_stream_out *s, uint32_t n, const SlotState *slots, uint32_t cap,
                                      uint32_t *counts, unsigned long long *bytes)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long b = 0;
    if (i < n) {
        const uint32_t f = frag_of(s[i]);
        const OutShape sh = out_shape(slots, cap, s[i].slot);
        const bool ok = sh.ok && !sh.tls13;
        counts[i] = ok ? (uint32_t) (((uint64_t) s[i].in_len + f - 1) / f) : 0u;
        b = ok ? s[i].in_len : 0;
    } else if (i == n) {
        counts[n] = 0;
    }
    wave_add_bytes(bytes, b);
}

__device__ __forceinline__ void dtls_seq(uint8_t ctr[8], const uint8_t base[8], uint64_t k)
{
    const uint64_t s = (ReplayWindow::seq48(base) + k) & 0xFFFFFFFFFFFFull;
    ctr[0] = base[0];
    ctr[1] = base[1];
#pragma unroll
    for (int b = 7; b >= 2; b--) ctr[b] = (uint8_t) (s >> (8 * (7 - b)));
}

/* One wave per record: the DTLS header (type after encryption, FE FD, epoch +
 * sequence, out_cid, protected length; mbedtls_ssl_write_record :2669-2727),
 * the descriptor, and the plaintext copied behind the header -- or, with
 * srcoff (nothing to copy), one thread per record (LPR = 1, as
 * out_frame_kernel). */
template <int LPR>
__device__ __forceinline__ void dtls_out_frame_one(const tlsrec_stream_out &si, uint32_t k, uint32_t j, uint32_t lane,
                                                   const SlotState *slots, uint32_t cap, const uint8_t *in,
                                                   uint8_t *out, tlsrec_batch_rec *recs, uint64_t *srcoff)
{
    const uint32_t f = frag_of(si);
    const OutShape sh = out_shape(slots, cap, si.slot);
    const uint32_t cid = dtls_cid_of(slots, si.slot), hdr = 13 + cid;
    const uint64_t src_off = (uint64_t) k * f;
    const uint64_t left = (uint64_t) si.in_len - src_off;
    const uint32_t len = left < f ? (uint32_t) left : f;
    const uint64_t pos = si.out_off + (uint64_t) k * (hdr + dtls_body(sh, cid, f));
    /* past the 48-bit wrap (:2741-2756): never protected, no bytes written --
     * record k would reuse sequence number (epoch, k - wrap), i.e. a nonce */
    if ((uint64_t) k > 0xFFFFFFFFFFFFull - ReplayWindow::seq48(si.out_ctr)) {
        if (lane == 0) {
            tlsrec_batch_rec d;
            memset(&d, 0, sizeof(d));
            d.slot = NO_SLOT;
            recs[j] = d;
        }
        return;
    }
    if (srcoff) {                                 /* (out_frame_kernel) */
        if (lane == 0) srcoff[j] = si.in_off + src_off;
    } else {
        const uint8_t *src = in + si.in_off + src_off;
        uint8_t *dst = out + pos + hdr + sh.head;
        const uint32_t nv = len / 16;
        for (uint32_t v = lane; v < nv; v += LPR) {
            uint4 w;
            __builtin_memcpy(&w, src + 16 * v, 16);
            __builtin_memcpy(dst + 16 * v, &w, 16);
        }
        for (uint32_t b = nv * 16 + lane; b < len; b += LPR) dst[b] = src[b];
    }
    if (lane == 0) {
        const uint32_t body = dtls_body(sh, cid, len);
        uint8_t *h = out + pos;
        tlsrec_batch_rec d;
        memset(&d, 0, sizeof(d));
        dtls_seq(d.ctr, si.out_ctr, k);
        h[0] = cid ? (uint8_t) TLSREC_MSG_CID : si.type;     /* the type encrypt_buf leaves (:2727) */
        h[1] = 0xfe;                                          /* mbedtls_ssl_write_version, DTLS 1.2 */
        h[2] = 0xfd;
        memcpy(h + 3, d.ctr, 8);
        memcpy(h + 11, slots[si.slot].cid, cid);              /* out_cid (:2712-2714) */
        h[11 + cid] = (uint8_t) (body >> 8);
        h[12 + cid] = (uint8_t) body;
        d.buf_off = pos + hdr;                                /* rec.buf = out_iv */
        d.buf_len = TLSREC_DTLS_OUT_BUFFER_LEN - hdr;         /* out_buf_len - (out_iv - out_buf) */
        d.data_offset = sh.head;
        d.data_len = len;
        d.slot = si.slot;
        d.type = si.type;
        d.ver[0] = 0xfe;
        d.ver[1] = 0xfd;
        recs[j] = d;
    }
}

template <int LPR>
__global__ void __launch_bounds__(256) dtls_out_frame_kernel(const tlsrec_stream_out *s, uint32_t n,
                                                             const uint32_t *offs, uint32_t total,
                                                             const SlotState *slots, uint32_t cap, const uint8_t *in,
                                                             uint8_t *out, tlsrec_batch_rec *recs, uint64_t *srcoff)
{
    const uint32_t j = blockIdx.x * (256 / LPR) + threadIdx.x / LPR, lane = threadIdx.x % LPR;
    if (j >= total) return;
    const uint32_t i = recs[j].slot;              /* connection of record j (out_map_kernel) */
    dtls_out_frame_one<LPR>(s[i], j - offs[i], j, lane, slots, cap, in, out, recs, srcoff);
}

/* (r06) The in-place send frame (srcoff) with a group of RG lanes per
 * connection: lane q frames records q, q + RG, ... of its connection, so no
 * out_map pass has to tell each record its connection (a 4-byte write into
 * every descriptor, 17-37 us of a 1 M-record send) and a connection's
 * descriptor is read once per group, not once per record. */
template <bool DTLS>
__global__ void __launch_bounds__(RX_THREADS) out_frame_conn_kernel(const tlsrec_stream_out *s, uint32_t n,
                                                                    const uint32_t *offs, const uint32_t *counts,
                                                                    const SlotState *slots, uint32_t cap,
                                                                    const uint8_t *in, uint8_t *out,
                                                                    tlsrec_batch_rec *recs, uint64_t *srcoff)
{
    const uint32_t i = blockIdx.x * RX_CONNS + threadIdx.x / RG, q = threadIdx.x % RG;
    if (i >= n) return;
    const tlsrec_stream_out si = s[i];
    const uint32_t first = offs[i], c = counts[i];
    for (uint32_t k = q; k < c; k += RG) {
        if constexpr (DTLS)
            dtls_out_frame_one<1>(si, k, first + k, 0, slots, cap, in, out, recs, srcoff);
        else
            out_frame_one<1>(si, k, first + k, 0, slots, cap, in, out, recs, srcoff);
    }
}

__global__ void dtls_out_finish_kernel(const tlsrec_stream_out *s, uint32_t n, const uint32_t *offs,
                                       const uint32_t *counts, const SlotState *slots, uint32_t cap,
                                       const tlsrec_batch_res *res, tlsrec_stream_out_res *sres)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tlsrec_stream_out si = s[i];
    const OutShape sh = out_shape(slots, cap, si.slot);
    int32_t st = (sh.ok && !sh.tls13) || si.in_len == 0 ? 0 : TLSREC_ERR_SSL_BAD_INPUT_DATA;
    const uint32_t cid = sh.ok ? dtls_cid_of(slots, si.slot) : 0, f = frag_of(si);
    uint8_t ctr[8];
    memcpy(ctr, si.out_ctr, 8);
    uint32_t nrec = 0, olen = 0;
    const uint32_t first = offs[i], cnt = counts[i];
    for (uint32_t k = 0; k < cnt && st == 0; k++) {
        const tlsrec_batch_res &r = res[first + k];
        if (r.status) { st = r.status; break; }
        const uint64_t left = (uint64_t) si.in_len - (uint64_t) k * f;
        const uint32_t len = left < f ? (uint32_t) left : f;
        if (r.data_offset != 0 || r.data_len != dtls_body(sh, cid, len)) {          /* :2697-2700 */
            st = TLSREC_ERR_SSL_INTERNAL_ERROR;
            break;
        }
        olen += 13 + cid + r.data_len;
        nrec++;
        int b;                                                 /* :2741-2756, ep_len = 2 */
        for (b = 8; b > 2; b--)
            if (++ctr[b - 1] != 0) break;
        if (b == 2) st = TLSREC_ERR_SSL_COUNTER_WRAPPING;
    }
    tlsrec_stream_out_res o;
    memset(&o, 0, sizeof(o));
    o.status = st;
    o.first = first;
    o.nrec = nrec;
    o.out_len = olen;
    memcpy(o.out_ctr, ctr, 8);
    o.nparsed = cnt;
    sres[i] = o;
}

/* The batch's record count and byte total to the host (r06): one wave sums
 * the spread byte counters and writes both into the calling thread's
 * host-mapped mailbox, then the call's sequence number after a release
 * fence.  Replaces two device-to-host copies and a stream synchronize: the
 * host reads the totals while the kernels queued behind this one (the
 * descriptor emit) still run.  (The copies cost 4 us each with a 20 us gap
 * between them, and the launch after the synchronize another 30 us, per
 * receive call; profiles/r06/ab/mailbox/.) */
__global__ void __launch_bounds__(64) totals_kernel(const uint32_t *total_p, const unsigned long long *spread,
                                                    TotMbox *mb, uint64_t seq)
{
    const int lane = threadIdx.x;
    unsigned long long v = lane < BYTES_SPREAD ? spread[lane * BYTES_STRIDE] : 0ull;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) {
        mb->total = *total_p;
        mb->bytes = v;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(&mb->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

} /* namespace tlsst */

using namespace tlsst;

/* ======================================================================
 * host side
 * ==================================================================== */
namespace {
struct Scratch {
    tlsrec_scratch_lease lease = { nullptr, nullptr };
    uint32_t *counts = nullptr, *offs = nullptr;
    HdrStop *stops = nullptr;
    unsigned long long *bytes = nullptr;   /* record bytes of the batch (its mean size steers the GCM launch) */
    unsigned long long *tstat = nullptr;   /* one-pass framing: tile status words (zeroed with bytes) */
    uint32_t *tctr = nullptr;              /* one-pass framing: tile counter */
    void *scan_tmp = nullptr;
    size_t scan_bytes = 0;
};
}

/* TLSREC_RX_FUSED=0: the DTLS receive framing as count, scan and emit
 * kernels (r05 / early r06), kept for A/B runs and as the tests' second path;
 * TLSREC_RX_FUSED_STREAM=1: the stream receive framing in one pass (measured
 * slower than its three kernels) */
static bool fused_env(void)
{
    const char *e = getenv("TLSREC_RX_FUSED");
    return !(e && atoi(e) == 0);
}
/* TLSREC_DTLS_STASH=0: the DTLS frame kernel's emit walks the headers again
 * instead of reading the count walk's LDS copy (A/B runs) */
static bool dtls_stash_env(void)
{
    const char *e = getenv("TLSREC_DTLS_STASH");
    return !(e && atoi(e) == 0);
}
/* TLSREC_RX_PREFILL=0: the receive batch runs its guard kernel although the
 * emit kernels wrote the guard results (A/B runs) */
static int prefill_env(void)
{
    const char *e = getenv("TLSREC_RX_PREFILL");
    return (e && atoi(e) == 0) ? 0 : 1;
}
/* lanes per connection of the receive header walk: the records a
 * connection can hold on average by the caller's capacity (max_records /
 * connections) -- 4, 8 or 16; TLSREC_RX_RG forces one */
static int rx_group(uint32_t n, uint32_t max_records)
{
    const char *e = getenv("TLSREC_RX_RG");
    if (e) {
        const int g = atoi(e);
        if (g == 4 || g == 8 || g == 16) return g;
    }
    const uint64_t per = n ? ((uint64_t) max_records + n - 1) / n : 16;
    return per <= 4 ? 4 : (per <= 8 ? 8 : 16);
}

template <int G>
static void launch_rx_count(uint32_t n, hipStream_t st, const tlsrec_stream_in *s, const uint8_t *arena,
                            uint32_t *counts, HdrStop *stops, unsigned long long *bytes)
{
    hipLaunchKernelGGL(in_count_group_kernel<G>, dim3((n + 1 + RX_THREADS / G - 1) / (RX_THREADS / G)),
                       dim3(RX_THREADS), 0, st, s, n, arena, counts, stops, bytes);
}

template <int G>
static void launch_rx_emit(uint32_t n, hipStream_t st, const tlsrec_stream_in *s, const uint8_t *arena,
                           const uint32_t *offs, const SlotState *slots, uint32_t cap, tlsrec_batch_rec *recs,
                           uint32_t max_records, tlsrec_batch_res *res)
{
    hipLaunchKernelGGL(in_emit_group_kernel<G>, dim3((n + RX_THREADS / G - 1) / (RX_THREADS / G)), dim3(RX_THREADS),
                       0, st, s, n, arena, offs, slots, cap, recs, max_records, res);
}

static bool fused_stream_env(void)
{
    const char *e = getenv("TLSREC_RX_FUSED_STREAM");
    return e && atoi(e) != 0;
}

/* the send paths read the application data in place (r05; TLSREC_STREAM_SRC=0
 * copies it into the output stream first, as r04 did) */
static bool src_env(void)
{
    const char *e = getenv("TLSREC_STREAM_SRC");
    return !(e && atoi(e) == 0);
}

/* tiles: the one-pass framing kernels' tile status words (0 = none) */
static int scratch_alloc(Scratch &sc, uint32_t n, hipStream_t st, uint32_t tiles = 0)
{
    sc.scan_bytes = tlsrec__scan_scratch_bytes(n + 1);
    const size_t a = 256, sz4 = (((size_t) n + 1) * 4 + a - 1) / a * a, szs = ((size_t) n * sizeof(HdrStop) + a) / a * a;
    constexpr size_t szb = BYTES_SPREAD * BYTES_STRIDE * 8;     /* the spread byte counters */
    const size_t szt = tiles ? ((size_t) tiles * 8 + a) / a * a + a : 0;   /* status words + the counter's line */
    const int lr = tlsrec__scratch_acquire(st, 1, 2 * sz4 + szs + szb + szt + sc.scan_bytes + a, &sc.lease);
    if (lr) return lr;
    uint8_t *m = (uint8_t *) sc.lease.mem;
    sc.counts = (uint32_t *) m;
    sc.offs = (uint32_t *) (m + sz4);
    sc.stops = (HdrStop *) (m + 2 * sz4);
    sc.bytes = (unsigned long long *) (m + 2 * sz4 + szs);
    if (tiles) {
        sc.tstat = (unsigned long long *) (m + 2 * sz4 + szs + szb);
        sc.tctr = (uint32_t *) (m + 2 * sz4 + szs + szb + szt - a);
    }
    sc.scan_tmp = m + 2 * sz4 + szs + szb + szt;
    return hipMemsetAsync(sc.bytes, 0, szb + szt, st) == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
}

/* The calling thread's host-mapped mailbox (allocated on first use, kept:
 * a thread's calls are sequential, so one mailbox per thread serves them) */
namespace {
struct Mailbox {
    TotMbox *h = nullptr, *d = nullptr;
    uint64_t seq = 0;
};
thread_local Mailbox t_mbox;
}

/* TLSREC_RX_MAILBOX=0: the totals come back by two copies and a stream
 * synchronize (before r06's second session), for A/B runs */
static bool mailbox_env(void)
{
    const char *e = getenv("TLSREC_RX_MAILBOX");
    return !(e && atoi(e) == 0);
}

/* the calling thread's mailbox (device pointer) and the next sequence
 * number; null with the copy path (TLSREC_RX_MAILBOX=0) or no mailbox */
static TotMbox *mailbox_next(uint64_t *seq)
{
    *seq = 0;
    if (!mailbox_env()) return nullptr;
    Mailbox &m = t_mbox;
    if (!m.h) {
        void *h = nullptr, *d = nullptr;
        if (hipHostMalloc(&h, 256, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
            return nullptr;
        memset(h, 0, 256);
        if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
            hipHostFree(h);
            return nullptr;
        }
        m.h = (TotMbox *) h;
        m.d = (TotMbox *) d;
    }
    *seq = ++m.seq;
    return m.d;
}

/* queue the totals kernel: offs[n] and the byte counters to the mailbox;
 * *seq = the value collect_totals waits for (0: the copy path, nothing queued) */
static int publish_totals(Scratch &sc, uint32_t n, hipStream_t st, uint64_t *seq)
{
    TotMbox *mb = mailbox_next(seq);
    if (!mb) {
        *seq = 0;
        return 0;
    }
    hipLaunchKernelGGL(totals_kernel, dim3(1), dim3(64), 0, st, sc.offs + n, sc.bytes, mb, *seq);
    return hipGetLastError() == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
}

/* the totals publish_totals queued (seq != 0), or by copies and a stream
 * synchronize (seq == 0); the mean record size into *avg_bytes */
static int collect_totals(Scratch &sc, uint32_t n, hipStream_t st, uint64_t seq, uint32_t *total,
                          uint32_t *avg_bytes)
{
    unsigned long long bytes = 0;
    if (seq) {
        TotMbox *h = t_mbox.h;
        for (uint64_t it = 0;; it++) {
            if (__atomic_load_n(&h->seq, __ATOMIC_ACQUIRE) == seq) break;
            if ((it & 1023) == 1023) {      /* a stream that failed or drained without the totals: an error */
                const hipError_t q = hipStreamQuery(st);
                if (q != hipSuccess && q != hipErrorNotReady) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
                if (q == hipSuccess && __atomic_load_n(&h->seq, __ATOMIC_ACQUIRE) != seq)
                    return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
            }
            /* queued behind long work on the stream: stop holding the CPU
             * after ~100 us of spinning */
            if (it > 65536) sched_yield();
        }
        *total = (uint32_t) __atomic_load_n(&h->total, __ATOMIC_RELAXED);
        bytes = __atomic_load_n(&h->bytes, __ATOMIC_RELAXED);
    } else {
        unsigned long long spread[BYTES_SPREAD * BYTES_STRIDE];
        if (hipMemcpyAsync(total, sc.offs + n, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(spread, sc.bytes, sizeof(spread), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        for (int k = 0; k < BYTES_SPREAD; k++) bytes += spread[k * BYTES_STRIDE];
    }
    if (avg_bytes) *avg_bytes = *total ? (uint32_t) (bytes / *total) : 0u;
    return 0;
}

/* after a one-pass framing kernel: offs[n] (the total) and the mean record
 * size to the host */
static int fetch_total(Scratch &sc, uint32_t n, hipStream_t st, uint32_t *total, uint32_t *avg_bytes)
{
    uint64_t seq;
    const int r = publish_totals(sc, n, st, &seq);
    return r ? r : collect_totals(sc, n, st, seq, total, avg_bytes);
}

/* TLSREC_RX_GROUPWALK=0: the r05 receive framing (one lane per connection
 * in the count and emit kernels), kept for A/B runs and as the tests' second
 * path */
static bool groupwalk_env(void)
{
    const char *e = getenv("TLSREC_RX_GROUPWALK");
    return !(e && atoi(e) == 0);
}

/* exclusive scan of counts[0..n] -> offs, and the totals queued to the
 * mailbox (*seq, see publish_totals): collect them with collect_totals */
static int scan_publish(Scratch &sc, uint32_t n, hipStream_t st, uint64_t *seq)
{
    if (tlsrec__exclusive_scan(sc.counts, sc.offs, n + 1, (uint32_t *) sc.scan_tmp, st) != hipSuccess)
        return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    return publish_totals(sc, n, st, seq);
}

/* exclusive scan of counts[0..n] -> offs; returns offs[n] (the total) on the
 * host, and the mean record size of the batch (0 if unknown) */
static int scan_total(Scratch &sc, uint32_t n, hipStream_t st, uint32_t *total, uint32_t *avg_bytes = nullptr)
{
    uint64_t seq;
    const int r = scan_publish(sc, n, st, &seq);
    return r ? r : collect_totals(sc, n, st, seq, total, avg_bytes);
}

static inline uint32_t blocks(uint32_t n, uint32_t t) { return (n + t - 1) / t; }

extern "C" int tlsrec_stream_decrypt(const tlsrec_keytab *kt, const tlsrec_stream_in *streams, uint32_t nstreams,
                                     uint8_t *arena, tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                     uint32_t max_records, tlsrec_stream_in_res *sres, uint32_t *nrecords,
                                     void *stream)
{
    if (nrecords) *nrecords = 0;
    if (!kt || (nstreams && (!streams || !arena || !sres))) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (nstreams == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    const SlotState *slots = tlsrec__keytab_slots(kt);
    const uint32_t cap = tlsrec_keytab_capacity(kt);
    Scratch sc;
    const bool fused = fused_stream_env() && groupwalk_env();
    /* one pass: G lanes per connection, tiles of 512 connections (G = 4:
     * two chunks of 128) or 128 (G = 16: eight chunks of 16) */
    const int frg = rx_group(nstreams, max_records);
    const uint32_t ftile = frg == 4 ? 2u * 64u : (frg == 8 ? 4u * 32u : 8u * 16u);
    const uint32_t tiles = blocks(nstreams, ftile);
    int r = scratch_alloc(sc, nstreams, st, fused ? tiles : 0u);
    uint32_t total = 0, avg = 0;
    const bool gw = groupwalk_env();
    if (r == 0 && fused) {
        /* count, scan and emit in one pass (descriptors up to max_records) */
        /* tiles of 128 connections: one chunk of 128 at 4 lanes (512 threads),
         * or chunks of 64 / 32 at 8 / 16 lanes */
        constexpr int FNT = TLSREC_RX_FRAME_NT;
        if (frg == 4)
            hipLaunchKernelGGL((in_frame_kernel<4, 512 / FNT, FNT>), dim3(tiles), dim3(FNT), 0, st, streams, nstreams,
                               (const uint8_t *) arena, slots, cap, sc.counts, sc.offs, sc.stops, sc.bytes, sc.tstat,
                               sc.tctr, recs, (recs && res) ? max_records : 0u, res);
        else if (frg == 8)
            hipLaunchKernelGGL((in_frame_kernel<8, 1024 / FNT, FNT>), dim3(tiles), dim3(FNT), 0, st, streams,
                               nstreams, (const uint8_t *) arena, slots, cap, sc.counts, sc.offs, sc.stops, sc.bytes,
                               sc.tstat, sc.tctr, recs, (recs && res) ? max_records : 0u, res);
        else
            hipLaunchKernelGGL((in_frame_kernel<16, 2048 / FNT, FNT>), dim3(tiles), dim3(FNT), 0, st, streams,
                               nstreams, (const uint8_t *) arena, slots, cap, sc.counts, sc.offs, sc.stops, sc.bytes,
                               sc.tstat, sc.tctr, recs, (recs && res) ? max_records : 0u, res);
        r = hipGetLastError() == hipSuccess ? fetch_total(sc, nstreams, st, &total, &avg)
                                            : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    } else if (r == 0) {
        const int rg = rx_group(nstreams, max_records);
        if (gw) {
            if (rg == 4)
                launch_rx_count<4>(nstreams, st, streams, (const uint8_t *) arena, sc.counts, sc.stops, sc.bytes);
            else if (rg == 8)
                launch_rx_count<8>(nstreams, st, streams, (const uint8_t *) arena, sc.counts, sc.stops, sc.bytes);
            else
                launch_rx_count<16>(nstreams, st, streams, (const uint8_t *) arena, sc.counts, sc.stops, sc.bytes);
        } else
            hipLaunchKernelGGL(in_count_kernel, dim3(blocks(nstreams + 1, 256)), dim3(256), 0, st, streams, nstreams,
                               (const uint8_t *) arena, sc.counts, sc.stops, sc.bytes);
        uint64_t seq = 0;
        r = hipGetLastError() == hipSuccess ? scan_publish(sc, nstreams, st, &seq) : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        /* the descriptors are emitted while the host collects the totals
         * (r06; at most max_records of them: the check follows) */
        if (r == 0 && recs && res) {
            if (gw && rg == 4)
                launch_rx_emit<4>(nstreams, st, streams, (const uint8_t *) arena, sc.offs, slots, cap, recs,
                                  max_records, res);
            else if (gw && rg == 8)
                launch_rx_emit<8>(nstreams, st, streams, (const uint8_t *) arena, sc.offs, slots, cap, recs,
                                  max_records, res);
            else if (gw)
                launch_rx_emit<16>(nstreams, st, streams, (const uint8_t *) arena, sc.offs, slots, cap, recs,
                                   max_records, res);
            else
                hipLaunchKernelGGL(in_emit_kernel, dim3(blocks(nstreams, 256)), dim3(256), 0, st, streams, nstreams,
                                   (const uint8_t *) arena, sc.offs, slots, cap, recs, max_records, res);
            if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        }
        if (r == 0) r = collect_totals(sc, nstreams, st, seq, &total, &avg);
    }
    if (r == 0 && total > max_records) r = TLSREC_ERR_SSL_BUFFER_TOO_SMALL;
    if (r == 0 && total && (!recs || !res)) r = TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (r == 0 && total) r = tlsrec__batch_sized(kt, recs, res, total, arena, arena, stream, 1, avg, prefill_env());
    if (r == 0) {
        hipLaunchKernelGGL(in_finish_kernel, dim3(blocks(nstreams, 256)), dim3(256), 0, st, streams, nstreams, sc.offs,
                           sc.counts, sc.stops, slots, cap, recs, res, sres);
        if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    tlsrec__scratch_release(&sc.lease);
    if (r == 0 && nrecords) *nrecords = total;
    return r;
}

extern "C" uint64_t tlsrec_stream_out_size(int tls_version, int cipher, uint32_t granularity, uint64_t in_len,
                                           uint32_t max_frag)
{
    if (tlsrec_cipher_keylen(cipher) == 0) return 0;
    const uint64_t tag = tlsrec_cipher_taglen(cipher);
    if (tls_version != TLSREC_VERSION_TLS1_2 && tls_version != TLSREC_VERSION_TLS1_3) return 0;
    const uint64_t f = max_frag ? max_frag : 16384;
    const uint64_t g = granularity ? granularity : 16;
    const uint64_t head = (tls_version == TLSREC_VERSION_TLS1_2 && cipher != TLSREC_CIPHER_CHACHA20_POLY1305) ? 8 : 0;
    auto body = [&](uint64_t n) -> uint64_t {
        if (tls_version == TLSREC_VERSION_TLS1_3) {
            const uint64_t inner = n + 1;
            return inner + (g - inner % g) % g + tag;
        }
        return head + n + tag;
    };
    const uint64_t full = in_len / f, rest = in_len % f;
    return full * (5 + body(f)) + (rest ? 5 + body(rest) : 0);
}

extern "C" int tlsrec_stream_encrypt(const tlsrec_keytab *kt, const tlsrec_stream_out *streams, uint32_t nstreams,
                                     const uint8_t *in_arena, uint8_t *out_arena, tlsrec_batch_rec *recs,
                                     tlsrec_batch_res *res, uint32_t max_records, tlsrec_stream_out_res *sres,
                                     uint32_t *nrecords, void *stream)
{
    if (nrecords) *nrecords = 0;
    if (!kt || (nstreams && (!streams || !in_arena || !out_arena || !sres))) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (nstreams == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    const SlotState *slots = tlsrec__keytab_slots(kt);
    const uint32_t cap = tlsrec_keytab_capacity(kt);
    Scratch sc;
    int r = scratch_alloc(sc, nstreams, st);
    uint32_t total = 0, avg = 0;
    if (r == 0) {
        hipLaunchKernelGGL(out_count_kernel, dim3(blocks(nstreams + 1, 256)), dim3(256), 0, st, streams, nstreams,
                           slots, cap, sc.counts, sc.bytes);
        r = hipGetLastError() == hipSuccess ? scan_total(sc, nstreams, st, &total, &avg)
                                            : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (r == 0 && total > max_records) r = TLSREC_ERR_SSL_BUFFER_TOO_SMALL;
    if (r == 0 && total && (!recs || !res)) r = TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (r == 0 && total) {
        /* AES-GCM / ChaCha20-Poly1305 tables: the AEAD reads the application
         * data in place (tlsrec__batch_src); other AEADs: copy, then in place */
        uint64_t *srcoff = nullptr;
        tlsrec_scratch_lease sl = { nullptr, nullptr };
        if (tlsrec__keytab_src_ok(kt) && src_env() &&
            tlsrec__scratch_acquire(st, 3, (size_t) total * sizeof(uint64_t), &sl) == 0)
            srcoff = (uint64_t *) sl.mem;
        if (srcoff) {
            hipLaunchKernelGGL(out_frame_conn_kernel<false>, dim3(blocks(nstreams, RX_CONNS)), dim3(RX_THREADS), 0, st,
                               streams, nstreams, sc.offs, sc.counts, slots, cap, in_arena, out_arena, recs, srcoff);
        } else {
            hipLaunchKernelGGL(out_map_kernel, dim3(blocks(nstreams, 4)), dim3(256), 0, st, nstreams, sc.offs,
                               sc.counts, recs);
            hipLaunchKernelGGL(out_frame_kernel<64>, dim3(blocks(total, 4)), dim3(256), 0, st, streams, nstreams,
                               sc.offs, total, slots, cap, in_arena, out_arena, recs, srcoff);
        }
        if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        if (r == 0)
            r = srcoff ? tlsrec__batch_src(kt, recs, res, total, in_arena, out_arena, stream, avg, srcoff)
                       : tlsrec__batch_sized(kt, recs, res, total, out_arena, out_arena, stream, 0, avg, 0);
        if (srcoff) tlsrec__scratch_release(&sl);
    }
    if (r == 0) {
        hipLaunchKernelGGL(out_finish_kernel, dim3(blocks(nstreams, 256)), dim3(256), 0, st, streams, nstreams,
                           sc.offs, sc.counts, slots, cap, res, sres);
        if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    tlsrec__scratch_release(&sc.lease);
    if (r == 0 && nrecords) *nrecords = total;
    return r;
}

extern "C" int tlsrec_stream_read(const tlsrec_stream_in_res *sres, uint32_t nstreams, const tlsrec_batch_rec *recs,
                                  const tlsrec_batch_res *res, uint8_t *arena, const tlsrec_stream_read_req *req,
                                  uint8_t *out_arena, tlsrec_stream_read_res *rres, void *stream)
{
    if (nstreams && (!sres || !recs || !res || !arena || !req || !out_arena || !rres)) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (nstreams == 0) return 0;
    hipLaunchKernelGGL(read_kernel, dim3(nstreams), dim3(256), 0, (hipStream_t) stream, sres, nstreams, recs, res,
                       arena, req, out_arena, rres);
    return hipGetLastError() == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
}

/* ---------------- DTLS host side ---------------------------------------- */
extern "C" int tlsrec_dtls_decrypt(const tlsrec_keytab *kt, const tlsrec_dtls_in *conns, uint32_t nconns,
                                   const tlsrec_dgram *dgrams, uint32_t ndgrams, uint8_t *arena,
                                   tlsrec_batch_rec *recs, tlsrec_batch_res *res, int32_t *disp,
                                   uint32_t max_records, tlsrec_dtls_in_res *cres, uint32_t *nrecords, void *stream)
{
    if (nrecords) *nrecords = 0;
    if (!kt || (nconns && (!conns || !cres || (ndgrams && (!dgrams || !arena))))) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (nconns == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    const SlotState *slots = tlsrec__keytab_slots(kt);
    const uint32_t cap = tlsrec_keytab_capacity(kt);
    Scratch sc;
    const bool fused = fused_env();
    const uint32_t tiles = blocks(nconns, DG_THREADS);
    int r = scratch_alloc(sc, nconns, st, fused ? tiles : 0u);
    uint32_t total = 0, avg = 0;
    tlsrec_scratch_lease dgl = { nullptr, nullptr };
    uint32_t *dgst = nullptr;
    if (r == 0 && fused) {
        /* count, scan and emit in one pass (descriptors up to max_records) */
        uint64_t seq = 0;
#ifndef TLSREC_DTLS_LASTTILE_MB
#define TLSREC_DTLS_LASTTILE_MB 1
#endif
        /* the frame kernel's last tile writes the totals into the mailbox
         * (r06; 0 in A/B builds: the totals kernel after the frame kernel) */
        TotMbox *mb = TLSREC_DTLS_LASTTILE_MB ? mailbox_next(&seq) : nullptr;
        /* the datagram summaries for the finish (none: it walks the headers) */
        if (ndgrams && tlsrec__scratch_acquire(st, 2, (size_t) ndgrams * 4, &dgl) == 0) dgst = (uint32_t *) dgl.mem;
        /* LDS for the records of a connection of mean size (4 / 16 records:
         * 24 / 96 KiB per workgroup); TLSREC_DTLS_STASH=0: the emit walks the
         * headers again */
        const uint32_t per = nconns ? (uint32_t) ((ndgrams + nconns - 1) / nconns) : 0;
#define TLSREC_DTLS_FRAME(S_) hipLaunchKernelGGL(dtls_frame_kernel<S_>, dim3(tiles), dim3(DG_THREADS), 0, st, conns, \
                           nconns, dgrams, ndgrams, (const uint8_t *) arena, slots, cap, sc.counts, sc.offs, sc.bytes, \
                           sc.tstat, sc.tctr, recs, (recs && res) ? max_records : 0u, res, mb, seq, dgst)
        if (!dtls_stash_env() || per > 16) TLSREC_DTLS_FRAME(0);
        else if (per > 4) TLSREC_DTLS_FRAME(16);
        else TLSREC_DTLS_FRAME(4);
#undef TLSREC_DTLS_FRAME
        if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        else if (mb) r = collect_totals(sc, nconns, st, seq, &total, &avg);
        else r = fetch_total(sc, nconns, st, &total, &avg);
    } else if (r == 0) {
        hipLaunchKernelGGL(dtls_count_kernel, dim3(blocks(nconns + 1, 256)), dim3(256), 0, st, conns, nconns, dgrams,
                           ndgrams, (const uint8_t *) arena, slots, cap, sc.counts, sc.bytes);
        uint64_t seq = 0;
        r = hipGetLastError() == hipSuccess ? scan_publish(sc, nconns, st, &seq) : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        if (r == 0 && recs && res) {   /* emitted while the host collects the totals (as the stream path) */
            hipLaunchKernelGGL(dtls_emit_kernel, dim3(blocks(nconns, 256)), dim3(256), 0, st, conns, nconns, dgrams,
                               ndgrams, (const uint8_t *) arena, sc.offs, slots, cap, recs, max_records, res);
            if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        }
        if (r == 0) r = collect_totals(sc, nconns, st, seq, &total, &avg);
    }
    if (r == 0 && total > max_records) r = TLSREC_ERR_SSL_BUFFER_TOO_SMALL;
    if (r == 0 && total && (!recs || !res || !disp)) r = TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (r == 0 && total) r = tlsrec__batch_sized(kt, recs, res, total, arena, arena, stream, 1, avg, prefill_env());
    if (r == 0) {
        if (fused)
            hipLaunchKernelGGL(dtls_finish_kernel<true>, dim3(blocks(nconns, 256)), dim3(256), 0, st, conns, nconns,
                               dgrams, ndgrams, arena, sc.offs, sc.counts, slots, cap, recs, res, disp, cres, dgst);
        else
            hipLaunchKernelGGL(dtls_finish_kernel<false>, dim3(blocks(nconns, 256)), dim3(256), 0, st, conns, nconns,
                               dgrams, ndgrams, arena, sc.offs, sc.counts, slots, cap, recs, res, disp, cres,
                               (const uint32_t *) nullptr);
        if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (dgl.mem) tlsrec__scratch_release(&dgl);
    tlsrec__scratch_release(&sc.lease);
    if (r == 0 && nrecords) *nrecords = total;
    return r;
}

extern "C" uint64_t tlsrec_dtls_out_size(int cipher, uint32_t granularity, uint32_t cid_len, uint64_t in_len,
                                         uint32_t max_frag)
{
    if (tlsrec_cipher_keylen(cipher) == 0 || cid_len > TLSREC_CID_LEN_MAX) return 0;
    const uint64_t tag = tlsrec_cipher_taglen(cipher);
    const uint64_t f = max_frag ? max_frag : 16384;
    const uint64_t g = granularity ? granularity : 16;
    const uint64_t head = cipher != TLSREC_CIPHER_CHACHA20_POLY1305 ? 8 : 0;
    auto body = [&](uint64_t n) -> uint64_t {
        if (cid_len) {
            const uint64_t inner = n + 1;
            return head + inner + (g - inner % g) % g + tag;
        }
        return head + n + tag;
    };
    const uint64_t full = in_len / f, rest = in_len % f;
    return full * (13 + cid_len + body(f)) + (rest ? 13 + cid_len + body(rest) : 0);
}

extern "C" int tlsrec_dtls_encrypt(const tlsrec_keytab *kt, const tlsrec_stream_out *streams, uint32_t nstreams,
                                   const uint8_t *in_arena, uint8_t *out_arena, tlsrec_batch_rec *recs,
                                   tlsrec_batch_res *res, uint32_t max_records, tlsrec_stream_out_res *sres,
                                   uint32_t *nrecords, void *stream)
{
    if (nrecords) *nrecords = 0;
    if (!kt || (nstreams && (!streams || !in_arena || !out_arena || !sres))) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (nstreams == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    const SlotState *slots = tlsrec__keytab_slots(kt);
    const uint32_t cap = tlsrec_keytab_capacity(kt);
    Scratch sc;
    int r = scratch_alloc(sc, nstreams, st);
    uint32_t total = 0, avg = 0;
    if (r == 0) {
        hipLaunchKernelGGL(dtls_out_count_kernel, dim3(blocks(nstreams + 1, 256)), dim3(256), 0, st, streams, nstreams,
                           slots, cap, sc.counts, sc.bytes);
        r = hipGetLastError() == hipSuccess ? scan_total(sc, nstreams, st, &total, &avg)
                                            : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (r == 0 && total > max_records) r = TLSREC_ERR_SSL_BUFFER_TOO_SMALL;
    if (r == 0 && total && (!recs || !res)) r = TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (r == 0 && total) {
        /* AES-GCM / ChaCha20-Poly1305 tables: the AEAD reads the application
         * data in place (tlsrec__batch_src); other AEADs: copy, then in place */
        uint64_t *srcoff = nullptr;
        tlsrec_scratch_lease sl = { nullptr, nullptr };
        if (tlsrec__keytab_src_ok(kt) && src_env() &&
            tlsrec__scratch_acquire(st, 3, (size_t) total * sizeof(uint64_t), &sl) == 0)
            srcoff = (uint64_t *) sl.mem;
        if (srcoff) {
            hipLaunchKernelGGL(out_frame_conn_kernel<true>, dim3(blocks(nstreams, RX_CONNS)), dim3(RX_THREADS), 0, st,
                               streams, nstreams, sc.offs, sc.counts, slots, cap, in_arena, out_arena, recs, srcoff);
        } else {
            hipLaunchKernelGGL(out_map_kernel, dim3(blocks(nstreams, 4)), dim3(256), 0, st, nstreams, sc.offs,
                               sc.counts, recs);
            hipLaunchKernelGGL(dtls_out_frame_kernel<64>, dim3(blocks(total, 4)), dim3(256), 0, st, streams, nstreams,
                               sc.offs, total, slots, cap, in_arena, out_arena, recs, srcoff);
        }
        if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        if (r == 0)
            r = srcoff ? tlsrec__batch_src(kt, recs, res, total, in_arena, out_arena, stream, avg, srcoff)
                       : tlsrec__batch_sized(kt, recs, res, total, out_arena, out_arena, stream, 0, avg, 0);
        if (srcoff) tlsrec__scratch_release(&sl);
    }
    if (r == 0) {
        hipLaunchKernelGGL(dtls_out_finish_kernel, dim3(blocks(nstreams, 256)), dim3(256), 0, st, streams, nstreams,
                           sc.offs, sc.counts, slots, cap, res, sres);
        if (hipGetLastError() != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    tlsrec__scratch_release(&sc.lease);
    if (r == 0 && nrecords) *nrecords = total;
    return r;
}
