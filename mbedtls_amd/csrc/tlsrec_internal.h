/*
 * tlsrec_internal.h -- layouts shared by the kernels and the engine (C++).
 */
#ifndef TLSREC_INTERNAL_H
#define TLSREC_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tlsrec.h"

namespace tlsrec {

/* Test hooks, the reference's MBEDTLS_TEST_HOOKS (ssl_misc.h:2685): only the
 * test build (libtlsrec_test.so, -DTLSREC_TEST_HOOKS, tests/ only) can leave a
 * record unreached by the kernels; in the release library the compare is
 * compiled out and no entry point sets it. */
#ifdef TLSREC_TEST_HOOKS
#define TLSREC_HOOK_SKIP(rec, skip) ((rec) == (skip))
#else
#define TLSREC_HOOK_SKIP(rec, skip) false
#endif

constexpr int KEY_TABLES = 7;                      /* H^1, H^2, ..., H^64 (4-bit position tables) */
/* plus H^8 as 5-bit position tables read in 8-byte halves (gmul5 in
 * tlsrec_device.h): 26 windows x 512 B, the 8-lane Horner multiplier */
constexpr int KEY_G5_POWER = 3;                     /* H^(2^3) */
constexpr int KEY_G5_WORDS = 26 * 32;               /* uint4 entries (13 KiB) */
constexpr int KEY_G5_OFF = KEY_TABLES * 512;        /* uint4 offset of the G5 table in a slot */
/* then H^1 .. H^64 as values (GCM-string words, 1 KiB): lane q of an L-lane
 * record multiplies its Horner sum by H^(L-q) once (the GCM kernel's lane
 * powers, GcmArgs::tm bit 3), and the record server's closing powers */
constexpr int KEY_HPOW_OFF = KEY_G5_OFF + KEY_G5_WORDS;
constexpr int KEY_HPOW_N = 64;
constexpr int KEY_TABLE_WORDS = KEY_TABLES * 512 + KEY_G5_WORDS + KEY_HPOW_N;   /* uint4 entries per slot (70 KiB) */

constexpr int GCM_WAVES = 16;                       /* default waves per workgroup (one WG per CU) */
/* The bucket pass counts ChaCha20-Poly1305 records (one class for every key:
 * the kernel takes each record's key itself) on CP_COUNTERS counters, a wave's
 * records on counter (wave index mod CP_COUNTERS): on one counter, 2 M records
 * round-robin over keys were 65 K same-address atomics, 0.75 ms of a c4s step.
 * (r06) The counters sit CP_STRIDE entries apart, one per 128-byte line: all
 * 64 in two lines still serialized the ChaCha half's 65 K atomics on two L2
 * channels (a c4s count kernel of 328 us); the class block spans CP_SPREAD
 * entries, the unused ones count nothing. */
constexpr uint32_t CP_COUNTERS = 64;
constexpr uint32_t CP_STRIDE = 32;
constexpr uint32_t CP_SPREAD = CP_COUNTERS * CP_STRIDE;
constexpr int CP_THREADS = 256;
constexpr int ARIA_GCM_WAVES = 16;   /* waves per ARIA-GCM workgroup (kernels.hip launch_gcm_aria) */
constexpr int CP_WAVES = CP_THREADS / 64;

/* Expanded per-slot state, 1024 bytes. */
struct SlotState {
    tlsrec_key_material km;   /* raw material as loaded */
    uint32_t rk[60];          /* AES round keys, little-endian column words */
    uint32_t rkr[60];         /* same, middle rounds 1..NR-1 stored rotr16 (aes_encrypt) */
    uint32_t nr;              /* 10 / 14, 0 for ChaCha20-Poly1305 */
    uint8_t h[16];            /* H = E_K(0^128) */
    uint8_t cid_len;          /* DTLS 1.2 connection ID of this transform direction */
    uint8_t cid[32];          /* (out_cid encrypting, in_cid decrypting), tlsrec_keytab_set_cid */
    uint8_t pad0[3];
    uint32_t ark[68];         /* ARIA: the nr + 1 round keys ek1.. (RFC 5794 2.2), 16 B each as LE words;
                                 Camellia: the 26 / 34 64-bit subkeys as (high, low) words */
    uint32_t hpow[4][4];      /* GCM: H^2, H^4, H^8, H^16 as GCM-string words (the table-free lane tree) */
    uint8_t pad[1024 - 64 - 240 - 240 - 4 - 16 - 33 - 3 - 272 - 64];
};
static_assert(sizeof(SlotState) == 1024, "SlotState layout");
static_assert(sizeof(tlsrec_key_material) == 64, "key material layout");
static_assert(sizeof(tlsrec_batch_rec) == 40, "batch record layout");
static_assert(sizeof(tlsrec_batch_res) == 16, "batch result layout");

/* Records a kernel processes: positions [*lo, *hi) of `perm` (record
 * indices grouped by key, built by the bucket pass), or, with perm == NULL,
 * positions [0, n) of the descriptor array itself (identity order: a table
 * holding a single key).  lo/hi live in device memory so the launches need
 * no host synchronisation. */
constexpr uint32_t GCM_DUMMY_BYTES = 65536;

struct GcmArgs {
    const SlotState *slots;
    const uint4 *ghtab;
    const tlsrec_batch_rec *recs;
    tlsrec_batch_res *res;
    uint64_t n;
    const uint32_t *perm;
    const uint32_t *lo, *hi;
    const uint8_t *in;
    uint8_t *out;
    uint32_t rpw;             /* records per wavefront chunk (<= 64) */
    uint32_t capacity;
    uint32_t cipher;          /* TLSREC_CIPHER_AES_128_GCM / _256_GCM / _192_GCM */
    uint32_t g5;              /* host-side launch choice: 5-bit GHASH Horner table (8-lane, 16-wave kernel) */
    uint32_t tm;              /* wave passes, table-free multiplies (tlsrec_clmul.h): bit 0 the 16-lane tree,
                                 bit 1 the 2- / 4- / 8- / 32-lane tree, bit 2 the AAD fold and final multiplies,
                                 bit 3 lane powers: AAD and length block in the lane layout, one multiply by
                                 H^(L-q) per lane and an XOR over the record's lanes instead of all of these */
    uint32_t skip;            /* test hook (tlsrec__test_skip_record): this record index is never reached */
    const tlsrec_batch_rec *srecs;   /* with perm: the descriptors in perm order (srecs[p] = recs[perm[p]],
                                        written by the bucket scatter), so a key pass reads its records'
                                        descriptors from one contiguous run instead of a line per record */
    uint8_t *dummy = nullptr;  /* r05: GCM_DUMMY_BYTES of device memory the idle lanes of a wave-pass round
                                  load from and store to, so the round still runs the mask-free body */
    const uint64_t *src_off = nullptr;  /* encrypt, r05: record i's content starts at in + src_off[i] (not in + buf_off
                                 + data_offset); its tail is read byte-wise, never past the content (the
                                 stream / DTLS send path reads the caller's application data in place) */
};

struct CpArgs {
    const SlotState *slots;
    const tlsrec_batch_rec *recs;
    tlsrec_batch_res *res;
    uint64_t n;
    const uint32_t *perm;
    const uint32_t *lo, *hi;
    const uint8_t *in;
    uint8_t *out;
    uint32_t rpw;
    uint32_t capacity;
    uint32_t cid;             /* the key table holds DTLS connection IDs: CID kernel variant */
    uint32_t skip;            /* test hook, as GcmArgs::skip */
    const uint64_t *src_off = nullptr;   /* encrypt: as GcmArgs::src_off */
};

/* Bucket pass: key index of a record = AES-128-GCM slot, AES-256-GCM slot,
 * AES-192-GCM slot, AES-CCM slot (cap-sized classes, in this order), then one
 * ChaCha20-Poly1305 class; no usable slot: BAD_INPUT_DATA. */
struct BucketArgs {
    const SlotState *slots;
    const uint8_t *cipher_of; /* [capacity] each slot's cipher (0 = none) */
    const tlsrec_batch_rec *recs;
    tlsrec_batch_res *res;
    uint32_t n;
    uint32_t capacity;
    uint32_t *counts;         /* [nk = 10 * capacity + CP_SPREAD + 1] records per (class, slot) */
    const uint32_t *offs;     /* [nk] their exclusive prefix sums (class start in perm) */
    uint2 *keyrank;           /* [n] each record's (key, rank within its key) from the count pass */
    uint32_t nk;
    uint32_t *perm;           /* [n] */
    tlsrec_batch_rec *srecs;  /* [n] descriptors in perm order (GcmArgs::srecs), or NULL */
};

/* AES-CCM records (ccm.hip): one lane per record, key passes per wave. */
struct CcmArgs {
    const SlotState *slots;
    const tlsrec_batch_rec *recs;
    tlsrec_batch_res *res;
    uint64_t n;
    const uint32_t *perm;
    const uint32_t *lo, *hi;
    const uint8_t *in;
    uint8_t *out;
    uint32_t capacity;
    uint32_t flag_nr;         /* identity order: the launch (AES rounds) that flags unusable slots */
    uint32_t cid;             /* the key table holds DTLS connection IDs: CID kernel variant */
    uint32_t skip;            /* test hook, as GcmArgs::skip */
};

} /* namespace tlsrec */

extern "C" {
hipError_t tlsrec__launch_ccm(const tlsrec::CcmArgs *a, int dec, uint32_t nr_mask, hipStream_t st);
hipError_t tlsrec__launch_keysetup(tlsrec::SlotState *slots, uint4 *ghtab, uint8_t *cipher_of,
                                   const tlsrec_key_material *keys,
                                   uint32_t first, uint32_t count, hipStream_t st);
hipError_t tlsrec__launch_gcm_aria(const tlsrec::GcmArgs *a, int dec, int nr, int cid, uint32_t grid, hipStream_t st);
hipError_t tlsrec__launch_gcm(const tlsrec::GcmArgs *a, int dec, int lanes, int nr, int waves, uint32_t grid,
                              hipStream_t st);
hipError_t tlsrec__launch_chachapoly(const tlsrec::CpArgs *a, int dec, int lanes, uint32_t grid,
                                     hipStream_t st);
/* Per-(device, stream, kind) device scratch, reused across calls (engine.hip).
 * Work enqueued on one stream is ordered, so a stream's scratch can be
 * reused by its next call without waiting; the lease's lock keeps two host
 * threads from interleaving their enqueues on one stream's scratch.  (The
 * stream-ordered allocator, hipMallocAsync / hipFreeAsync, was dropped:
 * under the system HIP 7.2 runtime a C host saw whole batches silently
 * skipped after a batch in the other direction -- results never written --
 * which plain allocations do not show.)  kind: 0 the bucket pass, 1 the
 * stream record layer (which calls the batch path inside its lease). */
typedef struct tlsrec_scratch_lease {
    void *mem;
    void *entry;
} tlsrec_scratch_lease;
int tlsrec__scratch_acquire(hipStream_t st, int kind, size_t bytes, tlsrec_scratch_lease *lease);
void tlsrec__scratch_release(tlsrec_scratch_lease *lease);
/* tlsrec_batch_encrypt (dec = 0) / _decrypt (dec = 1) with auto lanes, for a
 * caller that knows the batch's mean record size (the stream / DTLS layers);
 * prefilled: the caller's kernels already wrote INTERNAL_ERROR into every
 * result (the receive emit kernels, r06), so no guard kernel runs */
int tlsrec__batch_sized(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res, uint32_t n,
                        const uint8_t *in_arena, uint8_t *out_arena, void *stream, int dec, uint32_t avg_bytes,
                        int prefilled);
/* encrypt with each record's content read from in_arena + src_off[i] (GcmArgs::
 * src_off) and the records written to out_arena at buf_off: the stream / DTLS
 * send path without a copy of the application data.  Only for key tables of
 * AES-GCM and ChaCha20-Poly1305 keys without connection IDs
 * (tlsrec__keytab_src_ok). */
int tlsrec__batch_src(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res, uint32_t n,
                      const uint8_t *in_arena, uint8_t *out_arena, void *stream, uint32_t avg_bytes,
                      const uint64_t *src_off);
int tlsrec__keytab_src_ok(const tlsrec_keytab *kt);
hipError_t tlsrec__launch_bucket_zero(const tlsrec::BucketArgs *a, hipStream_t st);
hipError_t tlsrec__launch_bucket_count(const tlsrec::BucketArgs *a, hipStream_t st);
hipError_t tlsrec__launch_bucket_scatter(const tlsrec::BucketArgs *a, hipStream_t st);
/* exclusive scan of n uint32 (kernels.hip): two launches, scratch of
 * tlsrec__scan_scratch_bytes(n) bytes, in and out may not alias */
size_t tlsrec__scan_scratch_bytes(uint32_t n);
hipError_t tlsrec__exclusive_scan(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t *scratch, hipStream_t st);
/* server.hip: H^1 .. H^64 of one GCM key slot (64 uint4), from its GHASH tables */
/* every result of a batch to INTERNAL_ERROR before its AEAD kernels (fail closed, kernels.hip) */
hipError_t tlsrec__launch_res_guard(tlsrec_batch_res *res, uint32_t n, hipStream_t st);
}

#endif
