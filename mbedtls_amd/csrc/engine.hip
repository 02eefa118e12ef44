/*
 * engine.hip -- host side of the device engine: key tables, batch launches,
 * and the staging used by the single-record entry points.
 *
 * Everything here is plain HIP runtime C++ behind the extern "C" ABI of
 * include/tlsrec.h.  No torch types, no CPU crypto: a record is only ever
 * transformed by the kernels in kernels.hip.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "tlsrec.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"

using namespace tlsrec;

struct tlsrec_keytab {
    uint32_t capacity;
    int device;
    SlotState *d_slots;
    uint4 *d_ghtab;
    tlsrec_key_material *d_stage;
    uint8_t *h_cipher;        /* host mirror of each slot's cipher */
    uint32_t cipher_mask;     /* 1 << TLSREC_CIPHER_* of every loaded slot */
    uint32_t nloaded;         /* slots holding a key */
    uint32_t has_cid;         /* some slot was given a DTLS connection ID: launch the CID kernels */
};

static int hip_ok(hipError_t e) { return e == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED; }

extern "C" int tlsrec_device_check(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    return 0;
}

extern "C" const char *tlsrec_version_string(void)
{
    return "tlsrec 0.2 gfx950: aes-128/192/256-gcm(L=4/8/16/64, T-tables in LDS, GHASH 4-bit position tables) "
           "aes-ccm/ccm_8(lane per record) chacha20-poly1305(L=1/2/4/8, 26-bit limbs) "
           "tls13-key-schedule(hkdf-sha256/384) stream-record-layer aria-128/192/256-gcm/ccm camellia-128/192/256-gcm/ccm dtls1.2-cid";
}

extern "C" int tlsrec_keytab_create(tlsrec_keytab **out, uint32_t capacity)
{
    if (out == NULL || capacity == 0) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    *out = NULL;
    if (tlsrec_device_check() != 0) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    tlsrec_keytab *kt = (tlsrec_keytab *) calloc(1, sizeof(*kt));
    if (!kt) return TLSREC_ERR_SSL_ALLOC_FAILED;
    kt->capacity = capacity;
    hipGetDevice(&kt->device);
    kt->h_cipher = (uint8_t *) calloc(capacity, 1);
    if (!kt->h_cipher ||
        hipMalloc((void **) &kt->d_slots, sizeof(SlotState) * (size_t) capacity) != hipSuccess ||
        hipMalloc((void **) &kt->d_ghtab, sizeof(uint4) * (size_t) KEY_TABLE_WORDS * capacity) != hipSuccess ||
        hipMalloc((void **) &kt->d_stage, sizeof(tlsrec_key_material) * (size_t) capacity) != hipSuccess) {
        tlsrec_keytab_free(kt);
        return TLSREC_ERR_SSL_ALLOC_FAILED;
    }
    if (hipMemset(kt->d_slots, 0, sizeof(SlotState) * (size_t) capacity) != hipSuccess) {
        tlsrec_keytab_free(kt);
        return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    *out = kt;
    return 0;
}

extern "C" uint32_t tlsrec_keytab_capacity(const tlsrec_keytab *kt) { return kt ? kt->capacity : 0; }

extern "C" int tlsrec_keytab_set_cid(tlsrec_keytab *kt, uint32_t slot, const unsigned char *cid, size_t cid_len,
                                     void *stream)
{
    if (kt == NULL || slot >= kt->capacity || cid_len > TLSREC_CID_LEN_MAX || (cid_len && cid == NULL))
        return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    uint8_t v[1 + TLSREC_CID_LEN_MAX];
    memset(v, 0, sizeof(v));
    v[0] = (uint8_t) cid_len;
    if (cid_len) memcpy(v + 1, cid, cid_len);
    if (cid_len) kt->has_cid = 1;
    static_assert(offsetof(SlotState, cid) == offsetof(SlotState, cid_len) + 1, "SlotState CID layout");
    hipStream_t st = (hipStream_t) stream;
    hipError_t e = hipMemcpyAsync(&kt->d_slots[slot].cid_len, v, sizeof(v), hipMemcpyHostToDevice, st);
    /* and its mirror in the slot's key material, which the kernels hold */
    if (e == hipSuccess) e = hipMemcpyAsync(&kt->d_slots[slot].km.reserved[0], v, 1, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
}

extern "C" void tlsrec_keytab_free(tlsrec_keytab *kt)
{
    if (!kt) return;
    if (kt->d_slots) {
        /* zeroize key material (ssl_msg.c:6084-6099 zeroizes transforms) */
        hipMemset(kt->d_slots, 0, sizeof(SlotState) * (size_t) kt->capacity);
        hipMemset(kt->d_ghtab, 0, sizeof(uint4) * (size_t) KEY_TABLE_WORDS * kt->capacity);
        hipDeviceSynchronize();
    }
    hipFree(kt->d_slots);
    hipFree(kt->d_ghtab);
    hipFree(kt->d_stage);
    free(kt->h_cipher);
    free(kt);
}

static int check_material(const tlsrec_key_material *k)
{
    if (k->cipher < TLSREC_CIPHER_AES_128_GCM || k->cipher > TLSREC_CIPHER_MAX)
        return TLSREC_ERR_SSL_FEATURE_UNAVAILABLE;
    if (k->tls_minor != 3 && k->tls_minor != 4) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (k->taglen != tlsrec_cipher_taglen(k->cipher)) return TLSREC_ERR_SSL_FEATURE_UNAVAILABLE;
    if (k->fixed_ivlen != 12 && k->fixed_ivlen != 4) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    return 0;
}

extern "C" int tlsrec_keytab_load(tlsrec_keytab *kt, uint32_t first, uint32_t count,
                                  const tlsrec_key_material *keys, int keys_on_device, void *stream)
{
    if (!kt || !keys || first > kt->capacity || count > kt->capacity - first) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (count == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    tlsrec_key_material *host = NULL;
    if (keys_on_device) {
        host = (tlsrec_key_material *) malloc(sizeof(*host) * count);
        if (!host) return TLSREC_ERR_SSL_ALLOC_FAILED;
        if (hipMemcpyAsync(host, keys, sizeof(*host) * count, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {
            free(host);
            return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        }
    }
    const tlsrec_key_material *hk = keys_on_device ? host : keys;
    for (uint32_t i = 0; i < count; i++) {
        int r = check_material(&hk[i]);
        if (r) {
            free(host);
            return r;
        }
    }
    for (uint32_t i = 0; i < count; i++) {
        if (kt->h_cipher[first + i] == 0) kt->nloaded++;
        kt->h_cipher[first + i] = hk[i].cipher;
        kt->cipher_mask |= 1u << hk[i].cipher;
    }
    free(host);
    const tlsrec_key_material *src = keys;
    if (!keys_on_device) {
        if (hipMemcpyAsync(kt->d_stage + first, keys, sizeof(*keys) * count, hipMemcpyHostToDevice, st) != hipSuccess)
            return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        /* the staging copy must land before the host buffer may be reused */
        if (hipStreamSynchronize(st) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        src = kt->d_stage + first;
    }
    return hip_ok(tlsrec__launch_keysetup(kt->d_slots, kt->d_ghtab, src, first, count, st));
}

/* Device-side producers of key material (keysched.hip) write into the
 * table's staging area and then commit: bookkeeping as tlsrec_keytab_load,
 * then the key-setup kernel on the staged slots. */
extern "C" tlsrec_key_material *tlsrec__keytab_stage(tlsrec_keytab *kt) { return kt->d_stage; }
extern "C" const SlotState *tlsrec__keytab_slots(const tlsrec_keytab *kt) { return kt->d_slots; }
extern "C" const uint4 *tlsrec__keytab_ghtab(const tlsrec_keytab *kt) { return kt->d_ghtab; }

extern "C" int tlsrec__keytab_commit_staged(tlsrec_keytab *kt, uint32_t first, uint32_t count, int cipher,
                                            hipStream_t st)
{
    for (uint32_t i = 0; i < count; i++) {
        if (kt->h_cipher[first + i] == 0) kt->nloaded++;
        kt->h_cipher[first + i] = (uint8_t) cipher;
    }
    kt->cipher_mask |= 1u << cipher;
    return hip_ok(tlsrec__launch_keysetup(kt->d_slots, kt->d_ghtab, kt->d_stage + first, first, count, st));
}

/* waves per GCM workgroup: 16 (default) or 8; TLSREC_GCM_WAVES overrides */
static int gcm_waves(void)
{
    static int w = 0;
    if (w == 0) {
        const char *e = getenv("TLSREC_GCM_WAVES");
        w = (e && atoi(e) == 8) ? 8 : GCM_WAVES;
    }
    return w;
}

/* wave-pass GCM variant (per-wave key passes, H^L per wave in LDS) for
 * tables of many keys with very few records each (auto: < 8 per key, where
 * a workgroup-wide key pass leaves most waves idle; measured +17-20 % at 4
 * x 16 KiB per key, -45 % at 16 per key).  TLSREC_GCM_WP=1 forces it, =0
 * disables it. */
static int gcm_wp_env(void)
{
    const char *e = getenv("TLSREC_GCM_WP");   /* read per batch: tests switch it */
    return e ? atoi(e) : -1;
}

static uint32_t pick_rpw(uint64_t n, uint32_t waves_per_wg, uint32_t R, uint32_t target_wgs)
{
    uint64_t want = (n + (uint64_t) waves_per_wg * target_wgs - 1) / ((uint64_t) waves_per_wg * target_wgs);
    if (want < R) want = R;
    want = (want + R - 1) / R * R;
    if (want > 64) want = 64;
    return (uint32_t) want;
}

/* Device scratch of one bucketed batch (stream-ordered allocation). */
struct BucketScratch {
    void *mem = nullptr;
    uint32_t *counts, *offs, *cursor, *perm;
    void *scan_tmp;
    size_t scan_bytes;
};

static int bucket(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res, uint32_t n,
                  hipStream_t st, BucketScratch &b)
{
    /* AES-128-GCM, AES-256-GCM, AES-192-GCM, AES-CCM slots, ChaCha, ARIA-128/192/256-GCM,
     * Camellia-128/192/256-GCM slots, end */
    const size_t nk = 10 * (size_t) kt->capacity + 2;
    b.scan_bytes = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, b.scan_bytes, (uint32_t *) nullptr, (uint32_t *) nullptr,
                                         (int) nk, st) != hipSuccess)
        return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    const size_t al = 256;
    const size_t szk = (nk * 4 + al - 1) / al * al, szp = ((size_t) n * 4 + al - 1) / al * al;
    const size_t total = 3 * szk + szp + b.scan_bytes + al;
    if (hipMallocAsync(&b.mem, total, st) != hipSuccess) return TLSREC_ERR_SSL_ALLOC_FAILED;
    uint8_t *m = (uint8_t *) b.mem;
    b.counts = (uint32_t *) m;
    b.offs = (uint32_t *) (m + szk);
    b.cursor = (uint32_t *) (m + 2 * szk);
    b.perm = (uint32_t *) (m + 3 * szk);
    b.scan_tmp = m + 3 * szk + szp;
    BucketArgs a;
    a.slots = kt->d_slots;
    a.recs = recs;
    a.res = res;
    a.n = n;
    a.capacity = kt->capacity;
    a.counts = b.counts;
    a.cursor = b.cursor;
    a.perm = b.perm;
    if (hipMemsetAsync(b.counts, 0, nk * 4, st) != hipSuccess ||
        tlsrec__launch_bucket_count(&a, st) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(b.scan_tmp, b.scan_bytes, b.counts, b.offs, (int) nk, st) != hipSuccess ||
        hipMemcpyAsync(b.cursor, b.offs, nk * 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        tlsrec__launch_bucket_scatter(&a, st) != hipSuccess)
        return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    return 0;
}

static int batch(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res, uint32_t n,
                 const uint8_t *in, uint8_t *out, uint32_t lanes, void *stream, int dec)
{
    if (!kt || (!recs && n) || (!res && n)) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    int cu = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, kt->device) == hipSuccess && prop.multiProcessorCount > 0)
            cu = prop.multiProcessorCount;
    }
    /* A table holding a single key needs no grouping: the kernels walk the
     * descriptors in order and flag records naming an unusable slot.
     * Otherwise the bucket pass groups GCM records by key (then ChaCha). */
    BucketScratch bs;
    const bool identity = kt->nloaded == 1;
    if (!identity) {
        int r = bucket(kt, recs, res, n, st, bs);
        if (r) {
            if (bs.mem) hipFreeAsync(bs.mem, st);
            return r;
        }
    }
    const uint32_t cap = kt->capacity;
    int rc = 0;
    static const int gcm_ciphers[3] = { TLSREC_CIPHER_AES_128_GCM, TLSREC_CIPHER_AES_256_GCM,
                                        TLSREC_CIPHER_AES_192_GCM };
    for (int ci = 0; ci < 3 && !rc; ci++) {
        const int cipher = gcm_ciphers[ci];     /* bucket class ci: keys [ci * cap, (ci + 1) * cap) */
        if (!(kt->cipher_mask & (1u << cipher))) continue;
        /* (ARIA-GCM below: one configuration) */
        /* lanes per record: a key pass should still fill the 16 waves of a
         * workgroup.  8 for a single key or >= 128 records per key; 16
         * (4 records per wave) down to 48 records per key; 64 (one record per
         * wave) below that -- the many-connections, few-records regime of
         * the stream path. */
        const uint32_t rpk = kt->nloaded > 1 ? n / kt->nloaded : n;
        int L = (lanes == 4 || lanes == 8 || lanes == 16 || lanes == 64) ? (int) lanes
                : (kt->nloaded <= 1 || rpk >= 128) ? 8 : (rpk >= 48 ? 16 : 64);
        if (kt->has_cid) L = 8;     /* the CID variant: one configuration */
        GcmArgs a;
        a.slots = kt->d_slots;
        a.ghtab = kt->d_ghtab;
        a.recs = recs;
        a.res = res;
        a.n = n;
        a.perm = identity ? nullptr : bs.perm;
        a.lo = identity ? nullptr : bs.offs + (size_t) ci * cap;
        a.hi = identity ? nullptr : bs.offs + (size_t) (ci + 1) * cap;
        a.in = in;
        a.out = out;
        int nr = (int) tlsrec_cipher_nr(cipher);
        const int wpe = gcm_wp_env();
        const bool wp = !kt->has_cid && !identity && (L == 16 || L == 64) && nr != 12 && (wpe == 1 || (wpe != 0 && rpk < 8));
        const int waves = wp ? 8 : (kt->has_cid ? 16 : gcm_waves());
        a.rpw = pick_rpw(n, (uint32_t) waves, 64 / L, (uint32_t) cu);
        a.capacity = cap;
        a.cipher = (uint32_t) cipher;
        uint64_t per_wg = (uint64_t) waves * a.rpw;
        uint32_t grid = (uint32_t) ((n + per_wg - 1) / per_wg);
        if (tlsrec__launch_gcm(&a, dec, L, nr, wp ? -8 : (kt->has_cid ? -16 : waves), grid, st) != hipSuccess)
            rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    /* ARIA-GCM and Camellia-GCM: the GCM kernel around the LDS-table cipher
     * (8 lanes, 16 waves); bucket classes (4, 5, 6) cap + 1 and (7, 8, 9) cap + 1 */
    static const int alt_gcm[6] = { TLSREC_CIPHER_ARIA_128_GCM, TLSREC_CIPHER_ARIA_192_GCM, TLSREC_CIPHER_ARIA_256_GCM,
                                    TLSREC_CIPHER_CAMELLIA_128_GCM, TLSREC_CIPHER_CAMELLIA_192_GCM,
                                    TLSREC_CIPHER_CAMELLIA_256_GCM };
    for (int ci = 0; ci < 6 && !rc; ci++) {
        const int c = alt_gcm[ci];
        if (!(kt->cipher_mask & (1u << c))) continue;
        const size_t base = (size_t) (4 + ci) * cap + 1;
        GcmArgs a;
        a.slots = kt->d_slots;
        a.ghtab = kt->d_ghtab;
        a.recs = recs;
        a.res = res;
        a.n = n;
        a.perm = identity ? nullptr : bs.perm;
        a.lo = identity ? nullptr : bs.offs + base;
        a.hi = identity ? nullptr : bs.offs + base + cap;
        a.in = in;
        a.out = out;
        a.rpw = pick_rpw(n, (uint32_t) ARIA_GCM_WAVES, 8u, (uint32_t) cu);
        a.capacity = cap;
        a.cipher = (uint32_t) c;
        const uint64_t per_wg = (uint64_t) ARIA_GCM_WAVES * a.rpw;
        const uint32_t grid = (uint32_t) ((n + per_wg - 1) / per_wg);
        if (tlsrec__launch_gcm_aria(&a, dec, (int) tlsrec_cipher_alt_nr(c), (int) kt->has_cid, grid, st) != hipSuccess)
            rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    uint32_t ccm_nr = 0;
    for (int c = TLSREC_CIPHER_AES_128_CCM; c <= TLSREC_CIPHER_AES_256_CCM_8; c++)
        if (kt->cipher_mask & (1u << c)) ccm_nr |= 1u << tlsrec_cipher_nr(c);
    for (int c = TLSREC_CIPHER_ARIA_128_CCM; c <= TLSREC_CIPHER_CAMELLIA_256_CCM; c++)   /* ARIA / Camellia: bit nr + 4 */
        if (tlsrec_cipher_is_alt_ccm(c) && (kt->cipher_mask & (1u << c))) ccm_nr |= 1u << (tlsrec_cipher_alt_nr(c) + 4);
    if (!rc && ccm_nr) {
        CcmArgs a;
        a.slots = kt->d_slots;
        a.recs = recs;
        a.res = res;
        a.n = n;
        a.perm = identity ? nullptr : bs.perm;
        a.lo = identity ? nullptr : bs.offs + 3 * (size_t) cap;
        a.hi = identity ? nullptr : bs.offs + 4 * (size_t) cap;
        a.in = in;
        a.out = out;
        a.capacity = cap;
        a.flag_nr = 0;
        a.cid = kt->has_cid;
        if (tlsrec__launch_ccm(&a, dec, ccm_nr, st) != hipSuccess) rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (!rc && (kt->cipher_mask & (1u << TLSREC_CIPHER_CHACHA20_POLY1305))) {
        int L = (lanes == 1 || lanes == 2 || lanes == 4 || lanes == 8) ? (int) lanes : 2;
        if (kt->has_cid) L = 2;     /* the CID variant: one configuration */
        CpArgs a;
        a.slots = kt->d_slots;
        a.recs = recs;
        a.res = res;
        a.n = n;
        a.perm = identity ? nullptr : bs.perm;
        a.lo = identity ? nullptr : bs.offs + 4 * (size_t) cap;
        a.hi = identity ? nullptr : bs.offs + 4 * (size_t) cap + 1;
        a.in = in;
        a.out = out;
        a.rpw = pick_rpw(n, CP_WAVES, 64 / L, (uint32_t) cu * 4);
        a.capacity = cap;
        a.cid = kt->has_cid;
        uint64_t per_wg = (uint64_t) CP_WAVES * a.rpw;
        uint32_t grid = (uint32_t) ((n + per_wg - 1) / per_wg);
        if (tlsrec__launch_chachapoly(&a, dec, L, grid, st) != hipSuccess) rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (bs.mem && hipFreeAsync(bs.mem, st) != hipSuccess && !rc) rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    return rc;
}

extern "C" int tlsrec_batch_encrypt(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                    uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                                    uint32_t lanes_per_record, void *stream)
{
    return batch(kt, recs, res, n, in_arena, out_arena, lanes_per_record, stream, 0);
}

extern "C" int tlsrec_batch_decrypt(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                    uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                                    uint32_t lanes_per_record, void *stream)
{
    return batch(kt, recs, res, n, in_arena, out_arena, lanes_per_record, stream, 1);
}

/* ======================================================================
 * Engine used by the single-record API (tlsrec_host.c): a process-wide key
 * table with a slot allocator and a device staging area.
 * ==================================================================== */
#define TLSREC_ENGINE_SLOTS 4096

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static tlsrec_keytab *g_kt = NULL;
static uint8_t g_used[TLSREC_ENGINE_SLOTS];
static hipStream_t g_stream = NULL;
static uint8_t *g_dbuf = NULL;
static size_t g_dbuf_len = 0;
static void *g_dmeta = NULL;

static int engine_init_locked(void)
{
    if (g_kt) return 0;
    int r = tlsrec_keytab_create(&g_kt, TLSREC_ENGINE_SLOTS);
    if (r) return r;
    if (hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&g_dmeta, 64) != hipSuccess) {
        tlsrec_keytab_free(g_kt);
        g_kt = NULL;
        return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    return 0;
}

extern "C" int tlsrec__engine_slot_alloc(const tlsrec_key_material *km)
{
    pthread_mutex_lock(&g_mu);
    int r = engine_init_locked();
    int slot = -1;
    if (r == 0) {
        for (int i = 0; i < TLSREC_ENGINE_SLOTS; i++)
            if (!g_used[i]) { slot = i; break; }
        if (slot < 0) r = TLSREC_ERR_SSL_ALLOC_FAILED;
    }
    if (r == 0) {
        r = tlsrec_keytab_load(g_kt, (uint32_t) slot, 1, km, 0, g_stream);
        if (r == 0 && hipStreamSynchronize(g_stream) != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        if (r == 0) g_used[slot] = 1;
    }
    pthread_mutex_unlock(&g_mu);
    return r ? r : slot;
}

extern "C" void tlsrec__engine_slot_free(int slot)
{
    if (slot < 0 || slot >= TLSREC_ENGINE_SLOTS) return;
    pthread_mutex_lock(&g_mu);
    if (g_kt && g_used[slot]) {
        hipMemsetAsync(g_kt->d_slots + slot, 0, sizeof(SlotState), g_stream);
        hipMemsetAsync(g_kt->d_ghtab + (size_t) slot * KEY_TABLE_WORDS, 0, sizeof(uint4) * KEY_TABLE_WORDS,
                       g_stream);
        hipStreamSynchronize(g_stream);
        g_used[slot] = 0;
    }
    pthread_mutex_unlock(&g_mu);
}

extern "C" int tlsrec__engine_slot_set_cid(int slot, const unsigned char *cid, size_t cid_len)
{
    if (slot < 0 || slot >= TLSREC_ENGINE_SLOTS) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    pthread_mutex_lock(&g_mu);
    int r = g_kt && g_used[slot] ? tlsrec_keytab_set_cid(g_kt, (uint32_t) slot, cid, cid_len, g_stream)
                                 : TLSREC_ERR_SSL_INTERNAL_ERROR;
    pthread_mutex_unlock(&g_mu);
    return r;
}

/* Run one record through the batch kernels: host buffer -> device -> host.
 * A decrypted record's CID (cid_len bytes) is staged right after the buffer
 * (rec->cid_off = buf_len). */
extern "C" int tlsrec__engine_run(int dec, const tlsrec_batch_rec *rec, unsigned char *buf, size_t buf_len,
                                  const unsigned char *cid, tlsrec_batch_res *out)
{
    pthread_mutex_lock(&g_mu);
    int r = engine_init_locked();
    if (r == 0 && g_dbuf_len < buf_len + 16 + TLSREC_CID_LEN_MAX) {
        hipFree(g_dbuf);
        g_dbuf = NULL;
        g_dbuf_len = 0;
        size_t want = buf_len + 16 + TLSREC_CID_LEN_MAX > 65536 ? buf_len + 16 + TLSREC_CID_LEN_MAX : 65536;
        if (hipMalloc((void **) &g_dbuf, want) != hipSuccess) r = TLSREC_ERR_SSL_ALLOC_FAILED;
        else g_dbuf_len = want;
    }
    if (r == 0) {
        tlsrec_batch_rec d = *rec;
        d.buf_off = 0;
        tlsrec_batch_rec *d_rec = (tlsrec_batch_rec *) g_dmeta;
        tlsrec_batch_res *d_res = (tlsrec_batch_res *) ((uint8_t *) g_dmeta + 48);
        hipError_t e = hipSuccess;
        if (buf_len) e = hipMemcpyAsync(g_dbuf, buf, buf_len, hipMemcpyHostToDevice, g_stream);
        if (e == hipSuccess && d.cid_len) {
            e = hipMemcpyAsync(g_dbuf + buf_len, cid, d.cid_len, hipMemcpyHostToDevice, g_stream);
            const uint32_t off = (uint32_t) buf_len;
            d.cid_off[0] = (uint8_t) off; d.cid_off[1] = (uint8_t) (off >> 8);
            d.cid_off[2] = (uint8_t) (off >> 16); d.cid_off[3] = (uint8_t) (off >> 24);
        }
        if (e == hipSuccess) e = hipMemcpyAsync(d_rec, &d, sizeof(d), hipMemcpyHostToDevice, g_stream);
        if (e == hipSuccess) {
            r = batch(g_kt, d_rec, d_res, 1, g_dbuf, g_dbuf, 0, g_stream, dec);
            if (r == 0 && buf_len) e = hipMemcpyAsync(buf, g_dbuf, buf_len, hipMemcpyDeviceToHost, g_stream);
            if (r == 0 && e == hipSuccess) e = hipMemcpyAsync(out, d_res, sizeof(*out), hipMemcpyDeviceToHost, g_stream);
            if (e == hipSuccess) e = hipStreamSynchronize(g_stream);
        }
        if (e != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    pthread_mutex_unlock(&g_mu);
    return r;
}
