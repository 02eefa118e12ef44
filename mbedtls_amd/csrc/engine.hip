/*
 * engine.hip -- host side of the device engine: key tables, batch launches,
 * and the staging used by the single-record entry points.
 *
 * Everything here is plain HIP runtime C++ behind the extern "C" ABI of
 * include/tlsrec.h.  No torch types, no CPU crypto: a record is only ever
 * transformed by the kernels in kernels.hip.
 */
#include <hip/hip_runtime.h>
#include <algorithm>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tlsrec.h"
#include "tlsrec_frame.h"
#include "tlsrec_internal.h"

using namespace tlsrec;

struct HostPipe;   /* tlsrec_host_batch_*: device slots and streams, made on first use */

struct tlsrec_keytab {
    uint32_t capacity;
    int device;
    int cu;                   /* compute units of the device (launch sizing), read once at create */
    SlotState *d_slots;
    uint4 *d_ghtab;
    uint8_t *d_cipher;        /* each slot's cipher, one byte (the bucket pass reads it per record:
                                 an L2-resident array instead of a line of the 1 KiB slot) */
    tlsrec_key_material *d_stage;
    uint8_t *h_cipher;        /* host mirror of each slot's cipher */
    uint32_t cipher_mask;     /* 1 << TLSREC_CIPHER_* of every loaded slot */
    uint32_t nloaded;         /* slots holding a key */
    volatile uint32_t has_cid; /* some slot was given a DTLS connection ID: launch the CID kernels */
    uint8_t *d_dummy;         /* GcmArgs::dummy: 64 KiB the idle lanes of a wave-pass round load and store */
    HostPipe *pipe;
    pthread_mutex_t pipe_mu;
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
           "tls13-key-schedule(hkdf-sha256/384) stream-record-layer aria-128/192/256-gcm/ccm camellia-128/192/256-gcm/ccm dtls1.2-cid dtls1.2-datagram-record-layer(anti-replay) session-tickets";
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
    kt->cu = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, kt->device) == hipSuccess && prop.multiProcessorCount > 0)
            kt->cu = prop.multiProcessorCount;
    }
    pthread_mutex_init(&kt->pipe_mu, NULL);
    kt->h_cipher = (uint8_t *) calloc(capacity, 1);
    if (!kt->h_cipher ||
        hipMalloc((void **) &kt->d_slots, sizeof(SlotState) * (size_t) capacity) != hipSuccess ||
        hipMalloc((void **) &kt->d_ghtab, sizeof(uint4) * (size_t) KEY_TABLE_WORDS * capacity) != hipSuccess ||
        hipMalloc((void **) &kt->d_cipher, (size_t) capacity) != hipSuccess ||
        hipMalloc((void **) &kt->d_stage, sizeof(tlsrec_key_material) * (size_t) capacity) != hipSuccess ||
        hipMalloc((void **) &kt->d_dummy, GCM_DUMMY_BYTES) != hipSuccess) {
        tlsrec_keytab_free(kt);
        return TLSREC_ERR_SSL_ALLOC_FAILED;
    }
    if (hipMemset(kt->d_slots, 0, sizeof(SlotState) * (size_t) capacity) != hipSuccess ||
        hipMemset(kt->d_cipher, 0, (size_t) capacity) != hipSuccess) {
        tlsrec_keytab_free(kt);
        return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    *out = kt;
    return 0;
}

extern "C" uint32_t tlsrec_keytab_capacity(const tlsrec_keytab *kt) { return kt ? kt->capacity : 0; }

/* host mirror of a slot's cipher (0 = never loaded) */
extern "C" int tlsrec__keytab_cipher(const tlsrec_keytab *kt, uint32_t slot)
{
    return kt && slot < kt->capacity ? kt->h_cipher[slot] : 0;
}

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

static void host_pipe_free(HostPipe *p);

extern "C" void tlsrec_keytab_free(tlsrec_keytab *kt)
{
    if (!kt) return;
    host_pipe_free(kt->pipe);
    pthread_mutex_destroy(&kt->pipe_mu);
    if (kt->d_slots) {
        /* zeroize key material (ssl_msg.c:6084-6099 zeroizes transforms) */
        hipMemset(kt->d_slots, 0, sizeof(SlotState) * (size_t) kt->capacity);
        hipMemset(kt->d_ghtab, 0, sizeof(uint4) * (size_t) KEY_TABLE_WORDS * kt->capacity);
        if (kt->d_dummy) hipMemset(kt->d_dummy, 0, GCM_DUMMY_BYTES);   /* idle lanes' keystream under the keys */
        hipDeviceSynchronize();
    }
    hipFree(kt->d_dummy);
    hipFree(kt->d_slots);
    hipFree(kt->d_ghtab);
    hipFree(kt->d_cipher);
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
    return hip_ok(tlsrec__launch_keysetup(kt->d_slots, kt->d_ghtab, kt->d_cipher, src, first, count, st));
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
    return hip_ok(tlsrec__launch_keysetup(kt->d_slots, kt->d_ghtab, kt->d_cipher, kt->d_stage + first, first, count, st));
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
 * tables of many keys with very few records each (auto: < 12 per key, where
 * a workgroup-wide key pass leaves most waves idle).  Lanes per record in
 * it: 16 (a wave's 4 records share one key pass) from 3 records per key,
 * 64 below.  Measured, 256 K x 16 KiB AES-256-GCM decrypt (GiB/s):
 *   records/key        1     2     4     8    16    32
 *   wave passes L=16   90   177   415   423   429   433
 *   wave passes L=64  212   228   244   255   259   267
 *   workgroup passes   56   108   208   369   536   584
 * TLSREC_GCM_WP=1 forces it, =0 disables it. */
static int gcm_wp_env(void)
{
    const char *e = getenv("TLSREC_GCM_WP");   /* read per batch: tests switch it */
    return e ? atoi(e) : -1;
}

/* 8-lane GCM kernel with the 5-bit GHASH Horner table (gmul5: 104 instead of
 * 128 LDS cycles per multiply); TLSREC_GCM_G5=0 selects the 4-bit table
 * (read per batch: tests and A/B runs switch it) */
static uint32_t gcm_g5(void)
{
    const char *e = getenv("TLSREC_GCM_G5");
    return (e && atoi(e) == 0) ? 0u : 1u;
}

/* 16-lane wave passes: the lane tree by table-free multiplies (tlsrec_clmul.h)
 * instead of the key's H^8 / H^4 / H^2 / H^1 tables from HBM (24 KiB more per
 * key pass).  Same-box: k4 455 -> 461 GiB/s, stream 4 x 16 KiB per key
 * receive 424/429 -> 432/432.  TLSREC_GCM_TREEMUL=0 selects the tables. */
static uint32_t gcm_tm(bool pair, bool wp)
{
    /* bit 0: 16-lane wave passes (default on); bit 1: 2- and 4-lane ones
     * (default on for the paired passes: c4s 740 -> 750 GiB/s same-box; ±1 %
     * in the 8-wave passes); bit 2: the AAD fold and the two final multiplies
     * by H as a value too (default on for the paired passes, same-box: c4s
     * 720 -> 742, k4 549 -> 558, 64 K keys x 16 x 1.4 KiB 362 -> 377 GiB/s:
     * the key's 8 KiB H^1 table in global memory cost 32 lines per multiply);
     * bit 3 (r04): lane powers -- AAD and the length block in the lane
     * layout, one multiply by H^(d+1) per lane and a lane XOR replace the
     * fold, the tree and the final multiplies (the key-pass kernels then
     * stage only the Horner table).  Default on for the wave passes, whose
     * tails were table-free multiplies (same box: k4 582 -> 636 GiB/s, DTLS
     * 16 x 1.4 KiB +17 %); compiled into the wave-pass kernels only (the
     * 16-wave key passes' LDS-table tree is cheaper than a VALU multiply on an
     * LDS-bound kernel, and the run-time flag alone cost c2 5 %, tlsrec_gcm.h). */
    const char *e = getenv("TLSREC_GCM_TREEMUL");
    uint32_t tm = e ? (uint32_t) atoi(e) & 15u : (pair ? 15u : (wp ? 9u : 1u));
    /* bit 4 (r05): the paired passes build the key's Horner table in LDS
     * from H^L (tlsrec_clmul.h tlsrec_gtab4_window) instead of staging its
     * 8 KiB from HBM per key pass; TLSREC_GCM_HBUILD=0 stages it */
    const char *hb = getenv("TLSREC_GCM_HBUILD");
    if (pair && !(hb && atoi(hb) == 0)) tm |= 16u;
    return tm;
}

/* paired wave passes (16 waves, two per key table) for small records of many
 * keys; TLSREC_GCM_PAIR=0 keeps the 8-wave wave passes (read per batch) */
static int gcm_pair_env(void)
{
    const char *e = getenv("TLSREC_GCM_PAIR");
    return e ? atoi(e) : 1;
}

/* TLSREC_GROUPED=0: the stream / DTLS layers' batches go through the
 * bucket pass as in r05 (BatchOpt::grouped; A/B and the tests' second path) */
static bool grouped_env(void)
{
    const char *e = getenv("TLSREC_GROUPED");
    return !(e && atoi(e) == 0);
}

/* key-ordered descriptor copy for the GCM kernels (bucket scatter):
 * TLSREC_GCM_SRECS=1.  Off by default: same box, k4 665 vs 665-666, c4s 836
 * vs 840-843, c4 1032 vs 1035 GiB/s (profiles/r04h) -- the scattered 40-byte
 * writes cost what the contiguous reads save. */
static bool srecs_env(void)
{
    const char *e = getenv("TLSREC_GCM_SRECS");
    return e && atoi(e) == 1;
}

/* lanes per record of the paired passes over small records (2, 4 or 8):
 * measurement override of the records-per-key rule */
static int gcm_pair_l_env(void)
{
    const char *e = getenv("TLSREC_GCM_PAIR_L");
    const int v = e ? atoi(e) : 0;
    return (v == 2 || v == 4 || v == 8) ? v : 0;
}

/* Small records (<= 4 KiB) of many keys take the paired passes from 12 to
 * this many records per key, the 16-wave key passes from there
 * (TLSREC_GCM_PAIR_SMALL_MAX overrides; r04: 128). */
static uint32_t gcm_pair_small_max(void)
{
    const char *e = getenv("TLSREC_GCM_PAIR_SMALL_MAX");
    return e ? (uint32_t) atoi(e) : 256u;
}

/* ... and from this many (TLSREC_GCM_PAIR_SMALL_MIN overrides; r04: 12) */
static uint32_t gcm_pair_small_min(void)
{
    const char *e = getenv("TLSREC_GCM_PAIR_SMALL_MIN");
    return e ? (uint32_t) atoi(e) : 12u;
}

/* Lanes per record of the paired passes over small records, from the mean
 * records per key (r05).  Each half of a pair takes about rpk / 2 of a key's
 * records in rounds of R = 64 / L records, so a key pass fills
 *     eff(L) = (rpk / 2) / (R * ceil(rpk / (2 R)))
 * of its rounds; the L with the best eff(L) x base(L) wins, base = the
 * full-round rates measured at 64 / 128 records per key (1 400-B AES-256-GCM,
 * 2 : 4 : 8 lanes = 603 : 590 : 530 GiB/s).  The model against the same-box
 * sweep (profiles/r05/small_rpk/), best measured lane count in brackets:
 *   rpk      16  23  32  47  64  95  128  191
 *   model     8   4   4   8   2   4    2    2
 *   [best]    8   4   4   8   2   4    2    2
 * r04's rule (2 from 48, 4 from 24, else 8) lost 14-29 % at 47 and 95 per
 * key, and the 16-wave key passes it used from 128 per key 13-25 %. */
extern "C" uint32_t tlsrec__gcm_pair_small_l(uint32_t rpk)
{
    static const uint32_t Ls[3] = { 2, 4, 8 };
    static const double base[3] = { 1.0, 590.0 / 603.0, 530.0 / 603.0 };
    double best = -1.0;
    uint32_t bl = 8;
    const double h = rpk / 2.0;
    for (int i = 0; i < 3; i++) {
        const double R = 64.0 / Ls[i];
        const double rounds = ceil(h / R);
        const double score = rounds > 0 ? base[i] * h / (R * rounds) : 0.0;
        if (score > best + 1e-9) {
            best = score;
            bl = Ls[i];
        }
    }
    return bl;
}

/* Large records (> 4 KiB) take the paired passes below this many records per
 * key (r05: 40; r04: 12).  With the rounds starting at each key's first
 * position (tlsrec_gcm.h), 16 KiB records, 2^18 records (same box,
 * profiles/r05/pair_big), 16-wave key passes -> paired 16 lanes:
 *   records per key     16          23          32          47
 *   GiB/s            637 -> 705  638 -> 667  667 -> 711  668 -> 654
 * and the stream layer's 64 K connections x 16 x 16 KiB receive / send
 * 602 -> 685 / 497 -> 542.  At 64 per key one key fills a key pass's 16
 * waves exactly and the key passes stay (c4).  TLSREC_GCM_PAIR_BIG_MAX
 * overrides. */
static uint32_t gcm_pair_big_max(void)
{
    const char *e = getenv("TLSREC_GCM_PAIR_BIG_MAX");
    return e ? (uint32_t) atoi(e) : 40u;
}

/* lanes per GCM record when the caller passes 0 (auto): measurement override */
static uint32_t gcm_lanes_env(void)
{
    const char *e = getenv("TLSREC_GCM_LANES");
    return e ? (uint32_t) atoi(e) : 0u;
}

static uint32_t pick_rpw(uint64_t n, uint32_t waves_per_wg, uint32_t R, uint32_t target_wgs)
{
    uint64_t want = (n + (uint64_t) waves_per_wg * target_wgs - 1) / ((uint64_t) waves_per_wg * target_wgs);
    if (want < R) want = R;
    want = (want + R - 1) / R * R;
    if (want > 64) want = 64;
    return (uint32_t) want;
}

/* ---- per-stream device scratch (tlsrec_internal.h) ---- */
struct ScratchEntry {
    int device;
    hipStream_t stream;
    uintptr_t thread;         /* hipStreamPerThread: the calling thread (its own real stream) */
    int kind;
    void *mem;
    size_t bytes;
    pthread_mutex_t mu;
    ScratchEntry *next;
};
static pthread_mutex_t g_scratch_mu = PTHREAD_MUTEX_INITIALIZER;
static ScratchEntry *g_scratch = nullptr;

/* hipStreamPerThread entries belong to their thread: when it exits they are
 * marked orphaned, and the next acquire frees them, so a server whose
 * connections come and go on short-lived threads does not accumulate device
 * memory.  The exit hook itself makes no HIP call: it runs after
 * the HIP runtime's own thread-local state is gone.  hipFree waits for the
 * device, so work the dead thread left on its stream has finished by then. */
static const uintptr_t SCRATCH_ORPHAN = 1;     /* never a pthread_t of a live thread */
static pthread_key_t g_scratch_key;
static pthread_once_t g_scratch_once = PTHREAD_ONCE_INIT;
static volatile int g_scratch_orphans = 0;

static void scratch_thread_exit(void *)
{
    const uintptr_t me = (uintptr_t) pthread_self();
    pthread_mutex_lock(&g_scratch_mu);
    for (ScratchEntry *e = g_scratch; e; e = e->next)
        if (e->thread == me) {
            e->thread = SCRATCH_ORPHAN;
            g_scratch_orphans++;
        }
    pthread_mutex_unlock(&g_scratch_mu);
}

static void scratch_key_init(void) { pthread_key_create(&g_scratch_key, scratch_thread_exit); }

/* with g_scratch_mu held */
/* Under g_scratch_mu: unlink the orphaned entries (their threads exited) and
 * return them as a list; scratch_free_list frees them after the lock is
 * dropped -- hipFree waits for the device (a record-server grid, other
 * streams' kernels), and no other launcher should queue behind that. */
static ScratchEntry *scratch_reclaim_locked(void)
{
    ScratchEntry *dead = nullptr;
    for (ScratchEntry **pp = &g_scratch; *pp;) {
        ScratchEntry *e = *pp;
        if (e->thread == SCRATCH_ORPHAN) {
            *pp = e->next;
            e->next = dead;
            dead = e;
            g_scratch_orphans--;
        } else {
            pp = &e->next;
        }
    }
    return dead;
}

static void scratch_free_list(ScratchEntry *e)
{
    while (e) {
        ScratchEntry *next = e->next;
        if (e->mem) (void) hipFree(e->mem);
        pthread_mutex_destroy(&e->mu);
        free(e);
        e = next;
    }
}

extern "C" int tlsrec__scratch_acquire(hipStream_t st, int kind, size_t bytes, tlsrec_scratch_lease *lease)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    /* one handle, one ordered queue -- except hipStreamPerThread, which names
     * a different real stream in every thread: two threads' batches on it run
     * unordered on the GPU, so each thread gets its own scratch (the null
     * stream is one queue for every thread and needs nothing) */
    const uintptr_t thr = st == hipStreamPerThread ? (uintptr_t) pthread_self() : 0;
    pthread_mutex_lock(&g_scratch_mu);
    ScratchEntry *dead = g_scratch_orphans ? scratch_reclaim_locked() : nullptr;
    ScratchEntry *e = g_scratch;
    while (e && !(e->device == dev && e->stream == st && e->thread == thr && e->kind == kind)) e = e->next;
    if (!e) {
        e = (ScratchEntry *) calloc(1, sizeof(*e));
        if (!e) {
            pthread_mutex_unlock(&g_scratch_mu);
            scratch_free_list(dead);
            return TLSREC_ERR_SSL_ALLOC_FAILED;
        }
        e->device = dev;
        e->stream = st;
        e->thread = thr;
        e->kind = kind;
        pthread_mutex_init(&e->mu, NULL);
        e->next = g_scratch;
        g_scratch = e;
        if (thr) {
            pthread_once(&g_scratch_once, scratch_key_init);
            pthread_setspecific(g_scratch_key, (void *) 1);   /* non-NULL: the destructor runs */
        }
    }
    pthread_mutex_unlock(&g_scratch_mu);
    scratch_free_list(dead);
    pthread_mutex_lock(&e->mu);
    if (e->bytes < bytes) {
        /* grow: the stream's earlier work may still read the old buffer */
        if (e->mem && (hipStreamSynchronize(st) != hipSuccess || hipFree(e->mem) != hipSuccess)) {
            pthread_mutex_unlock(&e->mu);
            return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        }
        e->mem = nullptr;
        e->bytes = 0;
        const size_t want = bytes + bytes / 4 + 4096;
        if (hipMalloc(&e->mem, want) != hipSuccess) {
            e->mem = nullptr;
            pthread_mutex_unlock(&e->mu);
            return TLSREC_ERR_SSL_ALLOC_FAILED;
        }
        e->bytes = want;
    }
    lease->mem = e->mem;
    lease->entry = e;
    return 0;
}

/* diagnostics (tests): scratch entries alive, and their device bytes */
extern "C" uint32_t tlsrec__scratch_entries(uint64_t *bytes)
{
    uint32_t n = 0;
    uint64_t b = 0;
    pthread_mutex_lock(&g_scratch_mu);
    for (ScratchEntry *e = g_scratch; e; e = e->next) {
        n++;
        b += e->bytes;
    }
    pthread_mutex_unlock(&g_scratch_mu);
    if (bytes) *bytes = b;
    return n;
}

extern "C" void tlsrec__scratch_release(tlsrec_scratch_lease *lease)
{
    if (lease && lease->entry) {
        pthread_mutex_unlock(&((ScratchEntry *) lease->entry)->mu);
        lease->entry = nullptr;
        lease->mem = nullptr;
    }
}

/* Device scratch of one bucketed batch (the stream's kind-0 scratch). */
struct BucketScratch {
    tlsrec_scratch_lease lease = { nullptr, nullptr };
    uint32_t *counts, *offs, *perm;
    uint2 *keyrank;
    bool want_srecs = false;  /* GCM kernels will run: keep the descriptors in perm order too */
    tlsrec_batch_rec *srecs = nullptr;
    void *scan_tmp;           /* tlsrec__exclusive_scan's block sums */
    size_t scan_bytes;
};

static int bucket(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res, uint32_t n,
                  hipStream_t st, BucketScratch &b)
{
    /* AES-128-GCM, AES-256-GCM, AES-192-GCM, AES-CCM slots, ChaCha, ARIA-128/192/256-GCM,
     * Camellia-128/192/256-GCM slots, end */
    const size_t nk = 10 * (size_t) kt->capacity + CP_SPREAD + 1;
    b.scan_bytes = tlsrec__scan_scratch_bytes((uint32_t) nk);
    const size_t al = 256;
    const size_t szk = (nk * 4 + al - 1) / al * al, szp = ((size_t) n * 4 + al - 1) / al * al;
    const size_t szr = ((size_t) n * 8 + al - 1) / al * al;
    /* the descriptors in perm order for the GCM kernels (GcmArgs::srecs) */
    const size_t szs = b.want_srecs ? ((size_t) n * sizeof(tlsrec_batch_rec) + al - 1) / al * al : 0;
    const size_t total = 2 * szk + szp + szr + szs + b.scan_bytes + al;
    const int lr = tlsrec__scratch_acquire(st, 0, total, &b.lease);
    if (lr) return lr;
    uint8_t *m = (uint8_t *) b.lease.mem;
    b.counts = (uint32_t *) m;
    b.offs = (uint32_t *) (m + szk);
    b.perm = (uint32_t *) (m + 2 * szk);
    b.keyrank = (uint2 *) (m + 2 * szk + szp);
    b.srecs = szs ? (tlsrec_batch_rec *) (m + 2 * szk + szp + szr) : nullptr;
    b.scan_tmp = m + 2 * szk + szp + szr + szs;
    BucketArgs a;
    a.slots = kt->d_slots;
    a.cipher_of = kt->d_cipher;
    a.recs = recs;
    a.res = res;
    a.n = n;
    a.capacity = kt->capacity;
    a.counts = b.counts;
    a.offs = b.offs;
    a.keyrank = b.keyrank;
    a.nk = (uint32_t) nk;
    a.perm = b.perm;
    a.srecs = b.srecs;
    if (tlsrec__launch_bucket_zero(&a, st) != hipSuccess ||
        tlsrec__launch_bucket_count(&a, st) != hipSuccess ||
        tlsrec__exclusive_scan(b.counts, b.offs, (uint32_t) nk, (uint32_t *) b.scan_tmp, st) != hipSuccess ||
        tlsrec__launch_bucket_scatter(&a, st) != hipSuccess)
        return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    return 0;
}

/* only_cipher: launch only that cipher's kernel (the single-record engine,
 * which knows the record's slot on the host); 0 = every cipher loaded. */
/* avg_bytes: mean record size when the caller knows it (the stream / DTLS
 * layers and the host pipeline do; 0 = unknown) -- it decides the GCM launch
 * for many keys with little work each (below). */
/* Test hooks (tlsrec_internal.h TLSREC_HOOK_SKIP; the test build only, as the
 * reference compiles its own under MBEDTLS_TEST_HOOKS, ssl_misc.h:2685):
 *   tlsrec__test_skip_record   the AEAD kernels leave this record index
 *                              unreached, so a test can show that its result
 *                              stays INTERNAL_ERROR
 *   tlsrec__test_fail_staging  the next n staging-area allocations of the
 *                              single-record engine fail (ALLOC_FAILED path)
 *   tlsrec__test_server_shadow served records read their key state from
 *                              copies at addresses whose low 32 bits have bit
 *                              31 set (the readfirstlane sign-extension case) */
#ifdef TLSREC_TEST_HOOKS
static volatile uint32_t g_test_skip = 0xffffffffu;
static volatile int g_test_fail_staging = 0;
static uint8_t *g_test_shadow = nullptr;
static size_t g_test_shadow_bytes = 0;

extern "C" void tlsrec__test_skip_record(uint32_t index) { g_test_skip = index; }
extern "C" void tlsrec__test_fail_staging(int n) { g_test_fail_staging = n; }
extern "C" void tlsrec__test_server_shadow(void *dev, size_t bytes)
{
    g_test_shadow = (uint8_t *) dev;
    g_test_shadow_bytes = dev ? bytes : 0;
}
#else
static constexpr uint32_t g_test_skip = 0xffffffffu;
#endif

extern "C" int tlsrec__server_yield(void);
extern "C" void tlsrec__server_note_batch(hipStream_t stream, int counted);

/* Launch options of one batch:
 *   only_mask  launch only these ciphers' kernels (1 << TLSREC_CIPHER_*; the
 *              single-record engine knows its records' ciphers), 0 = every
 *              cipher the table holds
 *   avg_bytes  mean record size when the caller knows it (the stream / DTLS
 *              layers, the host pipeline; 0 = unknown) -- it decides the GCM
 *              launch for many keys with little work each (below)
 *   prefilled  the caller already wrote INTERNAL_ERROR into every result (the
 *              single-record engine stages it with the upload)
 *   coalesced  a few records of many connections gathered from concurrent
 *              single-record calls: identity order (no bucket pass: its four
 *              launches would cost more than the batch), GCM in 16-lane wave
 *              passes, so each wave serves its own record's key */
struct BatchOpt {
    uint32_t only_mask = 0;
    uint32_t avg_bytes = 0;
    bool prefilled = false;
    bool coalesced = false;
    bool grouped = false;                /* a key's records are contiguous (the stream / DTLS layers: a connection's
                                            records in order): no bucket pass, the kernels walk them in place */
    const uint64_t *src_off = nullptr;   /* encrypt: contents at in + src_off[i] (tlsrec__batch_src) */
};

static int batch(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res, uint32_t n,
                 const uint8_t *in, uint8_t *out, uint32_t lanes, void *stream, int dec, const BatchOpt &opt = BatchOpt())
{
    if (!kt || (!recs && n) || (!res && n)) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t) stream;
    const int cu = kt->cu;
    const uint32_t avg_bytes = opt.avg_bytes;
    const bool prefilled = opt.prefilled;
    const uint32_t cmask = opt.only_mask ? (kt->cipher_mask & opt.only_mask) : kt->cipher_mask;
    const uint32_t skip = g_test_skip;
    /* A table holding a single key, or a batch of one record, needs no
     * grouping: the kernels walk the descriptors in order and flag records
     * naming an unusable slot.  Otherwise the bucket pass groups GCM records
     * by key (then ChaCha).  Either way every result reads INTERNAL_ERROR
     * before the AEAD kernels run (the guard kernel, or the bucket count
     * kernel), so a record that no kernel reaches fails closed -- the
     * reference's auth_done check, ssl_msg.c:1260 / :1804. */
    /* batch work takes the CUs the record server holds (server.hip): yield
     * now, note the batch's stream on every way out (the server launches no
     * grid between the two) */
    struct YieldGuard {
        hipStream_t st;
        bool on;
        int counted;      /* the yield counted this batch as queueing (only then does the note uncount it) */
        ~YieldGuard() { if (on) tlsrec__server_note_batch(st, counted); }
    } yg{ st, !opt.coalesced, 0 };
    if (yg.on) yg.counted = tlsrec__server_yield();
    BucketScratch bs;
    /* (r05) a table of ChaCha20-Poly1305 keys only needs no grouping either:
     * its kernel walks records in arrival order, with or without the bucket
     * pass's permutation, and flags unusable slots in identity order -- the
     * count / scan / scatter kernels cost 5-6 % of a 1 M-record stream or
     * DTLS batch */
    /* (r06) records already grouped by key -- the stream and DTLS layers emit
     * each connection's records together -- need no bucket pass either: the
     * GCM passes find a key's run of records where they lie (the bucket
     * count / scan / scatter kernels were ~90 us of a 1 M-record call);
     * TLSREC_GROUPED=0 sends them through the bucket pass as before */
    const bool grouped = opt.grouped && grouped_env();
    const bool identity = kt->nloaded == 1 || n == 1 || opt.coalesced || grouped ||
                          kt->cipher_mask == (1u << TLSREC_CIPHER_CHACHA20_POLY1305);
    const bool keyrun = !identity || grouped;     /* the many-keys launch shapes apply */
    if (identity) {
        if (!prefilled && tlsrec__launch_res_guard(res, n, st) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    } else {
        const uint32_t gcm_mask = (1u << TLSREC_CIPHER_AES_128_GCM) | (1u << TLSREC_CIPHER_AES_256_GCM) |
                                  (1u << TLSREC_CIPHER_AES_192_GCM) | (1u << TLSREC_CIPHER_ARIA_128_GCM) |
                                  (1u << TLSREC_CIPHER_ARIA_192_GCM) | (1u << TLSREC_CIPHER_ARIA_256_GCM) |
                                  (1u << TLSREC_CIPHER_CAMELLIA_128_GCM) | (1u << TLSREC_CIPHER_CAMELLIA_192_GCM) |
                                  (1u << TLSREC_CIPHER_CAMELLIA_256_GCM);
        bs.want_srecs = (cmask & gcm_mask) != 0 && srecs_env();
        int r = bucket(kt, recs, res, n, st, bs);
        if (r) {
            tlsrec__scratch_release(&bs.lease);
            return r;
        }
    }
    const uint32_t cap = kt->capacity;
    int rc = 0;
    static const int gcm_ciphers[3] = { TLSREC_CIPHER_AES_128_GCM, TLSREC_CIPHER_AES_256_GCM,
                                        TLSREC_CIPHER_AES_192_GCM };
    const uint32_t lanes_in = lanes;
    if (!lanes) lanes = gcm_lanes_env();
    for (int ci = 0; ci < 3 && !rc; ci++) {
        const int cipher = gcm_ciphers[ci];     /* bucket class ci: keys [ci * cap, (ci + 1) * cap) */
        if (!(cmask & (1u << cipher))) continue;
        /* (ARIA-GCM below: one configuration) */
        /* lanes per record: a key pass should still fill the 16 waves of a
         * workgroup.  8 for a single key or >= 128 records per key; 16
         * (4 records per wave) down to 48 records per key; 64 (one record per
         * wave) below that -- the many-connections, few-records regime of
         * the stream path. */
        const uint32_t nl = kt->nloaded;     /* read once: the engine's pages change under it */
        const uint32_t rpk = nl > 1 ? n / nl : n;
        /* ... and the batch should fill the chip: with fewer than 8 records
         * per wave of a full grid (cu x 16 waves), more lanes per record
         * (measured at 16 K x 16 KiB records: L = 8 363, L = 16 611, L = 64
         * 536 GiB/s) */
        const uint64_t rpwave = (uint64_t) n / ((uint64_t) cu * GCM_WAVES);
        const int Lfill = rpwave >= 8 ? 8 : (rpwave >= 2 ? 16 : 64);
        int L = (lanes == 2 || lanes == 4 || lanes == 8 || lanes == 16 || lanes == 64) ? (int) lanes
                : (nl <= 1 || rpk >= 128) ? 8 : (rpk >= 48 ? 16 : 64);
        if (!(lanes == 2 || lanes == 4 || lanes == 8 || lanes == 16 || lanes == 64) && Lfill > L) L = Lfill;
        /* one key, small records (<= 4 KiB, size hint): 4 lanes per record
         * (16 records per wave round) once the batch fills the chip at that --
         * half the lane tree and twice the records in flight per wave.  Same
         * box (r04r): c2s 592/582 -> 652/661, c2se 610/604 -> 682/681 GiB/s;
         * 16 KiB records keep 8 (c2 750/742 at 8, 732/737 at 4). */
        if (!(lanes == 2 || lanes == 4 || lanes == 8 || lanes == 16 || lanes == 64) && nl <= 1 && L == 8 &&
            rpwave >= 16 && avg_bytes != 0 && avg_bytes <= 4096)
            L = 4;
        if (kt->has_cid) L = 8;     /* the CID variant: one configuration */
        GcmArgs a;
        a.slots = kt->d_slots;
        a.ghtab = kt->d_ghtab;
        a.dummy = kt->d_dummy;
        a.recs = recs;
        a.res = res;
        a.n = n;
        a.perm = identity ? nullptr : bs.perm;
        a.srecs = identity ? nullptr : bs.srecs;
        a.lo = identity ? nullptr : bs.offs + (size_t) ci * cap;
        a.hi = identity ? nullptr : bs.offs + (size_t) (ci + 1) * cap;
        a.in = in;
        a.out = out;
        int nr = (int) tlsrec_cipher_nr(cipher);
        const int wpe = gcm_wp_env();
        const bool auto_l = !(lanes == 2 || lanes == 4 || lanes == 8 || lanes == 16 || lanes == 64);
        /* wave passes (each wave stages only its key's H^L table, no
         * workgroup barriers) for few records per key, or -- when the record
         * size is known -- for keys with under 64 KiB of records each (same-box
         * measurements: 16 x 1.4 KiB per key 198 -> 313 GiB/s, DTLS 125 -> 231;
         * 16 x 16 KiB and 64 x 1.4 KiB per key stay faster with key passes) */
        /* 4 lanes (16 records of the key per wave round) when the keys'
         * records are small, 12..127 each, and the batch fills the chip at 16
         * records per wave: one GHASH lane tree per 16 records instead of per
         * 4, and only the tree tables H^1, H^2 read from HBM.  Same-box, 1.4 KiB
         * records (L = 16 wave passes or L = 16 key passes before):
         *   64 K keys x 16, DTLS AES-128-GCM   receive 232 -> 390, send 212 -> 328 GiB/s
         *   64 K keys x 16, stream AES-256-GCM receive 198 -> 335, send 200 -> 294
         *   16 K keys x 64, stream AES-256-GCM receive 317 -> 357, send 282 -> 324
         *   c4s (64 K keys x 64, GCM + ChaCha)  486 -> 541
         * and 2 lanes (32 records per round, the tree only H^1) from 48 records
         * per key: 16 K keys x 64 stream receive 353 -> 375, send 319 -> 332,
         * c4s 536 -> 549 (at 16 per key 2 lanes idle half the wave: 388 -> 254). */
        const bool small = avg_bytes != 0 && avg_bytes <= 4096 && rpk >= 12 && rpk < 128;
        const bool small2 = small && rpk >= 48 && (uint64_t) n >= (uint64_t) cu * 8 * 32;
        const bool small4 = small && !small2 && (uint64_t) n >= (uint64_t) cu * 8 * 16;
        const bool light = rpk < 12 || (avg_bytes != 0 && rpk < 48 && (uint64_t) rpk * avg_bytes < 65536u) ||
                           small2 || small4;
        if (auto_l && !kt->has_cid && keyrun && nr != 12 && wpe != 0 && light)
            L = small2 ? 2 : (small4 ? 4 : ((rpk >= 3 && Lfill <= 16) ? 16 : 64));
        bool wp = !kt->has_cid && keyrun && (L == 2 || L == 4 || L == 16 || L == 64) && nr != 12 &&
                  (wpe == 1 || (wpe != 0 && light));
        if (opt.coalesced && n > 1 && auto_l && !kt->has_cid && nr != 12) {
            L = 64;        /* a wave per record, 64 lanes on it: each wave its own record's key, in parallel */
            wp = true;
        }
        /* Paired wave passes: small records (<= 4 KiB), 12..127 per key.  The
         * 8-wave passes above hold one 8 KiB H^L table per wave beside the
         * 64 KiB T-tables, so they run at half the single-key kernel's
         * occupancy and wait on LDS latency (r02 PMC, DTLS 16 x 1.4 KiB per
         * key: LDS 35 %, VALU 53 % busy); with two waves per table, 16 waves
         * fit.  Each wave takes half of a key's records, so L is picked for
         * a round to hold that half: 2 lanes (32 records) from 48 records per
         * key, 4 from 24, 8 below. */
        /* Large records (known > 4 KiB) with 4..11 per key (k4, 16 KiB
         * streams): the same pairing at 16 or 32 lanes, 4 or 2 records of a key
         * per wave. */
        /* (r05: small records up to 255 per key, L by the round-fill model of
         * tlsrec__gcm_pair_small_l) */
        bool pair = false;
        /* (r06) the paired kernels hold lane powers only (tlsrec_gcm.h): a
         * coalesced call or a TREEMUL mode without bit 3 takes the 8-wave passes */
        if (auto_l && !kt->has_cid && keyrun && nr != 12 && wpe != 0 && gcm_pair_env() && avg_bytes != 0 &&
            !opt.coalesced && (gcm_tm(true, true) & 8u)) {
            int Lp = 0;
            const bool small_pair = avg_bytes <= 4096 && rpk >= gcm_pair_small_min() && rpk < gcm_pair_small_max();
            if (small_pair) Lp = (int) tlsrec__gcm_pair_small_l(rpk);
            if (small_pair && gcm_pair_l_env()) Lp = gcm_pair_l_env();     /* measurement override */
            else if (avg_bytes > 4096 && rpk >= 4 && rpk < gcm_pair_big_max()) Lp = rpk >= 8 ? 16 : 32;
            if (Lp && (uint64_t) n >= (uint64_t) cu * 16 * (uint64_t) (64 / Lp)) {
                L = Lp;
                wp = pair = true;
            }
        }
        if (L == 2 && !wp) L = 4;     /* 2 lanes: wave passes only */
        const int waves = pair ? 16 : (wp ? 8 : (kt->has_cid ? 16 : gcm_waves()));
        a.rpw = (opt.coalesced && wp) ? 1u : pick_rpw(n, (uint32_t) waves, 64 / L, (uint32_t) cu);
        a.src_off = dec ? nullptr : opt.src_off;
        a.capacity = cap;
        a.cipher = (uint32_t) cipher;
        a.g5 = gcm_g5();
        /* coalesced calls wait on the lane tree: from the key's tables (one
         * L2 round trip per level) rather than table-free (~1 700 dependent
         * VALU ticks per level) */
        a.tm = opt.coalesced ? 0u : gcm_tm(pair, wp);
        a.skip = skip;
        uint64_t per_wg = (uint64_t) waves * a.rpw;
        uint32_t grid = (uint32_t) ((n + per_wg - 1) / per_wg);
        if (tlsrec__launch_gcm(&a, dec, L, nr, pair ? -32 : (wp ? -8 : (kt->has_cid ? -16 : waves)), grid, st) !=
            hipSuccess)
            rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    /* ARIA-GCM and Camellia-GCM: the GCM kernel around the LDS-table cipher
     * (8 lanes, 16 waves); bucket classes (4, 5, 6) cap + CP_SPREAD and (7, 8, 9) cap + CP_SPREAD */
    static const int alt_gcm[6] = { TLSREC_CIPHER_ARIA_128_GCM, TLSREC_CIPHER_ARIA_192_GCM, TLSREC_CIPHER_ARIA_256_GCM,
                                    TLSREC_CIPHER_CAMELLIA_128_GCM, TLSREC_CIPHER_CAMELLIA_192_GCM,
                                    TLSREC_CIPHER_CAMELLIA_256_GCM };
    for (int ci = 0; ci < 6 && !rc; ci++) {
        const int c = alt_gcm[ci];
        if (!(cmask & (1u << c))) continue;
        const size_t base = (size_t) (4 + ci) * cap + CP_SPREAD;
        GcmArgs a;
        a.slots = kt->d_slots;
        a.ghtab = kt->d_ghtab;
        a.dummy = kt->d_dummy;
        a.recs = recs;
        a.res = res;
        a.n = n;
        a.perm = identity ? nullptr : bs.perm;
        a.srecs = identity ? nullptr : bs.srecs;
        a.lo = identity ? nullptr : bs.offs + base;
        a.hi = identity ? nullptr : bs.offs + base + cap;
        a.in = in;
        a.out = out;
        a.rpw = pick_rpw(n, (uint32_t) ARIA_GCM_WAVES, 8u, (uint32_t) cu);
        a.src_off = nullptr;
        a.capacity = cap;
        a.cipher = (uint32_t) c;
        a.g5 = 0;
        a.tm = 0;
        a.skip = skip;
        const uint64_t per_wg = (uint64_t) ARIA_GCM_WAVES * a.rpw;
        const uint32_t grid = (uint32_t) ((n + per_wg - 1) / per_wg);
        if (tlsrec__launch_gcm_aria(&a, dec, (int) tlsrec_cipher_alt_nr(c), (int) kt->has_cid, grid, st) != hipSuccess)
            rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    uint32_t ccm_nr = 0;
    for (int c = TLSREC_CIPHER_AES_128_CCM; c <= TLSREC_CIPHER_AES_256_CCM_8; c++)
        if (cmask & (1u << c)) ccm_nr |= 1u << tlsrec_cipher_nr(c);
    for (int c = TLSREC_CIPHER_ARIA_128_CCM; c <= TLSREC_CIPHER_CAMELLIA_256_CCM; c++)   /* ARIA / Camellia: bit nr + 4 */
        if (tlsrec_cipher_is_alt_ccm(c) && (cmask & (1u << c))) ccm_nr |= 1u << (tlsrec_cipher_alt_nr(c) + 4);
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
        a.skip = skip;
        if (tlsrec__launch_ccm(&a, dec, ccm_nr, st) != hipSuccess) rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (!rc && (cmask & (1u << TLSREC_CIPHER_CHACHA20_POLY1305))) {
        /* 2 lanes per record, more when the batch would not fill the chip
         * (cu x 8 resident waves: 2 per SIMD) */
        const uint64_t rpwave = (uint64_t) n / ((uint64_t) cu * 8);
        int L = (lanes_in == 1 || lanes_in == 2 || lanes_in == 4 || lanes_in == 8) ? (int) lanes_in
                : (rpwave >= 32 ? 2 : (rpwave >= 16 ? 4 : 8));
        if (kt->has_cid) L = 2;     /* the CID variant: one configuration */
        CpArgs a;
        a.slots = kt->d_slots;
        a.recs = recs;
        a.res = res;
        a.n = n;
        a.perm = identity ? nullptr : bs.perm;
        a.lo = identity ? nullptr : bs.offs + 4 * (size_t) cap;
        a.hi = identity ? nullptr : bs.offs + 4 * (size_t) cap + CP_SPREAD;
        a.in = in;
        a.out = out;
        a.rpw = pick_rpw(n, CP_WAVES, 64 / L, (uint32_t) cu * 4);
        a.capacity = cap;
        a.cid = kt->has_cid;
        a.skip = skip;
        a.src_off = dec ? nullptr : opt.src_off;
        uint64_t per_wg = (uint64_t) CP_WAVES * a.rpw;
        uint32_t grid = (uint32_t) ((n + per_wg - 1) / per_wg);
        if (tlsrec__launch_chachapoly(&a, dec, L, grid, st) != hipSuccess) rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    tlsrec__scratch_release(&bs.lease);
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

extern "C" int tlsrec_batch_encrypt_sized(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                          uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                                          uint32_t mean_record_bytes, void *stream)
{
    BatchOpt o;
    o.avg_bytes = mean_record_bytes;
    return batch(kt, recs, res, n, in_arena, out_arena, 0, stream, 0, o);
}

extern "C" int tlsrec_batch_decrypt_sized(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                          uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                                          uint32_t mean_record_bytes, void *stream)
{
    BatchOpt o;
    o.avg_bytes = mean_record_bytes;
    return batch(kt, recs, res, n, in_arena, out_arena, 0, stream, 1, o);
}

extern "C" int tlsrec__keytab_src_ok(const tlsrec_keytab *kt)
{
    const uint32_t ok = (1u << TLSREC_CIPHER_AES_128_GCM) | (1u << TLSREC_CIPHER_AES_192_GCM) |
                        (1u << TLSREC_CIPHER_AES_256_GCM) | (1u << TLSREC_CIPHER_CHACHA20_POLY1305);
    return kt && !kt->has_cid && (kt->cipher_mask & ~ok) == 0;   /* (the CID kernel variants read in place) */
}

extern "C" int tlsrec__batch_src(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                 uint32_t n, const uint8_t *in_arena, uint8_t *out_arena, void *stream,
                                 uint32_t avg_bytes, const uint64_t *src_off)
{
    if (!tlsrec__keytab_src_ok(kt) || !src_off) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    BatchOpt o;
    o.avg_bytes = avg_bytes;
    o.src_off = src_off;
    o.grouped = true;                    /* (the stream / DTLS send paths' records, connection by connection) */
    return batch(kt, recs, res, n, in_arena, out_arena, 0, stream, 0, o);
}

extern "C" int tlsrec__batch_sized(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                   uint32_t n, const uint8_t *in_arena, uint8_t *out_arena, void *stream, int dec,
                                   uint32_t avg_bytes, int prefilled)
{
    BatchOpt o;
    o.avg_bytes = avg_bytes;
    o.grouped = true;                    /* (the stream / DTLS layers' records, connection by connection) */
    o.prefilled = prefilled != 0;
    return batch(kt, recs, res, n, in_arena, out_arena, 0, stream, dec, o);
}


/* ======================================================================
 * Records in host memory: chunked H2D -> kernel -> D2H pipeline
 * (tlsrec_host_batch_*).  Records start and end in host socket buffers
 * (SURVEY.md 8(d)); a chunk is a run of consecutive records, its byte range
 * [buf_off of the first, end of the last) goes to one of NSLOT device slots,
 * is protected there in place, and comes back to the same offsets of the
 * output arena.  Three streams (H2D, kernels, D2H) chained by events keep
 * both copy directions and the kernels busy at once.
 * ==================================================================== */
static constexpr int PIPE_SLOTS = 3;

struct HostPipe {
    hipStream_t h2d, cmp, d2h;
    hipEvent_t ev_h2d[PIPE_SLOTS], ev_cmp[PIPE_SLOTS], ev_d2h[PIPE_SLOTS];
    uint8_t *slot[PIPE_SLOTS];
    size_t slot_bytes;
    tlsrec_batch_rec *d_recs;
    tlsrec_batch_res *d_res;
    size_t nrec_cap;
};

static void host_pipe_free(HostPipe *p)
{
    if (!p) return;
    if (p->h2d) hipStreamSynchronize(p->h2d);
    if (p->cmp) hipStreamSynchronize(p->cmp);
    if (p->d2h) hipStreamSynchronize(p->d2h);
    for (int i = 0; i < PIPE_SLOTS; i++) {
        hipFree(p->slot[i]);
        if (p->ev_h2d[i]) hipEventDestroy(p->ev_h2d[i]);
        if (p->ev_cmp[i]) hipEventDestroy(p->ev_cmp[i]);
        if (p->ev_d2h[i]) hipEventDestroy(p->ev_d2h[i]);
    }
    hipFree(p->d_recs);
    hipFree(p->d_res);
    if (p->h2d) hipStreamDestroy(p->h2d);
    if (p->cmp) hipStreamDestroy(p->cmp);
    if (p->d2h) hipStreamDestroy(p->d2h);
    delete p;
}

static int host_pipe_reserve(tlsrec_keytab *kt, size_t slot_bytes, size_t nrec)
{
    HostPipe *p = kt->pipe;
    if (!p) {
        p = new (std::nothrow) HostPipe();
        if (!p) return TLSREC_ERR_SSL_ALLOC_FAILED;
        kt->pipe = p;
        if (hipStreamCreateWithFlags(&p->h2d, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&p->cmp, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&p->d2h, hipStreamNonBlocking) != hipSuccess)
            return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        for (int i = 0; i < PIPE_SLOTS; i++)
            if (hipEventCreateWithFlags(&p->ev_h2d[i], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_cmp[i], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->ev_d2h[i], hipEventDisableTiming) != hipSuccess)
                return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (p->slot_bytes < slot_bytes) {
        for (int i = 0; i < PIPE_SLOTS; i++) {
            hipFree(p->slot[i]);
            p->slot[i] = NULL;
        }
        p->slot_bytes = 0;
        for (int i = 0; i < PIPE_SLOTS; i++)
            if (hipMalloc((void **) &p->slot[i], slot_bytes) != hipSuccess) return TLSREC_ERR_SSL_ALLOC_FAILED;
        p->slot_bytes = slot_bytes;
    }
    if (p->nrec_cap < nrec) {
        hipFree(p->d_recs);
        hipFree(p->d_res);
        p->d_recs = NULL;
        p->d_res = NULL;
        p->nrec_cap = 0;
        if (hipMalloc((void **) &p->d_recs, nrec * sizeof(tlsrec_batch_rec)) != hipSuccess ||
            hipMalloc((void **) &p->d_res, nrec * sizeof(tlsrec_batch_res)) != hipSuccess)
            return TLSREC_ERR_SSL_ALLOC_FAILED;
        p->nrec_cap = nrec;
    }
    return 0;
}

static int host_batch(tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res, uint32_t n,
                      const uint8_t *in, uint8_t *out, uint32_t lanes, uint64_t chunk_bytes, int dec)
{
    if (!kt || (n && (!recs || !res || !in || !out))) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (n == 0) return 0;
    if (chunk_bytes == 0) chunk_bytes = 64ull << 20;   /* measured best of 16 / 64 / 256 / 1024 MiB */
    /* records in ascending, non-overlapping order; chunks of whole records */
    struct Chunk { uint32_t first, count; uint64_t base, span; };
    Chunk *ch = (Chunk *) malloc(sizeof(Chunk) * n);
    if (!ch) return TLSREC_ERR_SSL_ALLOC_FAILED;
    uint32_t nch = 0;
    uint64_t maxspan = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t lo = recs[i].buf_off, hi = lo + recs[i].buf_len;
        if (i && lo < recs[i - 1].buf_off + recs[i - 1].buf_len) {
            free(ch);
            return TLSREC_ERR_SSL_BAD_INPUT_DATA;
        }
        if (nch && hi - ch[nch - 1].base <= chunk_bytes) {
            ch[nch - 1].count++;
            ch[nch - 1].span = hi - ch[nch - 1].base;
        } else {
            ch[nch++] = Chunk{ i, 1, lo, hi - lo };
        }
        if (ch[nch - 1].span > maxspan) maxspan = ch[nch - 1].span;
    }
    /* Output arena in pinned host memory the device can address: the kernels
     * write their output straight into it over PCIe (measured 48-49 GiB/s
     * for c2-shaped records, the link rate) while the next chunk's H2D copy
     * runs on the copy engine -- a D2H copy instead shares that engine with
     * the H2D copies and the two directions serialise.  Pageable output:
     * protect in place in the device slot and copy the chunk back. */
    uint8_t *zc = NULL;
    {
        hipPointerAttribute_t at;
        const char *zce = getenv("TLSREC_HOST_ZC");      /* =0: copy back even to pinned memory (measurement) */
        if (!(zce && atoi(zce) == 0) && hipPointerGetAttributes(&at, out) == hipSuccess && at.type == hipMemoryTypeHost &&
            at.devicePointer)
            zc = (uint8_t *) at.devicePointer;
        else
            (void) hipGetLastError();    /* pageable memory: clear the sticky error */
    }
    pthread_mutex_lock(&kt->pipe_mu);
    int rc = host_pipe_reserve(kt, (maxspan + 255) / 256 * 256, n);
    HostPipe *p = kt->pipe;
    if (!rc && hipMemcpyAsync(p->d_recs, recs, (size_t) n * sizeof(*recs), hipMemcpyHostToDevice, p->cmp) != hipSuccess)
        rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    for (uint32_t c = 0; c < nch && !rc; c++) {
        const int k = (int) (c % PIPE_SLOTS);
        const Chunk &C = ch[c];
        hipError_t e = hipSuccess;
        if (c >= PIPE_SLOTS) e = hipStreamWaitEvent(p->h2d, p->ev_d2h[k], 0);      /* slot drained */
        if (e == hipSuccess) e = hipMemcpyAsync(p->slot[k], in + C.base, C.span, hipMemcpyHostToDevice, p->h2d);
        if (e == hipSuccess) e = hipEventRecord(p->ev_h2d[k], p->h2d);
        if (e == hipSuccess) e = hipStreamWaitEvent(p->cmp, p->ev_h2d[k], 0);
        if (e != hipSuccess) {
            rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
            break;
        }
        /* the descriptors' buf_off are offsets into the host arena: shift the
         * device arena base so that base + buf_off lands in the slot */
        uint8_t *dev = (uint8_t *) ((uintptr_t) p->slot[k] - (uintptr_t) C.base);
        BatchOpt o;
        o.avg_bytes = (uint32_t) (C.span / (C.count ? C.count : 1));
        rc = batch(kt, p->d_recs + C.first, p->d_res + C.first, C.count, dev, zc ? zc : dev, lanes, p->cmp, dec, o);
        if (rc) break;
        e = hipEventRecord(p->ev_cmp[k], p->cmp);
        if (zc) {
            /* the slot is free once its kernel is done */
            if (e == hipSuccess) e = hipStreamWaitEvent(p->d2h, p->ev_cmp[k], 0);
        } else {
            if (e == hipSuccess) e = hipStreamWaitEvent(p->d2h, p->ev_cmp[k], 0);
            if (e == hipSuccess) e = hipMemcpyAsync(out + C.base, p->slot[k], C.span, hipMemcpyDeviceToHost, p->d2h);
        }
        if (e == hipSuccess) e = hipEventRecord(p->ev_d2h[k], p->d2h);
        if (e != hipSuccess) rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    if (!rc && (hipStreamSynchronize(p->cmp) != hipSuccess ||
                hipMemcpyAsync(res, p->d_res, (size_t) n * sizeof(*res), hipMemcpyDeviceToHost, p->d2h) != hipSuccess))
        rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    if (p) {
        /* drain every stream before the caller may reuse its buffers */
        if (hipStreamSynchronize(p->h2d) != hipSuccess || hipStreamSynchronize(p->cmp) != hipSuccess ||
            hipStreamSynchronize(p->d2h) != hipSuccess)
            rc = rc ? rc : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    }
    pthread_mutex_unlock(&kt->pipe_mu);
    free(ch);
    return rc;
}

extern "C" int tlsrec_host_batch_encrypt(tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                         uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                                         uint32_t lanes_per_record, uint64_t chunk_bytes)
{
    return host_batch(kt, recs, res, n, in_arena, out_arena, lanes_per_record, chunk_bytes, 0);
}

extern "C" int tlsrec_host_batch_decrypt(tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                                         uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                                         uint32_t lanes_per_record, uint64_t chunk_bytes)
{
    return host_batch(kt, recs, res, n, in_arena, out_arena, lanes_per_record, chunk_bytes, 1);
}

/* ======================================================================
 * Engine used by the single-record API (tlsrec_host.c).
 *
 * Key slots live in pages of ENGINE_PAGE_SLOTS (one key table each), added
 * as connections arrive -- ENGINE_MAX_PAGES x 4096 = 1 M slots, i.e. 512 K
 * connections per process.
 *
 * Concurrent calls are coalesced (flat combining, per page): a call queues
 * its record; if fewer than ENGINE_SETS batches of the page are in flight it
 * becomes the leader of the next one, takes every queued record (up to
 * ENGINE_BATCH, either direction), stages them in one pinned buffer, and runs
 * one H2D copy, one launch per direction and cipher (identity order: no
 * bucket pass), one D2H copy and one sync for all of them; the callers whose
 * records it carried are woken with their results.  A lone call is its own
 * leader: one record, one round trip.  Under load a round trip carries as
 * many records as arrived during the previous one.
 * ==================================================================== */
#define ENGINE_PAGE_SLOTS 4096
#define ENGINE_MAX_PAGES 256
#define ENGINE_SETS 2                    /* batches of a queue in flight at once (own streams) */
#define ENGINE_BATCH 256                 /* records per coalesced batch */
#define ENGINE_ALIGN 128                 /* record slots in the staging arena */

struct EngineReq {
    int dec;
    tlsrec_batch_rec d;                  /* slot = page-local */
    uint32_t cipher;
    unsigned char *buf;
    size_t buf_len;
    const unsigned char *cid;
    tlsrec_batch_res res;
    int rc;
    int done;                            /* guarded by the combiner's mutex */
    EngineReq *next;
};

/* one staging set: [descriptors][results][arena], pinned host memory the
 * device can address (hd = its device address), and a device copy */
struct EngineSet {
    hipStream_t st;
    uint8_t *h, *hd, *d;
    size_t cap;
    int busy;
};

/* Batches up to this many staged bytes run zero-copy: the kernels read the
 * records from, and write them back to, the pinned staging area over PCIe
 * (no copy-engine round trips: measured on MI355X, an H2D or D2H copy of a
 * small record costs ~12 us with its sync, a whole kernel launch ~10 us,
 * tools/probes/latency_probe.hip).  TLSREC_ENGINE_ZC=0 stages through device
 * memory always; =<bytes> moves the bound. */
static size_t engine_zc_max(void)
{
    static size_t v = (size_t) -1;
    if (v == (size_t) -1) {
        const char *e = getenv("TLSREC_ENGINE_ZC");
        v = e ? (size_t) strtoull(e, NULL, 0) : (size_t) (64u << 10);
    }
    return v;
}

struct Combiner {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    EngineReq *head, *tail;
    EngineSet set[ENGINE_SETS];
    uint64_t batches, records;           /* statistics (tlsrec__engine_stats) */
};

/* A page queues records per (AEAD family, direction): each batch is then one
 * kernel launch, and a call never waits behind another family's kernel --
 * CCM's CBC-MAC is one dependent AES chain per record (a 1.4 KiB record is
 * ~170 us on one lane), GCM and ChaCha20-Poly1305 records take ~25 us. */
#define ENGINE_QUEUES 6
static int engine_queue(uint32_t cipher, int dec)
{
    const int fam = cipher == TLSREC_CIPHER_CHACHA20_POLY1305 ? 1
                    : (tlsrec_cipher_is_ccm((int) cipher) || tlsrec_cipher_is_alt_ccm((int) cipher)) ? 2 : 0;
    return fam * 2 + (dec ? 1 : 0);
}

struct EnginePage {
    tlsrec_keytab *kt;
    uint8_t used[ENGINE_PAGE_SLOTS];
    uint8_t cid[ENGINE_PAGE_SLOTS];      /* the slot has a DTLS connection ID (the record server takes none) */
    uint32_t nused;
    Combiner *co[ENGINE_QUEUES];
};

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;   /* slot allocation, page growth */
static EnginePage g_pages[ENGINE_MAX_PAGES];
static volatile int g_npages = 0;
static hipStream_t g_load = NULL;
static volatile int g_ready = 0;

static int engine_init_locked(void)
{
    if (g_ready) return 0;
    if (tlsrec_device_check() != 0) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    if (hipStreamCreateWithFlags(&g_load, hipStreamNonBlocking) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    g_ready = 1;
    return 0;
}

static void combiner_free(Combiner *c)
{
    if (!c) return;
    for (int i = 0; i < ENGINE_SETS; i++) {
        if (c->set[i].st) {
            hipStreamSynchronize(c->set[i].st);
            hipStreamDestroy(c->set[i].st);
        }
        if (c->set[i].h) hipHostFree(c->set[i].h);
        if (c->set[i].d) hipFree(c->set[i].d);
    }
    pthread_cond_destroy(&c->cv);
    pthread_mutex_destroy(&c->mu);
    free(c);
}

static Combiner *combiner_new(void)
{
    Combiner *c = (Combiner *) calloc(1, sizeof(Combiner));
    if (!c) return NULL;
    pthread_mutex_init(&c->mu, NULL);
    pthread_cond_init(&c->cv, NULL);
    for (int i = 0; i < ENGINE_SETS; i++)
        if (hipStreamCreateWithFlags(&c->set[i].st, hipStreamNonBlocking) != hipSuccess) {
            c->set[i].st = NULL;
            combiner_free(c);      /* the streams created before this one */
            return NULL;
        }
    return c;
}

static tlsrec_keytab *slot_table(int slot, uint32_t *idx)
{
    if (slot < 0) return NULL;
    const int pg = slot / ENGINE_PAGE_SLOTS;
    if (pg >= g_npages) return NULL;
    *idx = (uint32_t) (slot % ENGINE_PAGE_SLOTS);
    return g_pages[pg].kt;
}

extern "C" int tlsrec__engine_slot_alloc(const tlsrec_key_material *km)
{
    pthread_mutex_lock(&g_mu);
    int r = engine_init_locked();
    int slot = -1;
    int pg = 0;
    if (r == 0) {
        for (pg = 0; pg < g_npages; pg++)
            if (g_pages[pg].nused < ENGINE_PAGE_SLOTS) break;
        if (pg == g_npages) {
            if (pg == ENGINE_MAX_PAGES) {
                r = TLSREC_ERR_SSL_ALLOC_FAILED;
            } else {
                EnginePage &N = g_pages[pg];
                r = tlsrec_keytab_create(&N.kt, ENGINE_PAGE_SLOTS);
                for (int q = 0; r == 0 && q < ENGINE_QUEUES; q++)
                    if (!(N.co[q] = combiner_new())) r = TLSREC_ERR_SSL_ALLOC_FAILED;
                if (r != 0) {
                    /* unwind the partial page: nothing of it stays allocated or pointed at */
                    for (int q = 0; q < ENGINE_QUEUES; q++) {
                        combiner_free(N.co[q]);
                        N.co[q] = NULL;
                    }
                    if (N.kt) tlsrec_keytab_free(N.kt);
                    N.kt = NULL;
                }
                if (r == 0) g_npages = pg + 1;
            }
        }
    }
    if (r == 0) {
        EnginePage &P = g_pages[pg];
        for (int i = 0; i < ENGINE_PAGE_SLOTS; i++)
            if (!P.used[i]) { slot = i; break; }
        r = tlsrec_keytab_load(P.kt, (uint32_t) slot, 1, km, 0, g_load);
        if (r == 0 && hipStreamSynchronize(g_load) != hipSuccess) r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
        if (r == 0) {
            P.used[slot] = 1;
            P.cid[slot] = 0;
            P.nused++;
            slot += pg * ENGINE_PAGE_SLOTS;
        }
    }
    pthread_mutex_unlock(&g_mu);
    return r ? r : slot;
}

extern "C" void tlsrec__engine_slot_free(int slot)
{
    pthread_mutex_lock(&g_mu);
    uint32_t i = 0;
    tlsrec_keytab *kt = slot_table(slot, &i);
    EnginePage *P = kt ? &g_pages[slot / ENGINE_PAGE_SLOTS] : NULL;
    if (kt && P->used[i]) {
        /* zeroize (ssl_msg.c:6084-6099); the slot's cipher stays recorded in the
         * table's mask, so a later batch of this page may launch one kernel more */
        hipMemsetAsync(kt->d_slots + i, 0, sizeof(SlotState), g_load);
        hipMemsetAsync(kt->d_cipher + i, 0, 1, g_load);
        hipMemsetAsync(kt->d_ghtab + (size_t) i * KEY_TABLE_WORDS, 0, sizeof(uint4) * KEY_TABLE_WORDS, g_load);
        /* (the GHASH tables end with H^1..H^64, the record server's closing powers) */
        hipStreamSynchronize(g_load);
        kt->h_cipher[i] = 0;
        kt->nloaded--;
        P->used[i] = 0;
        P->nused--;
    }
    pthread_mutex_unlock(&g_mu);
}

#ifdef TLSREC_TEST_HOOKS
/* test hook: the device bytes of an engine slot -- its SlotState (1024 B),
 * the first 1024 B of its GHASH tables and its 64 record-server powers
 * (1024 B) -- copied to host, to show what slot_free leaves behind */
extern "C" int tlsrec__test_engine_slot_dump(int slot, void *state, void *ghtab, void *hpw)
{
    pthread_mutex_lock(&g_mu);
    uint32_t i = 0;
    tlsrec_keytab *kt = slot_table(slot, &i);
    int r = kt ? 0 : TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (!r && (hipMemcpy(state, kt->d_slots + i, sizeof(SlotState), hipMemcpyDeviceToHost) != hipSuccess ||
               hipMemcpy(ghtab, kt->d_ghtab + (size_t) i * KEY_TABLE_WORDS, 1024, hipMemcpyDeviceToHost) != hipSuccess ||
               hipMemcpy(hpw, kt->d_ghtab + (size_t) i * KEY_TABLE_WORDS + KEY_HPOW_OFF, 1024,
                         hipMemcpyDeviceToHost) != hipSuccess))
        r = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    pthread_mutex_unlock(&g_mu);
    return r;
}
#endif

extern "C" int tlsrec__engine_slot_set_cid(int slot, const unsigned char *cid, size_t cid_len)
{
    pthread_mutex_lock(&g_mu);
    uint32_t i = 0;
    tlsrec_keytab *kt = slot_table(slot, &i);
    int r = kt && g_pages[slot / ENGINE_PAGE_SLOTS].used[i] ? tlsrec_keytab_set_cid(kt, i, cid, cid_len, g_load)
                                                            : TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (r == 0) g_pages[slot / ENGINE_PAGE_SLOTS].cid[i] = cid_len != 0;
    pthread_mutex_unlock(&g_mu);
    return r;
}

static size_t al(size_t x, size_t a) { return (x + a - 1) / a * a; }

/* Leader: stage `n` records (linked from `first`), run them, fill in their
 * results.  Records of one direction are contiguous in the staging area
 * (encrypt first), each in its own ENGINE_ALIGN-aligned arena slot with its
 * CID bytes behind the buffer. */
static int run_batch(tlsrec_keytab *kt, EngineSet &S, EngineReq *first, uint32_t n)
{
    EngineReq *v[ENGINE_BATCH];
    uint32_t k = 0, ne = 0;
    for (EngineReq *r = first; r && k < n; r = r->next) v[k++] = r;
    /* encrypt records first */
    std::stable_partition(v, v + n, [](const EngineReq *r) { return !r->dec; });
    while (ne < n && !v[ne]->dec) ne++;
    const size_t off_res = al((size_t) n * sizeof(tlsrec_batch_rec), 256);
    const size_t off_arena = al(off_res + (size_t) n * sizeof(tlsrec_batch_res), 256);
    size_t used = 0;
    size_t boff[ENGINE_BATCH];
    for (uint32_t i = 0; i < n; i++) {
        boff[i] = used;
        used = al(used + v[i]->buf_len + v[i]->d.cid_len + 16, ENGINE_ALIGN);
    }
    const size_t need = off_arena + used + ENGINE_ALIGN;
    bool fail_alloc = false;
#ifdef TLSREC_TEST_HOOKS
    if (g_test_fail_staging > 0) {
        g_test_fail_staging--;
        fail_alloc = true;
    }
#endif
    if (S.cap < need || fail_alloc) {
        hipStreamSynchronize(S.st);
        hipHostFree(S.h);
        hipFree(S.d);
        S.h = S.hd = S.d = NULL;
        S.cap = 0;
        const size_t want = need > (1u << 20) ? need + need / 2 : (1u << 20);
        if (fail_alloc || hipHostMalloc((void **) &S.h, want, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void **) &S.hd, S.h, 0) != hipSuccess ||
            hipMalloc((void **) &S.d, want) != hipSuccess) {
            /* no request of this batch ran: each caller gets the error, never
             * the unfilled result (ssl_msg.c:1260 / :1804) */
            if (S.h) hipHostFree(S.h);
            if (S.d) hipFree(S.d);
            S.h = S.hd = S.d = NULL;
            for (uint32_t i = 0; i < n; i++) v[i]->rc = TLSREC_ERR_SSL_ALLOC_FAILED;
            return TLSREC_ERR_SSL_ALLOC_FAILED;
        }
        S.cap = want;
    }
    tlsrec_batch_rec *hd = (tlsrec_batch_rec *) S.h;
    tlsrec_batch_res *hr = (tlsrec_batch_res *) (S.h + off_res);
    uint8_t *ha = S.h + off_arena;
    uint32_t mask_e = 0, mask_d = 0;
    for (uint32_t i = 0; i < n; i++) {
        EngineReq *r = v[i];
        tlsrec_batch_rec d = r->d;
        d.buf_off = boff[i];
        if (r->buf_len) memcpy(ha + boff[i], r->buf, r->buf_len);
        if (d.cid_len) {
            memcpy(ha + boff[i] + r->buf_len, r->cid, d.cid_len);
            const uint32_t o = (uint32_t) r->buf_len;
            d.cid_off[0] = (uint8_t) o; d.cid_off[1] = (uint8_t) (o >> 8);
            d.cid_off[2] = (uint8_t) (o >> 16); d.cid_off[3] = (uint8_t) (o >> 24);
        }
        hd[i] = d;
        /* each result goes up as INTERNAL_ERROR: only a kernel turns it into a
         * verdict (ssl_msg.c:1260 / :1804, auth_done) */
        memset(&hr[i], 0, sizeof(hr[i]));
        hr[i].status = TLSREC_ERR_SSL_INTERNAL_ERROR;
        (r->dec ? mask_d : mask_e) |= 1u << r->cipher;
    }
    const size_t total = off_arena + used;
    const bool zc = total <= engine_zc_max();
    uint8_t *base = zc ? S.hd : S.d;
    hipError_t e = zc ? hipSuccess : hipMemcpyAsync(S.d, S.h, total, hipMemcpyHostToDevice, S.st);
    int rc = e == hipSuccess ? 0 : TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    tlsrec_batch_rec *dd = (tlsrec_batch_rec *) base;
    tlsrec_batch_res *dr = (tlsrec_batch_res *) (base + off_res);
    uint8_t *da = base + off_arena;
    BatchOpt o;
    o.prefilled = true;
    o.coalesced = true;     /* identity order, a wave per GCM record (one record too: 8 KiB of tables, not 56) */
    if (!rc && ne) {
        o.only_mask = mask_e;
        rc = batch(kt, dd, dr, ne, da, da, 0, S.st, 0, o);
    }
    if (!rc && n > ne) {
        o.only_mask = mask_d;
        rc = batch(kt, dd + ne, dr + ne, n - ne, da, da, 0, S.st, 1, o);
    }
    if (!rc) {
        e = zc ? hipSuccess : hipMemcpyAsync(S.h + off_res, S.d + off_res, total - off_res, hipMemcpyDeviceToHost, S.st);
        if (e == hipSuccess) e = hipStreamSynchronize(S.st);
        if (e != hipSuccess) rc = TLSREC_ERR_SSL_HW_ACCEL_FAILED;
    } else {
        hipStreamSynchronize(S.st);
    }
    for (uint32_t i = 0; i < n; i++) {
        EngineReq *r = v[i];
        r->rc = rc;
        if (!rc) {
            r->res = hr[i];
            if (r->buf_len) memcpy(r->buf, ha + boff[i], r->buf_len);
        }
    }
    return rc;
}

/* server.hip: the resident record server (AES-GCM, ChaCha20-Poly1305) */
extern "C" int tlsrec__server_run(int dec, uint32_t cipher, uint32_t nr, const tlsrec_batch_rec *rec,
                                  const void *slot_state, const void *ghtab, const void *hpw, unsigned char *buf,
                                  size_t buf_len, const void *plan, int skip, tlsrec_batch_res *out);

/* Run one record through the kernels: host buffer -> device -> host.  A
 * decrypted record's CID (cid_len bytes) is staged right after the buffer.
 * AES-GCM and ChaCha20-Poly1305 records of transforms without connection IDs
 * go to the record server first (plan: the record's framing plan, as the
 * host entry points computed it); the coalescing launch path below takes
 * every other record, and any the server does not take. */
extern "C" int tlsrec__engine_run(int dec, const tlsrec_batch_rec *rec, unsigned char *buf, size_t buf_len,
                                  const unsigned char *cid, const void *plan, tlsrec_batch_res *out)
{
    if (!g_ready) {
        pthread_mutex_lock(&g_mu);
        int r = engine_init_locked();
        pthread_mutex_unlock(&g_mu);
        if (r) return r;
    }
    uint32_t idx = 0;
    tlsrec_keytab *kt = slot_table((int) rec->slot, &idx);
    if (!kt) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    const uint32_t cipher = kt->h_cipher[idx];
    if (cipher == 0) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (buf_len > 0xffffffffu - 64) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    /* per slot, not the page's has_cid: one CID connection must not take the
     * server away from the page's other 4095 slots */
    if ((tlsrec_cipher_is_gcm((int) cipher) || cipher == TLSREC_CIPHER_CHACHA20_POLY1305) &&
        !g_pages[rec->slot / ENGINE_PAGE_SLOTS].cid[idx] && rec->cid_len == 0) {
        tlsrec_batch_rec d = *rec;
        d.slot = idx;
        const void *p_state = kt->d_slots + idx;
        const void *p_ghtab = kt->d_ghtab + (size_t) idx * KEY_TABLE_WORDS;
        const void *p_hpw = kt->d_ghtab + (size_t) idx * KEY_TABLE_WORDS + KEY_HPOW_OFF;
#ifdef TLSREC_TEST_HOOKS
        if (g_test_shadow) {
            /* copies at the first address of the test's buffer whose low word
             * has bit 31 set, all three inside that half of the 4 GiB window */
            const size_t sz[3] = { sizeof(SlotState), sizeof(uint4) * KEY_TABLE_WORDS, 0 };
            const size_t tot = sz[0] + sz[1] + sz[2];
            const uintptr_t b0 = (uintptr_t) g_test_shadow, end = b0 + g_test_shadow_bytes;
            uintptr_t at = (b0 + 255) & ~(uintptr_t) 255;
            if (!(at & 0x80000000u) || (at & 0xffffffffu) + tot > 0x100000000ull)
                at = ((at & 0xffffffffu) + tot > 0x100000000ull ? (at | 0xffffffffull) + 1 : at & ~(uintptr_t) 0xffffffffu) |
                     0x80000000u;
            if (at + tot > end) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
            const void *src[3] = { p_state, p_ghtab, p_hpw };
            uint8_t *dst = (uint8_t *) at;
            const void *dsts[3];
            for (int k = 0; k < 3; k++) {
                if (hipMemcpyAsync(dst, src[k], sz[k], hipMemcpyDeviceToDevice, g_load) != hipSuccess)
                    return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
                dsts[k] = dst;
                dst += sz[k];
            }
            if (hipStreamSynchronize(g_load) != hipSuccess) return TLSREC_ERR_SSL_HW_ACCEL_FAILED;
            p_state = dsts[0];
            p_ghtab = dsts[1];
            p_hpw = (const uint4 *) dsts[1] + KEY_HPOW_OFF;    /* the powers inside the copied tables */
        }
#endif
        const int r = tlsrec__server_run(dec, cipher, tlsrec_cipher_nr((int) cipher), &d, p_state, p_ghtab, p_hpw,
                                         buf, buf_len, plan, g_test_skip == 0, out);
        if (r <= 0) return r;
    }
    Combiner *co = g_pages[rec->slot / ENGINE_PAGE_SLOTS].co[engine_queue(cipher, dec)];
    EngineReq me;
    me.dec = dec;
    me.d = *rec;
    me.d.slot = idx;
    me.cipher = cipher;
    me.buf = buf;
    me.buf_len = buf_len;
    me.cid = cid;
    /* fail closed: a request no batch filled in reads as an error, never as
     * the success its zeroed result would say */
    me.rc = TLSREC_ERR_SSL_INTERNAL_ERROR;
    memset(&me.res, 0, sizeof(me.res));
    me.res.status = TLSREC_ERR_SSL_INTERNAL_ERROR;
    me.done = 0;
    me.next = NULL;
    pthread_mutex_lock(&co->mu);
    if (co->tail) co->tail->next = &me; else co->head = &me;
    co->tail = &me;
    while (!me.done) {
        int si = -1;
        for (int i = 0; i < ENGINE_SETS; i++)
            if (!co->set[i].busy) { si = i; break; }
        if (si < 0 || co->head == NULL) {
            pthread_cond_wait(&co->cv, &co->mu);
            continue;
        }
        /* leader: take the queue (up to ENGINE_BATCH records) */
        EngineSet &S = co->set[si];
        S.busy = 1;
        EngineReq *first = co->head;
        uint32_t n = 0;
        EngineReq *last = NULL;
        for (EngineReq *r = first; r && n < ENGINE_BATCH; r = r->next) { last = r; n++; }
        co->head = last->next;
        if (!co->head) co->tail = NULL;
        last->next = NULL;
        co->batches++;
        co->records += n;
        pthread_mutex_unlock(&co->mu);
        run_batch(kt, S, first, n);
        pthread_mutex_lock(&co->mu);
        for (EngineReq *r = first, *nx; r; r = nx) {
            nx = r->next;
            r->done = 1;
        }
        S.busy = 0;
        pthread_cond_broadcast(&co->cv);
    }
    pthread_mutex_unlock(&co->mu);
    if (me.rc) return me.rc;
    *out = me.res;
    return 0;
}

/* coalescing statistics over every page: batches run and records carried */
extern "C" void tlsrec__engine_stats(uint64_t *batches, uint64_t *records)
{
    uint64_t b = 0, r = 0;
    for (int pg = 0; pg < g_npages; pg++)
        for (int q = 0; q < ENGINE_QUEUES; q++) {
            Combiner *c = g_pages[pg].co[q];
            if (!c) continue;
            pthread_mutex_lock(&c->mu);
            b += c->batches;
            r += c->records;
            pthread_mutex_unlock(&c->mu);
        }
    if (batches) *batches = b;
    if (records) *records = r;
}
