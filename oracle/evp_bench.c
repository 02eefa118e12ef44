/*
 * evp_bench.c -- CPU baseline leg "OpenSSL EVP" of bench.py (test / baseline
 * infrastructure, never the product path).
 *
 * The reference's x86 CPU path runs its AEADs on AES-NI + PCLMULQDQ (AES-NI is
 * enabled by default, /root/reference/ChangeLog:1021-1024, :5335), which the
 * table-driven restatement in oracle.c does not model.  The TF-PSA-Crypto
 * sources are absent, so this leg stands in for that accelerated path with
 * OpenSSL 3 libcrypto (AES-NI / VAES / VPCLMULQDQ GCM, AVX2 / AVX-512
 * ChaCha20-Poly1305): the record framing of mbedtls_ssl_encrypt_buf /
 * mbedtls_ssl_decrypt_buf (nonce ssl_msg.c:768-781, AAD :568-735, TLS 1.3
 * inner plaintext :466-514, TLS 1.2 explicit IV :1066-1075 / :1353-1365)
 * around one EVP AEAD call per record, one thread per host core, one key
 * context per thread (the PSA key slot of a connection).
 *
 * evp_bench_records() returns the wall time of the pass; every record's
 * status lands in status[] (0, or -0x7180 for a failed tag).
 */
#define _POSIX_C_SOURCE 200809L
#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <pthread.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#define EB_AES_128_GCM 1
#define EB_AES_256_GCM 2
#define EB_CHACHA20_POLY1305 3

typedef struct {
    int cipher, tls13, dir;
    const uint8_t *key, *iv;
    uint8_t *arena;
    size_t stride, data_len;
    uint64_t lo, hi, seq0;
    int32_t *status;
} eb_job;

static const EVP_CIPHER *eb_cipher(int c)
{
    switch (c) {
        case EB_AES_128_GCM: return EVP_aes_128_gcm();
        case EB_AES_256_GCM: return EVP_aes_256_gcm();
        case EB_CHACHA20_POLY1305: return EVP_chacha20_poly1305();
        default: return NULL;
    }
}

/* The cipher fetched from a library context of the calling thread's own.
 * With the default context every thread's EVP_CipherInit_ex (the per-record
 * nonce re-init) updates the one shared provider cipher object: measured in
 * this container, 8 threads of ChaCha20-Poly1305 1.4 KiB records ran 3.2 GiB/s
 * on the shared context and 5.4 GiB/s with a context per thread (1 thread:
 * 0.7 / 0.8 GiB/s).  Free with EVP_CIPHER_free. */
static EVP_CIPHER *eb_fetch(OSSL_LIB_CTX *lc, int c)
{
    const char *name = c == EB_AES_128_GCM ? "AES-128-GCM"
                       : c == EB_AES_256_GCM ? "AES-256-GCM"
                       : c == EB_CHACHA20_POLY1305 ? "ChaCha20-Poly1305" : NULL;
    return name ? EVP_CIPHER_fetch(lc, name, NULL) : NULL;
}

/* One record through an EVP context that already holds its connection's key:
 * the framing of mbedtls_ssl_encrypt_buf / _decrypt_buf around one AEAD. */
/* v0 v1: the version bytes of the TLS 1.2 AAD (3 3; DTLS 1.2 writes fe fd,
 * and its 8-byte sequence is epoch || seq48) */
static int32_t eb_record_v(EVP_CIPHER_CTX *ctx, int cipher, int tls13, int dir, const uint8_t *iv, uint8_t *buf,
                           size_t data_len, uint64_t seq, uint8_t v0, uint8_t v1)
{
    const int explicit_iv = !tls13 && cipher != EB_CHACHA20_POLY1305;   /* ivlen != fixed_ivlen, :739-743 */
    uint8_t ctr[8], nonce[12], aad[13];
    for (int k = 7; k >= 0; k--) { ctr[k] = (uint8_t) seq; seq >>= 8; }
    /* ssl_build_record_nonce: fixed IV ^ (0^4 || seq), or iv4 || seq (TLS 1.2 GCM) */
    if (explicit_iv) {
        memcpy(nonce, iv, 4);
        memcpy(nonce + 4, ctr, 8);
    } else {
        memcpy(nonce, iv, 12);
        for (int k = 0; k < 8; k++) nonce[4 + k] ^= ctr[k];
    }
    int ok;
    int outl = 0;
    if (dir) {
        /* encrypt: content at buf[off], TLS 1.3 inner plaintext = content || 23 || 0^pad */
        size_t off = explicit_iv ? 8 : 0, len = data_len;
        uint8_t *p = buf + off;
        if (tls13) {
            p[len++] = 23;
            size_t pad = (16 - len % 16) % 16;
            memset(p + len, 0, pad);
            len += pad;
        }
        size_t aadlen;
        if (tls13) {
            const size_t l = len + 16;
            aad[0] = 23; aad[1] = 3; aad[2] = 3; aad[3] = (uint8_t) (l >> 8); aad[4] = (uint8_t) l;
            aadlen = 5;
        } else {
            memcpy(aad, ctr, 8);
            aad[8] = 23; aad[9] = v0; aad[10] = v1; aad[11] = (uint8_t) (len >> 8); aad[12] = (uint8_t) len;
            aadlen = 13;
        }
        ok = EVP_CipherInit_ex(ctx, NULL, NULL, NULL, nonce, 1) == 1 &&
             EVP_CipherUpdate(ctx, NULL, &outl, aad, (int) aadlen) == 1 &&
             EVP_CipherUpdate(ctx, p, &outl, p, (int) len) == 1 &&
             EVP_CipherFinal_ex(ctx, p + len, &outl) == 1 &&
             EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, p + len) == 1;
        if (explicit_iv) memcpy(buf, ctr, 8);
        return ok ? 0 : -1;
    }
    /* decrypt: record body at buf[0] (explicit IV first for TLS 1.2 GCM) */
    size_t off = explicit_iv ? 8 : 0;
    if (data_len < off + 16) return -0x7180;
    size_t len = data_len - off - 16;
    uint8_t *p = buf + off;
    if (explicit_iv) memcpy(nonce + 4, buf, 8);
    size_t aadlen;
    if (tls13) {
        const size_t l = len + 16;
        aad[0] = 23; aad[1] = 3; aad[2] = 3; aad[3] = (uint8_t) (l >> 8); aad[4] = (uint8_t) l;
        aadlen = 5;
    } else {
        memcpy(aad, ctr, 8);
        aad[8] = 23; aad[9] = v0; aad[10] = v1; aad[11] = (uint8_t) (len >> 8); aad[12] = (uint8_t) len;
        aadlen = 13;
    }
    ok = EVP_CipherInit_ex(ctx, NULL, NULL, NULL, nonce, 0) == 1 &&
         EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, 16, p + len) == 1 &&
         EVP_CipherUpdate(ctx, NULL, &outl, aad, (int) aadlen) == 1 &&
         EVP_CipherUpdate(ctx, p, &outl, p, (int) len) == 1 &&
         EVP_CipherFinal_ex(ctx, p + len, &outl) == 1;
    if (!ok) {
        memset(p, 0, len);                 /* PSA wipes the output on a bad tag */
        return -0x7180;                    /* MBEDTLS_ERR_SSL_INVALID_MAC */
    }
    if (tls13) {
        /* ssl_parse_inner_plaintext: strip zero padding, recover the type */
        size_t k = len;
        while (k > 0 && p[k - 1] == 0) k--;
        return k == 0 ? -0x7200 : 0;
    }
    return 0;
}

static int32_t eb_record(EVP_CIPHER_CTX *ctx, int cipher, int tls13, int dir, const uint8_t *iv, uint8_t *buf,
                         size_t data_len, uint64_t seq)
{
    return eb_record_v(ctx, cipher, tls13, dir, iv, buf, data_len, seq, 3, 3);
}

static void *eb_worker(void *arg)
{
    eb_job *j = (eb_job *) arg;
    OSSL_LIB_CTX *lc = OSSL_LIB_CTX_new();
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    EVP_CIPHER *ev = lc ? eb_fetch(lc, j->cipher) : NULL;
    /* the connection's key, set once (psa_import_key at transform setup) */
    if (!ctx || !ev || EVP_CipherInit_ex(ctx, ev, NULL, j->key, NULL, j->dir) != 1) {
        for (uint64_t i = j->lo; i < j->hi; i++) j->status[i] = -1;
    } else {
        for (uint64_t i = j->lo; i < j->hi; i++)
            j->status[i] = eb_record(ctx, j->cipher, j->tls13, j->dir, j->iv, j->arena + i * j->stride, j->data_len,
                                     j->seq0 + i);
    }
    EVP_CIPHER_CTX_free(ctx);
    EVP_CIPHER_free(ev);
    OSSL_LIB_CTX_free(lc);
    return NULL;
}

/* dir 1 = encrypt (content_len bytes of content per record), 0 = decrypt
 * (data_len = the whole protected record body); record i at arena + i*stride,
 * sequence number seq0 + i, one key for the batch. */
double evp_bench_records(int cipher, int tls13, const uint8_t *key, const uint8_t *iv, int dir, uint8_t *arena,
                         size_t stride, size_t data_len, uint64_t n, uint64_t seq0, int threads, int32_t *status)
{
    if (threads < 1) threads = 1;
    if (threads > 512) threads = 512;
    pthread_t tid[512];
    eb_job jobs[512];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < threads; i++) {
        jobs[i] = (eb_job) { cipher, tls13, dir, key, iv, arena, stride, data_len,
                             n * (uint64_t) i / (uint64_t) threads, n * (uint64_t) (i + 1) / (uint64_t) threads,
                             seq0, status };
        if (pthread_create(&tid[i], NULL, eb_worker, &jobs[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);   /* started workers use the caller's buffers */
            return -1.0;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double) (b.tv_sec - a.tv_sec) + 1e-9 * (double) (b.tv_nsec - a.tv_nsec);
}

/* ---- many connections: one EVP context per connection -------------------
 * The multi-connection configs (c4 / c4s): record i belongs to connection
 * i % nconn (records round-robin over connections, as the GPU batch), each
 * connection has its own key context (the reference keeps one transform per
 * connection, ssl_misc.h:1073-1120), and a connection is served by one thread
 * (thread = connection % threads).  evp_mixed_create sets every key once
 * (untimed: psa_import_key at transform setup). */
typedef struct {
    uint32_t nconn;
    int tls13, threads;
    EVP_CIPHER_CTX **ctx;
    uint8_t *cipher;
    uint8_t (*iv)[12];
    OSSL_LIB_CTX **lc;        /* one library context per serving thread (eb_fetch) */
    EVP_CIPHER **ev;          /* [threads][3]: that thread's fetched ciphers */
    const uint8_t *keys;      /* setup only */
    int setup_ok;
} eb_mixed;

void evp_mixed_free(eb_mixed *m);

typedef struct {
    eb_mixed *m;
    int t;
    int ok;
} eb_setup;

static void *eb_setup_worker(void *arg)
{
    eb_setup *s = (eb_setup *) arg;
    eb_mixed *m = s->m;
    s->ok = 1;
    m->lc[s->t] = OSSL_LIB_CTX_new();
    if (!m->lc[s->t]) { s->ok = 0; return NULL; }
    for (int c = 1; c <= 3; c++) m->ev[3 * s->t + c - 1] = eb_fetch(m->lc[s->t], c);
    for (uint32_t c = (uint32_t) s->t; c < m->nconn; c += (uint32_t) m->threads) {
        EVP_CIPHER *ev = m->cipher[c] >= 1 && m->cipher[c] <= 3 ? m->ev[3 * s->t + m->cipher[c] - 1] : NULL;
        m->ctx[c] = EVP_CIPHER_CTX_new();
        if (!ev || !m->ctx[c] || EVP_CipherInit_ex(m->ctx[c], ev, NULL, m->keys + 32 * (size_t) c, NULL, 1) != 1) {
            s->ok = 0;
            return NULL;
        }
    }
    return NULL;
}

/* connection c is served by thread c % threads, whose library context holds
 * its key context (made by that thread: untimed, psa_import_key at setup) */
eb_mixed *evp_mixed_create(uint32_t nconn, const uint8_t *ciphers, const uint8_t *keys /* 32 B each */,
                           const uint8_t *ivs /* 12 B each */, int tls13, int threads)
{
    if (threads < 1) threads = 1;
    if (threads > 512) threads = 512;
    eb_mixed *m = calloc(1, sizeof(*m));
    if (!m) return NULL;
    m->nconn = nconn;
    m->tls13 = tls13;
    m->threads = threads;
    m->ctx = calloc(nconn, sizeof(*m->ctx));
    m->cipher = malloc(nconn);
    m->iv = malloc((size_t) nconn * 12);
    m->lc = calloc((size_t) threads, sizeof(*m->lc));
    m->ev = calloc((size_t) threads * 3, sizeof(*m->ev));
    if (!m->ctx || !m->cipher || !m->iv || !m->lc || !m->ev) { evp_mixed_free(m); return NULL; }
    memcpy(m->cipher, ciphers, nconn);
    memcpy(m->iv, ivs, (size_t) nconn * 12);
    m->keys = keys;
    pthread_t tid[512];
    eb_setup st[512];
    int ok = 1;
    for (int i = 0; i < threads; i++) {
        st[i] = (eb_setup) { m, i, 0 };
        if (pthread_create(&tid[i], NULL, eb_setup_worker, &st[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);   /* started workers use the caller's buffers */
            return evp_mixed_free(m), NULL;
        }
    }
    for (int i = 0; i < threads; i++) {
        pthread_join(tid[i], NULL);
        ok &= st[i].ok;
    }
    m->keys = NULL;
    if (!ok) { evp_mixed_free(m); return NULL; }
    return m;
}

void evp_mixed_free(eb_mixed *m)
{
    if (!m) return;
    if (m->ctx)
        for (uint32_t c = 0; c < m->nconn; c++) EVP_CIPHER_CTX_free(m->ctx[c]);
    if (m->ev)
        for (int i = 0; i < 3 * m->threads; i++) EVP_CIPHER_free(m->ev[i]);
    if (m->lc)
        for (int i = 0; i < m->threads; i++) OSSL_LIB_CTX_free(m->lc[i]);
    free(m->ctx);
    free(m->cipher);
    free(m->iv);
    free(m->lc);
    free(m->ev);
    free(m);
}

typedef struct {
    const eb_mixed *m;
    int dir, t, threads;
    uint8_t *arena;
    size_t stride, data_len;
    uint64_t n;
    int32_t *status;
} eb_mjob;

static void *eb_mworker(void *arg)
{
    eb_mjob *j = (eb_mjob *) arg;
    const eb_mixed *m = j->m;
    for (uint64_t i = 0; i < j->n; i++) {
        const uint32_t c = (uint32_t) (i % m->nconn);
        if ((int) (c % (uint32_t) j->threads) != j->t) continue;
        j->status[i] = eb_record(m->ctx[c], m->cipher[c], m->tls13, j->dir, m->iv[c], j->arena + i * j->stride,
                                 j->data_len, i / m->nconn);   /* the connection's own sequence number */
    }
    return NULL;
}

double evp_mixed_records(const eb_mixed *m, int dir, uint8_t *arena, size_t stride, size_t data_len, uint64_t n,
                         int32_t *status)
{
    const int threads = m->threads;    /* the serving threads of evp_mixed_create */
    pthread_t tid[512];
    eb_mjob jobs[512];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < threads; i++) {
        jobs[i] = (eb_mjob) { m, dir, i, threads, arena, stride, data_len, n, status };
        if (pthread_create(&tid[i], NULL, eb_mworker, &jobs[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);   /* started workers use the caller's buffers */
            return -1.0;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double) (b.tv_sec - a.tv_sec) + 1e-9 * (double) (b.tv_nsec - a.tv_nsec);
}

/* Where an EVP record's time goes (bench.py reports it beside the EVP leg):
 * out[0] = nonce re-init + AAD, out[1] = the payload update, out[2] = final,
 * out[3] = tag ctrl, each in microseconds per record (encrypt, len bytes,
 * one context, warm cache).  OpenSSL 3's provider dispatch costs ~0.1-0.5 us
 * per call, which at 1.4 KiB is as much as the ChaCha20-Poly1305 arithmetic. */
static double eb_now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double) t.tv_sec + 1e-9 * (double) t.tv_nsec;
}

int evp_call_profile(int cipher, size_t len, int iters, double out[4])
{
    const EVP_CIPHER *ev = eb_cipher(cipher);
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    uint8_t key[32] = { 1 }, nonce[12] = { 2 }, aad[5] = { 23, 3, 3, 0, 0 }, tag[16];
    uint8_t *buf = calloc(1, len + 32);
    if (!ev || !ctx || !buf || EVP_CipherInit_ex(ctx, ev, NULL, key, NULL, 1) != 1) {
        EVP_CIPHER_CTX_free(ctx);
        free(buf);
        return -1;
    }
    double t[4] = { 0, 0, 0, 0 };
    int outl = 0, ok = 1;
    for (int i = 0; i < iters; i++) {
        nonce[11] = (uint8_t) i;
        nonce[10] = (uint8_t) (i >> 8);
        const double a = eb_now();
        ok &= EVP_CipherInit_ex(ctx, NULL, NULL, NULL, nonce, 1) == 1;
        ok &= EVP_CipherUpdate(ctx, NULL, &outl, aad, 5) == 1;
        const double b = eb_now();
        ok &= EVP_CipherUpdate(ctx, buf, &outl, buf, (int) len) == 1;
        const double c = eb_now();
        ok &= EVP_CipherFinal_ex(ctx, buf + len, &outl) == 1;
        const double d = eb_now();
        ok &= EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1;
        const double e = eb_now();
        t[0] += b - a; t[1] += c - b; t[2] += d - c; t[3] += e - d;
    }
    for (int k = 0; k < 4; k++) out[k] = t[k] / iters * 1e6;
    EVP_CIPHER_CTX_free(ctx);
    free(buf);
    return ok ? 0 : -1;
}

/* ---- bulk independent parity (tests/test_evp_parity_gpu.py) --------------
 * Records of any length under a few keys, checked against OpenSSL EVP with
 * the ssl_msg.c framing of eb_record:
 *   mode 0: seal record i in place (content at off[i] + head, for GPU decrypt)
 *   mode 1: seal a copy of record i's plaintext (plain + off[i] + head) and
 *           compare the wire bytes with got + off[i] (the GPU's encrypt output)
 *   mode 2: compare the content bytes of got (decrypted by the GPU) with plain
 * head = 8 for TLS 1.2 GCM (explicit nonce), else 0.  result[i] = 0 when the
 * record matches (mode 0: the EVP status), 1 when it does not. */
typedef struct {
    int mode, cipher, tls13, t, threads;
    uint32_t nkeys;
    const uint8_t *keys, *ivs;
    uint64_t n;
    const uint32_t *keyidx, *len;
    const uint64_t *seq, *off;
    uint8_t *plain;
    const uint8_t *got;
    int32_t *result;
} eb_vjob;

static void *eb_vworker(void *arg)
{
    eb_vjob *j = (eb_vjob *) arg;
    const EVP_CIPHER *ev = eb_cipher(j->cipher);
    EVP_CIPHER_CTX **ctx = calloc(j->nkeys, sizeof(*ctx));
    uint8_t *scratch = malloc(16384 + 64);
    const size_t head = (!j->tls13 && j->cipher != EB_CHACHA20_POLY1305) ? 8 : 0;
    int ok = ev && ctx && scratch;
    for (uint32_t k = 0; ok && k < j->nkeys; k++) {
        ctx[k] = EVP_CIPHER_CTX_new();
        ok = ctx[k] && EVP_CipherInit_ex(ctx[k], ev, NULL, j->keys + 32 * (size_t) k, NULL, 1) == 1;
    }
    for (uint64_t i = (uint64_t) j->t; i < j->n; i += (uint64_t) j->threads) {
        if (!ok || j->keyidx[i] >= j->nkeys || j->len[i] > 16384) { j->result[i] = -1; continue; }
        const uint32_t k = j->keyidx[i];
        const size_t len = j->len[i];
        const size_t inner = j->tls13 ? len + 1 + (16 - (len + 1) % 16) % 16 : len;
        const size_t wire = head + inner + 16;
        if (j->mode == 0) {
            j->result[i] = eb_record(ctx[k], j->cipher, j->tls13, 1, j->ivs + 12 * (size_t) k, j->plain + j->off[i],
                                     len, j->seq[i]);
        } else if (j->mode == 1) {
            memset(scratch, 0, wire);
            memcpy(scratch + head, j->plain + j->off[i] + head, len);
            const int32_t st = eb_record(ctx[k], j->cipher, j->tls13, 1, j->ivs + 12 * (size_t) k, scratch, len,
                                         j->seq[i]);
            j->result[i] = st != 0 || memcmp(scratch, j->got + j->off[i], wire) != 0;
        } else {
            j->result[i] = memcmp(j->plain + j->off[i] + head, j->got + j->off[i] + head, len) != 0;
        }
    }
    if (ctx)
        for (uint32_t k = 0; k < j->nkeys; k++) EVP_CIPHER_CTX_free(ctx[k]);
    free(ctx);
    free(scratch);
    return NULL;
}

int evp_check_records(int mode, int cipher, int tls13, uint32_t nkeys, const uint8_t *keys, const uint8_t *ivs,
                      uint64_t n, const uint32_t *keyidx, const uint64_t *seq, const uint64_t *off,
                      const uint32_t *len, uint8_t *plain, const uint8_t *got, int threads, int32_t *result)
{
    if (threads < 1) threads = 1;
    if (threads > 512) threads = 512;
    pthread_t tid[512];
    eb_vjob jobs[512];
    for (int i = 0; i < threads; i++) {
        jobs[i] = (eb_vjob) { mode, cipher, tls13, i, threads, nkeys, keys, ivs, n, keyidx, len, seq, off, plain, got,
                              result };
        if (pthread_create(&tid[i], NULL, eb_vworker, &jobs[i]) != 0) {
            /* the workers already started write into result: join them before
             * the caller may reuse it */
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);
            return -1;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    return 0;
}

/* ---- the SURVEY §8(f) rows: record framing of a connection around EVP -----
 * tools/bench_stream.py / bench_dtls.py's "evp" CPU leg.  Connection c (its
 * key context made by evp_mixed_create, served by thread c % threads) sends
 * or receives its records in order, as one thread serving that socket would:
 *   stream receive: the header walk of ssl_get_next_record
 *     (ssl_parse_record_header ssl_msg.c:3561-3776: type, version, length
 *     checks), decrypt_buf (one EVP AEAD), the zero-length and counter rules of
 *     ssl_prepare_record_content (:3914-3966);
 *   stream send: mbedtls_ssl_write_record (:2648-2793): max_frag records, the
 *     5-byte header, encrypt_buf (one EVP AEAD), counter increment;
 *   DTLS receive: the 13-byte header (epoch, explicit 48-bit sequence), the
 *     anti-replay window check and update (mbedtls_ssl_dtls_replay_check /
 *     _update, :4240-4330), decrypt_buf;
 *   DTLS send: the 13-byte header with epoch || seq, encrypt_buf.
 * status[c]: 0, or the first error of the connection. */
typedef struct {
    const eb_mixed *m;
    int dtls, dir, t;
    uint8_t *in;
    size_t in_stride, in_len;
    uint8_t *out;
    size_t out_stride, max_frag;
    int32_t *status;
} eb_rjob;

static int32_t eb_stream_recv(const eb_mixed *m, uint32_t c, uint8_t *b, size_t len)
{
    size_t pos = 0;
    uint64_t seq = 0;
    int nb_zero = 0;
    while (len - pos >= 5) {
        uint8_t *h = b + pos;
        if (h[0] < 20 || h[0] > 23) return -0x7200;                 /* ssl_check_record_type */
        if (((h[1] << 8) | h[2]) > 0x0304) return -0x7200;
        const size_t dlen = ((size_t) h[3] << 8) | h[4];
        if (dlen == 0) return -0x7200;
        if (5 + dlen > 5 + 16384 + 256) return -0x7100;
        if (len - pos < 5 + dlen) break;
        const int32_t r = eb_record(m->ctx[c], m->cipher[c], m->tls13, 0, m->iv[c], h + 5, dlen, seq);
        if (r) return r;
        /* TLS 1.3: eb_record strips the padding (an all-zero inner plaintext is
         * INVALID_RECORD); no zero-length application data in this workload */
        nb_zero = 0;
        if (++seq == 0) return -0x6B80;                              /* COUNTER_WRAPPING */
        pos += 5 + dlen;
    }
    (void) nb_zero;
    return pos == len ? 0 : -0x7200;
}

static int32_t eb_stream_send(const eb_mixed *m, uint32_t c, const uint8_t *pt, size_t len, uint8_t *out,
                              size_t cap, size_t max_frag)
{
    size_t off = 0, pos = 0;
    uint64_t seq = 0;
    const int tls13 = m->tls13;
    const int explicit_iv = !tls13 && m->cipher[c] != EB_CHACHA20_POLY1305;
    while (off < len) {
        const size_t n = len - off < max_frag ? len - off : max_frag;
        const size_t inner = tls13 ? n + 1 + (16 - (n + 1) % 16) % 16 : n;
        const size_t body = (explicit_iv ? 8 : 0) + inner + 16;
        if (pos + 5 + body > cap) return -0x6A00;                    /* BUFFER_TOO_SMALL */
        uint8_t *h = out + pos;
        memcpy(h + 5 + (explicit_iv ? 8 : 0), pt + off, n);
        const int32_t r = eb_record(m->ctx[c], m->cipher[c], tls13, 1, m->iv[c], h + 5, n, seq);
        if (r) return r;
        h[0] = 23;
        h[1] = 3;
        h[2] = 3;
        h[3] = (uint8_t) (body >> 8);
        h[4] = (uint8_t) body;
        pos += 5 + body;
        off += n;
        seq++;
    }
    return 0;
}

static int32_t eb_dtls_recv(const eb_mixed *m, uint32_t c, uint8_t *b, size_t len, size_t dgram)
{
    uint64_t top = 0, window = 0;
    int any = 0;
    size_t nd = 0, accepted = 0;
    for (size_t d = 0; d + dgram <= len; d += dgram, nd++) {
        uint8_t *h = b + d;
        if (h[0] < 20 || h[0] > 23 || h[1] != 0xfe || h[2] != 0xfd) continue;   /* dropped datagram */
        const uint16_t epoch = (uint16_t) (h[3] << 8 | h[4]);
        uint64_t rs = 0;
        for (int k = 5; k < 11; k++) rs = rs << 8 | h[k];
        const size_t dlen = ((size_t) h[11] << 8) | h[12];
        if (epoch != 1 || 13 + dlen > dgram) continue;
        /* anti-replay check */
        if (any && rs + 64 <= top) continue;
        if (any && rs <= top && (window >> (top - rs)) & 1) continue;
        const int32_t r = eb_record_v(m->ctx[c], m->cipher[c], 0, 0, m->iv[c], h + 13, dlen,
                                      (uint64_t) epoch << 48 | rs, 0xfe, 0xfd);
        if (r == -0x7180) continue;                                   /* bad MAC: dropped (badmac_limit 0) */
        if (r) return r;
        /* anti-replay update */
        if (!any || rs > top) {
            const uint64_t shift = any ? rs - top : 64;
            window = shift >= 64 ? 1 : (window << shift) | 1;
            top = rs;
            any = 1;
        } else {
            window |= (uint64_t) 1 << (top - rs);
        }
        accepted++;
    }
    /* the bench workload is all-valid: a dropped datagram is an error here */
    return accepted == nd ? 0 : -0x7200;
}

static int32_t eb_dtls_send(const eb_mixed *m, uint32_t c, const uint8_t *pt, size_t len, uint8_t *out, size_t cap,
                            size_t max_frag)
{
    size_t off = 0, pos = 0;
    uint64_t seq = 0;
    const int explicit_iv = m->cipher[c] != EB_CHACHA20_POLY1305;
    while (off < len) {
        const size_t n = len - off < max_frag ? len - off : max_frag;
        const size_t body = (explicit_iv ? 8 : 0) + n + 16;
        if (pos + 13 + body > cap) return -0x6A00;
        uint8_t *h = out + pos;
        const uint64_t ctr = (uint64_t) 1 << 48 | seq;                /* epoch 1 */
        memcpy(h + 13 + (explicit_iv ? 8 : 0), pt + off, n);
        const int32_t r = eb_record_v(m->ctx[c], m->cipher[c], 0, 1, m->iv[c], h + 13, n, ctr, 0xfe, 0xfd);
        if (r) return r;
        h[0] = 23;
        h[1] = 0xfe;
        h[2] = 0xfd;
        for (int k = 0; k < 8; k++) h[3 + k] = (uint8_t) (ctr >> (56 - 8 * k));
        h[11] = (uint8_t) (body >> 8);
        h[12] = (uint8_t) body;
        pos += 13 + body;
        off += n;
        seq++;
    }
    return 0;
}

static void *eb_rworker(void *arg)
{
    eb_rjob *j = (eb_rjob *) arg;
    const eb_mixed *m = j->m;
    for (uint32_t c = (uint32_t) j->t; c < m->nconn; c += (uint32_t) m->threads) {
        uint8_t *in = j->in + (size_t) c * j->in_stride;
        uint8_t *out = j->out ? j->out + (size_t) c * j->out_stride : NULL;
        int32_t r;
        if (j->dir)
            r = j->dtls ? eb_dtls_send(m, c, in, j->in_len, out, j->out_stride, j->max_frag)
                        : eb_stream_send(m, c, in, j->in_len, out, j->out_stride, j->max_frag);
        else
            r = j->dtls ? eb_dtls_recv(m, c, in, j->in_len, j->max_frag) : eb_stream_recv(m, c, in, j->in_len);
        j->status[c] = r;
    }
    return NULL;
}

/* dir 1 = send (in: in_len bytes of application data per connection, out:
 * its records), 0 = receive (in: in_len wire bytes per connection, decrypted
 * in place; DTLS: max_frag = the wire size of one datagram).  Seconds. */
double evp_mixed_stream(const eb_mixed *m, int dtls, int dir, uint8_t *in, size_t in_stride, size_t in_len,
                        uint8_t *out, size_t out_stride, size_t max_frag, int32_t *status)
{
    const int threads = m->threads;
    pthread_t tid[512];
    eb_rjob jobs[512];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < threads; i++) {
        jobs[i] = (eb_rjob) { m, dtls, dir, i, in, in_stride, in_len, out, out_stride, max_frag, status };
        if (pthread_create(&tid[i], NULL, eb_rworker, &jobs[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);
            return -1.0;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double) (b.tv_sec - a.tv_sec) + 1e-9 * (double) (b.tv_nsec - a.tv_nsec);
}
