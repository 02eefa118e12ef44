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
#include <openssl/evp.h>
#include <pthread.h>
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

static void *eb_worker(void *arg)
{
    eb_job *j = (eb_job *) arg;
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    const EVP_CIPHER *ev = eb_cipher(j->cipher);
    const int explicit_iv = !j->tls13 && j->cipher != EB_CHACHA20_POLY1305;   /* ivlen != fixed_ivlen, :739-743 */
    /* the connection's key, set once (psa_import_key at transform setup) */
    if (!ctx || !ev || EVP_CipherInit_ex(ctx, ev, NULL, j->key, NULL, j->dir) != 1) {
        for (uint64_t i = j->lo; i < j->hi; i++) j->status[i] = -1;
        EVP_CIPHER_CTX_free(ctx);
        return NULL;
    }
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint8_t *buf = j->arena + i * j->stride;
        uint8_t ctr[8], nonce[12], aad[13];
        uint64_t s = j->seq0 + i;
        for (int k = 7; k >= 0; k--) { ctr[k] = (uint8_t) s; s >>= 8; }
        /* ssl_build_record_nonce: fixed IV ^ (0^4 || seq), or iv4 || seq (TLS 1.2 GCM) */
        if (explicit_iv) {
            memcpy(nonce, j->iv, 4);
            memcpy(nonce + 4, ctr, 8);
        } else {
            memcpy(nonce, j->iv, 12);
            for (int k = 0; k < 8; k++) nonce[4 + k] ^= ctr[k];
        }
        int ok;
        int outl = 0;
        if (j->dir) {
            /* encrypt: content at buf[off], TLS 1.3 inner plaintext = content || 23 || 0^pad */
            size_t off = explicit_iv ? 8 : 0, len = j->data_len;
            uint8_t *p = buf + off;
            if (j->tls13) {
                p[len++] = 23;
                size_t pad = (16 - len % 16) % 16;
                memset(p + len, 0, pad);
                len += pad;
            }
            size_t aadlen;
            if (j->tls13) {
                const size_t l = len + 16;
                aad[0] = 23; aad[1] = 3; aad[2] = 3; aad[3] = (uint8_t) (l >> 8); aad[4] = (uint8_t) l;
                aadlen = 5;
            } else {
                memcpy(aad, ctr, 8);
                aad[8] = 23; aad[9] = 3; aad[10] = 3; aad[11] = (uint8_t) (len >> 8); aad[12] = (uint8_t) len;
                aadlen = 13;
            }
            ok = EVP_CipherInit_ex(ctx, NULL, NULL, NULL, nonce, 1) == 1 &&
                 EVP_CipherUpdate(ctx, NULL, &outl, aad, (int) aadlen) == 1 &&
                 EVP_CipherUpdate(ctx, p, &outl, p, (int) len) == 1 &&
                 EVP_CipherFinal_ex(ctx, p + len, &outl) == 1 &&
                 EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, p + len) == 1;
            if (explicit_iv) memcpy(buf, ctr, 8);
            j->status[i] = ok ? 0 : -1;
        } else {
            /* decrypt: record body at buf[0] (explicit IV first for TLS 1.2 GCM) */
            size_t off = explicit_iv ? 8 : 0;
            if (j->data_len < off + 16) { j->status[i] = -0x7180; continue; }
            size_t len = j->data_len - off - 16;
            uint8_t *p = buf + off;
            if (explicit_iv) memcpy(nonce + 4, buf, 8);
            size_t aadlen;
            if (j->tls13) {
                const size_t l = len + 16;
                aad[0] = 23; aad[1] = 3; aad[2] = 3; aad[3] = (uint8_t) (l >> 8); aad[4] = (uint8_t) l;
                aadlen = 5;
            } else {
                memcpy(aad, ctr, 8);
                aad[8] = 23; aad[9] = 3; aad[10] = 3; aad[11] = (uint8_t) (len >> 8); aad[12] = (uint8_t) len;
                aadlen = 13;
            }
            ok = EVP_CipherInit_ex(ctx, NULL, NULL, NULL, nonce, 0) == 1 &&
                 EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, 16, p + len) == 1 &&
                 EVP_CipherUpdate(ctx, NULL, &outl, aad, (int) aadlen) == 1 &&
                 EVP_CipherUpdate(ctx, p, &outl, p, (int) len) == 1 &&
                 EVP_CipherFinal_ex(ctx, p + len, &outl) == 1;
            if (!ok) {
                memset(p, 0, len);                 /* PSA wipes the output on a bad tag */
                j->status[i] = -0x7180;            /* MBEDTLS_ERR_SSL_INVALID_MAC */
                continue;
            }
            if (j->tls13) {
                /* ssl_parse_inner_plaintext: strip zero padding, recover the type */
                size_t k = len;
                while (k > 0 && p[k - 1] == 0) k--;
                j->status[i] = k == 0 ? -0x7200 : 0;
            } else {
                j->status[i] = 0;
            }
        }
    }
    EVP_CIPHER_CTX_free(ctx);
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
        if (pthread_create(&tid[i], NULL, eb_worker, &jobs[i]) != 0) return -1.0;
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double) (b.tv_sec - a.tv_sec) + 1e-9 * (double) (b.tv_nsec - a.tv_nsec);
}
