/*
 * abi_host.c -- a plain C host of libtlsrec.so, compiled with gcc against
 * include/tlsrec.h only (no HIP headers, no Python): the way an Mbed TLS
 * build would call the engine in place of mbedtls_ssl_encrypt_buf /
 * mbedtls_ssl_decrypt_buf.
 *
 *   abi_host layout                         tlsrec_record vs a mirror of
 *                                           mbedtls_record (ssl_misc.h:1163-1188),
 *                                           field by field (offsetof); no GPU
 *   abi_host kat <endpoint> <ctr> <server_key> <server_iv> <client_key> <client_iv> <pt> <ct>
 *                                           one TLS 1.3 record KAT of
 *                                           test_suite_ssl.data:2776-2834 at padding
 *                                           granularity 1 (ssl_tls13_record_protection,
 *                                           test_suite_ssl.function:2201-2299)
 *   abi_host latency <cipher> <tls> <content> <iters>
 *                                           p50 / p99 / mean microseconds of
 *                                           tlsrec_encrypt_buf and tlsrec_decrypt_buf
 *   abi_host threads <threads> <records>    one transform per thread, concurrent
 *                                           round trips, every payload checked
 *
 * Prints one JSON line; exit status 0 = pass.
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "tlsrec.h"

/* mbedtls_record with MBEDTLS_SSL_DTLS_CONNECTION_ID and CID_LEN_MAX 32
 * (the default configuration, mbedtls_config.h / ssl.h:423-429) */
typedef struct {
    uint8_t ctr[8];
    uint8_t type;
    uint8_t ver[2];
    unsigned char *buf;
    size_t buf_len;
    size_t data_offset;
    size_t data_len;
    uint8_t cid_len;
    unsigned char cid[32];
} mirror_mbedtls_record;

static int layout(void)
{
    struct { const char *f; size_t a, b; } rows[] = {
        { "ctr", offsetof(tlsrec_record, ctr), offsetof(mirror_mbedtls_record, ctr) },
        { "type", offsetof(tlsrec_record, type), offsetof(mirror_mbedtls_record, type) },
        { "ver", offsetof(tlsrec_record, ver), offsetof(mirror_mbedtls_record, ver) },
        { "buf", offsetof(tlsrec_record, buf), offsetof(mirror_mbedtls_record, buf) },
        { "buf_len", offsetof(tlsrec_record, buf_len), offsetof(mirror_mbedtls_record, buf_len) },
        { "data_offset", offsetof(tlsrec_record, data_offset), offsetof(mirror_mbedtls_record, data_offset) },
        { "data_len", offsetof(tlsrec_record, data_len), offsetof(mirror_mbedtls_record, data_len) },
        { "cid_len", offsetof(tlsrec_record, cid_len), offsetof(mirror_mbedtls_record, cid_len) },
        { "cid", offsetof(tlsrec_record, cid), offsetof(mirror_mbedtls_record, cid) },
        { "sizeof", sizeof(tlsrec_record), sizeof(mirror_mbedtls_record) },
    };
    int ok = 1;
    printf("{\"layout\": {");
    for (size_t i = 0; i < sizeof(rows) / sizeof(rows[0]); i++) {
        printf("%s\"%s\": [%zu, %zu]", i ? ", " : "", rows[i].f, rows[i].a, rows[i].b);
        ok &= rows[i].a == rows[i].b;
    }
    /* the batch layouts the kernels assume */
    ok &= sizeof(tlsrec_batch_rec) == 40 && sizeof(tlsrec_batch_res) == 16 && sizeof(tlsrec_key_material) == 64;
    printf("}, \"batch_rec\": %zu, \"batch_res\": %zu, \"key_material\": %zu, \"ok\": %s}\n",
           sizeof(tlsrec_batch_rec), sizeof(tlsrec_batch_res), sizeof(tlsrec_key_material), ok ? "true" : "false");
    return ok ? 0 : 1;
}

static size_t unhex(const char *s, unsigned char *out, size_t cap)
{
    size_t n = strlen(s) / 2;
    if (n > cap) return (size_t) -1;
    for (size_t i = 0; i < n; i++) {
        unsigned v;
        if (sscanf(s + 2 * i, "%2x", &v) != 1) return (size_t) -1;
        out[i] = (unsigned char) v;
    }
    return n;
}

static int kat(char **a)
{
    unsigned char sk[32], si[16], ck[32], ci[16], pt[512], ct[512];
    const int client = strcmp(a[0], "client") == 0;
    const int ctr = atoi(a[1]);
    size_t skl = unhex(a[2], sk, 32), sil = unhex(a[3], si, 16), ckl = unhex(a[4], ck, 32), cil = unhex(a[5], ci, 16);
    size_t ptl = unhex(a[6], pt, sizeof(pt)), ctl = unhex(a[7], ct, sizeof(ct));
    if (skl != 16 || ckl != 16 || sil != 12 || cil != 12 || ptl == (size_t) -1 || ctl == (size_t) -1) return 2;
    tlsrec_transform send, recv;
    /* the sender's write key/iv encrypt; the receiver uses the same (its read side) */
    const unsigned char *wk = client ? ck : sk, *wi = client ? ci : si, *rk = client ? sk : ck, *ri = client ? si : ci;
    int r = tlsrec_transform_setup_ex(&send, TLSREC_VERSION_TLS1_3, TLSREC_CIPHER_AES_128_GCM, wk, rk, wi, ri, 1);
    if (r == 0) r = tlsrec_transform_setup_ex(&recv, TLSREC_VERSION_TLS1_3, TLSREC_CIPHER_AES_128_GCM, rk, wk, ri, wi, 1);
    if (r != 0) {
        printf("{\"kat\": \"setup\", \"ret\": %d}\n", r);
        return 1;
    }
    unsigned char buf[600];
    memset(buf, 0, sizeof(buf));
    memcpy(buf, pt, ptl);
    tlsrec_record rec;
    memset(&rec, 0, sizeof(rec));
    rec.ctr[7] = (uint8_t) ctr;
    rec.type = TLSREC_MSG_APPLICATION_DATA;
    rec.ver[0] = 3;
    rec.ver[1] = 3;
    rec.buf = buf;
    rec.buf_len = ctl + 16;
    rec.data_offset = 0;
    rec.data_len = ptl;
    int re = tlsrec_encrypt_buf(NULL, &send, &rec);
    int enc_ok = re == 0 && rec.data_len == ctl && memcmp(buf + rec.data_offset, ct, ctl) == 0 && rec.type == 23;
    int rd = tlsrec_decrypt_buf(NULL, &recv, &rec);
    int dec_ok = rd == 0 && rec.data_len == ptl && memcmp(buf + rec.data_offset, pt, ptl) == 0 && rec.type == 23;
    printf("{\"kat\": \"%s ctr %d\", \"encrypt_ret\": %d, \"ciphertext_equal\": %s, \"decrypt_ret\": %d, "
           "\"plaintext_equal\": %s}\n", a[0], ctr, re, enc_ok ? "true" : "false", rd, dec_ok ? "true" : "false");
    tlsrec_transform_free(&send);
    tlsrec_transform_free(&recv);
    return enc_ok && dec_ok ? 0 : 1;
}

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return 1e6 * (double) t.tv_sec + 1e-3 * (double) t.tv_nsec;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *) a, y = *(const double *) b;
    return (x > y) - (x < y);
}

/* libtlsrec internal: how many coalesced batches carried how many records,
 * and the record server's requests (served, sent back to the launch path) and
 * grid launches */
void tlsrec__engine_stats(uint64_t *batches, uint64_t *records);
void tlsrec__server_stats(uint64_t *served, uint64_t *fallback, uint64_t *launches);
void tlsrec__server_why(uint64_t out[4]);
uint64_t tlsrec__server_closing(void);

static void print_server_stats(void)
{
    uint64_t s = 0, f = 0, l = 0;
    uint64_t why[4] = { 0, 0, 0, 0 };
    tlsrec__server_stats(&s, &f, &l);
    tlsrec__server_why(why);
    /* why: launch-path fallbacks by reason (batch work pending, other set not
     * drained, withdrawn, no free slot); closing: claims that found a grid
     * leaving idle */
    printf(", \"server_served\": %llu, \"server_fallback\": %llu, \"server_launches\": %llu, "
           "\"server_why\": {\"batch\": %llu, \"drain\": %llu, \"withdrawn\": %llu, \"noslot\": %llu}, "
           "\"server_closing\": %llu}\n",
           (unsigned long long) s, (unsigned long long) f, (unsigned long long) l, (unsigned long long) why[0],
           (unsigned long long) why[1], (unsigned long long) why[2], (unsigned long long) why[3],
           (unsigned long long) tlsrec__server_closing());
}

static int latency(char **a)
{
    const int cipher = atoi(a[0]);
    const int tls = strcmp(a[1], "1.2") == 0 ? TLSREC_VERSION_TLS1_2 : TLSREC_VERSION_TLS1_3;
    const size_t content = (size_t) atol(a[2]);
    const int iters = atoi(a[3]);
    unsigned char key[32], iv[16];
    for (int i = 0; i < 32; i++) key[i] = (unsigned char) (i * 7 + 1);
    for (int i = 0; i < 16; i++) iv[i] = (unsigned char) (i * 13 + 5);
    tlsrec_transform t;
    int r = tlsrec_transform_setup(&t, tls, cipher, key, key, iv, iv);
    if (r) {
        printf("{\"latency\": \"setup\", \"ret\": %d}\n", r);
        return 1;
    }
    const size_t head = tls == TLSREC_VERSION_TLS1_2 && cipher != TLSREC_CIPHER_CHACHA20_POLY1305 ? 8 : 0;
    const size_t buf_len = head + content + 64;
    unsigned char *buf = malloc(buf_len), *plain = malloc(content + 1);
    for (size_t i = 0; i < content; i++) plain[i] = (unsigned char) (i * 31 + 3);
    double *te = malloc(sizeof(double) * iters), *td = malloc(sizeof(double) * iters);
    int bad = 0;
    for (int it = -20; it < iters; it++) {          /* 20 warm-up round trips */
        memset(buf, 0, buf_len);
        memcpy(buf + head, plain, content);
        tlsrec_record rec;
        memset(&rec, 0, sizeof(rec));
        uint64_t seq = (uint64_t) (it + 20);
        for (int k = 7; k >= 0; k--) { rec.ctr[k] = (uint8_t) seq; seq >>= 8; }
        rec.type = 23;
        rec.ver[0] = rec.ver[1] = 3;
        rec.buf = buf;
        rec.buf_len = buf_len;
        rec.data_offset = head;
        rec.data_len = content;
        double t0 = now_us();
        int re = tlsrec_encrypt_buf(NULL, &t, &rec);
        double t1 = now_us();
        int rd = tlsrec_decrypt_buf(NULL, &t, &rec);
        double t2 = now_us();
        bad += re != 0 || rd != 0 || rec.data_len != content || memcmp(buf + rec.data_offset, plain, content) != 0;
        if (it >= 0) {
            te[it] = t1 - t0;
            td[it] = t2 - t1;
        }
    }
    double me = 0, md = 0;
    for (int i = 0; i < iters; i++) { me += te[i]; md += td[i]; }
    qsort(te, iters, sizeof(double), cmp_d);
    qsort(td, iters, sizeof(double), cmp_d);
    const int i50 = iters / 2, i99 = (int) ((iters - 1) * 0.99);
    printf("{\"latency_us\": {\"cipher\": %d, \"tls\": \"%s\", \"content\": %zu, \"iters\": %d, "
           "\"encrypt_p50\": %.1f, \"encrypt_p99\": %.1f, \"encrypt_mean\": %.1f, "
           "\"decrypt_p50\": %.1f, \"decrypt_p99\": %.1f, \"decrypt_mean\": %.1f}, \"bad\": %d",
           cipher, a[1], content, iters, te[i50], te[i99], me / iters, td[i50], td[i99], md / iters, bad);
    print_server_stats();
    tlsrec_transform_free(&t);
    free(buf);
    free(plain);
    free(te);
    free(td);
    return bad ? 1 : 0;
}

typedef struct { int id, records, bad, mix; double us; pthread_barrier_t *go; } thr_job;

static void *thr_main(void *arg)
{
    thr_job *j = (thr_job *) arg;
    /* mix: AES-256-GCM, ChaCha20-Poly1305 and AES-128-CCM threads (CCM runs on
     * the launch path); otherwise the north star's two AEADs */
    const int ciphers[3] = { TLSREC_CIPHER_AES_256_GCM, TLSREC_CIPHER_CHACHA20_POLY1305, TLSREC_CIPHER_AES_128_CCM };
    const int cipher = ciphers[j->id % (j->mix ? 3 : 2)];
    unsigned char key[32], iv[16];
    for (int i = 0; i < 32; i++) key[i] = (unsigned char) (i + j->id * 17);
    for (int i = 0; i < 16; i++) iv[i] = (unsigned char) (i * 3 + j->id);
    tlsrec_transform t;
    if (tlsrec_transform_setup(&t, TLSREC_VERSION_TLS1_3, cipher, key, key, iv, iv) != 0) {
        j->bad = j->records;
        pthread_barrier_wait(j->go);
        return NULL;
    }
    unsigned char buf[2048], plain[1400];
    pthread_barrier_wait(j->go);          /* every transform set up: time the records only */
    const double t0 = now_us();
    for (int n = 0; n < j->records; n++) {
        const size_t len = (size_t) (1 + (n * 97 + j->id * 13) % 1400);
        for (size_t i = 0; i < len; i++) plain[i] = (unsigned char) (i ^ n ^ j->id);
        memset(buf, 0, sizeof(buf));
        memcpy(buf, plain, len);
        tlsrec_record rec;
        memset(&rec, 0, sizeof(rec));
        rec.ctr[7] = (uint8_t) n;
        rec.ctr[6] = (uint8_t) (n >> 8);
        rec.type = 23;
        rec.ver[0] = rec.ver[1] = 3;
        rec.buf = buf;
        rec.buf_len = sizeof(buf);
        rec.data_offset = 0;
        rec.data_len = len;
        if (tlsrec_encrypt_buf(NULL, &t, &rec) != 0 || tlsrec_decrypt_buf(NULL, &t, &rec) != 0 ||
            rec.data_len != len || memcmp(buf + rec.data_offset, plain, len) != 0)
            j->bad++;
    }
    j->us = now_us() - t0;
    tlsrec_transform_free(&t);
    return NULL;
}

static int threads(char **a, int mix)
{
    const int nt = atoi(a[0]), records = atoi(a[1]);
    pthread_t tid[64];
    thr_job jobs[64];
    if (nt < 1 || nt > 64) return 2;
    pthread_barrier_t go;
    pthread_barrier_init(&go, NULL, (unsigned) nt);
    for (int i = 0; i < nt; i++) {
        jobs[i] = (thr_job) { i, records, 0, mix, 0, &go };
        pthread_create(&tid[i], NULL, thr_main, &jobs[i]);
    }
    int bad = 0;
    double us = 0;                        /* the slowest thread's record loop */
    for (int i = 0; i < nt; i++) {
        pthread_join(tid[i], NULL);
        bad += jobs[i].bad;
        if (jobs[i].us > us) us = jobs[i].us;
    }
    pthread_barrier_destroy(&go);
    uint64_t nb = 0, nr = 0;
    tlsrec__engine_stats(&nb, &nr);
    printf("{\"threads\": %d, \"ciphers\": \"%s\", \"records_per_thread\": %d, \"round_trips_per_s\": %.0f, "
           "\"bad\": %d, \"engine_batches\": %llu, \"engine_records\": %llu, \"records_per_batch\": %.2f",
           nt, mix ? "gcm+chacha+ccm" : "gcm+chacha", records, 1e6 * nt * records / us, bad, (unsigned long long) nb,
           (unsigned long long) nr, nb ? (double) nr / nb : 0.0);
    print_server_stats();
    return bad ? 1 : 0;
}

int main(int argc, char **argv)
{
    if (argc >= 2 && strcmp(argv[1], "layout") == 0) return layout();
    if (tlsrec_device_check() != 0) {
        printf("{\"error\": \"no gfx950 device\"}\n");
        return 3;
    }
    if (argc == 10 && strcmp(argv[1], "kat") == 0) return kat(argv + 2);
    if (argc == 6 && strcmp(argv[1], "latency") == 0) return latency(argv + 2);
    if (argc == 4 && strcmp(argv[1], "threads") == 0) return threads(argv + 2, 1);
    if (argc == 5 && strcmp(argv[1], "threads") == 0) return threads(argv + 2, strcmp(argv[4], "mix") == 0);
    fprintf(stderr, "usage: abi_host layout | kat ... | latency <cipher> <1.2|1.3> <content> <iters> | "
                    "threads <n> <records> [mix|gcm_chacha]\n");
    return 2;
}
