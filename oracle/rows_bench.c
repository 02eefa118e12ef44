/*
 * rows_bench.c -- CPU baselines of the SURVEY §8(f) rows, "port" leg: the
 * oracle's restatements of the stream record layer (stream.c), the DTLS 1.2
 * datagram layer (dtls.c) and the TLS 1.3 key schedule (keysched.c), timed
 * over many connections on the host's cores.
 *
 * TEST INFRASTRUCTURE ONLY: tools/bench_{stream,dtls,keysched}.py call it
 * for the `cpu_baseline` of their lines, beside the GPU rows they measure.
 * Nothing in the product links or loads it.
 *
 * Work split: connection c is served by thread c % threads, as one CPU thread
 * would serve a socket's records in order (ssl_get_next_record,
 * ssl_msg.c:4700-4907; mbedtls_ssl_write_record, :2648-2793).
 */
#define _POSIX_C_SOURCE 200809L
#include "oracle.h"

#include <pthread.h>
#include <string.h>
#include <time.h>

typedef struct {
    const orc_transform *const *ts;
    uint32_t nconn;
    int dtls, dir, id, threads;
    uint8_t *in;
    size_t in_stride, in_len;
    uint8_t *out;
    size_t out_stride, max_frag;
    int32_t *status;
} rows_job;

static void *rows_worker(void *arg)
{
    rows_job *j = (rows_job *) arg;
    for (uint32_t c = (uint32_t) j->id; c < j->nconn; c += (uint32_t) j->threads) {
        const orc_transform *t = j->ts[c];
        uint8_t *in = j->in + (size_t) c * j->in_stride;
        int r;
        if (j->dir) {
            /* send: the connection's application data -> records of max_frag */
            uint8_t *out = j->out + (size_t) c * j->out_stride;
            size_t out_len = 0;
            uint32_t nrec = 0;
            uint8_t ctr[8] = { 0 };
            if (j->dtls) {
                ctr[1] = 1;                                        /* epoch 1, sequence 0 */
                r = orc_dtls_encrypt(t, in, j->in_len, 23, ctr, j->max_frag, out, j->out_stride, &out_len, &nrec);
            } else {
                r = orc_stream_encrypt(t, in, j->in_len, 23, ctr, j->max_frag, 16384 + 2048, out, j->out_stride,
                                       &out_len, &nrec);
            }
        } else if (j->dtls) {
            /* receive: the connection's datagrams (one record each, wire bytes
             * back to back in `in`), anti-replay on, epoch 1 */
            orc_dtls_state st;
            memset(&st, 0, sizeof(st));
            st.in_epoch = 1;
            st.anti_replay = 1;
            uint64_t doff[64];
            uint32_t dlen[64];
            orc_dtls_rec recs[64];
            orc_dtls_res res;
            const size_t nd = j->max_frag ? j->in_len / j->max_frag : 0;   /* max_frag = datagram wire size here */
            r = nd > 64 ? ORC_ERR_SSL_BAD_INPUT_DATA : 0;
            if (!r) {
                for (size_t d = 0; d < nd; d++) {
                    doff[d] = d * j->max_frag;
                    dlen[d] = (uint32_t) j->max_frag;
                }
                r = orc_dtls_decrypt(t, &st, in, doff, dlen, nd, recs, 64, &res);
                if (!r && res.naccepted != nd) r = ORC_ERR_SSL_INVALID_RECORD;
            }
        } else {
            /* receive: the connection's record stream, decrypted in place */
            orc_stream_rec recs[64];
            orc_stream_res res;
            const uint8_t ctr[8] = { 0 };
            r = orc_stream_decrypt(t, in, j->in_len, ctr, 0, 5 + 16384 + 256, ORC_VERSION_TLS1_3, recs, 64, &res);
            if (!r && res.consumed != j->in_len) r = ORC_ERR_SSL_INVALID_RECORD;
        }
        j->status[c] = r;
    }
    return NULL;
}

static double elapsed(const struct timespec *a, const struct timespec *b)
{
    return (double) (b->tv_sec - a->tv_sec) + 1e-9 * (double) (b->tv_nsec - a->tv_nsec);
}

/* dir 1 = send (in: in_len bytes of application data per connection, out:
 * the records), 0 = receive (in: in_len wire bytes per connection, decrypted
 * in place; DTLS: max_frag = the wire size of one datagram).  Seconds. */
double orc_bench_stream_rows(const orc_transform *const *ts, uint32_t nconn, int dtls, int dir, uint8_t *in,
                             size_t in_stride, size_t in_len, uint8_t *out, size_t out_stride, size_t max_frag,
                             int threads, int32_t *status)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    rows_job jobs[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < threads; i++) {
        jobs[i] = (rows_job) { ts, nconn, dtls, dir, i, threads, in, in_stride, in_len, out, out_stride, max_frag,
                               status };
        if (pthread_create(&tid[i], NULL, rows_worker, &jobs[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);
            return -1.0;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return elapsed(&a, &b);
}

/* ---- the TLS 1.3 key schedule: KeyUpdate + traffic keys per connection --- */
typedef struct {
    int alg, update, id, threads;
    const uint8_t *secrets;
    uint32_t count;
    size_t keylen;
    uint8_t *out;             /* keylen + 12 bytes per connection */
    int32_t *status;
} ks_job;

static void *ks_worker(void *arg)
{
    ks_job *j = (ks_job *) arg;
    const size_t H = orc_hash_len(j->alg);
    for (uint32_t c = (uint32_t) j->id; c < j->count; c += (uint32_t) j->threads) {
        const uint8_t *s = j->secrets + (size_t) c * 48;
        uint8_t next[64];
        int r = 0;
        if (j->update) {
            r = orc_tls13_update_traffic_secret(j->alg, s, next);   /* RFC 8446 7.2 */
            s = next;
        }
        uint8_t *o = j->out + (size_t) c * (j->keylen + 12);
        if (!r)
            r = orc_tls13_hkdf_expand_label(j->alg, s, H, (const uint8_t *) "key", 3, NULL, 0, o, j->keylen);
        if (!r) r = orc_tls13_hkdf_expand_label(j->alg, s, H, (const uint8_t *) "iv", 2, NULL, 0, o + j->keylen, 12);
        j->status[c] = r;
    }
    return NULL;
}

/* secrets: 48 bytes per connection (the hash length used).  Seconds. */
double orc_bench_keysched(int alg, const uint8_t *secrets, uint32_t count, int update, size_t keylen, int threads,
                          uint8_t *out, int32_t *status)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    ks_job jobs[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int i = 0; i < threads; i++) {
        jobs[i] = (ks_job) { alg, update, i, threads, secrets, count, keylen, out, status };
        if (pthread_create(&tid[i], NULL, ks_worker, &jobs[i]) != 0) {
            for (int k = 0; k < i; k++) pthread_join(tid[k], NULL);
            return -1.0;
        }
    }
    for (int i = 0; i < threads; i++) pthread_join(tid[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return elapsed(&a, &b);
}
