/*
 * dtls_host.c -- a C host of the DTLS 1.2 datagram record layer
 * (tlsrec_dtls_encrypt / tlsrec_dtls_decrypt, include/tlsrec.h), compiled
 * with gcc against the header and the HIP runtime API only: what a DTLS
 * server built on Mbed TLS would run per poll of its sockets
 * (INTEGRATION.md section 2b').
 *
 *   sender:   per connection, application data -> one record per datagram
 *             (mbedtls_ssl_write_record, ssl_msg.c:2648-2793), epoch 1
 *   network:  datagram k of connection i, plus a replayed copy of datagram 0
 *             and a copy of datagram 1 renumbered to a fresh sequence number
 *             with a flipped tag byte (passes the replay check, fails the MAC)
 *   receiver: tlsrec_dtls_decrypt with the anti-replay window on
 *             (ssl_get_next_record's datagram branch, ssl_msg.c:4700-4873)
 *
 *   dtls_host [connections] [datagrams] [content] [cipher]
 *
 * Checks every accepted plaintext, the replay (UNEXPECTED_RECORD), the bad MAC
 * (INVALID_MAC, datagram dropped) and the window afterwards.  Prints one JSON
 * line; exit status 0 = pass.
 */
#define _POSIX_C_SOURCE 200809L
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tlsrec.h"

#define CK(x) do { if ((x) != hipSuccess) { printf("{\"pass\": false, \"hip\": \"%s\"}\n", #x); return 1; } } while (0)

static uint64_t splitmix(uint64_t *s)
{
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static uint8_t pt_byte(uint32_t conn, uint64_t j) { return (uint8_t) (conn * 131u + j * 7u + (j >> 8)); }

int main(int argc, char **argv)
{
    const uint32_t C = argc > 1 ? (uint32_t) atoi(argv[1]) : 64;
    const uint32_t D = argc > 2 ? (uint32_t) atoi(argv[2]) : 8;
    const uint32_t L = argc > 3 ? (uint32_t) atoi(argv[3]) : 1200;
    const int cipher = argc > 4 ? atoi(argv[4]) : TLSREC_CIPHER_AES_128_GCM;
    if (C == 0 || D < 2 || L == 0 || L > 16384) return 2;
    if (tlsrec_device_check() != 0) {
        printf("{\"pass\": false, \"error\": \"no gfx950 device\"}\n");
        return 1;
    }
    /* one TLS 1.2 key per connection; the sender's and the receiver's slot hold the same key */
    tlsrec_key_material *km = calloc(C, sizeof(*km));
    uint64_t s = 0x64746c73ull;
    for (uint32_t i = 0; i < C; i++) {
        km[i].cipher = (uint8_t) cipher;
        km[i].tls_minor = 3;
        km[i].fixed_ivlen = cipher == TLSREC_CIPHER_CHACHA20_POLY1305 ? 12 : 4;
        km[i].taglen = (cipher >= TLSREC_CIPHER_AES_128_CCM_8 && cipher <= TLSREC_CIPHER_AES_256_CCM_8) ? 8 : 16;
        for (int b = 0; b < 32; b++) km[i].key[b] = (uint8_t) splitmix(&s);
        for (int b = 0; b < 12; b++) km[i].iv[b] = (uint8_t) splitmix(&s);
    }
    tlsrec_keytab *kt = NULL;
    if (tlsrec_keytab_create(&kt, C) != 0 || tlsrec_keytab_load(kt, 0, C, km, 0, NULL) != 0) {
        printf("{\"pass\": false, \"error\": \"key table\"}\n");
        return 1;
    }
    /* ---- send ---- */
    const uint64_t in_len = (uint64_t) D * L;
    const uint64_t out_len = tlsrec_dtls_out_size(cipher, 0, 0, in_len, L);
    const uint32_t wire = (uint32_t) (out_len / D);
    uint8_t *h_in = malloc(C * in_len), *h_out = malloc(C * out_len);
    for (uint32_t i = 0; i < C; i++)
        for (uint64_t j = 0; j < in_len; j++) h_in[i * in_len + j] = pt_byte(i, j);
    tlsrec_stream_out *so = calloc(C, sizeof(*so));
    for (uint32_t i = 0; i < C; i++) {
        so[i].in_off = (uint64_t) i * in_len;
        so[i].in_len = (uint32_t) in_len;
        so[i].slot = i;
        so[i].out_off = (uint64_t) i * out_len;
        so[i].out_ctr[1] = 1;                      /* epoch 1, sequence 0 */
        so[i].max_frag = L;
        so[i].type = TLSREC_MSG_APPLICATION_DATA;
    }
    const uint32_t n = C * D;
    uint8_t *d_in, *d_out;
    tlsrec_stream_out *d_so;
    tlsrec_batch_rec *d_recs;
    tlsrec_batch_res *d_res;
    tlsrec_stream_out_res *d_sres;
    CK(hipMalloc((void **) &d_in, C * in_len));
    CK(hipMalloc((void **) &d_out, C * out_len + 4096));
    CK(hipMalloc((void **) &d_so, C * sizeof(*so)));
    CK(hipMalloc((void **) &d_recs, (n + 2 * C) * sizeof(tlsrec_batch_rec)));
    CK(hipMalloc((void **) &d_res, (n + 2 * C) * sizeof(tlsrec_batch_res)));
    CK(hipMalloc((void **) &d_sres, C * sizeof(tlsrec_stream_out_res)));
    CK(hipMemcpy(d_in, h_in, C * in_len, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_so, so, C * sizeof(*so), hipMemcpyHostToDevice));
    uint32_t nrec = 0;
    int r = tlsrec_dtls_encrypt(kt, d_so, C, d_in, d_out, d_recs, d_res, n, d_sres, &nrec, NULL);
    tlsrec_stream_out_res *sres = calloc(C, sizeof(*sres));
    CK(hipMemcpy(sres, d_sres, C * sizeof(*sres), hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_out, d_out, C * out_len, hipMemcpyDeviceToHost));
    int send_ok = r == 0 && nrec == n;
    for (uint32_t i = 0; i < C; i++) send_ok &= sres[i].status == 0 && sres[i].nrec == D && sres[i].out_len == out_len;
    /* ---- the network: per connection its D datagrams, then a replay of
     * datagram 0 and a copy of datagram 1 with its last (tag) byte flipped ---- */
    const uint32_t G = D + 2;
    uint8_t *h_rx = malloc((uint64_t) C * G * wire);
    tlsrec_dgram *dg = calloc((size_t) C * G, sizeof(*dg));
    tlsrec_dtls_in *ci = calloc(C, sizeof(*ci));
    for (uint32_t i = 0; i < C; i++) {
        for (uint32_t k = 0; k < G; k++) {
            const uint32_t src = k < D ? k : (k == D ? 0 : 1);
            const uint64_t off = ((uint64_t) i * G + k) * wire;
            memcpy(h_rx + off, h_out + (uint64_t) i * out_len + (uint64_t) src * wire, wire);
            if (k == D + 1) {                      /* a fresh sequence number D, so the replay check passes */
                for (int b = 0; b < 6; b++) h_rx[off + 5 + b] = (uint8_t) ((uint64_t) D >> (8 * (5 - b)));
                h_rx[off + wire - 1] ^= 0x5a;      /* and the AAD / tag no longer authenticate */
            }
            dg[i * G + k].off = off;
            dg[i * G + k].len = wire;
        }
        ci[i].first_dgram = i * G;
        ci[i].ndgram = G;
        ci[i].slot = i;
        ci[i].in_epoch = 1;
        ci[i].flags = TLSREC_DTLS_ANTI_REPLAY;
    }
    uint8_t *d_rx;
    tlsrec_dgram *d_dg;
    tlsrec_dtls_in *d_ci;
    tlsrec_dtls_in_res *d_cres;
    int32_t *d_disp;
    const uint32_t nmax = C * G;
    CK(hipMalloc((void **) &d_rx, (uint64_t) C * G * wire));
    CK(hipMalloc((void **) &d_dg, (size_t) C * G * sizeof(*dg)));
    CK(hipMalloc((void **) &d_ci, C * sizeof(*ci)));
    CK(hipMalloc((void **) &d_cres, C * sizeof(tlsrec_dtls_in_res)));
    CK(hipMalloc((void **) &d_disp, nmax * sizeof(int32_t)));
    CK(hipFree(d_recs));
    CK(hipFree(d_res));
    CK(hipMalloc((void **) &d_recs, nmax * sizeof(tlsrec_batch_rec)));
    CK(hipMalloc((void **) &d_res, nmax * sizeof(tlsrec_batch_res)));
    CK(hipMemcpy(d_rx, h_rx, (uint64_t) C * G * wire, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_dg, dg, (size_t) C * G * sizeof(*dg), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ci, ci, C * sizeof(*ci), hipMemcpyHostToDevice));
    uint32_t listed = 0;
    r = tlsrec_dtls_decrypt(kt, d_ci, C, d_dg, C * G, d_rx, d_recs, d_res, d_disp, nmax, d_cres, &listed, NULL);
    tlsrec_dtls_in_res *cres = calloc(C, sizeof(*cres));
    tlsrec_batch_rec *recs = calloc(nmax, sizeof(*recs));
    tlsrec_batch_res *res = calloc(nmax, sizeof(*res));
    int32_t *disp = calloc(nmax, sizeof(int32_t));
    CK(hipMemcpy(cres, d_cres, C * sizeof(*cres), hipMemcpyDeviceToHost));
    CK(hipMemcpy(recs, d_recs, nmax * sizeof(*recs), hipMemcpyDeviceToHost));
    CK(hipMemcpy(res, d_res, nmax * sizeof(*res), hipMemcpyDeviceToHost));
    CK(hipMemcpy(disp, d_disp, nmax * sizeof(int32_t), hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_rx, d_rx, (uint64_t) C * G * wire, hipMemcpyDeviceToHost));
    int recv_ok = r == 0 && listed == C * G;
    uint32_t accepted = 0, replays = 0, badmacs = 0, bytes_ok = 0;
    for (uint32_t i = 0; i < C && recv_ok; i++) {
        const tlsrec_dtls_in_res *c = &cres[i];
        recv_ok &= c->status == 0 && c->nrec == G && c->naccepted == D && c->dgrams_done == G &&
                   c->window_top == D - 1 && c->window == (D >= 64 ? ~0ull : ((1ull << D) - 1));
        for (uint32_t k = 0; k < G; k++) {
            const uint32_t x = c->first + k;
            if (k < D) {
                const int ok = disp[x] == 0 && res[x].data_len == L && res[x].type == TLSREC_MSG_APPLICATION_DATA;
                accepted += disp[x] == 0;
                if (ok) {
                    const uint8_t *p = h_rx + recs[x].buf_off + res[x].data_offset;
                    uint32_t j = 0;
                    while (j < L && p[j] == pt_byte(i, (uint64_t) k * L + j)) j++;
                    bytes_ok += j == L;
                }
                recv_ok &= ok;
            } else if (k == D) {
                replays += disp[x] == TLSREC_ERR_SSL_UNEXPECTED_RECORD;
            } else {
                badmacs += disp[x] == TLSREC_ERR_SSL_INVALID_MAC;
            }
        }
    }
    recv_ok &= accepted == C * D && bytes_ok == C * D && replays == C && badmacs == C;
    printf("{\"pass\": %s, \"connections\": %u, \"datagrams\": %u, \"content\": %u, \"cipher\": %d, \"wire\": %u, "
           "\"send_ok\": %s, \"accepted\": %u, \"plaintext_ok\": %u, \"replays_skipped\": %u, \"bad_mac_dropped\": %u}\n",
           send_ok && recv_ok ? "true" : "false", C, D, L, cipher, wire, send_ok ? "true" : "false", accepted, bytes_ok,
           replays, badmacs);
    tlsrec_keytab_free(kt);
    return send_ok && recv_ok ? 0 : 1;
}
