/*
 * oracle.h -- CPU restatement of the Mbed TLS 4.1.0 record-protection path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in mbedtls_amd/ links, loads or calls
 * this code; only tests/, __graft_entry__.smoke() (as the checker) and the
 * cpu_baseline leg of bench.py use it.
 *
 * What it restates (reference = /root/reference, Mbed TLS 4.1.0):
 *   - record framing of library/ssl_msg.c:
 *       ssl_compute_padding_length        ssl_msg.c:431-435
 *       ssl_build_inner_plaintext         ssl_msg.c:466-491
 *       ssl_parse_inner_plaintext         ssl_msg.c:496-514
 *       ssl_extract_add_data_from_record  ssl_msg.c:568-735 (incl. the RFC 9146
 *                                         DTLS 1.2 CID branch, :667-733)
 *       ssl_transform_aead_dynamic_iv_is_explicit ssl_msg.c:739-743
 *       ssl_build_record_nonce            ssl_msg.c:768-781
 *       mbedtls_ssl_encrypt_buf (AEAD)    ssl_msg.c:784-1078
 *       mbedtls_ssl_decrypt_buf (AEAD)    ssl_msg.c:1270-1433, 1803-1818
 *   - transform population (ivlen / fixed_ivlen / taglen / minlen):
 *       TLS 1.3: library/ssl_tls13_keys.c:974-998
 *       TLS 1.2: library/ssl_tls.c:7768-7797
 *   - PSA error mapping: library/ssl_tls.c:2157-2166
 *
 * The AEAD arithmetic itself lives in the TF-PSA-Crypto submodule, which is
 * NOT vendored in /root/reference (.gitmodules:4-6; the directory is empty).
 * It is restated here from the published standards it implements:
 *   - AES: FIPS-197 (S-box derived from the GF(2^8) inverse + affine map)
 *   - GCM: NIST SP 800-38D (GHASH with 4-bit Shoup tables, the Mbed TLS
 *     builtin design class, ChangeLog:439-441)
 *   - ChaCha20 / Poly1305 / AEAD: RFC 8439 sections 2.3, 2.5, 2.8
 *
 * Pinning: see oracle/README.md.  The AES-128-GCM TLS 1.3 record path is
 * pinned by the reference's own 4 KATs (tests/suites/test_suite_ssl.data:
 * 2776-2834).  AES-256-GCM and ChaCha20-Poly1305 have no record KAT in the
 * reference; they are pinned by standards vectors (SP 800-38D test cases,
 * RFC 8439 2.8.2) and a differential check against OpenSSL libcrypto.
 */
#ifndef TLSREC_ORACLE_H
#define TLSREC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes: the values of include/mbedtls/ssl.h:40-125 and the PSA codes
 * they alias (MBEDTLS_ERR_SSL_BAD_INPUT_DATA = PSA_ERROR_INVALID_ARGUMENT
 * = -135, MBEDTLS_ERR_SSL_BUFFER_TOO_SMALL = PSA_ERROR_BUFFER_TOO_SMALL = -138). */
#define ORC_ERR_SSL_BAD_INPUT_DATA     (-135)
#define ORC_ERR_SSL_BUFFER_TOO_SMALL   (-138)
#define ORC_ERR_SSL_INVALID_MAC        (-0x7180)
#define ORC_ERR_SSL_INVALID_RECORD     (-0x7200)
#define ORC_ERR_SSL_INTERNAL_ERROR     (-0x6C00)
#define ORC_ERR_SSL_FEATURE_UNAVAILABLE (-0x7080)
#define ORC_ERR_SSL_UNEXPECTED_CID     (-0x6000)   /* ssl.h:156 */
#define ORC_SSL_MSG_CID                25          /* MBEDTLS_SSL_MSG_CID, ssl.h:528 */
#define ORC_CID_LEN_MAX                32          /* MBEDTLS_SSL_CID_{IN,OUT}_LEN_MAX, ssl.h:423-429 */

#define ORC_VERSION_TLS1_2 0x0303
#define ORC_VERSION_TLS1_3 0x0304

#define ORC_CIPHER_AES_128_GCM        1
#define ORC_CIPHER_AES_256_GCM        2
#define ORC_CIPHER_CHACHA20_POLY1305  3
/* the remaining AES AEADs of mbedtls_ssl_cipher_to_psa
 * (ssl_tls.c:2168-2363); *_CCM_8 = the MBEDTLS_CIPHERSUITE_SHORT_TAG suites
 * (taglen 8, ssl_tls.c:7707-7708, ssl_tls13_keys.c:981-985) */
#define ORC_CIPHER_AES_192_GCM        4
#define ORC_CIPHER_AES_128_CCM        5
#define ORC_CIPHER_AES_192_CCM        6
#define ORC_CIPHER_AES_256_CCM        7
#define ORC_CIPHER_AES_128_CCM_8      8
#define ORC_CIPHER_AES_192_CCM_8      9
#define ORC_CIPHER_AES_256_CCM_8      10
/* ARIA-GCM (PSA_KEY_TYPE_ARIA, ssl_tls.c:2248-2289; RFC 6209 suites) */
#define ORC_CIPHER_ARIA_128_GCM       11
#define ORC_CIPHER_ARIA_192_GCM       12
#define ORC_CIPHER_ARIA_256_GCM       13
/* ARIA-CCM (PSA_ALG_CCM with PSA_KEY_TYPE_ARIA, ssl_tls.c:2241-2282), 16-byte tag */
#define ORC_CIPHER_ARIA_128_CCM       14
#define ORC_CIPHER_ARIA_192_CCM       15
#define ORC_CIPHER_ARIA_256_CCM       16
/* Camellia-GCM / -CCM (PSA_KEY_TYPE_CAMELLIA, ssl_tls.c:2297-2345; RFC 6367 suites) */
#define ORC_CIPHER_CAMELLIA_128_GCM   17
#define ORC_CIPHER_CAMELLIA_192_GCM   18
#define ORC_CIPHER_CAMELLIA_256_GCM   19
#define ORC_CIPHER_CAMELLIA_128_CCM   20
#define ORC_CIPHER_CAMELLIA_192_CCM   21
#define ORC_CIPHER_CAMELLIA_256_CCM   22

#define ORC_OUT_CONTENT_LEN 16384     /* MBEDTLS_SSL_OUT_CONTENT_LEN, ssl.h:409 */

/* ---- primitives ------------------------------------------------------- */
/* Block-cipher context of the GCM / CCM code: AES (kind 0), ARIA (kind 1,
 * oracle/aria.c; nr = 12/14/16 rounds, ark = the nr + 1 round keys) or
 * Camellia (kind 2, oracle/camellia.c; nr = 18/24, ark = the 64-bit subkeys). */
typedef struct {
    uint32_t rk[60];
    int nr;
    int kind;
    uint8_t ark[17][16];
} orc_aes_ctx;

int  orc_aes_setkey_enc(orc_aes_ctx *ctx, const uint8_t *key, unsigned keybits);
void orc_aes_encrypt_block(const orc_aes_ctx *ctx, const uint8_t in[16], uint8_t out[16]);
/* ARIA (RFC 5794) in the same context type; orc_aes_encrypt_block dispatches */
int  orc_aria_setkey_enc(orc_aes_ctx *ctx, const uint8_t *key, unsigned keybits);
void orc_aria_encrypt_block(const orc_aes_ctx *ctx, const uint8_t in[16], uint8_t out[16]);
const uint8_t *orc_aria_sbox(int i);   /* SB1..SB4 as i = 0..3 */
/* Camellia (RFC 3713) in the same context type */
int  orc_camellia_setkey_enc(orc_aes_ctx *ctx, const uint8_t *key, unsigned keybits);
void orc_camellia_encrypt_block(const orc_aes_ctx *ctx, const uint8_t in[16], uint8_t out[16]);
const uint8_t *orc_camellia_sbox1(void);
const uint8_t *orc_aes_sbox(void);

typedef struct {
    orc_aes_ctx aes;
    uint64_t hl[16], hh[16];   /* Shoup 4-bit table of n*H */
    uint8_t h[16];
} orc_gcm_ctx;

int  orc_gcm_setkey(orc_gcm_ctx *ctx, const uint8_t *key, unsigned keybits);
/* GCM over AES (bc 0), ARIA (bc 1) or Camellia (bc 2) */
int  orc_gcm_setkey_ex(orc_gcm_ctx *ctx, const uint8_t *key, unsigned keybits, int bc);
void orc_ghash_mult(const orc_gcm_ctx *ctx, const uint8_t x[16], uint8_t out[16]);
/* one-shot GCM with a 12-byte IV; tag_len <= 16 */
void orc_gcm_encrypt(const orc_gcm_ctx *ctx, const uint8_t iv[12],
                     const uint8_t *aad, size_t aad_len,
                     const uint8_t *in, size_t len, uint8_t *out,
                     uint8_t *tag, size_t tag_len);
/* returns 0 or ORC_ERR_SSL_INVALID_MAC */
int  orc_gcm_decrypt(const orc_gcm_ctx *ctx, const uint8_t iv[12],
                     const uint8_t *aad, size_t aad_len,
                     const uint8_t *in, size_t len, uint8_t *out,
                     const uint8_t *tag, size_t tag_len);
/* GHASH over (aad, ct) with the length block, raw (no E(J0) mask) */
void orc_ghash(const orc_gcm_ctx *ctx, const uint8_t *aad, size_t aad_len,
               const uint8_t *ct, size_t ct_len, uint8_t out[16]);
void orc_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]);

/* CCM (NIST SP 800-38C) with a 12-byte nonce (q = 3), tag_len 4..16 */
void orc_ccm_encrypt(const orc_aes_ctx *aes, const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                     const uint8_t *in, size_t len, uint8_t *out, uint8_t *tag, size_t tag_len);
int  orc_ccm_decrypt(const orc_aes_ctx *aes, const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                     const uint8_t *in, size_t len, uint8_t *out, const uint8_t *tag, size_t tag_len);

void orc_chacha20_block(const uint8_t key[32], uint32_t counter,
                        const uint8_t nonce[12], uint8_t out[64]);
void orc_chacha20_xor(const uint8_t key[32], uint32_t counter,
                      const uint8_t nonce[12], const uint8_t *in,
                      uint8_t *out, size_t len);
void orc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len,
                  uint8_t tag[16]);
void orc_chachapoly_encrypt(const uint8_t key[32], const uint8_t nonce[12],
                            const uint8_t *aad, size_t aad_len,
                            const uint8_t *in, size_t len, uint8_t *out,
                            uint8_t tag[16]);
int  orc_chachapoly_decrypt(const uint8_t key[32], const uint8_t nonce[12],
                            const uint8_t *aad, size_t aad_len,
                            const uint8_t *in, size_t len, uint8_t *out,
                            const uint8_t tag[16]);

/* ---- record layer ------------------------------------------------------ */

/* Mirror of the AEAD-relevant fields of struct mbedtls_ssl_transform
 * (library/ssl_misc.h:1073-1120) with raw keys in place of PSA key ids. */
typedef struct {
    size_t minlen, ivlen, fixed_ivlen, maclen, taglen;
    uint8_t iv_enc[16], iv_dec[16];
    int tls_version;
    int cipher;
    size_t keylen;
    uint8_t key_enc[32], key_dec[32];
    orc_gcm_ctx gcm_enc, gcm_dec;   /* expanded GCM state (its AES context serves CCM) */
    size_t granularity;             /* MBEDTLS_SSL_CID_TLS1_3_PADDING_GRANULARITY */
    /* DTLS 1.2 connection IDs (ssl_misc.h transform in_cid / out_cid) */
    uint8_t in_cid_len, out_cid_len;
    uint8_t in_cid[ORC_CID_LEN_MAX], out_cid[ORC_CID_LEN_MAX];
} orc_transform;

/* Mirror of mbedtls_record (library/ssl_misc.h:1163-1188). */
typedef struct {
    uint8_t ctr[8];
    uint8_t type;
    uint8_t ver[2];
    uint8_t *buf;
    size_t buf_len;
    size_t data_offset;
    size_t data_len;
    uint8_t cid_len;
    uint8_t cid[ORC_CID_LEN_MAX];
} orc_record;

/* Populate a transform as ssl_tls13_keys.c:922-1042 / ssl_tls.c:7639-7979
 * (AEAD branch) would.  granularity = 16 for the default config. */
int orc_transform_setup(orc_transform *t, int tls_version, int cipher,
                        const uint8_t *key_enc, const uint8_t *key_dec,
                        const uint8_t *iv_enc, const uint8_t *iv_dec,
                        size_t granularity);

/* Set the transform's DTLS 1.2 connection IDs (what ssl_tls12_populate_transform
 * copies from ssl->own_cid / handshake->peer_cid, ssl_tls.c). */
int orc_transform_set_cid(orc_transform *t, const uint8_t *in_cid, size_t in_len,
                          const uint8_t *out_cid, size_t out_len);

int orc_encrypt_buf(const orc_transform *t, orc_record *rec);
int orc_decrypt_buf(const orc_transform *t, orc_record *rec);

/* ---- CPU baseline batch driver (bench.py cpu_baseline leg) ------------- */
/* Decrypt (dir=0) or encrypt (dir=1) `n` TLS records laid out at a fixed
 * stride, all under one transform, with record i using seq = seq0 + i, on
 * `threads` pthreads.  Returns elapsed seconds (CLOCK_MONOTONIC) or < 0. */
double orc_bench_records(const orc_transform *t, int dir, uint8_t *arena,
                         size_t stride, size_t data_len, uint64_t n,
                         uint64_t seq0, int threads, int32_t *status);
/* record i under ts[i % nconn] with sequence number i / nconn (c4 / c4s CPU leg) */
double orc_bench_records_multi(const orc_transform *const *ts, uint32_t nconn, int dir, uint8_t *arena,
                               size_t stride, size_t data_len, uint64_t n, int threads, int32_t *status);

/* ---- TLS 1.3 key schedule (oracle/keysched.c) -------------------------- */
/* hash identifiers: the psa_algorithm_t values PSA_ALG_SHA_256 / _384 of the
 * PSA Crypto API (the reference passes psa_algorithm_t hash_alg) */
#define ORC_HASH_SHA256 0x02000009
#define ORC_HASH_SHA384 0x0200000a
#define ORC_TLS13_CONTEXT_UNHASHED 0     /* MBEDTLS_SSL_TLS1_3_CONTEXT_UNHASHED, ssl_tls13_keys.h */
#define ORC_TLS13_CONTEXT_HASHED   1

size_t orc_hash_len(int alg);
int orc_hash(int alg, const uint8_t *msg, size_t len, uint8_t *out);
int orc_hmac(int alg, const uint8_t *key, size_t klen, const uint8_t *msg, size_t len, uint8_t *out);
int orc_hkdf_extract(int alg, const uint8_t *salt, size_t salt_len, const uint8_t *ikm, size_t ikm_len,
                     uint8_t *prk);
int orc_hkdf_expand(int alg, const uint8_t *prk, size_t prk_len, const uint8_t *info, size_t info_len,
                    uint8_t *out, size_t out_len);
size_t orc_tls13_encode_label(size_t desired, const uint8_t *label, size_t label_len, const uint8_t *ctx,
                              size_t ctx_len, uint8_t *dst);
int orc_tls13_hkdf_expand_label(int alg, const uint8_t *secret, size_t secret_len, const uint8_t *label,
                                size_t label_len, const uint8_t *ctx, size_t ctx_len, uint8_t *buf, size_t buf_len);
int orc_tls13_derive_secret(int alg, const uint8_t *secret, size_t secret_len, const uint8_t *label,
                            size_t label_len, const uint8_t *ctx, size_t ctx_len, int ctx_hashed, uint8_t *dst,
                            size_t dst_len);
int orc_tls13_evolve_secret(int alg, const uint8_t *secret_old, const uint8_t *input, size_t input_len,
                            uint8_t *secret_new);
int orc_tls13_make_traffic_keys(int alg, const uint8_t *client_secret, const uint8_t *server_secret,
                                size_t secret_len, size_t key_len, size_t iv_len, uint8_t *client_key,
                                uint8_t *client_iv, uint8_t *server_key, uint8_t *server_iv);
int orc_tls13_exporter(int alg, const uint8_t *secret, size_t secret_len, const uint8_t *label, size_t label_len,
                       const uint8_t *context, size_t context_len, uint8_t *out, size_t out_len);
int orc_tls13_update_traffic_secret(int alg, const uint8_t *secret, uint8_t *next);

/* ---- stream record loops (oracle/stream.c) ------------------------------ */
#define ORC_ERR_SSL_COUNTER_WRAPPING (-0x6B80)   /* ssl.h */
#define ORC_IN_CONTENT_LEN 16384                 /* MBEDTLS_SSL_IN_CONTENT_LEN, ssl.h:405 */
/* AEAD-only build: IN_BUFFER_LEN (13 + 16 + 16 + 16384) minus the 8-byte
 * in_hdr offset = largest header+body fetch_input accepts; OUT buffer space
 * from out_iv = 16416 (ssl_misc.h:300-392). */
#define ORC_MAX_IN_RECORD 16421
#define ORC_OUT_BUF_SPACE 16416

typedef struct { uint32_t off, data_offset, data_len; uint8_t type; } orc_stream_rec;
typedef struct {
    int32_t status;          /* error that ended the stream, 0 = all complete records accepted */
    uint32_t nrec;           /* records accepted */
    uint32_t consumed;       /* bytes of the accepted records */
    uint8_t in_ctr[8];
    uint8_t nb_zero;
} orc_stream_res;

int orc_stream_decrypt(const orc_transform *t, uint8_t *buf, size_t len, const uint8_t in_ctr[8], uint8_t nb_zero,
                       size_t max_record, int max_version, orc_stream_rec *out, size_t max_out,
                       orc_stream_res *res);
size_t orc_stream_record_wire(const orc_transform *t, size_t n);
int orc_stream_read(uint8_t *buf, const orc_stream_rec *recs, size_t nrec, uint8_t *out, size_t cap,
                    size_t *copied, size_t *records, size_t *left);
int orc_stream_encrypt(const orc_transform *t, const uint8_t *pt, size_t len, uint8_t type, uint8_t out_ctr[8],
                       size_t max_frag, size_t out_buf_space, uint8_t *out, size_t out_cap, size_t *out_len,
                       uint32_t *nrec);

/* ---- DTLS 1.2 datagram record loops (oracle/dtls.c) ---------------------- */
#define ORC_ERR_SSL_UNEXPECTED_RECORD (-0x6700)  /* ssl.h:136 */
#define ORC_ERR_SSL_EARLY_MESSAGE     (-0x6480)  /* ssl.h:146 */
#define ORC_ERR_SSL_CONN_EOF          (-0x7280)  /* ssl.h:46 */
/* MBEDTLS_SSL_IN_BUFFER_LEN / OUT_BUFFER_LEN of the AEAD-only build with DTLS
 * connection IDs (ssl_misc.h:300-392): 13 + (16 IV + 16 tag + 16 CID
 * padding + 16384) + 32 CID; in_hdr = in_buf for DTLS (ssl_msg.c:5264-5266) */
#define ORC_DTLS_MAX_DATAGRAM   16477
#define ORC_DTLS_OUT_BUFFER_LEN 16477
/* record dispositions besides 0 (accepted) and the MBEDTLS_ERR_SSL_* code that
 * skipped or dropped the record */
#define ORC_DTLS_DROPPED     1   /* discarded with the rest of its datagram */
#define ORC_DTLS_NOT_REACHED 2   /* after the connection's fatal error */

/* the mbedtls_ssl_context / config fields the DTLS read loop uses */
typedef struct {
    uint64_t window_top, window;      /* in_window_top / in_window (anti-replay) */
    uint32_t badmac_seen, badmac_limit;
    uint16_t in_epoch;
    uint8_t cid_len;                  /* conf->cid_len: CID length of incoming tls12_cid records */
    uint8_t anti_replay;              /* conf->anti_replay */
    uint8_t ignore_unexpected_cid;    /* conf->ignore_unexpected_cid */
    uint8_t nb_zero;
} orc_dtls_state;

typedef struct {
    uint32_t dgram, off;              /* datagram index, header offset in it */
    uint32_t data_offset, data_len;   /* rec fields after processing (offset from the header) */
    int32_t disp;
    uint8_t type;
} orc_dtls_rec;

typedef struct {
    int32_t status;                   /* the fatal error mbedtls_ssl_read returns, 0 = none */
    uint32_t nrec;                    /* records listed (every record a header walk finds) */
    uint32_t naccepted;
    uint32_t dgrams_done;             /* datagrams processed before a fatal error */
    uint32_t invalid_dgrams;          /* datagrams cut short by a header error */
} orc_dtls_res;

int orc_dtls_replay_check(const orc_dtls_state *st, const uint8_t ctr[8]);
void orc_dtls_replay_update(orc_dtls_state *st, const uint8_t ctr[8]);
int orc_dtls_decrypt(const orc_transform *t, orc_dtls_state *st, uint8_t *buf, const uint64_t *doff,
                     const uint32_t *dlen, size_t nd, orc_dtls_rec *out, size_t max_out, orc_dtls_res *res);
size_t orc_dtls_record_wire(const orc_transform *t, size_t n);
int orc_dtls_encrypt(const orc_transform *t, const uint8_t *pt, size_t len, uint8_t type, uint8_t out_ctr[8],
                     size_t max_frag, uint8_t *out, size_t out_cap, size_t *out_len, uint32_t *nrec);

/* ---- session tickets (oracle/ticket.c) ----------------------------------- */
#define ORC_ERR_SSL_SESSION_TICKET_EXPIRED (-0x6D80)   /* ssl.h:111 */
typedef struct {
    int cipher;              /* ORC_CIPHER_AES_*_GCM / _CCM (16-byte tag) / CHACHA20_POLY1305 */
    uint8_t key[32];
    uint8_t name[4];
} orc_ticket_key;
int orc_ticket_write(const orc_ticket_key keys[2], int active, uint8_t *start, size_t space, size_t clear_len,
                     size_t *tlen);
int orc_ticket_parse(const orc_ticket_key keys[2], uint8_t *buf, size_t len, size_t *clear_len);

#ifdef __cplusplus
}
#endif
#endif
