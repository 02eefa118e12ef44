/*
 * tlsrec.h -- C ABI of the MI355X TLS record-protection engine (libtlsrec.so).
 *
 * Drop-in boundary for the AEAD record path of Mbed TLS 4.1.0:
 *
 *   reference (internal, library/ssl_misc.h:1724-1732)     this library
 *   ---------------------------------------------------    ----------------------
 *   int mbedtls_ssl_encrypt_buf(ssl, transform, rec)       tlsrec_encrypt_buf
 *       library/ssl_msg.c:784-1268
 *   int mbedtls_ssl_decrypt_buf(ssl, transform, rec)       tlsrec_decrypt_buf
 *       library/ssl_msg.c:1270-1834
 *   struct mbedtls_ssl_transform (ssl_misc.h:1073-1120)    tlsrec_transform
 *   mbedtls_record               (ssl_misc.h:1163-1188)    tlsrec_record
 *   mbedtls_ssl_tls13_populate_transform                   tlsrec_transform_setup
 *       (library/ssl_tls13_keys.c:922-1042) and the AEAD
 *       branch of ssl_tls12_populate_transform
 *       (library/ssl_tls.c:7768-7797)
 *   mbedtls_ssl_transform_free (ssl_msg.c:6084-6099)       tlsrec_transform_free
 *   psa_aead_encrypt / psa_aead_decrypt (TF-PSA-Crypto,    the HIP kernels behind
 *       called at ssl_msg.c:1043 and :1412)                 every entry point
 *
 * plus a device-resident batch extension (tlsrec_batch_encrypt/decrypt) that
 * applies the same per-record semantics to many records already in HBM, and a
 * key table (tlsrec_keytab_*) that holds per-connection keys on the GPU.
 *
 * Semantics and error codes are those of the reference: 0 on success or a
 * negative MBEDTLS_ERR_SSL_* value (include/mbedtls/ssl.h:40-125); the record
 * is transformed in place and its data_offset / data_len / type are updated
 * exactly as the reference updates them.  Only the AEAD suites are supported
 * (AES-128/192/256-GCM, AES-128/192/256-CCM and CCM_8, ChaCha20-Poly1305,
 * ARIA-128/192/256-GCM and -CCM;
 * TLS 1.2 and 1.3, and DTLS 1.2 records with an RFC 9146 connection ID).
 *
 * Every entry point that touches record data runs on the GPU; there is no CPU
 * fallback.  Without a usable HIP device they return
 * TLSREC_ERR_SSL_HW_ACCEL_FAILED (MBEDTLS_ERR_SSL_HW_ACCEL_FAILED).
 */
#ifndef TLSREC_H
#define TLSREC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants (values of include/mbedtls/ssl.h) ---------------------- */
#define TLSREC_ERR_SSL_BAD_INPUT_DATA        (-135)    /* PSA_ERROR_INVALID_ARGUMENT, ssl.h:40 */
#define TLSREC_ERR_SSL_BUFFER_TOO_SMALL      (-138)    /* PSA_ERROR_BUFFER_TOO_SMALL, ssl.h:125 */
#define TLSREC_ERR_SSL_ALLOC_FAILED          (-141)    /* PSA_ERROR_INSUFFICIENT_MEMORY, ssl.h:101 */
#define TLSREC_ERR_SSL_FEATURE_UNAVAILABLE   (-0x7080) /* ssl.h:38 */
#define TLSREC_ERR_SSL_INVALID_MAC           (-0x7180) /* ssl.h:42 */
#define TLSREC_ERR_SSL_INVALID_RECORD        (-0x7200) /* ssl.h:44 */
#define TLSREC_ERR_SSL_HW_ACCEL_FAILED       (-0x7F80) /* ssl.h:103 */
#define TLSREC_ERR_SSL_INTERNAL_ERROR        (-0x6C00) /* ssl.h:117 */
#define TLSREC_ERR_SSL_UNEXPECTED_CID        (-0x6000) /* ssl.h:156 */

#define TLSREC_VERSION_TLS1_2   0x0303   /* MBEDTLS_SSL_VERSION_TLS1_2 */
#define TLSREC_VERSION_TLS1_3   0x0304   /* MBEDTLS_SSL_VERSION_TLS1_3 */

#define TLSREC_CIPHER_AES_128_GCM        1
#define TLSREC_CIPHER_AES_256_GCM        2
#define TLSREC_CIPHER_CHACHA20_POLY1305  3
/* the other AES AEADs of mbedtls_ssl_cipher_to_psa
 * (ssl_tls.c:2168-2363).  The _CCM_8 ids are the MBEDTLS_CIPHERSUITE_SHORT_TAG
 * suites (taglen 8: ssl_tls.c:7707-7708, ssl_tls13_keys.c:981-985). */
#define TLSREC_CIPHER_AES_192_GCM        4
#define TLSREC_CIPHER_AES_128_CCM        5
#define TLSREC_CIPHER_AES_192_CCM        6
#define TLSREC_CIPHER_AES_256_CCM        7
#define TLSREC_CIPHER_AES_128_CCM_8      8
#define TLSREC_CIPHER_AES_192_CCM_8      9
#define TLSREC_CIPHER_AES_256_CCM_8      10
/* ARIA-GCM (RFC 5794 block cipher; PSA_KEY_TYPE_ARIA + PSA_ALG_GCM in
 * mbedtls_ssl_cipher_to_psa, ssl_tls.c:2248-2289; the RFC 6209 TLS 1.2 suites) */
#define TLSREC_CIPHER_ARIA_128_GCM       11
#define TLSREC_CIPHER_ARIA_192_GCM       12
#define TLSREC_CIPHER_ARIA_256_GCM       13
/* ARIA-CCM (PSA_KEY_TYPE_ARIA + PSA_ALG_CCM, ssl_tls.c:2241-2282), 16-byte tag */
#define TLSREC_CIPHER_ARIA_128_CCM       14
#define TLSREC_CIPHER_ARIA_192_CCM       15
#define TLSREC_CIPHER_ARIA_256_CCM       16
/* Camellia-GCM / -CCM (RFC 3713 block cipher; PSA_KEY_TYPE_CAMELLIA with
 * PSA_ALG_GCM / PSA_ALG_CCM, ssl_tls.c:2297-2345; the RFC 6367 suites), 16-byte tag */
#define TLSREC_CIPHER_CAMELLIA_128_GCM   17
#define TLSREC_CIPHER_CAMELLIA_192_GCM   18
#define TLSREC_CIPHER_CAMELLIA_256_GCM   19
#define TLSREC_CIPHER_CAMELLIA_128_CCM   20
#define TLSREC_CIPHER_CAMELLIA_192_CCM   21
#define TLSREC_CIPHER_CAMELLIA_256_CCM   22
#define TLSREC_CIPHER_MAX                22

#define TLSREC_MSG_APPLICATION_DATA  23      /* ssl.h:527 */
#define TLSREC_MSG_CID               25      /* MBEDTLS_SSL_MSG_CID, ssl.h:528 */
#define TLSREC_CID_LEN_MAX           32      /* MBEDTLS_SSL_CID_{IN,OUT}_LEN_MAX, ssl.h:423-429 */
#define TLSREC_OUT_CONTENT_LEN       16384   /* MBEDTLS_SSL_OUT_CONTENT_LEN, ssl.h:409 */
#define TLSREC_PADDING_GRANULARITY   16      /* MBEDTLS_SSL_CID_TLS1_3_PADDING_GRANULARITY, ssl.h:432 */

/* ---- single-record API (host buffers) --------------------------------- */

/* AEAD fields of struct mbedtls_ssl_transform, with raw key bytes and
 * device key-table slots in place of the PSA key ids psa_key_enc/dec. */
typedef struct tlsrec_transform {
    size_t minlen;           /* min. ciphertext length */
    size_t ivlen;            /* 12 */
    size_t fixed_ivlen;      /* 12, or 4 for TLS 1.2 GCM */
    size_t maclen;           /* 0 for AEAD */
    size_t taglen;           /* 16 */
    unsigned char iv_enc[16];
    unsigned char iv_dec[16];
    int tls_version;         /* TLSREC_VERSION_* */
    int cipher;              /* TLSREC_CIPHER_* */
    size_t keylen;           /* 16, 24 or 32 */
    unsigned char key_enc[32];
    unsigned char key_dec[32];
    int32_t slot_enc;        /* device key slots (engine key table), -1 = none */
    int32_t slot_dec;
    uint32_t granularity;    /* MBEDTLS_SSL_CID_TLS1_3_PADDING_GRANULARITY (16) */
    /* DTLS 1.2 connection IDs (ssl_misc.h transform in_cid / out_cid); set
     * with tlsrec_transform_set_cid, zero after tlsrec_transform_setup */
    uint8_t in_cid_len;
    uint8_t out_cid_len;
    unsigned char in_cid[TLSREC_CID_LEN_MAX];
    unsigned char out_cid[TLSREC_CID_LEN_MAX];
} tlsrec_transform;

/* mbedtls_record (ssl_misc.h:1163-1188). */
typedef struct tlsrec_record {
    uint8_t ctr[8];          /* implicit sequence number (DTLS: epoch + seq), big endian */
    uint8_t type;            /* record content type */
    uint8_t ver[2];          /* version as on the wire */
    unsigned char *buf;      /* host buffer enclosing the record content */
    size_t buf_len;
    size_t data_offset;
    size_t data_len;
    uint8_t cid_len;         /* connection ID of the record (0 = none) */
    unsigned char cid[TLSREC_CID_LEN_MAX];
} tlsrec_record;

/* Populate `t` like mbedtls_ssl_tls13_populate_transform (TLS 1.3) or the
 * AEAD branch of ssl_tls12_populate_transform (TLS 1.2) and import both keys
 * into the engine's device key table.  iv_* point at 12 bytes (TLS 1.3,
 * ChaChaPoly) or at least fixed_ivlen bytes (TLS 1.2 GCM: 4). */
int tlsrec_transform_setup(tlsrec_transform *t, int tls_version, int cipher,
                           const unsigned char *key_enc, const unsigned char *key_dec,
                           const unsigned char *iv_enc, const unsigned char *iv_dec);
/* As tlsrec_transform_setup with an explicit TLS 1.3 padding granularity
 * (the reference's compile-time MBEDTLS_SSL_CID_TLS1_3_PADDING_GRANULARITY;
 * its record KATs are generated with 1). */
int tlsrec_transform_setup_ex(tlsrec_transform *t, int tls_version, int cipher,
                              const unsigned char *key_enc, const unsigned char *key_dec,
                              const unsigned char *iv_enc, const unsigned char *iv_dec,
                              unsigned granularity);
/* DTLS 1.2 connection IDs of a transform: in_cid (records it decrypts must
 * carry it, else TLSREC_ERR_SSL_UNEXPECTED_CID) and out_cid (records it
 * encrypts get it and become DTLSInnerPlaintext of type TLSREC_MSG_CID) --
 * what ssl_tls12_populate_transform copies from ssl->own_cid and the peer's
 * CID (library/ssl_tls.c).  Lengths <= TLSREC_CID_LEN_MAX, 0 = none.  Also
 * sets the CID of the transform's device key slots. */
int tlsrec_transform_set_cid(tlsrec_transform *t, const unsigned char *in_cid, size_t in_len,
                             const unsigned char *out_cid, size_t out_len);
/* Release the key slots and zeroize the transform. */
void tlsrec_transform_free(tlsrec_transform *t);

/* Same contract as mbedtls_ssl_encrypt_buf / mbedtls_ssl_decrypt_buf;
 * `ssl` is accepted for signature parity and only used for debugging in the
 * reference, it may be NULL. */
int tlsrec_encrypt_buf(void *ssl, tlsrec_transform *t, tlsrec_record *rec);
int tlsrec_decrypt_buf(const void *ssl, tlsrec_transform *t, tlsrec_record *rec);

/* ---- device key table -------------------------------------------------- */

/* One direction of one connection: the raw material a handshake produces
 * (what the RCCL broadcast carries).  64 bytes. */
typedef struct tlsrec_key_material {
    uint8_t cipher;          /* TLSREC_CIPHER_* */
    uint8_t tls_minor;       /* 3 = TLS 1.2, 4 = TLS 1.3 */
    uint8_t fixed_ivlen;     /* 12, or 4 for TLS 1.2 GCM */
    uint8_t taglen;          /* 16, or 8 for TLSREC_CIPHER_AES_*_CCM_8 */
    uint8_t granularity;     /* TLS 1.3 padding granularity, 0 = 16 (ssl.h:432) */
    uint8_t reserved[11];    /* zero (the device copy keeps the slot's CID length in [0]) */
    uint8_t iv[16];          /* static IV, first fixed_ivlen bytes used */
    uint8_t key[32];         /* 16, 24 or 32 bytes used */
} tlsrec_key_material;

typedef struct tlsrec_keytab tlsrec_keytab;

/* Device table of `capacity` slots on the current HIP device. */
int tlsrec_keytab_create(tlsrec_keytab **kt, uint32_t capacity);
/* Load `count` slots starting at `first` from `keys` (host memory, or device
 * memory when keys_on_device != 0) and expand them on the GPU (AES key
 * schedule, H = E_K(0), GHASH tables).  Enqueued on `stream` (hipStream_t,
 * NULL = default stream). */
int tlsrec_keytab_load(tlsrec_keytab *kt, uint32_t first, uint32_t count,
                       const tlsrec_key_material *keys, int keys_on_device,
                       void *stream);
/* Connection ID of slot `slot` (a transform direction: out_cid for an
 * encrypting slot, in_cid for a decrypting one); a (re)load resets it to
 * none.  Enqueued on `stream` and waited for. */
int tlsrec_keytab_set_cid(tlsrec_keytab *kt, uint32_t slot, const unsigned char *cid, size_t cid_len,
                          void *stream);
uint32_t tlsrec_keytab_capacity(const tlsrec_keytab *kt);
void tlsrec_keytab_free(tlsrec_keytab *kt);

/* ---- device-resident batch API ----------------------------------------- */

/* mbedtls_record with offsets into a device arena (40 bytes). */
typedef struct tlsrec_batch_rec {
    uint64_t buf_off;        /* rec->buf = arena + buf_off */
    uint32_t buf_len;
    uint32_t data_offset;
    uint32_t data_len;
    uint32_t slot;           /* key-table slot = the transform direction */
    uint8_t  ctr[8];         /* sequence number, big endian */
    uint8_t  type;
    uint8_t  ver[2];
    uint8_t  cid_len;        /* decrypt: the record's connection ID length (0 = none) */
    uint8_t  cid_off[4];     /* decrypt: its bytes at in_arena + buf_off + cid_off
                                (little-endian u32; the DTLS header holds them) */
} tlsrec_batch_rec;

/* The fields of the record after the call, plus its status (16 bytes). */
typedef struct tlsrec_batch_res {
    int32_t  status;         /* 0 or MBEDTLS_ERR_SSL_* */
    uint32_t data_offset;
    uint32_t data_len;
    uint8_t  type;
    uint8_t  cid_len;        /* encrypt: rec->cid_len as the reference leaves it
                                (the slot's CID once ssl_msg.c:874 has run) */
    uint8_t  reserved[2];
} tlsrec_batch_res;

/* Protect / unprotect `n` records.  `recs` and `res` are device arrays; the
 * record buffers live in `in_arena`; results are written to the same offsets
 * of `out_arena` (== in_arena for the reference's in-place behaviour).
 * Per-record semantics are those of mbedtls_ssl_encrypt_buf / _decrypt_buf
 * under the slot's key; a record naming a slot past the table or never
 * loaded gets TLSREC_ERR_SSL_BAD_INPUT_DATA and is left untouched.
 * Records may reference any mix of slots and ciphers in any order (the
 * engine groups them by key on the device); 128-byte aligned record buffers
 * avoid partial-line HBM writes.
 * lanes_per_record: 0 = auto, else lanes of a wavefront sharing one record:
 * 4/8/16/64 for AES-GCM, 1/2/4/8 for ChaCha20-Poly1305 (other values: auto).
 * Asynchronous on `stream` (hipStream_t, NULL = default stream); per-record
 * status lands in `res`. */
int tlsrec_batch_encrypt(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs,
                         tlsrec_batch_res *res, uint32_t n, const uint8_t *in_arena,
                         uint8_t *out_arena, uint32_t lanes_per_record, void *stream);
int tlsrec_batch_decrypt(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs,
                         tlsrec_batch_res *res, uint32_t n, const uint8_t *in_arena,
                         uint8_t *out_arena, uint32_t lanes_per_record, void *stream);

/* The same with the caller's mean record size (buf_len bytes, 0 = unknown)
 * as a launch hint: the host cannot read device-resident descriptors without
 * a sync, and with many keys of small records (<= 4 KiB, 12..127 per key)
 * the GCM kernels then take per-wave key passes at 2 or 4 lanes per record (the
 * stream / DTLS layers and the host pipeline pass the size themselves).
 * Results are identical with any hint; lanes are chosen automatically. */
int tlsrec_batch_encrypt_sized(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs,
                               tlsrec_batch_res *res, uint32_t n, const uint8_t *in_arena,
                               uint8_t *out_arena, uint32_t mean_record_bytes, void *stream);
int tlsrec_batch_decrypt_sized(const tlsrec_keytab *kt, const tlsrec_batch_rec *recs,
                               tlsrec_batch_res *res, uint32_t n, const uint8_t *in_arena,
                               uint8_t *out_arena, uint32_t mean_record_bytes, void *stream);

/* Records in HOST memory (the socket-buffer boundary of ssl_msg.c:2058 /
 * :1855): the same per-record semantics as tlsrec_batch_*, with `recs` /
 * `res` host arrays and buf_off offsets into the host arenas in_arena /
 * out_arena (pinned memory, e.g. hipHostMalloc, gives the full PCIe rate).
 * The batch is cut into chunks of consecutive records of at most
 * chunk_bytes (0 = 64 MiB) of arena; each chunk's byte range is copied to
 * the device and protected there, copies and kernels overlapped on separate
 * streams.  Output: if out_arena is pinned host memory the device can
 * address (hipHostMalloc, hipHostRegister), the kernels write straight into
 * it -- exactly the bytes tlsrec_batch_* writes to its out_arena, so with
 * out_arena != in_arena the other bytes of a record are left as they were;
 * otherwise each chunk is protected in place on the device and its whole byte
 * range copied back to the same offsets of out_arena (gaps between records
 * carry the input bytes).  Records must be in ascending buf_off order and must not
 * overlap (else TLSREC_ERR_SSL_BAD_INPUT_DATA).  Synchronous: returns when
 * every result is in `res`. */
int tlsrec_host_batch_encrypt(tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                              uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                              uint32_t lanes_per_record, uint64_t chunk_bytes);
int tlsrec_host_batch_decrypt(tlsrec_keytab *kt, const tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                              uint32_t n, const uint8_t *in_arena, uint8_t *out_arena,
                              uint32_t lanes_per_record, uint64_t chunk_bytes);

/* Host-only: run the record-framing checks of encrypt_buf / decrypt_buf
 * (everything decided before the AEAD, tlsrec_frame.h) for one batch record
 * under `km`.  Returns 1 if the record proceeds to the AEAD (aead_pos /
 * aead_len filled), 0 if it stops early (`early` holds the status and the
 * record fields the reference would leave).  Needs no GPU. */
int tlsrec_frame_check(int decrypt, const tlsrec_key_material *km, const tlsrec_batch_rec *rec,
                       tlsrec_batch_res *early, uint32_t *aead_pos, uint32_t *aead_len);

/* Host-only: rank `rank`'s contiguous share of a batch of n_records split
 * over `world` GPUs (one process per GPU): ranks differ
 * by at most one record, every record has exactly one owner.  The key table
 * reaches the ranks by a broadcast of rank 0's tlsrec_key_material array
 * (ncclBroadcast over RCCL/xGMI) followed by tlsrec_keytab_load with
 * keys_on_device = 1 -- tests/c/mgpu_shard.c shows the sequence. */
int tlsrec_shard_bounds(uint64_t n_records, uint32_t rank, uint32_t world, uint64_t *start, uint64_t *count);

/* ---- TLS 1.3 key schedule (library/ssl_tls13_keys.c) --------------------
 * HKDF-SHA256/384 on the GPU: the reference's single-shot functions with the
 * same arguments and return codes, plus a batch that derives many
 * connections' record keys straight into a device key table.  Hash
 * identifiers are the psa_algorithm_t values the reference passes. */
#define TLSREC_ALG_SHA_256   0x02000009   /* PSA_ALG_SHA_256 */
#define TLSREC_ALG_SHA_384   0x0200000a   /* PSA_ALG_SHA_384 */
#define TLSREC_TLS13_CONTEXT_UNHASHED 0   /* MBEDTLS_SSL_TLS1_3_CONTEXT_UNHASHED, ssl_tls13_keys.h:35 */
#define TLSREC_TLS13_CONTEXT_HASHED   1   /* MBEDTLS_SSL_TLS1_3_CONTEXT_HASHED, ssl_tls13_keys.h:36 */

/* struct mbedtls_ssl_key_set, library/ssl_misc.h:604-618 */
typedef struct tlsrec_key_set {
    unsigned char client_write_key[32];
    unsigned char server_write_key[32];
    unsigned char client_write_iv[16];
    unsigned char server_write_iv[16];
    size_t key_len;
    size_t iv_len;
} tlsrec_key_set;

/* mbedtls_ssl_tls13_hkdf_expand_label, ssl_tls13_keys.c:138-217 (label
 * without the "tls13 " prefix, <= 249 B; ctx <= 64 B; buf_len <= 255*64) */
int tlsrec_tls13_hkdf_expand_label(int hash_alg, const unsigned char *secret, size_t secret_len,
                                   const unsigned char *label, size_t label_len,
                                   const unsigned char *ctx, size_t ctx_len,
                                   unsigned char *buf, size_t buf_len);
/* mbedtls_ssl_tls13_derive_secret, ssl_tls13_keys.c:293-330 */
int tlsrec_tls13_derive_secret(int hash_alg, const unsigned char *secret, size_t secret_len,
                               const unsigned char *label, size_t label_len,
                               const unsigned char *ctx, size_t ctx_len, int ctx_hashed,
                               unsigned char *dstbuf, size_t dstbuf_len);
/* mbedtls_ssl_tls13_evolve_secret, ssl_tls13_keys.c:332-419 (secret_old may
 * be NULL: initial stage; input NULL or empty: all-zero IKM) */
int tlsrec_tls13_evolve_secret(int hash_alg, const unsigned char *secret_old,
                               const unsigned char *input, size_t input_len,
                               unsigned char *secret_new);
/* mbedtls_ssl_tls13_make_traffic_keys, ssl_tls13_keys.c:262-291 */
int tlsrec_tls13_make_traffic_keys(int hash_alg, const unsigned char *client_secret,
                                   const unsigned char *server_secret, size_t secret_len,
                                   size_t key_len, size_t iv_len, tlsrec_key_set *keys);
/* mbedtls_ssl_tls13_exporter, ssl_tls13_keys.c:1828-1858 */
int tlsrec_tls13_exporter(int hash_alg, const unsigned char *secret, size_t secret_len,
                          const unsigned char *label, size_t label_len,
                          const unsigned char *context_value, size_t context_len,
                          unsigned char *out, size_t out_len);
/* KeyUpdate (RFC 8446 7.2; label "traffic upd", ssl_tls13_keys.h:16):
 * next = HKDF-Expand-Label(secret, "traffic upd", "", Hash.length) */
int tlsrec_tls13_update_traffic_secret(int hash_alg, const unsigned char *secret,
                                       unsigned char *next);

/* One direction's traffic secret (client_application_traffic_secret_N or
 * server_...), 48 bytes; SHA-256 suites use the first 32. */
typedef struct tlsrec_tls13_secret {
    uint8_t secret[48];
} tlsrec_tls13_secret;

/* Batch: for each of `count` device-resident secrets, optionally first apply
 * a KeyUpdate in place (key_update != 0), then derive write_key / write_iv as
 * ssl_tls13_make_traffic_key does (ssl_tls13_keys.c:219-246) and load them
 * into slots first..first+count-1 of `kt` as TLS 1.3 keys of `cipher` (the
 * suite fixes the hash: AES-256-GCM -> SHA-384, others -> SHA-256; key
 * expansion and GHASH tables as tlsrec_keytab_load).  Asynchronous on
 * `stream`; the secrets buffer must stay valid until the stream reaches it. */
int tlsrec_tls13_keytab_derive(tlsrec_keytab *kt, uint32_t first, uint32_t count, int cipher,
                               tlsrec_tls13_secret *secrets, int key_update, void *stream);

/* ---- TLS stream record layer --------------------------
 * Whole-connection framing on the device: received byte streams are split at
 * their 5-byte record headers, checked and decrypted in place; application
 * data is split into records, framed and encrypted into record streams.  Per
 * connection the result is what repeated ssl_get_next_record calls
 * (ssl_msg.c:4700-4900: ssl_parse_record_header :3561-3776,
 * ssl_prepare_record_content :3810-4017) or repeated mbedtls_ssl_write calls
 * (mbedtls_ssl_write_record :2648-2793) produce.  All arrays are device
 * memory; the calls synchronise `stream` once (to size the record batch). */
#define TLSREC_MAX_IN_RECORD  16421  /* header + body limit of mbedtls_ssl_fetch_input (AEAD-only build:
                                        MBEDTLS_SSL_IN_BUFFER_LEN 16429 minus the 8-byte in_hdr offset) */
#define TLSREC_OUT_BUF_SPACE  16416  /* out_buf_len - (out_iv - out_buf), ssl_msg.c:2688 (AEAD-only build) */
#define TLSREC_ERR_SSL_COUNTER_WRAPPING (-0x6B80)   /* ssl.h:119 */

/* One connection's received bytes, starting at a record header (ssl->in_hdr). */
typedef struct tlsrec_stream_in {
    uint64_t off;            /* first byte in the arena */
    uint32_t len;            /* bytes received (ssl->in_left) */
    uint32_t slot;           /* key slot of transform_in */
    uint8_t  in_ctr[8];      /* ssl->in_ctr */
    uint8_t  nb_zero;        /* ssl->nb_zero */
    uint8_t  reserved[7];
} tlsrec_stream_in;

typedef struct tlsrec_stream_in_res {
    int32_t  status;         /* 0: every complete record accepted (a trailing partial record waits);
                                else the error the reference returns for the first bad record */
    uint32_t first;          /* this connection's records are recs/res[first .. first+nparsed) */
    uint32_t nrec;           /* records accepted, in order; record k's plaintext is at
                                arena + recs[first+k].buf_off + res[first+k].data_offset */
    uint32_t consumed;       /* bytes of the accepted records (the next call starts there) */
    uint8_t  in_ctr[8];      /* ssl->in_ctr afterwards */
    uint8_t  nb_zero;
    uint8_t  reserved[3];
    uint32_t nparsed;        /* records framed (bytes of records after a failing one are unspecified) */
} tlsrec_stream_in_res;

/* `recs` / `res`: device arrays of max_records entries, filled by the call.
 * *nrecords (host, may be NULL) = records framed over all connections.
 * Returns TLSREC_ERR_SSL_BUFFER_TOO_SMALL (nothing decrypted) if the
 * connections hold more than max_records complete records. */
int tlsrec_stream_decrypt(const tlsrec_keytab *kt, const tlsrec_stream_in *streams, uint32_t nstreams,
                          uint8_t *arena, tlsrec_batch_rec *recs, tlsrec_batch_res *res,
                          uint32_t max_records, tlsrec_stream_in_res *sres, uint32_t *nrecords,
                          void *stream);

/* Read side of mbedtls_ssl_read over the records tlsrec_stream_decrypt
 * accepted: per connection, ssl_read_application_data (ssl_msg.c:5627-5650)
 * in record order -- copy at most out_cap bytes of application data (type 23
 * records; other content types are the caller's) to out_arena + out_off and
 * zeroize the plaintext handed out; a record only partly consumed keeps its
 * tail (in_offt += n). */
typedef struct tlsrec_stream_read_req {
    uint64_t out_off;        /* the caller's buffer (buf of mbedtls_ssl_read) in out_arena */
    uint32_t out_cap;        /* len */
    uint32_t reserved;
} tlsrec_stream_read_req;

typedef struct tlsrec_stream_read_res {
    uint32_t copied;         /* bytes written to the caller's buffer */
    uint32_t records;        /* accepted records fully consumed (non-application ones included) */
    uint32_t left;           /* bytes still unread in the next record (in_msglen) */
    uint32_t reserved;
} tlsrec_stream_read_res;

int tlsrec_stream_read(const tlsrec_stream_in_res *sres, uint32_t nstreams, const tlsrec_batch_rec *recs,
                       const tlsrec_batch_res *res, uint8_t *arena, const tlsrec_stream_read_req *req,
                       uint8_t *out_arena, tlsrec_stream_read_res *rres, void *stream);

/* One connection's application data to send. */
typedef struct tlsrec_stream_out {
    uint64_t in_off;         /* plaintext in the input arena */
    uint32_t in_len;
    uint32_t slot;           /* key slot of transform_out */
    uint64_t out_off;        /* record stream destination in the output arena */
    uint8_t  out_ctr[8];     /* ssl->cur_out_ctr */
    uint32_t max_frag;       /* mbedtls_ssl_get_max_out_record_payload(); 0 = 16384 */
    uint8_t  type;           /* ssl->out_msgtype, normally 23 */
    uint8_t  reserved[3];
} tlsrec_stream_out;

typedef struct tlsrec_stream_out_res {
    int32_t  status;         /* 0 or the first record's error (COUNTER_WRAPPING after the record) */
    uint32_t first;          /* records recs/res[first .. first+nparsed) */
    uint32_t nrec;           /* records written */
    uint32_t out_len;        /* bytes of record stream written at out_off */
    uint8_t  out_ctr[8];     /* cur_out_ctr afterwards */
    uint32_t nparsed;
    uint8_t  reserved[4];
} tlsrec_stream_out_res;

/* Bytes of record stream `in_len` bytes of application data become (host
 * helper for sizing out_arena; 0 for an unsupported suite). */
uint64_t tlsrec_stream_out_size(int tls_version, int cipher, uint32_t granularity, uint64_t in_len,
                                uint32_t max_frag);
int tlsrec_stream_encrypt(const tlsrec_keytab *kt, const tlsrec_stream_out *streams, uint32_t nstreams,
                          const uint8_t *in_arena, uint8_t *out_arena, tlsrec_batch_rec *recs,
                          tlsrec_batch_res *res, uint32_t max_records, tlsrec_stream_out_res *sres,
                          uint32_t *nrecords, void *stream);

/* ---- DTLS 1.2 datagram record layer (DTLS branch) -------
 * The datagram-transport form of the same loops: received datagrams are
 * split at their 13-byte DTLS record headers (plus conf->cid_len CID bytes
 * for tls12_cid records) with the DTLS checks of ssl_parse_record_header
 * (ssl_msg.c:3561-3776: datagram holds the record, epoch, anti-replay window
 * :3248-3306), decrypted in place by the AEAD kernels, and ssl_get_next_record's
 * datagram rules applied per connection in arrival order (ssl_msg.c:4727-4873:
 * unexpected records skipped, a header error or a bad MAC drops the rest of
 * the datagram, badmac_limit, ignore_unexpected_cid) together with
 * ssl_prepare_record_content's DTLS post-rules (explicit sequence numbers, no
 * in_ctr step, mbedtls_ssl_dtls_replay_update).  Send writes one record per
 * mbedtls_ssl_write, each its own datagram (mbedtls_ssl_write_record,
 * :2648-2793: FE FD, epoch + 48-bit sequence, out_cid).  DTLS 1.2 only (the
 * reference has no DTLS 1.3): slots must hold TLS 1.2 keys. */
#define TLSREC_ERR_SSL_UNEXPECTED_RECORD (-0x6700)   /* ssl.h:136 */
#define TLSREC_ERR_SSL_EARLY_MESSAGE     (-0x6480)   /* ssl.h:146 */
#define TLSREC_ERR_SSL_CONN_EOF          (-0x7280)   /* ssl.h:46 */
/* MBEDTLS_SSL_IN_BUFFER_LEN / OUT_BUFFER_LEN of the AEAD-only build with DTLS
 * connection IDs (ssl_misc.h:300-392): 13 + 16 + 16 + 16 + 16384 + 32.  A
 * longer datagram is read truncated, as f_recv into that buffer would be. */
#define TLSREC_DTLS_MAX_DATAGRAM   16477
#define TLSREC_DTLS_OUT_BUFFER_LEN 16477
/* record dispositions (besides 0 = accepted and the MBEDTLS_ERR_SSL_* code
 * that skipped or dropped the record: UNEXPECTED_RECORD / EARLY_MESSAGE
 * (other epoch or replayed; skipped), INVALID_MAC (datagram dropped),
 * UNEXPECTED_CID (ignored), or the connection's fatal error) */
#define TLSREC_DTLS_DROPPED     1    /* discarded with the rest of its datagram */
#define TLSREC_DTLS_NOT_REACHED 2    /* after the connection's fatal error */
#define TLSREC_DTLS_ANTI_REPLAY            1   /* conf->anti_replay */
#define TLSREC_DTLS_IGNORE_UNEXPECTED_CID  2   /* conf->ignore_unexpected_cid */

/* One received datagram (one f_recv result) in the arena. */
typedef struct tlsrec_dgram {
    uint64_t off;
    uint32_t len;
    uint32_t reserved;
} tlsrec_dgram;

/* One connection's receive state (the mbedtls_ssl_context / config fields the
 * DTLS read loop uses) and its datagrams, in arrival order.  Datagram ranges
 * of different connections must not overlap. */
typedef struct tlsrec_dtls_in {
    uint64_t window_top;     /* ssl->in_window_top */
    uint64_t window;         /* ssl->in_window */
    uint32_t first_dgram;    /* dgrams[first_dgram .. first_dgram + ndgram) */
    uint32_t ndgram;
    uint32_t slot;           /* key slot of transform_in (TLS 1.2 key) */
    uint32_t badmac_seen;    /* ssl->badmac_seen */
    uint32_t badmac_limit;   /* conf->badmac_limit, 0 = no limit */
    uint16_t in_epoch;       /* ssl->in_epoch */
    uint8_t  cid_len;        /* conf->cid_len: CID length of incoming tls12_cid records */
    uint8_t  flags;          /* TLSREC_DTLS_ANTI_REPLAY | TLSREC_DTLS_IGNORE_UNEXPECTED_CID */
    uint8_t  nb_zero;        /* ssl->nb_zero */
    uint8_t  reserved[7];
} tlsrec_dtls_in;

typedef struct tlsrec_dtls_in_res {
    uint64_t window_top;     /* state afterwards */
    uint64_t window;
    int32_t  status;         /* 0, or the fatal error mbedtls_ssl_read returns (processing stops) */
    uint32_t first;          /* this connection's records are recs/res/disp[first .. first+nrec) */
    uint32_t nrec;           /* records a header walk finds in its datagrams, in order */
    uint32_t naccepted;      /* records with disposition 0: plaintext at
                                arena + recs[k].buf_off + res[k].data_offset, res[k].data_len, res[k].type */
    uint32_t dgrams_done;    /* datagrams fully processed before a fatal error */
    uint32_t invalid_dgrams; /* datagrams cut short by a header error (INVALID_RECORD) */
    uint32_t badmac_seen;
    uint8_t  nb_zero;
    uint8_t  reserved[3];
} tlsrec_dtls_in_res;

/* recs / res / disp: device arrays of max_records entries.  *nrecords (host,
 * may be NULL) = records listed over all connections.  Records skipped or
 * dropped keep unspecified bytes (the reference discards them too). */
int tlsrec_dtls_decrypt(const tlsrec_keytab *kt, const tlsrec_dtls_in *conns, uint32_t nconns,
                        const tlsrec_dgram *dgrams, uint32_t ndgrams, uint8_t *arena, tlsrec_batch_rec *recs,
                        tlsrec_batch_res *res, int32_t *disp, uint32_t max_records, tlsrec_dtls_in_res *cres,
                        uint32_t *nrecords, void *stream);

/* Bytes of datagrams `in_len` bytes of application data become under a TLS
 * 1.2 key with an out_cid of cid_len bytes (0 for an unsupported suite). */
uint64_t tlsrec_dtls_out_size(int cipher, uint32_t granularity, uint32_t cid_len, uint64_t in_len,
                              uint32_t max_frag);
/* tlsrec_stream_out with out_ctr = epoch (2 bytes) + 48-bit sequence number;
 * record k of a connection is one datagram: its header starts at
 * out_arena + recs[first + k].buf_off - 13 - cid_len and it is
 * 13 + cid_len + res[first + k].data_len bytes long. */
int tlsrec_dtls_encrypt(const tlsrec_keytab *kt, const tlsrec_stream_out *streams, uint32_t nstreams,
                        const uint8_t *in_arena, uint8_t *out_arena, tlsrec_batch_rec *recs,
                        tlsrec_batch_res *res, uint32_t max_records, tlsrec_stream_out_res *sres,
                        uint32_t *nrecords, void *stream);

/* ---- session tickets (library/ssl_ticket.c) ------------
 * mbedtls_ssl_ticket_write / mbedtls_ssl_ticket_parse for a batch of tickets
 * in device memory.  Ticket = key_name[4] || iv[12] || len16 || state ||
 * tag[16] (ssl_ticket.c:44-55); AEAD nonce = iv, AAD = the 18 header bytes.
 * The ticket keys are key-table slots holding an AES-GCM, AES-CCM (16-byte
 * tag) or ChaCha20-Poly1305 key (the cipher of mbedtls_ssl_ticket_setup). */
#define TLSREC_ERR_SSL_SESSION_TICKET_EXPIRED (-0x6D80)   /* ssl.h:111 */
#define TLSREC_TICKET_MIN_LEN 34                          /* TICKET_MIN_LEN, ssl_ticket.c:49-52 */

/* the keys[2] / active fields of mbedtls_ssl_ticket_context */
typedef struct tlsrec_ticket_keys {
    uint32_t slot[2];        /* key-table slots of keys[0], keys[1] */
    uint8_t  name[2][4];     /* their key names */
    uint32_t active;         /* ctx->active: the key new tickets use */
} tlsrec_ticket_keys;

typedef struct tlsrec_ticket {
    uint64_t off;            /* ticket start in the arena */
    uint32_t len;            /* write: end - start (space); parse: ticket length */
    uint32_t clear_len;      /* write: serialized session length; the state is at off + 18 and the caller's
                                random IV at off + 4 (psa_generate_random, ssl_ticket.c:255) */
} tlsrec_ticket;

typedef struct tlsrec_ticket_res {
    int32_t  status;         /* 0 or MBEDTLS_ERR_SSL_* as the reference returns it */
    uint32_t tlen;           /* write: *tlen; parse: clear_len (state decrypted in place at off + 18) */
    uint32_t reserved[2];
} tlsrec_ticket_res;

int tlsrec_ticket_write(const tlsrec_keytab *kt, const tlsrec_ticket_keys *keys, const tlsrec_ticket *tickets,
                        uint32_t n, uint8_t *arena, tlsrec_ticket_res *res, void *stream);
int tlsrec_ticket_parse(const tlsrec_keytab *kt, const tlsrec_ticket_keys *keys, const tlsrec_ticket *tickets,
                        uint32_t n, uint8_t *arena, tlsrec_ticket_res *res, void *stream);

/* ---- engine ------------------------------------------------------------- */
/* 0 if a gfx950 device is usable, else TLSREC_ERR_SSL_HW_ACCEL_FAILED. */
int tlsrec_device_check(void);
/* Library build string (kernel variants, arch). */
const char *tlsrec_version_string(void);

#ifdef __cplusplus
}
#endif
#endif /* TLSREC_H */
