/*
 * tlsrec_host.c -- single-record entry points (host C).
 *
 * tlsrec_encrypt_buf / tlsrec_decrypt_buf keep the contract of
 * mbedtls_ssl_encrypt_buf / mbedtls_ssl_decrypt_buf (library/ssl_msg.c:784,
 * :1270): the record's buffer is protected in place, data_offset / data_len /
 * type are updated, 0 or MBEDTLS_ERR_SSL_* is returned.  Checks that need no
 * record bytes are decided here with the same framing plan the kernels use
 * (tlsrec_frame.h); everything else -- the AEAD, the tag check, the TLS 1.3
 * unpadding -- runs on the GPU through the batch kernels with a batch of one.
 */
#include <stdint.h>
#include <string.h>

#include "tlsrec.h"
#include "tlsrec_frame.h"

/* engine.hip */
int tlsrec__engine_slot_alloc(const tlsrec_key_material *km);
void tlsrec__engine_slot_free(int slot);
int tlsrec__engine_run(int dec, const tlsrec_batch_rec *rec, unsigned char *buf, size_t buf_len,
                       const unsigned char *cid, const void *plan, tlsrec_batch_res *out);
int tlsrec__engine_slot_set_cid(int slot, const unsigned char *cid, size_t cid_len);

static void zeroize(void *p, size_t n)
{
    volatile unsigned char *v = (volatile unsigned char *) p;
    while (n--) *v++ = 0;
}

int tlsrec_transform_setup(tlsrec_transform *t, int tls_version, int cipher,
                           const unsigned char *key_enc, const unsigned char *key_dec,
                           const unsigned char *iv_enc, const unsigned char *iv_dec)
{
    return tlsrec_transform_setup_ex(t, tls_version, cipher, key_enc, key_dec, iv_enc, iv_dec,
                                     TLSREC_PADDING_GRANULARITY);
}

int tlsrec_transform_setup_ex(tlsrec_transform *t, int tls_version, int cipher,
                              const unsigned char *key_enc, const unsigned char *key_dec,
                              const unsigned char *iv_enc, const unsigned char *iv_dec,
                              unsigned granularity)
{
    if (t == NULL || key_enc == NULL || key_dec == NULL || iv_enc == NULL || iv_dec == NULL)
        return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (granularity == 0 || granularity > 255) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    memset(t, 0, sizeof(*t));
    t->slot_enc = t->slot_dec = -1;
    t->granularity = granularity;
    t->keylen = tlsrec_cipher_keylen(cipher);   /* mbedtls_ssl_cipher_to_psa, ssl_tls.c:2168-2363 */
    if (t->keylen == 0) return TLSREC_ERR_SSL_FEATURE_UNAVAILABLE;
    t->cipher = cipher;
    t->tls_version = tls_version;
    t->ivlen = 12;
    t->taglen = tlsrec_cipher_taglen(cipher);   /* short-tag suites: ssl_tls.c:7707-7708 */
    t->maclen = 0;
    if (tls_version == TLSREC_VERSION_TLS1_3) {           /* ssl_tls13_keys.c:985-998 */
        t->fixed_ivlen = t->ivlen;
        t->minlen = t->taglen + granularity;
    } else if (tls_version == TLSREC_VERSION_TLS1_2) {    /* ssl_tls.c:7768-7797 */
        t->fixed_ivlen = cipher == TLSREC_CIPHER_CHACHA20_POLY1305 ? 12 : 4;
        t->minlen = (t->ivlen - t->fixed_ivlen) + t->taglen;
    } else {
        return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    }
    memcpy(t->key_enc, key_enc, t->keylen);
    memcpy(t->key_dec, key_dec, t->keylen);
    memcpy(t->iv_enc, iv_enc, t->fixed_ivlen);
    memcpy(t->iv_dec, iv_dec, t->fixed_ivlen);

    tlsrec_key_material km;
    memset(&km, 0, sizeof(km));
    km.cipher = (uint8_t) cipher;
    km.tls_minor = tls_version == TLSREC_VERSION_TLS1_3 ? 4 : 3;
    km.fixed_ivlen = (uint8_t) t->fixed_ivlen;
    km.taglen = (uint8_t) t->taglen;
    km.granularity = (uint8_t) granularity;
    memcpy(km.iv, iv_enc, t->fixed_ivlen);
    memcpy(km.key, key_enc, t->keylen);
    int r = tlsrec__engine_slot_alloc(&km);
    if (r < 0) {
        zeroize(&km, sizeof(km));
        zeroize(t, sizeof(*t));
        return r;
    }
    t->slot_enc = r;
    memcpy(km.iv, iv_dec, t->fixed_ivlen);
    memcpy(km.key, key_dec, t->keylen);
    r = tlsrec__engine_slot_alloc(&km);
    zeroize(&km, sizeof(km));
    if (r < 0) {
        tlsrec__engine_slot_free(t->slot_enc);
        zeroize(t, sizeof(*t));
        return r;
    }
    t->slot_dec = r;
    return 0;
}

/* transform->in_cid / out_cid (ssl_tls12_populate_transform, library/ssl_tls.c);
 * the encrypt slot gets out_cid, the decrypt slot in_cid */
int tlsrec_transform_set_cid(tlsrec_transform *t, const unsigned char *in_cid, size_t in_len,
                             const unsigned char *out_cid, size_t out_len)
{
    if (t == NULL || in_len > TLSREC_CID_LEN_MAX || out_len > TLSREC_CID_LEN_MAX ||
        (in_len && in_cid == NULL) || (out_len && out_cid == NULL))
        return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    if (t->slot_enc < 0 || t->slot_dec < 0) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    int r = tlsrec__engine_slot_set_cid(t->slot_enc, out_cid, out_len);
    if (r == 0) r = tlsrec__engine_slot_set_cid(t->slot_dec, in_cid, in_len);
    if (r != 0) return r;
    memset(t->in_cid, 0, sizeof(t->in_cid));
    memset(t->out_cid, 0, sizeof(t->out_cid));
    if (in_len) memcpy(t->in_cid, in_cid, in_len);
    if (out_len) memcpy(t->out_cid, out_cid, out_len);
    t->in_cid_len = (uint8_t) in_len;
    t->out_cid_len = (uint8_t) out_len;
    return 0;
}

void tlsrec_transform_free(tlsrec_transform *t)
{
    if (t == NULL) return;
    if (t->slot_enc >= 0) tlsrec__engine_slot_free(t->slot_enc);
    if (t->slot_dec >= 0) tlsrec__engine_slot_free(t->slot_dec);
    zeroize(t, sizeof(*t));
    t->slot_enc = t->slot_dec = -1;
}

static tlsrec_plan_key pkey(const tlsrec_transform *t, int dec)
{
    tlsrec_plan_key k;
    k.tls13 = t->tls_version == TLSREC_VERSION_TLS1_3;
    k.fixed_ivlen = (uint32_t) t->fixed_ivlen;
    k.taglen = (uint32_t) t->taglen;
    k.iv = dec ? t->iv_dec : t->iv_enc;
    k.cid_len = dec ? t->in_cid_len : t->out_cid_len;
    k.cid = dec ? t->in_cid : t->out_cid;
    return k;
}

static int run(int dec, tlsrec_transform *t, tlsrec_record *rec, const tlsrec_plan *p)
{
    tlsrec_batch_rec d;
    tlsrec_batch_res res;
    memset(&d, 0, sizeof(d));
    d.buf_off = 0;
    d.buf_len = (uint32_t) rec->buf_len;
    d.data_offset = (uint32_t) rec->data_offset;
    d.data_len = (uint32_t) rec->data_len;
    d.slot = (uint32_t) (dec ? t->slot_dec : t->slot_enc);
    memcpy(d.ctr, rec->ctr, 8);
    d.type = rec->type;
    d.ver[0] = rec->ver[0];
    d.ver[1] = rec->ver[1];
    d.cid_len = dec ? rec->cid_len : 0;
    int r = tlsrec__engine_run(dec, &d, rec->buf, rec->buf_len, rec->cid, p, &res);
    if (r != 0) return r;
    /* no kernel reached the record: the staged INTERNAL_ERROR is returned and
     * rec is left as it was (ssl_msg.c:1260 / :1804, auth_done != 1) */
    if (res.status == TLSREC_ERR_SSL_INTERNAL_ERROR) return res.status;
    rec->data_offset = res.data_offset;
    rec->data_len = res.data_len;
    rec->type = res.type;
    if (!dec && res.cid_len) {                       /* ssl_msg.c:874-875 */
        rec->cid_len = res.cid_len;
        memcpy(rec->cid, t->out_cid, res.cid_len);
    }
    return res.status;
}

/* mbedtls_ssl_encrypt_buf (ssl_msg.c:784-1268), AEAD transforms */
int tlsrec_encrypt_buf(void *ssl, tlsrec_transform *t, tlsrec_record *rec)
{
    (void) ssl;   /* debug-only in the reference (ssl_msg.c:802-806) */
    if (t == NULL) return TLSREC_ERR_SSL_INTERNAL_ERROR;                       /* :810-813 */
    if (rec == NULL || rec->buf == NULL) return TLSREC_ERR_SSL_INTERNAL_ERROR; /* :814-823 */
    if (rec->buf_len > 0xffffffffu) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    tlsrec_plan_key k = pkey(t, 0);
    tlsrec_plan p;
    tlsrec_plan_encrypt(&p, &k, rec->ctr, rec->type, rec->ver, rec->buf_len, rec->data_offset,
                        rec->data_len, t->granularity);
    if (p.cid_set) {                                 /* ssl_msg.c:874-875 */
        rec->cid_len = p.cid_len;
        memcpy(rec->cid, t->out_cid, p.cid_len);
    }
    if (p.status != 0) {
        if (p.side_type) {
            rec->buf[p.side_pos] = rec->type;
            memset(rec->buf + p.side_pos + 1, 0, p.side_zeros);
        }
        rec->data_offset = p.data_offset;
        rec->data_len = p.data_len;
        rec->type = p.type;
        return p.status;
    }
    if (t->slot_enc < 0) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    return run(0, t, rec, &p);
}

/* mbedtls_ssl_decrypt_buf (ssl_msg.c:1270-1834), AEAD transforms */
int tlsrec_decrypt_buf(const void *ssl, tlsrec_transform *t, tlsrec_record *rec)
{
    (void) ssl;
    if (rec == NULL || rec->buf == NULL) return TLSREC_ERR_SSL_INTERNAL_ERROR; /* :1301-1307 */
    if (t == NULL) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    if (rec->buf_len > 0xffffffffu) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    tlsrec_plan_key k = pkey(t, 1);
    tlsrec_plan p;
    if (rec->cid_len > TLSREC_CID_LEN_MAX) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    tlsrec_plan_decrypt(&p, &k, rec->ctr, rec->type, rec->ver, rec->buf_len, rec->data_offset, rec->data_len,
                        rec->cid, rec->cid_len);
    if (p.status != 0) {
        rec->data_offset = p.data_offset;
        rec->data_len = p.data_len;
        return p.status;
    }
    if (t->slot_dec < 0) return TLSREC_ERR_SSL_INTERNAL_ERROR;
    return run(1, t, rec, &p);
}

int tlsrec_frame_check(int decrypt, const tlsrec_key_material *km, const tlsrec_batch_rec *rec,
                       tlsrec_batch_res *early, uint32_t *aead_pos, uint32_t *aead_len)
{
    tlsrec_plan_key k;
    tlsrec_plan p;
    k.tls13 = km->tls_minor == 4;
    k.fixed_ivlen = km->fixed_ivlen;
    k.taglen = km->taglen;
    k.iv = km->iv;
    k.cid_len = 0;      /* framing of records without a connection ID */
    k.cid = NULL;
    if (decrypt)
        tlsrec_plan_decrypt(&p, &k, rec->ctr, rec->type, rec->ver, rec->buf_len, rec->data_offset,
                            rec->data_len, NULL, 0);
    else
        tlsrec_plan_encrypt(&p, &k, rec->ctr, rec->type, rec->ver, rec->buf_len, rec->data_offset,
                            rec->data_len, km->granularity ? km->granularity : TLSREC_PADDING_GRANULARITY);
    if (early) {
        early->status = p.status;
        early->data_offset = p.data_offset;
        early->data_len = p.data_len;
        early->type = p.type;
        early->cid_len = p.cid_set ? p.cid_len : 0;
        early->reserved[0] = early->reserved[1] = 0;
    }
    if (aead_pos) *aead_pos = p.aead_pos;
    if (aead_len) *aead_len = p.aead_len;
    return p.status == 0;
}

/* Contiguous balanced record shard of one rank (mbedtls_amd/shard.py
 * shard_bounds): the first n % world ranks take one
 * extra record, so every record has exactly one owner. */
int tlsrec_shard_bounds(uint64_t n_records, uint32_t rank, uint32_t world, uint64_t *start, uint64_t *count)
{
    if (world == 0 || rank >= world || !start || !count) return TLSREC_ERR_SSL_BAD_INPUT_DATA;
    const uint64_t base = n_records / world, extra = n_records % world;
    *start = (uint64_t) rank * base + (rank < extra ? rank : extra);
    *count = base + (rank < extra ? 1u : 0u);
    return 0;
}
