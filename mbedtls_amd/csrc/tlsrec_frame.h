/*
 * tlsrec_frame.h -- per-record framing plan for the AEAD record path.
 *
 * Restates, as straight-line integer code shared by the host C library and
 * the HIP kernels, every decision mbedtls_ssl_encrypt_buf /
 * mbedtls_ssl_decrypt_buf take before and after their psa_aead_* call:
 *
 *   structure checks            ssl_msg.c:814-823 (enc), :1301-1307 (dec)
 *   content length limit        ssl_msg.c:831-839
 *   TLS 1.3 inner plaintext     ssl_msg.c:853-868 with :431-435, :466-491
 *   tag room                    ssl_msg.c:995-998
 *   nonce                       ssl_msg.c:768-781, :1012-1019, :1383-1388
 *   additional data             ssl_msg.c:568-735 (incl. the DTLS 1.2 CID
 *                               branch of RFC 9146, :683-724)
 *   DTLS 1.2 + CID              ssl_msg.c:874-897 (enc), :1313-1320 (dec)
 *   explicit IV (TLS 1.2 GCM)   ssl_msg.c:1066-1075 (enc), :1352-1365 (dec)
 *   short-record checks         ssl_msg.c:1356-1377
 *
 * The plan says what the device must do (AEAD over which bytes, with which
 * nonce and AAD) and what the record fields / status are if it stops early.
 * The AEAD itself and the TLS 1.3 unpadding (ssl_msg.c:1809-1818) run in the
 * kernels.
 */
#ifndef TLSREC_FRAME_H
#define TLSREC_FRAME_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TLSREC_HD __host__ __device__ static inline
/* rare paths (DTLS connection IDs) kept out of the record kernels' register
 * allocation */
#define TLSREC_HD_COLD __host__ __device__ static __attribute__((noinline))
#else
#define TLSREC_HD static inline
#define TLSREC_HD_COLD static
#endif

#define TLSREC_E_BAD_INPUT_DATA   (-135)
#define TLSREC_E_BUFFER_TOO_SMALL (-138)
#define TLSREC_E_INVALID_MAC      (-0x7180)
#define TLSREC_E_INVALID_RECORD   (-0x7200)
#define TLSREC_E_INTERNAL_ERROR   (-0x6C00)
#define TLSREC_E_UNEXPECTED_CID   (-0x6000)
#define TLSREC_MSG_CID_TYPE       25           /* MBEDTLS_SSL_MSG_CID, ssl.h:528 */

/* Cipher properties (mbedtls_ssl_cipher_to_psa, ssl_tls.c:2168-2363; the
 * _CCM_8 ids are the short-tag suites).  Ids: include/tlsrec.h. */
TLSREC_HD uint32_t tlsrec_cipher_keylen(int c)
{
    switch (c) {
        case 1: case 5: case 8: case 11: case 14: case 17: case 20: return 16;   /* AES-128, ARIA-128, Camellia-128 */
        case 4: case 6: case 9: case 12: case 15: case 18: case 21: return 24;   /* AES-192, ARIA-192, Camellia-192 */
        case 2: case 3: case 7: case 10: case 13: case 16: case 19: case 22: return 32;  /* AES-256, ChaCha20-Poly1305, ARIA-256, Camellia-256 */
        default: return 0;
    }
}
TLSREC_HD uint32_t tlsrec_cipher_taglen(int c) { return (c >= 8 && c <= 10) ? 8u : 16u; }
TLSREC_HD int tlsrec_cipher_is_gcm(int c) { return c == 1 || c == 2 || c == 4; }   /* AES-GCM */
TLSREC_HD int tlsrec_cipher_is_aria_gcm(int c) { return c >= 11 && c <= 13; }      /* ARIA-GCM */
TLSREC_HD int tlsrec_cipher_is_aria_ccm(int c) { return c >= 14 && c <= 16; }      /* ARIA-CCM */
TLSREC_HD int tlsrec_cipher_is_aria(int c) { return c >= 11 && c <= 16; }          /* ARIA, any mode */
/* ARIA rounds (RFC 5794 2.1): 12 / 14 / 16 */
TLSREC_HD uint32_t tlsrec_cipher_aria_nr(int c) { return tlsrec_cipher_is_aria(c) ? tlsrec_cipher_keylen(c) / 4 + 8 : 0u; }
/* Camellia-GCM / -CCM (PSA_KEY_TYPE_CAMELLIA, ssl_tls.c:2297-2345) */
TLSREC_HD int tlsrec_cipher_is_cam_gcm(int c) { return c >= 17 && c <= 19; }
TLSREC_HD int tlsrec_cipher_is_cam_ccm(int c) { return c >= 20 && c <= 22; }
TLSREC_HD int tlsrec_cipher_is_cam(int c) { return c >= 17 && c <= 22; }
/* Camellia rounds (RFC 3713 2.3): 18 for 128-bit keys, 24 for 192 / 256 */
TLSREC_HD uint32_t tlsrec_cipher_cam_nr(int c) { return tlsrec_cipher_is_cam(c) ? (tlsrec_cipher_keylen(c) == 16 ? 18u : 24u) : 0u; }
/* The LDS-table block ciphers that share the GCM / CCM kernels' ARIA slot,
 * told apart by their round count (ARIA 12 / 14 / 16, Camellia 18 / 24) */
TLSREC_HD int tlsrec_cipher_is_alt_gcm(int c) { return tlsrec_cipher_is_aria_gcm(c) || tlsrec_cipher_is_cam_gcm(c); }
TLSREC_HD int tlsrec_cipher_is_alt_ccm(int c) { return tlsrec_cipher_is_aria_ccm(c) || tlsrec_cipher_is_cam_ccm(c); }
TLSREC_HD uint32_t tlsrec_cipher_alt_nr(int c) { return tlsrec_cipher_is_aria(c) ? tlsrec_cipher_aria_nr(c) : tlsrec_cipher_cam_nr(c); }
TLSREC_HD int tlsrec_cipher_is_ccm(int c) { return c >= 5 && c <= 10; }
/* AES rounds of an AES-based cipher, 0 otherwise */
TLSREC_HD uint32_t tlsrec_cipher_nr(int c) { return (c == 3 || c > 10) ? 0u : tlsrec_cipher_keylen(c) / 4 + 6; }

typedef struct tlsrec_plan {
    int32_t  status;          /* error found before the AEAD (no AEAD runs) */
    int32_t  post_status;     /* error the reference returns after its AEAD */
    uint32_t data_offset;     /* rec->data_offset when the call returns */
    uint32_t data_len;        /* rec->data_len when the call returns (enc) /
                                 after tag removal (dec, before unpadding) */
    uint8_t  type;            /* rec->type when the call returns (enc) */
    uint8_t  tls13;
    uint8_t  explicit_iv;     /* TLS 1.2 GCM: 8-byte nonce travels in the record */
    uint8_t  aad_len;         /* 5 (TLS 1.3), 13 (TLS 1.2) or 23 + cid_len (CID) */
    uint32_t aead_pos;        /* buffer offset of the AEAD input/output */
    uint32_t aead_len;        /* AEAD plaintext length (ciphertext w/o tag) */
    uint32_t content_len;     /* encrypt: bytes taken from the buffer; the
                                 remaining aead_len - content_len bytes are
                                 the inner type byte and zero padding */
    uint8_t  inner_type;      /* encrypt TLS 1.3: real content type */
    uint8_t  side_type;       /* early error still wrote the type byte ... */
    uint16_t side_zeros;      /* ... and this many zero pad bytes after it */
    uint32_t side_pos;        /* at this buffer offset */
    uint8_t  aad[16];         /* first 16 bytes of the AAD (all of it unless CID) */
    uint8_t  nonce[12];       /* decrypt + explicit_iv: bytes 4..11 come from
                                 the record (buffer offset data_offset) */
    uint8_t  inner;           /* AEAD plaintext is a (D)TLSInnerPlaintext:
                                 TLS 1.3, or DTLS 1.2 with a CID */
    uint8_t  cid_len;         /* CID in the AAD (0 = none) */
    uint8_t  cid_set;         /* encrypt: the reference has set rec->cid (:874) */
} tlsrec_plan;

/* Key-slot parameters the plan needs (from the transform / key material). */
typedef struct tlsrec_plan_key {
    int tls13;
    uint32_t fixed_ivlen;     /* 12 or 4 */
    uint32_t taglen;          /* 16, or 8 for the CCM_8 suites */
    const uint8_t *iv;        /* fixed IV (iv_enc for encrypt, iv_dec for decrypt) */
    uint32_t cid_len;         /* DTLS 1.2 CID: out_cid (encrypt) / in_cid (decrypt) */
    const uint8_t *cid;
} tlsrec_plan_key;

TLSREC_HD void tlsrec__nonce(uint8_t nonce[12], const uint8_t *fixed, uint32_t fixed_len,
                             const uint8_t dyn[8])
{
    /* ssl_build_record_nonce (ssl_msg.c:768-781) */
    for (int i = 0; i < 12; i++) nonce[i] = (uint32_t) i < fixed_len ? fixed[i] : 0;
    for (int i = 0; i < 8; i++) nonce[4 + i] ^= dyn[i];
}

/* Byte k of the RFC 9146 AAD of a DTLS 1.2 record with a CID
 * (ssl_extract_add_data_from_record, ssl_msg.c:683-724):
 *   0xff x 8 || type || cid_len || type || ver || epoch+seq || cid || len16 */
TLSREC_HD uint8_t tlsrec_cid_aad_byte(uint32_t k, uint8_t type, const uint8_t ver[2], const uint8_t ctr[8],
                                      const uint8_t *cid, uint32_t cid_len, uint32_t len_field)
{
    if (k < 8) return 0xff;                          /* seq_num_placeholder */
    if (k == 8 || k == 10) return type;              /* tls12_cid, type */
    if (k == 9) return (uint8_t) cid_len;
    if (k == 11 || k == 12) return ver[k - 11];
    if (k < 21) return ctr[k - 13];
    if (k < 21 + cid_len) return cid[k - 21];
    if (k == 21 + cid_len) return (uint8_t) (len_field >> 8);
    if (k == 22 + cid_len) return (uint8_t) len_field;
    return 0;
}

/* aad[0..15] of a CID record; returns the AAD length */
TLSREC_HD_COLD uint8_t tlsrec__cid_aad_head(uint8_t aad[16], const uint8_t ctr[8], uint8_t type, const uint8_t ver[2],
                                           uint32_t len_field, const uint8_t *cid, uint32_t cid_len)
{
    for (uint32_t i = 0; i < 16; i++) aad[i] = tlsrec_cid_aad_byte(i, type, ver, ctr, cid, cid_len, len_field);
    return (uint8_t) (23 + cid_len);
}

/* rec->cid == transform->in_cid (ssl_msg.c:1317-1318) */
TLSREC_HD_COLD int tlsrec__cid_equal(const uint8_t *a, const uint8_t *b, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++)
        if (a[i] != b[i]) return 0;
    return 1;
}

TLSREC_HD uint8_t tlsrec__aad(uint8_t aad[16], int tls13, const uint8_t ctr[8], uint8_t type,
                              const uint8_t ver[2], uint32_t len_field, const uint8_t *cid, uint32_t cid_len)
{
    /* ssl_extract_add_data_from_record (ssl_msg.c:568-735):
     * TLS 1.3: type || ver || len(TLSCiphertext)        (:671-677, :727-731)
     * TLS 1.2: seq  || type || ver || len(plaintext)    (:700-703, :727-731)
     * DTLS 1.2 + CID: tlsrec_cid_aad_byte; aad[] keeps its first 16 bytes */
    for (int i = 0; i < 16; i++) aad[i] = 0;
    if (!tls13 && cid_len != 0) return tlsrec__cid_aad_head(aad, ctr, type, ver, len_field, cid, cid_len);
    /* constant positions in each branch: a runtime offset would make the
     * kernels keep the whole plan in scratch memory */
    if (!tls13) {
        for (int i = 0; i < 8; i++) aad[i] = ctr[i];
        aad[8] = type;
        aad[9] = ver[0];
        aad[10] = ver[1];
        aad[11] = (uint8_t) (len_field >> 8);
        aad[12] = (uint8_t) len_field;
        return 13;
    }
    aad[0] = type;
    aad[1] = ver[0];
    aad[2] = ver[1];
    aad[3] = (uint8_t) (len_field >> 8);
    aad[4] = (uint8_t) len_field;
    return 5;
}

/* mbedtls_ssl_encrypt_buf, AEAD mode.  buf_len/data_offset/data_len are the
 * mbedtls_record fields; granularity is MBEDTLS_SSL_CID_TLS1_3_PADDING_GRANULARITY. */
TLSREC_HD void tlsrec_plan_encrypt(tlsrec_plan *p, const tlsrec_plan_key *k,
                                   const uint8_t ctr[8], uint8_t type, const uint8_t ver[2],
                                   uint64_t buf_len, uint64_t data_offset, uint64_t data_len,
                                   uint32_t granularity)
{
    p->status = 0;
    p->post_status = 0;
    p->data_offset = (uint32_t) data_offset;
    p->data_len = (uint32_t) data_len;
    p->type = type;
    p->tls13 = (uint8_t) k->tls13;
    p->explicit_iv = (uint8_t) (k->fixed_ivlen != 12);
    p->aad_len = 0;
    p->aead_pos = (uint32_t) data_offset;
    p->aead_len = 0;
    p->content_len = (uint32_t) data_len;
    p->inner_type = type;
    p->side_type = 0;
    p->side_zeros = 0;
    p->side_pos = 0;
    p->inner = (uint8_t) k->tls13;
    p->cid_len = 0;
    p->cid_set = 0;

    if (buf_len < data_offset || buf_len - data_offset < data_len) {    /* :814-823 */
        p->status = TLSREC_E_INTERNAL_ERROR;
        return;
    }
    if (data_len > 16384) {                                            /* :831-839 */
        p->status = TLSREC_E_BAD_INPUT_DATA;
        return;
    }
    uint64_t post_avail = buf_len - (data_len + data_offset);
    uint64_t len = data_len;
    /* (D)TLSInnerPlaintext: TLS 1.3 (:853-868), or DTLS 1.2 with a CID
     * (:874-897; a TLS 1.3 transform carries no CID) */
    const int cid = !k->tls13 && k->cid_len != 0;
    if (cid) {
        p->cid_len = (uint8_t) k->cid_len;
        p->cid_set = 1;                                                /* :874-875 */
    }
    if (k->tls13 || cid) {
        uint32_t g = granularity ? granularity : 16;
        /* data_len <= 16384 here: 32-bit, and a mask for a power-of-two
         * granularity (the 64-bit remainder cost the GCM encrypt kernels
         * registers in every round) */
        const uint32_t dl1 = (uint32_t) data_len + 1;
        const uint64_t pad = (g & (g - 1)) == 0 ? (0u - dl1) & (g - 1) : (g - dl1 % g) % g;   /* :431-435 */
        if (post_avail == 0) {                                         /* :473-475 */
            p->status = TLSREC_E_BUFFER_TOO_SMALL;
            return;
        }
        if (post_avail - 1 < pad) {                                    /* :480-482 */
            /* the real type byte has already been written (:476) */
            p->side_type = 1;
            p->side_pos = (uint32_t) (data_offset + data_len);
            p->status = TLSREC_E_BUFFER_TOO_SMALL;
            return;
        }
        len = data_len + 1 + pad;
        p->data_len = (uint32_t) len;
        p->type = cid ? TLSREC_MSG_CID_TYPE : 23;                      /* :867, :896 */
        p->inner = 1;
        post_avail = buf_len - (len + data_offset);
        if (post_avail < k->taglen) {                                  /* :995-998 */
            /* inner plaintext was built in the buffer before this check */
            p->side_type = 1;
            p->side_zeros = (uint16_t) pad;
            p->side_pos = (uint32_t) (data_offset + data_len);
            p->status = TLSREC_E_BUFFER_TOO_SMALL;
            return;
        }
    } else if (post_avail < k->taglen) {                               /* :995-998 */
        p->status = TLSREC_E_BUFFER_TOO_SMALL;
        return;
    }
    tlsrec__nonce(p->nonce, k->iv, k->fixed_ivlen, ctr);               /* :1012-1019 */
    p->aad_len = tlsrec__aad(p->aad, k->tls13, ctr, p->type, ver,
                             (uint32_t) (k->tls13 ? len + k->taglen : len), k->cid, p->cid_len);
    p->aead_len = (uint32_t) len;
    p->data_len = (uint32_t) (len + k->taglen);                        /* psa_aead_encrypt output */
    if (p->explicit_iv) {                                              /* :1066-1075 */
        if (data_offset < 8) {
            p->post_status = TLSREC_E_BUFFER_TOO_SMALL;
        } else {
            p->data_offset = (uint32_t) (data_offset - 8);
            p->data_len += 8;
        }
    }
}

/* mbedtls_ssl_decrypt_buf, AEAD mode (up to, not including, the AEAD call).
 * rec_cid / rec_cid_len: the record's connection ID (rec->cid). */
TLSREC_HD void tlsrec_plan_decrypt(tlsrec_plan *p, const tlsrec_plan_key *k,
                                   const uint8_t ctr[8], uint8_t type, const uint8_t ver[2],
                                   uint64_t buf_len, uint64_t data_offset, uint64_t data_len,
                                   const uint8_t *rec_cid, uint32_t rec_cid_len)
{
    p->status = 0;
    p->post_status = 0;
    p->data_offset = (uint32_t) data_offset;
    p->data_len = (uint32_t) data_len;
    p->type = type;
    p->tls13 = (uint8_t) k->tls13;
    p->explicit_iv = (uint8_t) (k->fixed_ivlen != 12);
    p->aad_len = 0;
    p->aead_pos = (uint32_t) data_offset;
    p->aead_len = 0;
    p->content_len = 0;
    p->inner_type = 0;
    p->side_type = 0;
    p->side_zeros = 0;
    p->side_pos = 0;
    p->cid_set = 0;
    p->cid_len = (uint8_t) rec_cid_len;
    /* TLS 1.3 and DTLS 1.2 + CID end with ssl_parse_inner_plaintext (:1809-1829) */
    p->inner = (uint8_t) (k->tls13 || rec_cid_len != 0);

    if (buf_len < data_offset || buf_len - data_offset < data_len) {    /* :1301-1307 */
        p->status = TLSREC_E_INTERNAL_ERROR;
        return;
    }
    if (rec_cid_len != k->cid_len ||                                   /* :1313-1320 */
        (rec_cid_len != 0 && !tlsrec__cid_equal(rec_cid, k->cid, rec_cid_len))) {
        p->status = TLSREC_E_UNEXPECTED_CID;
        return;
    }
    uint64_t off = data_offset, len = data_len;
    if (p->explicit_iv) {                                              /* :1352-1365 */
        if (len < 8) {
            p->status = TLSREC_E_INVALID_MAC;
            return;
        }
        off += 8;
        len -= 8;
        p->data_offset = (uint32_t) off;
        p->data_len = (uint32_t) len;
    }
    if (len < k->taglen) {                                             /* :1371-1377 */
        p->status = TLSREC_E_INVALID_MAC;
        return;
    }
    len -= k->taglen;
    p->data_len = (uint32_t) len;
    p->aead_pos = (uint32_t) off;
    p->aead_len = (uint32_t) len;
    /* the dynamic part is rec->ctr, or the explicit IV read from the record */
    tlsrec__nonce(p->nonce, k->iv, k->fixed_ivlen, ctr);
    p->aad_len = tlsrec__aad(p->aad, k->tls13, ctr, type, ver,
                             (uint32_t) (k->tls13 ? len + k->taglen : len), rec_cid, rec_cid_len);
}

#endif /* TLSREC_FRAME_H */
