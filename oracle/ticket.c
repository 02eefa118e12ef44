/*
 * ticket.c -- CPU restatement of the session-ticket protection of Mbed TLS
 * 4.1.0 (library/ssl_ticket.c), SURVEY.md 8(f)-4.
 *
 * TEST INFRASTRUCTURE ONLY (scope and pinning: oracle.h, oracle/README.md).
 *
 * Ticket layout (ssl_ticket.c:44-55, :233-236):
 *     key_name[4] || iv[12] || len16 || enc_state[len] || tag[16]
 * AAD = key_name || iv || len16 (TICKET_ADD_DATA_LEN = 18), nonce = iv.
 *   mbedtls_ssl_ticket_write  :210-306 (the IV comes from the caller's RNG,
 *                                       psa_generate_random at :255; the
 *                                       serialized session is already at
 *                                       start + 18, mbedtls_ssl_session_save)
 *   mbedtls_ssl_ticket_parse  :334-412 (key chosen by name :319-332, else
 *                                       SESSION_TICKET_EXPIRED; session_load
 *                                       is the caller's)
 * The AEAD is the ticket key's: AES-GCM, AES-CCM (16-byte tag) or
 * ChaCha20-Poly1305, the primitives of oracle.c.
 */
#include "oracle.h"

#include <string.h>

#define TKT_NAME 4
#define TKT_IV 12
#define TKT_LEN 2
#define TKT_TAG 16
#define TKT_MIN (TKT_NAME + TKT_IV + TKT_LEN + TKT_TAG)
#define TKT_AAD (TKT_NAME + TKT_IV + TKT_LEN)

/* The ticket key's AEAD: mbedtls_ssl_ticket_setup (ssl_ticket.c:188-209)
 * takes any PSA AEAD key type -- AES, ARIA and Camellia with GCM or CCM
 * (16-byte tag, :185), and ChaCha20-Poly1305. */
static int tkt_cipher_ok(int c)
{
    return (c >= ORC_CIPHER_AES_128_GCM && c <= ORC_CIPHER_AES_256_CCM) ||
           (c >= ORC_CIPHER_ARIA_128_GCM && c <= ORC_CIPHER_CAMELLIA_256_CCM);
}

static size_t tkt_keylen(int c)
{
    switch (c) {
        case ORC_CIPHER_AES_128_GCM: case ORC_CIPHER_AES_128_CCM: case ORC_CIPHER_ARIA_128_GCM:
        case ORC_CIPHER_ARIA_128_CCM: case ORC_CIPHER_CAMELLIA_128_GCM: case ORC_CIPHER_CAMELLIA_128_CCM:
            return 16;
        case ORC_CIPHER_AES_192_GCM: case ORC_CIPHER_AES_192_CCM: case ORC_CIPHER_ARIA_192_GCM:
        case ORC_CIPHER_ARIA_192_CCM: case ORC_CIPHER_CAMELLIA_192_GCM: case ORC_CIPHER_CAMELLIA_192_CCM:
            return 24;
        default: return 32;
    }
}

/* block cipher of the GCM / CCM code: 0 AES, 1 ARIA, 2 Camellia */
static int tkt_bc(int c)
{
    return c >= ORC_CIPHER_CAMELLIA_128_GCM ? 2 : (c >= ORC_CIPHER_ARIA_128_GCM ? 1 : 0);
}

static int tkt_is_ccm(int c)
{
    return (c >= ORC_CIPHER_AES_128_CCM && c <= ORC_CIPHER_AES_256_CCM) ||
           (c >= ORC_CIPHER_ARIA_128_CCM && c <= ORC_CIPHER_ARIA_256_CCM) || c >= ORC_CIPHER_CAMELLIA_128_CCM;
}

static void tkt_bc_setkey(orc_aes_ctx *a, int c, const uint8_t *key)
{
    const unsigned bits = (unsigned) tkt_keylen(c) * 8;
    const int bc = tkt_bc(c);
    if (bc == 2) orc_camellia_setkey_enc(a, key, bits);
    else if (bc == 1) orc_aria_setkey_enc(a, key, bits);
    else orc_aes_setkey_enc(a, key, bits);
}

static void tkt_seal(const orc_ticket_key *k, const uint8_t *aad, uint8_t *data, size_t len, uint8_t *tag)
{
    const uint8_t *iv = aad + TKT_NAME;
    if (k->cipher == ORC_CIPHER_CHACHA20_POLY1305) {
        orc_chachapoly_encrypt(k->key, iv, aad, TKT_AAD, data, len, data, tag);
    } else if (tkt_is_ccm(k->cipher)) {
        orc_aes_ctx a;
        tkt_bc_setkey(&a, k->cipher, k->key);
        orc_ccm_encrypt(&a, iv, aad, TKT_AAD, data, len, data, tag, TKT_TAG);
    } else {
        orc_gcm_ctx g;
        orc_gcm_setkey_ex(&g, k->key, (unsigned) tkt_keylen(k->cipher) * 8, tkt_bc(k->cipher));
        orc_gcm_encrypt(&g, iv, aad, TKT_AAD, data, len, data, tag, TKT_TAG);
    }
}

static int tkt_open(const orc_ticket_key *k, const uint8_t *aad, uint8_t *data, size_t len, const uint8_t *tag)
{
    const uint8_t *iv = aad + TKT_NAME;
    if (k->cipher == ORC_CIPHER_CHACHA20_POLY1305)
        return orc_chachapoly_decrypt(k->key, iv, aad, TKT_AAD, data, len, data, tag);
    if (tkt_is_ccm(k->cipher)) {
        orc_aes_ctx a;
        tkt_bc_setkey(&a, k->cipher, k->key);
        return orc_ccm_decrypt(&a, iv, aad, TKT_AAD, data, len, data, tag, TKT_TAG);
    }
    orc_gcm_ctx g;
    orc_gcm_setkey_ex(&g, k->key, (unsigned) tkt_keylen(k->cipher) * 8, tkt_bc(k->cipher));
    return orc_gcm_decrypt(&g, iv, aad, TKT_AAD, data, len, data, tag, TKT_TAG);
}

/* mbedtls_ssl_ticket_write, ssl_ticket.c:210-306 */
int orc_ticket_write(const orc_ticket_key keys[2], int active, uint8_t *start, size_t space, size_t clear_len,
                     size_t *tlen)
{
    if (space < TKT_MIN) return ORC_ERR_SSL_BUFFER_TOO_SMALL;             /* MBEDTLS_SSL_CHK_BUF_PTR :236 */
    const orc_ticket_key *k = &keys[active];
    if (!tkt_cipher_ok(k->cipher)) return ORC_ERR_SSL_BAD_INPUT_DATA;
    memcpy(start, k->name, TKT_NAME);                                      /* :253 */
    uint8_t *state = start + TKT_AAD;
    if (clear_len > space - TKT_AAD) return ORC_ERR_SSL_BUFFER_TOO_SMALL;   /* session_save into end - state */
    if (clear_len > 65535) return 0;                                      /* :262-266: ret is 0 here */
    start[16] = (uint8_t) (clear_len >> 8);                                /* :268 */
    start[17] = (uint8_t) clear_len;
    if (clear_len + TKT_TAG > space - TKT_AAD) return ORC_ERR_SSL_BUFFER_TOO_SMALL;   /* PSA output size */
    tkt_seal(k, start, state, clear_len, state + clear_len);              /* :271-279 */
    *tlen = TKT_MIN + clear_len;                                           /* :305 */
    return 0;
}

/* mbedtls_ssl_ticket_parse, ssl_ticket.c:334-412 (up to mbedtls_ssl_session_load) */
int orc_ticket_parse(const orc_ticket_key keys[2], uint8_t *buf, size_t len, size_t *clear_len)
{
    if (len < TKT_MIN) return ORC_ERR_SSL_BAD_INPUT_DATA;                  /* :356-358 */
    size_t enc_len = ((size_t) buf[16] << 8) | buf[17];                    /* :370 */
    if (len != TKT_MIN + enc_len) return ORC_ERR_SSL_BAD_INPUT_DATA;       /* :372-375 */
    const orc_ticket_key *k = NULL;
    for (int i = 0; i < 2; i++)                                           /* ssl_ticket_select_key :319-332 */
        if (memcmp(buf, keys[i].name, TKT_NAME) == 0) { k = &keys[i]; break; }
    if (k == NULL) return ORC_ERR_SSL_SESSION_TICKET_EXPIRED;               /* :378-381 */
    if (!tkt_cipher_ok(k->cipher)) return ORC_ERR_SSL_BAD_INPUT_DATA;
    uint8_t *ticket = buf + TKT_AAD;
    if (tkt_open(k, buf, ticket, enc_len, ticket + enc_len) != 0) {         /* :384-391 */
        memset(ticket, 0, enc_len);                                        /* PSA clears its output */
        return ORC_ERR_SSL_INVALID_MAC;
    }
    *clear_len = enc_len;
    return 0;
}
