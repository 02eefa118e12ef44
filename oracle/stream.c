/*
 * stream.c -- CPU restatement of the TLS (stream transport) record read and
 * write loops of Mbed TLS 4.1.0 around the AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY (scope and pinning: oracle.h, oracle/README.md).
 *
 * Read side, one connection's received bytes, as repeated
 * ssl_get_next_record (library/ssl_msg.c:4700-4900) would consume them:
 *   mbedtls_ssl_fetch_input size check          ssl_msg.c:~2208 (nb_want > in_buf_len - hdr off:
 *                                                BAD_INPUT_DATA)
 *   ssl_parse_record_header (TLS branch)        ssl_msg.c:3561-3776 (type check :3529-3539,
 *                                                version <= max_tls_version, data_len != 0)
 *   ssl_prepare_record_content                  ssl_msg.c:3810-4017 (TLS 1.3 CCS passes undecrypted,
 *                                                decrypt_buf, zero-length rules, in_ctr
 *                                                increment + COUNTER_WRAPPING, IN_CONTENT_LEN)
 * Write side, one connection's application data, as mbedtls_ssl_write called
 * until every byte is sent (one record of at most max_frag bytes per call):
 *   mbedtls_ssl_write_record                    ssl_msg.c:2648-2793 (version 0x0303 on the wire
 *                                                for TLS 1.3, rec.buf = out_iv, header length =
 *                                                protected length, cur_out_ctr increment)
 */
#include "oracle.h"

#include <string.h>

static int bump_ctr(uint8_t ctr[8])
{
    /* ssl_msg.c:3954-3963 / :2749-2756, TLS: mbedtls_ssl_ep_len() == 0 */
    int i;
    for (i = 8; i > 0; i--)
        if (++ctr[i - 1] != 0) break;
    return i == 0 ? ORC_ERR_SSL_COUNTER_WRAPPING : 0;
}

int orc_stream_decrypt(const orc_transform *t, uint8_t *buf, size_t len, const uint8_t in_ctr[8], uint8_t nb_zero,
                       size_t max_record, int max_version, orc_stream_rec *out, size_t max_out,
                       orc_stream_res *res)
{
    memset(res, 0, sizeof(*res));
    memcpy(res->in_ctr, in_ctr, 8);
    res->nb_zero = nb_zero;
    size_t pos = 0;
    for (;;) {
        if (len - pos < 5) break;                                   /* fetch_input(5): wait for more */
        uint8_t *hdr = buf + pos;
        const uint8_t type = hdr[0];
        if (type != 20 && type != 21 && type != 22 && type != 23) { /* ssl_check_record_type */
            res->status = ORC_ERR_SSL_INVALID_RECORD;
            break;
        }
        const int ver = (hdr[1] << 8) | hdr[2];
        if (ver > max_version) {                                    /* tls_version > max_tls_version */
            res->status = ORC_ERR_SSL_INVALID_RECORD;
            break;
        }
        const size_t dlen = ((size_t) hdr[3] << 8) | hdr[4];
        if (dlen == 0) {                                            /* ssl_msg.c:3723-3726 */
            res->status = ORC_ERR_SSL_INVALID_RECORD;
            break;
        }
        if (5 + dlen > max_record) {                                /* fetch_input(rec.buf_len) */
            res->status = ORC_ERR_SSL_BAD_INPUT_DATA;
            break;
        }
        if (len - pos < 5 + dlen) break;                            /* incomplete record: wait */
        orc_record rec;
        rec.cid_len = 0;   /* no DTLS connection ID on this path */
        memcpy(rec.ctr, res->in_ctr, 8);
        rec.type = type;
        rec.ver[0] = hdr[1];
        rec.ver[1] = hdr[2];
        rec.buf = hdr;
        rec.buf_len = 5 + dlen;
        rec.data_offset = 5;
        rec.data_len = dlen;
        int ccs = t->tls_version == ORC_VERSION_TLS1_3 && type == 20;
        if (!ccs) {
            int r = orc_decrypt_buf(t, &rec);
            if (r) {
                res->status = r;
                break;
            }
            /* the content type may change in decryption (TLS 1.3 / CID inner
             * plaintext): re-checked, fatal this time (ssl_msg.c:3914-3917) */
            if (rec.type != 20 && rec.type != 21 && rec.type != 22 && rec.type != 23) {
                res->status = ORC_ERR_SSL_INVALID_RECORD;
                break;
            }
            if (rec.data_len == 0) {
                if (t->tls_version == ORC_VERSION_TLS1_2 && rec.type != 23) {
                    res->status = ORC_ERR_SSL_INVALID_RECORD;
                    break;
                }
                if (++res->nb_zero > 3) {
                    res->status = ORC_ERR_SSL_INVALID_MAC;
                    break;
                }
            } else {
                res->nb_zero = 0;
            }
            r = bump_ctr(res->in_ctr);
            if (r) {
                res->status = r;
                break;
            }
        }
        if (rec.data_len > ORC_IN_CONTENT_LEN) {
            res->status = ORC_ERR_SSL_INVALID_RECORD;
            break;
        }
        if (res->nrec < max_out) {
            out[res->nrec].off = (uint32_t) pos;
            out[res->nrec].data_offset = (uint32_t) rec.data_offset;
            out[res->nrec].data_len = (uint32_t) rec.data_len;
            out[res->nrec].type = rec.type;
        }
        res->nrec++;
        pos += 5 + dlen;
        res->consumed = (uint32_t) pos;
    }
    return res->status;
}

size_t orc_stream_record_wire(const orc_transform *t, size_t n)
{
    size_t body;
    if (t->tls_version == ORC_VERSION_TLS1_3) {
        size_t g = t->granularity;
        size_t inner = n + 1;
        body = inner + (g - inner % g) % g + t->taglen;
    } else {
        body = (t->ivlen - t->fixed_ivlen) + n + t->taglen;
    }
    return 5 + body;
}

int orc_stream_encrypt(const orc_transform *t, const uint8_t *pt, size_t len, uint8_t type, uint8_t out_ctr[8],
                       size_t max_frag, size_t out_buf_space, uint8_t *out, size_t out_cap, size_t *out_len,
                       uint32_t *nrec)
{
    size_t off = 0, pos = 0;
    *nrec = 0;
    *out_len = 0;
    const size_t head = t->ivlen - t->fixed_ivlen;                  /* out_msg - out_iv (explicit IV) */
    while (off < len) {
        const size_t n = len - off < max_frag ? len - off : max_frag;
        const size_t wire = orc_stream_record_wire(t, n);
        if (pos + wire > out_cap) return ORC_ERR_SSL_BUFFER_TOO_SMALL;
        uint8_t tmp[16 * 1024 + 512];
        memset(tmp, 0, sizeof(tmp));
        memcpy(tmp + head, pt + off, n);
        orc_record rec;
        rec.cid_len = 0;   /* no DTLS connection ID on this path */
        memcpy(rec.ctr, out_ctr, 8);
        rec.type = type;
        rec.ver[0] = 3;                                             /* TLS 1.3 writes 0x0303 (:2669-2674) */
        rec.ver[1] = 3;
        rec.buf = tmp;
        rec.buf_len = out_buf_space;
        rec.data_offset = head;
        rec.data_len = n;
        int r = orc_encrypt_buf(t, &rec);
        if (r) return r;
        if (rec.data_offset != 0) return ORC_ERR_SSL_INTERNAL_ERROR;   /* :2704-2707 */
        uint8_t *h = out + pos;
        h[0] = rec.type;
        h[1] = 3;
        h[2] = 3;
        h[3] = (uint8_t) (rec.data_len >> 8);
        h[4] = (uint8_t) rec.data_len;
        memcpy(h + 5, tmp, rec.data_len);
        pos += 5 + rec.data_len;
        off += n;
        (*nrec)++;
        *out_len = pos;
        r = bump_ctr(out_ctr);
        if (r) return r;
    }
    return 0;
}

/* The read side of mbedtls_ssl_read over a connection's accepted records:
 * ssl_read_application_data (ssl_msg.c:5627-5650) copies at most the
 * caller's remaining space from each application-data record in order and
 * zeroizes the bytes it handed out (mbedtls_platform_zeroize(in_offt, n));
 * a record only partly consumed keeps its tail (in_offt += n).  Records of
 * other content types are left to the caller (not application data). */
int orc_stream_read(uint8_t *buf, const orc_stream_rec *recs, size_t nrec, uint8_t *out, size_t cap,
                    size_t *copied, size_t *records, size_t *left)
{
    size_t done = 0, full = 0, rest = 0;
    for (size_t k = 0; k < nrec; k++) {
        if (recs[k].type != 23) {
            full++;
            continue;
        }
        uint8_t *src = buf + recs[k].off + recs[k].data_offset;
        size_t n = recs[k].data_len < cap - done ? recs[k].data_len : cap - done;
        memcpy(out + done, src, n);
        memset(src, 0, n);
        done += n;
        if (n < recs[k].data_len) {
            rest = recs[k].data_len - n;
            break;
        }
        full++;
    }
    *copied = done;
    *records = full;
    *left = rest;
    return 0;
}
