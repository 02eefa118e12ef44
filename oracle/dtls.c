/*
 * dtls.c -- CPU restatement of the DTLS 1.2 (datagram transport) record read
 * and write loops of Mbed TLS 4.1.0 around the AEAD path.
 *
 * TEST INFRASTRUCTURE ONLY (scope and pinning: oracle.h, oracle/README.md).
 *
 * Read side, one connection's received datagrams in arrival order, as
 * repeated ssl_get_next_record (library/ssl_msg.c:4700-4900) would consume
 * them after the handshake:
 *   mbedtls_ssl_fetch_input, DTLS branch        ssl_msg.c:1877-2000 (a whole datagram per
 *                                                read, truncated to the in buffer; a 0-byte
 *                                                read is CONN_EOF; 1..12 bytes left after a
 *                                                record is INTERNAL_ERROR, :1921-1926)
 *   ssl_parse_record_header, DTLS branch        ssl_msg.c:3561-3776 (13-byte header, CID header
 *                                                of conf->cid_len bytes for type tls12_cid, type
 *                                                check :3529-3539, mbedtls_ssl_read_version
 *                                                :6215-6228 <= max_tls_version (TLS 1.2 for
 *                                                DTLS, ssl_tls.c:5514-5517), data_len != 0,
 *                                                datagram holds the record, epoch, anti-replay)
 *   ssl_get_next_record dispositions            ssl_msg.c:4727-4800 (UNEXPECTED_RECORD skips the
 *                                                record, EARLY_MESSAGE too once the handshake is
 *                                                over, any other header error drops the rest of
 *                                                the datagram), :4837-4873 (INVALID_MAC drops the
 *                                                datagram and counts against badmac_limit)
 *   ssl_prepare_record_content                  ssl_msg.c:3810-4017 (decrypt_buf, ignored
 *                                                UNEXPECTED_CID, type re-check :3914-3917,
 *                                                zero-length rules, no in_ctr step for DTLS,
 *                                                mbedtls_ssl_dtls_replay_update, IN_CONTENT_LEN)
 *   mbedtls_ssl_dtls_replay_check / _update     ssl_msg.c:3248-3306 (64-record window)
 * Write side, one connection's application data, one mbedtls_ssl_write per
 * record of at most max_frag bytes, each record flushed as its own datagram:
 *   mbedtls_ssl_write_record                    ssl_msg.c:2648-2793 (header type / FE FD /
 *                                                epoch+seq / out_cid / length, rec.buf =
 *                                                out_iv, 48-bit sequence increment with
 *                                                COUNTER_WRAPPING, :2749-2756 with ep_len 2)
 */
#include "oracle.h"

#include <string.h>

static uint64_t load48(const uint8_t *b)
{
    uint64_t v = 0;
    for (int i = 0; i < 6; i++) v = (v << 8) | b[i];
    return v;
}

/* mbedtls_ssl_dtls_replay_check, ssl_msg.c:3248-3271 (0 = acceptable) */
int orc_dtls_replay_check(const orc_dtls_state *st, const uint8_t ctr[8])
{
    const uint64_t seq = load48(ctr + 2);
    if (!st->anti_replay) return 0;
    if (seq > st->window_top) return 0;
    const uint64_t bit = st->window_top - seq;
    if (bit >= 64) return -1;
    if (st->window & ((uint64_t) 1 << bit)) return -1;
    return 0;
}

/* mbedtls_ssl_dtls_replay_update, ssl_msg.c:3277-3306 */
void orc_dtls_replay_update(orc_dtls_state *st, const uint8_t ctr[8])
{
    const uint64_t seq = load48(ctr + 2);
    if (!st->anti_replay) return;
    if (seq > st->window_top) {
        const uint64_t shift = seq - st->window_top;
        if (shift >= 64) {
            st->window = 1;
        } else {
            st->window <<= shift;
            st->window |= 1;
        }
        st->window_top = seq;
    } else {
        const uint64_t bit = st->window_top - seq;
        if (bit < 64) st->window |= (uint64_t) 1 << bit;
    }
}

/* mbedtls_ssl_read_version, datagram transport (ssl_msg.c:6215-6228) */
static uint16_t read_version_dtls(const uint8_t v[2])
{
    const uint16_t w = (uint16_t) ((v[0] << 8) | v[1]);
    return (uint16_t) ~(w - (w == 0xfeff ? 0x0202 : 0x0201));
}

/* Header of the record at b[0 .. rem): the checks of ssl_parse_record_header
 * that decide where the record ends (every failure here is INVALID_RECORD,
 * which drops the rest of the datagram).  Fills rec and returns 0. */
static int parse_header(const orc_dtls_state *st, uint8_t *b, size_t rem, orc_record *rec)
{
    size_t len_off = 11;                                           /* :3591-3596 */
    if (rem < len_off + 2) return ORC_ERR_SSL_INVALID_RECORD;      /* :3598-3606 */
    rec->type = b[0];
    rec->cid_len = 0;
    if (st->cid_len != 0 && rec->type == ORC_SSL_MSG_CID) {            /* :3616-3649 */
        len_off += st->cid_len;
        if (rem < len_off + 2) return ORC_ERR_SSL_INVALID_RECORD;
        rec->cid_len = st->cid_len;
        memcpy(rec->cid, b + 11, st->cid_len);
    } else if (rec->type < 20 || rec->type > 23) {                 /* :3651-3657 */
        return ORC_ERR_SSL_INVALID_RECORD;
    }
    rec->ver[0] = b[1];
    rec->ver[1] = b[2];
    if (read_version_dtls(b + 1) > ORC_VERSION_TLS1_2) return ORC_ERR_SSL_INVALID_RECORD;   /* :3662-3676 */
    memcpy(rec->ctr, b + 3, 8);                                    /* explicit sequence number :3683-3687 */
    rec->data_offset = len_off + 2;
    rec->data_len = ((size_t) b[len_off] << 8) | b[len_off + 1];
    rec->buf = b;
    rec->buf_len = rec->data_offset + rec->data_len;
    if (rec->data_len == 0) return ORC_ERR_SSL_INVALID_RECORD;     /* :3723-3726 */
    if (rem < rec->data_offset + rec->data_len) return ORC_ERR_SSL_INVALID_RECORD;   /* :3745-3753 */
    return 0;
}

/* the state-dependent part of ssl_parse_record_header: epoch (:3755-3768)
 * and the anti-replay check (:3769-3776) */
static int header_disposition(const orc_dtls_state *st, const orc_record *rec)
{
    const unsigned epoch = ((unsigned) rec->ctr[0] << 8) | rec->ctr[1];
    if (epoch != st->in_epoch)
        return epoch == (unsigned) st->in_epoch + 1 ? ORC_ERR_SSL_EARLY_MESSAGE : ORC_ERR_SSL_UNEXPECTED_RECORD;
    if (orc_dtls_replay_check(st, rec->ctr) != 0) return ORC_ERR_SSL_UNEXPECTED_RECORD;
    return 0;
}

static void list_rec(orc_dtls_rec *out, size_t max_out, orc_dtls_res *res, uint32_t dg, size_t off,
                     const orc_record *rec, int32_t disp)
{
    if (res->nrec < max_out) {
        orc_dtls_rec *o = &out[res->nrec];
        o->dgram = dg;
        o->off = (uint32_t) off;
        o->data_offset = (uint32_t) rec->data_offset;
        o->data_len = (uint32_t) rec->data_len;
        o->disp = disp;
        o->type = rec->type;
    }
    res->nrec++;
}

/* List the records of b[pos .. len) that a structural walk finds, without
 * processing them (the rest of a dropped datagram, or datagrams after the
 * connection's fatal error), with disposition `disp`. */
static void list_rest(const orc_dtls_state *st, uint8_t *b, size_t pos, size_t len, uint32_t dg, int32_t disp,
                      orc_dtls_rec *out, size_t max_out, orc_dtls_res *res)
{
    while (len - pos >= 13) {
        orc_record rec;
        if (parse_header(st, b + pos, len - pos, &rec) != 0) break;
        list_rec(out, max_out, res, dg, pos, &rec, disp);
        pos += rec.buf_len;
    }
}

int orc_dtls_decrypt(const orc_transform *t, orc_dtls_state *st, uint8_t *buf, const uint64_t *doff,
                     const uint32_t *dlen, size_t nd, orc_dtls_rec *out, size_t max_out, orc_dtls_res *res)
{
    memset(res, 0, sizeof(*res));
    if (t->tls_version != ORC_VERSION_TLS1_2) res->status = ORC_ERR_SSL_BAD_INPUT_DATA;   /* no DTLS 1.3 */
    for (size_t d = 0; d < nd; d++) {
        uint8_t *b = buf + doff[d];
        /* f_recv into the in buffer (in_hdr = in_buf for DTLS, :5264-5266) */
        const size_t len = dlen[d] < ORC_DTLS_MAX_DATAGRAM ? dlen[d] : ORC_DTLS_MAX_DATAGRAM;
        if (res->status) {
            list_rest(st, b, 0, len, (uint32_t) d, ORC_DTLS_NOT_REACHED, out, max_out, res);
            continue;
        }
        if (len == 0) {                                            /* f_recv returned 0 (:1968-1970) */
            res->status = ORC_ERR_SSL_CONN_EOF;
            continue;
        }
        size_t pos = 0;
        while (pos < len) {
            if (len - pos < 13) {                                  /* fetch_input(13) */
                if (pos == 0) {                                    /* a new datagram: the header check fails */
                    res->invalid_dgrams++;
                } else {                                           /* :1921-1926 */
                    res->status = ORC_ERR_SSL_INTERNAL_ERROR;
                }
                break;
            }
            orc_record rec;
            if (parse_header(st, b + pos, len - pos, &rec) != 0) { /* drop the rest of the datagram */
                res->invalid_dgrams++;
                break;
            }
            const size_t here = pos;
            pos += rec.buf_len;                                    /* next_record_offset (:4786, :4806) */
            int r = header_disposition(st, &rec);
            if (r != 0) {                                          /* skip this record only */
                list_rec(out, max_out, res, (uint32_t) d, here, &rec, r);
                continue;
            }
            int32_t disp = 0;
            r = orc_decrypt_buf(t, &rec);                          /* ssl_prepare_record_content */
            if (r == ORC_ERR_SSL_UNEXPECTED_CID && st->ignore_unexpected_cid) {   /* :3872-3879 */
                list_rec(out, max_out, res, (uint32_t) d, here, &rec, r);
                continue;
            }
            if (r == 0) {
                if (rec.type < 20 || rec.type > 23) {              /* :3914-3917 */
                    r = ORC_ERR_SSL_INVALID_RECORD;
                } else if (rec.data_len == 0) {                    /* :3920-3941 */
                    if (rec.type != 23) r = ORC_ERR_SSL_INVALID_RECORD;
                    else if (++st->nb_zero > 3) r = ORC_ERR_SSL_INVALID_MAC;
                } else {
                    st->nb_zero = 0;
                }
            }
            if (r == 0) {
                orc_dtls_replay_update(st, rec.ctr);               /* :4003-4007 */
                if (rec.data_len > ORC_IN_CONTENT_LEN) r = ORC_ERR_SSL_INVALID_RECORD;   /* :4011-4014 */
            }
            if (r == ORC_ERR_SSL_INVALID_MAC) {                    /* ssl_get_next_record :4837-4873 */
                disp = r;
                list_rec(out, max_out, res, (uint32_t) d, here, &rec, disp);
                if (st->badmac_limit != 0 && ++st->badmac_seen >= st->badmac_limit) {
                    res->status = r;
                } else {
                    list_rest(st, b, pos, len, (uint32_t) d, ORC_DTLS_DROPPED, out, max_out, res);
                }
                break;
            }
            if (r != 0) {                                          /* fatal */
                list_rec(out, max_out, res, (uint32_t) d, here, &rec, r);
                res->status = r;
                break;
            }
            list_rec(out, max_out, res, (uint32_t) d, here, &rec, 0);
            res->naccepted++;
        }
        if (res->status) {
            list_rest(st, b, pos, len, (uint32_t) d, ORC_DTLS_NOT_REACHED, out, max_out, res);
        } else {
            res->dgrams_done = (uint32_t) d + 1;
        }
    }
    return res->status;
}

size_t orc_dtls_record_wire(const orc_transform *t, size_t n)
{
    const size_t cid = t->out_cid_len;
    size_t body = t->ivlen - t->fixed_ivlen;                       /* explicit IV */
    if (cid) {
        const size_t g = t->granularity, inner = n + 1;            /* DTLSInnerPlaintext (:874-897) */
        body += inner + (g - inner % g) % g;
    } else {
        body += n;
    }
    return 13 + cid + body + t->taglen;
}

int orc_dtls_encrypt(const orc_transform *t, const uint8_t *pt, size_t len, uint8_t type, uint8_t out_ctr[8],
                     size_t max_frag, uint8_t *out, size_t out_cap, size_t *out_len, uint32_t *nrec)
{
    *nrec = 0;
    *out_len = 0;
    if (t->tls_version != ORC_VERSION_TLS1_2) return ORC_ERR_SSL_BAD_INPUT_DATA;
    size_t off = 0, pos = 0;
    const size_t cid = t->out_cid_len;
    const size_t head = t->ivlen - t->fixed_ivlen;                 /* out_msg - out_iv */
    const size_t hdr = 13 + cid;                                   /* out_iv - out_hdr (update_out_pointers) */
    while (off < len) {
        const size_t n = len - off < max_frag ? len - off : max_frag;
        const size_t wire = orc_dtls_record_wire(t, n);
        if (pos + wire > out_cap) return ORC_ERR_SSL_BUFFER_TOO_SMALL;
        uint8_t tmp[16 * 1024 + 512];
        memset(tmp, 0, sizeof(tmp));
        memcpy(tmp + head, pt + off, n);
        orc_record rec;
        rec.cid_len = 0;                                           /* set by encrypt_buf (:2686-2689) */
        memcpy(rec.ctr, out_ctr, 8);
        rec.type = type;
        rec.ver[0] = 0xfe;                                         /* mbedtls_ssl_write_version, DTLS 1.2 */
        rec.ver[1] = 0xfd;
        rec.buf = tmp;
        rec.buf_len = ORC_DTLS_OUT_BUFFER_LEN - hdr;               /* out_buf_len - (out_iv - out_buf) */
        rec.data_offset = head;
        rec.data_len = n;
        int r = orc_encrypt_buf(t, &rec);
        if (r) return r;
        if (rec.data_offset != 0) return ORC_ERR_SSL_INTERNAL_ERROR;   /* :2697-2700 */
        uint8_t *h = out + pos;
        h[0] = rec.type;                                           /* updated type (:2727) */
        h[1] = 0xfe;
        h[2] = 0xfd;
        memcpy(h + 3, out_ctr, 8);
        memcpy(h + 11, rec.cid, rec.cid_len);
        h[11 + rec.cid_len] = (uint8_t) (rec.data_len >> 8);
        h[12 + rec.cid_len] = (uint8_t) rec.data_len;
        memcpy(h + 13 + rec.cid_len, tmp, rec.data_len);
        pos += 13 + rec.cid_len + rec.data_len;
        off += n;
        (*nrec)++;
        *out_len = pos;
        int i;                                                     /* :2741-2756, ep_len = 2 */
        for (i = 8; i > 2; i--)
            if (++out_ctr[i - 1] != 0) break;
        if (i == 2) return ORC_ERR_SSL_COUNTER_WRAPPING;
    }
    return 0;
}
