/* CPU check of mbedtls_amd/csrc/tlsrec_clmul.h (the table-free GF(2^128)
 * multiply the GCM kernels can use): a shared object with one entry point,
 * called by tests/test_clmul.py against the oracle's bitwise orc_gf128_mul. */
#include <stdint.h>
#include <string.h>

#include "tlsrec_clmul.h"

void clmul_check_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16])
{
    uint32_t a[4], b[4], r[4];
    memcpy(a, x, 16);   /* little-endian host: the kernels' uint4 words */
    memcpy(b, y, 16);
    tlsrec_gf128_mul(a, b, r);
    memcpy(out, r, 16);
}

/* the 4-bit position table of p (32 windows x 16 entries x 16 B) as the
 * paired GCM passes build it: lane (window k0 < 4, entry n) starts at
 * B_k0 and steps by X^16 to windows k0 + 4, k0 + 8, ... */
void clmul_check_gtab4(const uint8_t p[16], uint8_t out[8192])
{
    uint32_t a[4];
    memcpy(a, p, 16);
    for (uint32_t k0 = 0; k0 < 4; k0++)
        for (uint32_t n = 0; n < 16; n++) {
            uint64_t bh, bl;
            tlsrec_gtab4_base(a, k0, &bh, &bl);
            for (uint32_t k = k0; k < 32; k += 4) {
                uint64_t eh, el;
                uint32_t w[4];
                tlsrec_gtab4_entry(bh, bl, n, &eh, &el);
                tlsrec_g_to_words(eh, el, w);
                memcpy(out + k * 256 + n * 16, w, 16);
                tlsrec_gf128_shr(&bh, &bl, 16);
            }
        }
}

/* the same table from tlsrec_gtab4_quad, the r06 build of the paired GCM
 * passes: lane (window k, quarter q) makes entries 4q .. 4q + 3 */
void clmul_check_gtab4_quad(const uint8_t p[16], uint8_t out[8192])
{
    uint32_t a[4];
    memcpy(a, p, 16);
    for (uint32_t k = 0; k < 32; k++)
        for (uint32_t q = 0; q < 4; q++) {
            uint32_t w[4][4];
            tlsrec_gtab4_quad(a, k, q, w);
            memcpy(out + k * 256 + q * 64, w, 64);
        }
}
