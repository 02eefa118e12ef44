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
