// CPU check of the bitsliced AES counter mode (tlsrec_bitslice.h) against a
// byte-wise FIPS-197 AES: g++ -O2 -std=c++17 -Itools -Imbedtls_amd/csrc tools/bs_check.cpp -o /tmp/bs_check
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "tlsrec_bitslice.h"

static uint8_t S[256];
static uint8_t xt(uint8_t s) { return (uint8_t) ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)); }
static void gen_sbox()
{
    uint8_t ex[256], lg[256] = {0}, x = 1;
    for (int i = 0; i < 255; i++) { ex[i] = x; lg[x] = (uint8_t) i; x = (uint8_t) (xt(x) ^ x); }
    for (int a = 0; a < 256; a++) {
        uint8_t inv = a ? ex[(255 - lg[a]) % 255] : 0, s = inv, r = inv;
        for (int k = 0; k < 4; k++) { r = (uint8_t) ((r << 1) | (r >> 7)); s ^= r; }
        S[a] = s ^ 0x63;
    }
}
static void expand(const uint8_t *key, int nk, uint32_t *rk)
{
    const int nr = nk + 6, total = 4 * (nr + 1);
    for (int i = 0; i < nk; i++) rk[i] = key[4*i] | (key[4*i+1] << 8) | (key[4*i+2] << 16) | ((uint32_t) key[4*i+3] << 24);
    uint32_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = (t >> 8) | (t << 24);
            t = S[t & 255] | (S[(t >> 8) & 255] << 8) | (S[(t >> 16) & 255] << 16) | ((uint32_t) S[t >> 24] << 24);
            t ^= rcon; rcon = xt((uint8_t) rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = S[t & 255] | (S[(t >> 8) & 255] << 8) | (S[(t >> 16) & 255] << 16) | ((uint32_t) S[t >> 24] << 24);
        }
        rk[i] = rk[i - nk] ^ t;
    }
}
static void enc(const uint32_t *rk, int nr, uint8_t st[16])
{
    for (int i = 0; i < 16; i++) st[i] ^= (uint8_t) (rk[i / 4] >> (8 * (i % 4)));
    for (int r = 1; r <= nr; r++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++) for (int row = 0; row < 4; row++) t[4*c+row] = S[st[4*((c+row)&3)+row]];
        if (r != nr) for (int c = 0; c < 4; c++) {
            uint8_t a0 = t[4*c], a1 = t[4*c+1], a2 = t[4*c+2], a3 = t[4*c+3], all = a0^a1^a2^a3;
            t[4*c] ^= all ^ xt(a0^a1); t[4*c+1] ^= all ^ xt(a1^a2); t[4*c+2] ^= all ^ xt(a2^a3); t[4*c+3] ^= all ^ xt(a3^a0);
        }
        for (int i = 0; i < 16; i++) st[i] = t[i] ^ (uint8_t) (rk[4*r + i/4] >> (8 * (i % 4)));
    }
}
int main()
{
    gen_sbox();
    /* S-box circuit exhaustively: 256 values in 8 x 32-bit planes */
    for (int base = 0; base < 256; base += 32) {
        uint32_t x[8] = {0};
        for (int j = 0; j < 32; j++) for (int k = 0; k < 8; k++) x[k] |= (uint32_t) (((base + j) >> k) & 1) << j;
        tlsrec::bs::sbox(x);
        for (int j = 0; j < 32; j++) {
            int v = 0; for (int k = 0; k < 8; k++) v |= ((x[k] >> j) & 1) << k;
            if (v != S[base + j]) { printf("sbox mismatch at %d\n", base + j); return 1; }
        }
    }
    /* transpose */
    {
        uint32_t A[32], B[32];
        for (int i = 0; i < 32; i++) A[i] = B[i] = (uint32_t) rand() * 2654435761u ^ (uint32_t) rand();
        tlsrec::bs::transpose32(A);
        for (int i = 0; i < 32; i++) for (int j = 0; j < 32; j++)
            if (((A[i] >> j) & 1) != ((B[j] >> i) & 1)) { printf("transpose mismatch %d %d\n", i, j); return 1; }
    }
    /* FIPS-197 C.3 */
    uint8_t key[32]; for (int i = 0; i < 32; i++) key[i] = (uint8_t) i;
    uint32_t rk[60]; expand(key, 8, rk);
    uint8_t st[16]; for (int i = 0; i < 16; i++) st[i] = (uint8_t) (i * 0x11);
    enc(rk, 14, st);
    static const uint8_t c3[16] = {0x8e,0xa2,0xb7,0xca,0x51,0x67,0x45,0xbf,0xea,0xfc,0x49,0x90,0x4b,0x49,0x60,0x89};
    if (memcmp(st, c3, 16)) { printf("byte AES wrong\n"); return 1; }
    /* counter mode, random keys / nonces / bases, AES-128 and AES-256 */
    int fails = 0;
    for (int trial = 0; trial < 200; trial++) {
        const int nk = (trial & 1) ? 8 : 4, nr = nk + 6;
        for (int i = 0; i < 32; i++) key[i] = (uint8_t) rand();
        expand(key, nk, rk);
        uint32_t n[3] = { (uint32_t) rand() ^ ((uint32_t) rand() << 16), (uint32_t) rand() ^ ((uint32_t) rand() << 16), (uint32_t) rand() ^ ((uint32_t) rand() << 16) };
        uint32_t c0 = (uint32_t) (rand() % 2048) * 32;
        uint32_t out[4][32];
        if (nr == 14) tlsrec::bs::ctr32<14>(rk, S, n[0], n[1], n[2], c0, out);
        else tlsrec::bs::ctr32<10>(rk, S, n[0], n[1], n[2], c0, out);
        for (int j = 0; j < 32; j++) {
            uint8_t b[16];
            for (int i = 0; i < 12; i++) b[i] = (uint8_t) (n[i / 4] >> (8 * (i % 4)));
            const uint32_t ctr = c0 + j;
            b[12] = (uint8_t) (ctr >> 24); b[13] = (uint8_t) (ctr >> 16); b[14] = (uint8_t) (ctr >> 8); b[15] = (uint8_t) ctr;
            enc(rk, nr, b);
            for (int c = 0; c < 4; c++) {
                uint32_t w = b[4*c] | (b[4*c+1] << 8) | (b[4*c+2] << 16) | ((uint32_t) b[4*c+3] << 24);
                if (w != out[c][j]) { fails++; break; }
            }
        }
    }
    printf("ctr32 fails: %d\n", fails);
    return fails != 0;
}
