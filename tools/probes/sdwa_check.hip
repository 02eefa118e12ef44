// Checks rotl16(d ^ a) built from two SDWA XORs against the plain form.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(uint32_t *o, const uint32_t *a, const uint32_t *d)
{
    const int i = threadIdx.x;
    uint32_t r;
    asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n\t"
                 "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1"
                 : "=&v"(r) : "v"(d[i]), "v"(a[i]));
    o[2 * i] = r;
    uint32_t r2;
    asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0"
                 : "=&v"(r2) : "v"(d[i]), "v"(a[i]));
    o[2 * i + 1] = r2;
}
int main()
{
    uint32_t ha[64], hd[64], ho[128];
    for (int i = 0; i < 64; i++) { ha[i] = 0x01234567u * (i + 1); hd[i] = 0x89abcdefu ^ (i * 0x10001u); }
    uint32_t *a, *d, *o;
    (void) hipMalloc(&a, 256); (void) hipMalloc(&d, 256); (void) hipMalloc(&o, 512);
    (void) hipMemcpy(a, ha, 256, hipMemcpyHostToDevice);
    (void) hipMemcpy(d, hd, 256, hipMemcpyHostToDevice);
    k<<<1, 64>>>(o, a, d);
    (void) hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64; i++) {
        uint32_t x = ha[i] ^ hd[i], want = (x << 16) | (x >> 16);
        if (ho[2 * i] != want) bad++;
        if (i < 4) printf("a %08x d %08x want %08x got %08x first-only %08x\n", ha[i], hd[i], want, ho[2 * i], ho[2 * i + 1]);
    }
    printf("bad %d\n", bad);
    return 0;
}
