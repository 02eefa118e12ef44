// Issue rate of the integer ops Poly1305 can be built from (one SIMD's view):
// 8 independent chains per lane, 16 waves/CU, cycles per wave-instruction.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools_bin/valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int ITER = 4096;

template <int V>
__global__ __launch_bounds__(1024) void valu(uint32_t *out, unsigned long long *clk)
{
    const unsigned long long c0 = clock64();
    uint32_t a[8];
    uint64_t w[8];
    double f[8];
    for (int i = 0; i < 8; i++) { a[i] = threadIdx.x * (i + 3); w[i] = a[i]; f[i] = a[i]; }
    const uint32_t m = threadIdx.x | 0x10001u;
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (V == 0) a[i] = a[i] + m;                                          // v_add_u32
            if (V == 2) a[i] = __umul24(a[i], m) + m;             // v_mad_u32_u24
            if (V == 3) a[i] = __umulhi(a[i] & 0xffffff, m & 0xffffff) ^ a[i];        // v_mul_hi_u32_u24
            if (V == 4) f[i] = __builtin_fma(f[i], 1.0000001, 0.5);               // v_fma_f64
            if (V == 5) a[i] = a[i] * m;                                          // v_mul_lo_u32
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s += a[i] + (uint32_t) w[i] + (uint32_t) f[i];
    out[blockIdx.x * 1024 + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = clock64() - c0;
}

__global__ __launch_bounds__(1024) void mad64(uint32_t *out, unsigned long long *clk)
{
    const unsigned long long c0 = clock64();
    uint64_t w[8];
    for (int i = 0; i < 8; i++) w[i] = threadIdx.x * (i + 3);
    const uint32_t m = threadIdx.x | 0x10001u;
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) w[i] = (uint64_t) (uint32_t) w[i] * m + w[i];   // v_mad_u64_u32
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s += (uint32_t) w[i] + (uint32_t) (w[i] >> 32);
    out[blockIdx.x * 1024 + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = clock64() - c0;
}

static void report(const char *name, unsigned long long *clk)
{
    unsigned long long h[256];
    (void) hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    double c = 0;
    for (int i = 0; i < 256; i++) c += h[i];
    c /= 256;
    /* 16 waves/CU = 4 per SIMD; instr per wave = ITER*8 */
    printf("%-22s %.2f SIMD cycles per wave-instruction\n", name, c / (ITER * 8.0 * 4));
}

int main()
{
    uint32_t *out;
    unsigned long long *clk;
    (void) hipMalloc(&out, 256 * 1024 * 4);
    (void) hipMalloc(&clk, 256 * 8);
    valu<0><<<256, 1024>>>(out, clk); (void) hipDeviceSynchronize();
    valu<0><<<256, 1024>>>(out, clk); (void) hipDeviceSynchronize(); report("v_add_u32", clk);
    mad64<<<256, 1024>>>(out, clk); (void) hipDeviceSynchronize(); report("v_mad_u64_u32", clk);
    valu<2><<<256, 1024>>>(out, clk); (void) hipDeviceSynchronize(); report("v_mad_u32_u24 (+add)", clk);
    valu<3><<<256, 1024>>>(out, clk); (void) hipDeviceSynchronize(); report("v_mul_hi_u32_u24 (+xor)", clk);
    valu<4><<<256, 1024>>>(out, clk); (void) hipDeviceSynchronize(); report("v_fma_f64", clk);
    valu<5><<<256, 1024>>>(out, clk); (void) hipDeviceSynchronize(); report("v_mul_lo_u32", clk);
    return 0;
}
