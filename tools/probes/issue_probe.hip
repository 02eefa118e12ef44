// VALU issue model on gfx950: cycles per wave-instruction of v_bitop3_b32 for
// C independent chains per lane at W waves per SIMD (one workgroup per CU).
//   hipcc --offload-arch=gfx950 -O3 tools/issue_probe.hip -o tools_bin/issue_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int ITER = 2048;

template <int C>
__global__ void issue(uint32_t *out, unsigned long long *clk)
{
    uint32_t a[C];
    for (int i = 0; i < C; i++) a[i] = threadIdx.x * (i + 3);
    uint32_t b = threadIdx.x ^ 0x1234, c = threadIdx.x * 7;
    __syncthreads();
    const unsigned long long c0 = clock64();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int i = 0; i < C; i++)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
    }
    const unsigned long long c1 = clock64();
    uint32_t s = 0;
    for (int i = 0; i < C; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = c1 - c0;
}

template <int C>
static void run(int waves_per_simd, uint32_t *out, unsigned long long *clk)
{
    const int threads = waves_per_simd * 4 * 64;
    issue<C><<<256, threads>>>(out, clk);
    hipDeviceSynchronize();
    unsigned long long h[256];
    hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256; i++) s += h[i];
    s /= 256;
    /* instructions per SIMD = waves_per_simd * ITER * 8 * C */
    printf("chains=%2d waves/SIMD=%d  %.2f SIMD cycles per wave-instruction\n", C, waves_per_simd,
           s / ((double) waves_per_simd * ITER * 8 * C));
}

int main()
{
    uint32_t *out; unsigned long long *clk;
    hipMalloc(&out, 256 * 1024 * 4);
    hipMalloc(&clk, 256 * 8);
    for (int w = 1; w <= 4; w *= 2) {
        run<1>(w, out, clk); run<2>(w, out, clk); run<4>(w, out, clk); run<8>(w, out, clk);
    }
    return 0;
}
