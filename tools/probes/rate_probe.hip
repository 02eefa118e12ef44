// VALU issue cost of one wave-instruction on gfx950, 4 waves per SIMD x 8
// independent chains (issue_probe.hip's saturating point), for the Poly1305
// candidates: v_add_u32 (reference), v_mad_u64_u32, v_mul_lo_u32,
// v_mad_u32_u24, v_mul_hi_u32_u24, v_fma_f64.  Ratio to v_add_u32 = passes.
//   hipcc --offload-arch=gfx950 -O3 tools/rate_probe.hip -o rate_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int ITER = 1024, C = 8;

template <int OP>
__global__ __launch_bounds__(1024) void rate(uint64_t *out, unsigned long long *clk)
{
    uint64_t a[C];
    uint32_t u[C];
    double d[C];
    for (int i = 0; i < C; i++) { a[i] = threadIdx.x * (i + 3) + 1; u[i] = (uint32_t) a[i]; d[i] = 1.0 + threadIdx.x * 1e-9 * (i + 1); }
    uint32_t b = threadIdx.x ^ 0x1234, c = threadIdx.x * 7 + 1;
    double db = 1.0000001, dc = 1e-12;
    __syncthreads();
    const unsigned long long c0 = wall_clock64(), k0 = clock64();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int i = 0; i < C; i++) {
                if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(b));
                if constexpr (OP == 1) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
                if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[i]) : "v"(b));
                if constexpr (OP == 3) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(u[i]) : "v"(b), "v"(c));
                if constexpr (OP == 4) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(u[i]) : "v"(b));
                if constexpr (OP == 5) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[i]) : "v"(db), "v"(dc));
                if constexpr (OP == 6) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[i]) : "v"(b));
                if constexpr (OP == 7) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[i]) : "v"(b));
                if constexpr (OP == 8) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(u[i]));
                if constexpr (OP == 9) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(u[i]) : "v"(b), "v"(c));
                if constexpr (OP == 10) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(b), "v"(c));
                if constexpr (OP == 11) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(b), "v"(c));
                if constexpr (OP == 12) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(u[i]) : "v"(b));
            }
    }
    const unsigned long long c1 = wall_clock64(), k1 = clock64();
    uint64_t s = 0;
    for (int i = 0; i < C; i++) s += a[i] + u[i] + (uint64_t) d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = c1 - c0; clk[2 * blockIdx.x + 1] = k1 - k0; }
}

static const char *NAME[] = { "v_add_u32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mad_u32_u24", "v_mul_hi_u32_u24",
                              "v_fma_f64", "v_mul_hi_u32", "v_xor_b32", "v_alignbit_b32", "v_bitop3_b32", "v_perm_b32",
                              "v_add3_u32", "v_add_u32_e64" };

template <int OP>
static double run(uint64_t *out, unsigned long long *clk, int grid)
{
    hipEvent_t e0, e1;
    (void) hipEventCreate(&e0); (void) hipEventCreate(&e1);
    rate<OP><<<grid, 1024>>>(out, clk);
    (void) hipEventRecord(e0);
    rate<OP><<<grid, 1024>>>(out, clk);
    (void) hipEventRecord(e1);
    (void) hipEventSynchronize(e1);
    float ms = 0;
    (void) hipEventElapsedTime(&ms, e0, e1);
    /* wave-instructions per SIMD: grid/256 WGs per CU x 16 waves / 4 SIMDs x ITER x 8 x C */
    const double per_simd = (double) grid / 256 * 4 * ITER * 8 * C;
    const double ns = ms * 1e6 / per_simd;
    unsigned long long h[2];
    (void) hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    const double ghz = (double) h[1] / ((double) h[0] / 100e6) / 1e9;   /* clock64 ticks per wall second */
    printf("%-18s %.3f ms  %.3f ns per wave-instruction per SIMD  clock64 %.3f GHz -> %.2f ticks\n", NAME[OP], ms, ns,
           ghz, ns * ghz);
    return ns;
}

int main()
{
    uint64_t *out; unsigned long long *clk;
    const int grid = 256 * 2;
    (void) hipMalloc(&out, (size_t) grid * 1024 * 8);
    (void) hipMalloc(&clk, grid * 16);
    const double base = run<0>(out, clk, grid);
    const double r[12] = { run<1>(out, clk, grid), run<2>(out, clk, grid), run<3>(out, clk, grid),
                           run<4>(out, clk, grid), run<5>(out, clk, grid), run<6>(out, clk, grid),
                           run<7>(out, clk, grid), run<8>(out, clk, grid), run<9>(out, clk, grid),
                           run<10>(out, clk, grid), run<11>(out, clk, grid), run<12>(out, clk, grid) };
    for (int i = 0; i < 12; i++) printf("%-18s %.2f x v_add_u32\n", NAME[i + 1], r[i] / base);
    /* clock: s_memtime ticks over one v_add_u32 run (shader clock) */
    return 0;
}
