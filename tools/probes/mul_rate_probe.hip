/*
 * mul_rate_probe.hip -- issue cost of the multipliers Poly1305 can use on
 * gfx950, in cycles per wave instruction: v_mad_u64_u32 (the 26-bit limb
 * products), v_fma_f64 (exact below 2^53), v_cvt_f64_u32, against v_add_u32.
 * 8 independent chains per lane, 256 CUs x 8 waves; each kernel's time over
 * its instruction count gives wave-instructions per cycle per SIMD; plus the
 * 32-bit ALU forms the ChaCha20 quarter round and limb splitting use.
 *   hipcc --offload-arch=gfx950 -O3 mul_rate_probe.hip -o mul_rate_probe
 */
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 4096, CH = 8;

__global__ __launch_bounds__(256) void k_add(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_mad64(uint32_t *out, uint32_t seed)
{
    uint64_t a[CH];
    const uint32_t m = seed | 1u;
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++)
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a[c]) : "v"(m), "v"(m + c) : "vcc");
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= (uint32_t) a[c] ^ (uint32_t) (a[c] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma64(uint32_t *out, uint32_t seed)
{
    double a[CH];
    const double m = 1.0000001 + seed * 1e-9;
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a[c]) : "v"(m));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= (uint32_t) a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_cvt64(uint32_t *out, uint32_t seed)
{
    double a[CH];
    uint32_t v = seed + threadIdx.x;
    for (int c = 0; c < CH; c++) a[c] = 0;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(a[c]) : "v"(v + c));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= (uint32_t) a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}


__global__ __launch_bounds__(256) void k_op0(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op1(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op2(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op3(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op4(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op5(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op6(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op7(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op8(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_bfe_u32 %0, %0, 3, 22" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_op9(uint32_t *out, uint32_t seed)
{
    uint32_t a[CH];
    for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
    for (int i = 0; i < ITERS; i++)
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a[c]) : "v"(seed));
    uint32_t s = 0;
    for (int c = 0; c < CH; c++) s ^= a[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K> static float run(K k, uint32_t *d)
{
    hipEvent_t e0, e1;
    (void) hipEventCreate(&e0);
    (void) hipEventCreate(&e1);
    hipLaunchKernelGGL(k, 2048, 256, 0, 0, d, 7u);
    (void) hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, 2048, 256, 0, 0, d, 7u + r);
    (void) hipEventRecord(e1, 0);
    (void) hipEventSynchronize(e1);
    float ms = 0;
    (void) hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main()
{
    uint32_t *d = nullptr;
    (void) hipMalloc((void **) &d, 2048 * 256 * 4);
    hipDeviceProp_t pr;
    (void) hipGetDeviceProperties(&pr, 0);
    const double clk = pr.clockRate * 1e3;   /* Hz */
    const double winstr = 2048.0 * 4 * ITERS * CH;      /* wave instructions per launch */
    const double simds = pr.multiProcessorCount * 4.0;
    const char *names[] = { "v_add_u32", "v_mad_u64_u32", "v_fma_f64", "v_cvt_f64_u32", "v_xor_b32", "v_alignbit_b32", "v_perm_b32", "v_xad_u32", "v_add3_u32", "v_pk_add_u16_opsel_swap", "v_pk_add_u16", "v_mul_lo_u32", "v_bfe_u32", "v_bitop3_b32" };
    float t[] = { run(k_add, d), run(k_mad64, d), run(k_fma64, d), run(k_cvt64, d), run(k_op0, d), run(k_op1, d), run(k_op2, d), run(k_op3, d), run(k_op4, d), run(k_op5, d), run(k_op6, d), run(k_op7, d), run(k_op8, d), run(k_op9, d) };
    for (int i = 0; i < (int) (sizeof(t) / sizeof(t[0])); i++) {
        const double cyc = t[i] * 1e-3 * clk * simds / winstr;   /* SIMD cycles per wave instruction */
        printf("{\"instr\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_instr_at_max_clock\": %.2f}\n", names[i], t[i], cyc);
    }
    printf("{\"cus\": %d, \"clock_mhz\": %.0f, \"err\": \"%s\"}\n", pr.multiProcessorCount, clk / 1e6,
           hipGetErrorString(hipGetLastError()));
    return 0;
}
