// Can the vector-memory path (L1/TCP) take AES T-table lookups beside the LDS?
// M of the 16 lookups per round read T0..T3 from a 4 KiB table in global
// memory (L1-resident); the rest read the 32-copy LDS T0/T1 image.  Prints
// ns per round per wave (lower = better) for M = 0..12; all variants compute
// the same AES rounds, checked against M = 0.
//   hipcc --offload-arch=gfx950 -O3 tools/tcp_probe.hip -o tools_bin/tcp_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }

typedef __attribute__((address_space(1))) const uint32_t gu32;

template <int M>
__device__ __forceinline__ uint32_t look(const uint8_t *lds, gu32 *gt, uint32_t w, uint32_t lb, int c, int j)
{
    if (c * 4 + j < M) {
        const uint32_t x = (w >> (8 * j)) & 0xffu;
        return gt[j * 256 + x];                       /* T_j[x] */
    }
    const uint32_t a = __builtin_amdgcn_perm(w, lb, 0x0C0C0000u | ((4u + j) << 8));
    const uint32_t v = *reinterpret_cast<const uint32_t *>(lds + a + (j & 1) * 128);
    return (j >= 2) ? rotl16(v) : v;                  /* T2 = rotl16(T0), T3 = rotl16(T1) */
}

template <int M>
__global__ __launch_bounds__(1024) void probe(const uint32_t *gtab, uint32_t *out, int iters)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
    gu32 *gt = (gu32 *) (uintptr_t) gtab;
    for (int t = threadIdx.x; t < 256 * 64; t += blockDim.x) {
        const int x = t >> 6, c = t & 63;             /* c < 32: T0 copy, else T1 copy */
        const uint32_t v = gtab[(c >> 5) * 256 + x];
        *reinterpret_cast<uint32_t *>(lds + x * 256 + (c >> 5) * 128 + (c & 31) * 4) = v;
    }
    __syncthreads();
    const uint32_t lb = (threadIdx.x & 31) << 2;
    uint32_t s0 = threadIdx.x * 0x9E3779B9u + blockIdx.x, s1 = s0 * 3u + 7u, s2 = s1 ^ 0x5bd1e995u, s3 = s2 * 5u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 14; r++) {
            const uint32_t t0 = xor3(look<M>(lds, gt, s0, lb, 0, 0), look<M>(lds, gt, s1, lb, 0, 1),
                                     xor3(look<M>(lds, gt, s2, lb, 0, 2), look<M>(lds, gt, s3, lb, 0, 3), r));
            const uint32_t t1 = xor3(look<M>(lds, gt, s1, lb, 1, 0), look<M>(lds, gt, s2, lb, 1, 1),
                                     xor3(look<M>(lds, gt, s3, lb, 1, 2), look<M>(lds, gt, s0, lb, 1, 3), r));
            const uint32_t t2 = xor3(look<M>(lds, gt, s2, lb, 2, 0), look<M>(lds, gt, s3, lb, 2, 1),
                                     xor3(look<M>(lds, gt, s0, lb, 2, 2), look<M>(lds, gt, s1, lb, 2, 3), r));
            const uint32_t t3 = xor3(look<M>(lds, gt, s3, lb, 3, 0), look<M>(lds, gt, s0, lb, 3, 1),
                                     xor3(look<M>(lds, gt, s1, lb, 3, 2), look<M>(lds, gt, s2, lb, 3, 3), r));
            s0 = t0; s1 = t1; s2 = t2; s3 = t3;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3;
}

template <int M>
static void run(const uint32_t *gt, uint32_t *out, uint32_t *ref, int grid, int iters)
{
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    probe<M><<<grid, 1024>>>(gt, out, iters);
    hipEventRecord(a);
    probe<M><<<grid, 1024>>>(gt, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    static uint32_t h[1 << 22], r0[1 << 22];
    const size_t n = (size_t) grid * 1024;
    hipMemcpy(h, out, n * 4, hipMemcpyDeviceToHost);
    if (M == 0) hipMemcpy(r0, out, n * 4, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) bad += h[i] != r0[i];
    const double waves = (double) grid * 16, rounds = (double) iters * 14;
    /* per CU: waves/256 waves, each `rounds` rounds */
    const double lookups = waves * 64 * rounds * 16;
    printf("M=%2d  %.3f ms  %.1f G lookups/s  %.2f lookups/clk/CU@2.1GHz  mismatches %zu\n", M, ms,
           lookups / ms / 1e6, lookups / (ms * 1e-3) / 256 / 2.1e9, bad);
    (void) ref;
}

int main()
{
    uint8_t sb[256];
    {   /* AES S-box */
        uint8_t p = 1, q = 1;
        do {
            p = p ^ (p << 1) ^ (p & 0x80 ? 0x1B : 0);
            q ^= q << 1; q ^= q << 2; q ^= q << 4; if (q & 0x80) q ^= 0x09;
            uint8_t x = q ^ (q << 1 | q >> 7) ^ (q << 2 | q >> 6) ^ (q << 3 | q >> 5) ^ (q << 4 | q >> 4);
            sb[p] = x ^ 0x63;
        } while (p != 1);
        sb[0] = 0x63;
    }
    uint32_t t[1024];
    for (int x = 0; x < 256; x++) {
        uint32_t s = sb[x], s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff, s3 = s2 ^ s;
        uint32_t t0 = s2 | (s << 8) | (s << 16) | (s3 << 24);
        for (int j = 0; j < 4; j++) t[j * 256 + x] = j ? ((t0 << (8 * j)) | (t0 >> (32 - 8 * j))) : t0;
    }
    uint32_t *gt, *out;
    hipMalloc(&gt, sizeof t);
    hipMemcpy(gt, t, sizeof t, hipMemcpyHostToDevice);
    const int grid = 256 * 4, iters = 200;
    hipMalloc(&out, (size_t) grid * 1024 * 4);
    run<0>(gt, out, nullptr, grid, iters);
    run<2>(gt, out, nullptr, grid, iters);
    run<4>(gt, out, nullptr, grid, iters);
    run<6>(gt, out, nullptr, grid, iters);
    run<8>(gt, out, nullptr, grid, iters);
    run<10>(gt, out, nullptr, grid, iters);
    run<12>(gt, out, nullptr, grid, iters);
    run<16>(gt, out, nullptr, grid, iters);
    return 0;
}
