// Occupancy x ILP probe for the fused counter-mode AES + GHASH step:
// W waves per workgroup (one workgroup per CU), NB independent chains per lane.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Imbedtls_amd/csrc tools/ilp_probe.hip -o tools_bin/ilp_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "tlsrec_device.h"

using namespace tlsrec;
constexpr int AESOFF = 40960;   /* after 5 GHASH tables */
constexpr int ITER = 128;   /* x 8 lanes x 16 B = one 16 KiB record per lane group */

template <int W, int NB, int MEM>
__global__ __launch_bounds__(W * 64) void ilp(const uint32_t *rk_g, uint4 *out, unsigned long long *clk,
                                               const uint4 *src, uint4 *dst)
{
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    __shared__ __attribute__((aligned(16))) uint8_t lds[AESOFF + 65536];
    const int tid = threadIdx.x;
    aes_fill_tables(lds + AESOFF, tid, W * 64);
    for (int i = tid; i < AESOFF / 16; i += W * 64) reinterpret_cast<uint4 *>(lds)[i] = make_uint4(i, 3 * i, 5 * i, 7 * i);
    __syncthreads();
    const kconst_u32 *rk = (const kconst_u32 *) (uintptr_t) rk_g;
    const uint32_t lb = (uint32_t) (tid & 31) << 2;
    CtrCache cc = ctr_cache<AESOFF>(lds, lb, rk, tid, blockIdx.x, 7);
    uint4 z[NB], xp[NB];
    for (int b = 0; b < NB; b++) { z[b] = make_uint4(tid, b, 1, 2); xp[b] = make_uint4(0, 0, 0, 0); }
    uint4 sink = make_uint4(0, 0, 0, 0);
    /* record r = global wave * 8 + lane / 8, 16 KiB each (1024 x 16 B), lane q = lane % 8 */
    const size_t rec = ((size_t) blockIdx.x * W + (tid >> 6)) * 8 + ((tid & 63) >> 3);
    const size_t base = rec * 1024 + (tid & 7);
    for (int it = 0; it < ITER; it++) {
        uint32_t ctrw[NB];
        uint4 y[NB], ks[NB], pr[NB], blk[NB];
        for (int b = 0; b < NB; b++) {
            ctrw[b] = bswap32(it * NB + b + 2);
            y[b] = xor4(z[b], xp[b]);
            if (MEM) blk[b] = src[base + (size_t) (((it * NB + b) * 8) & 1023)];
        }
        aes_ghash_n<14, AESOFF, 4, NB>(lds, lb, rk, cc, ctrw, y, ks, pr);
        for (int b = 0; b < NB; b++) {
            z[b] = pr[b];
            if (MEM) {
                dst[base + (size_t) (((it * NB + b) * 8) & 1023)] = xor4(blk[b], ks[b]);
                xp[b] = blk[b];
            } else {
                xp[b] = ks[b];
                sink = xor4(sink, ks[b]);
            }
        }
    }
    for (int b = 0; b < NB; b++) sink = xor4(sink, z[b]);
    out[blockIdx.x * 1024 + tid] = sink;
    if (tid == 0) {
        const unsigned long long c1 = clock64(), w1 = wall_clock64();
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = w1 - w0;
    }
}

template <int W, int NB, int MEM>
static void run(const uint32_t *rk, uint4 *out, unsigned long long *clk, const uint4 *src, uint4 *dst, int grid)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    ilp<W, NB, MEM><<<grid, W * 64>>>(rk, out, clk, src, dst);
    (void) hipEventRecord(a);
    ilp<W, NB, MEM><<<grid, W * 64>>>(rk, out, clk, src, dst);
    (void) hipEventRecord(b);
    (void) hipEventSynchronize(b);
    float ms = 0;
    (void) hipEventElapsedTime(&ms, a, b);
    const double blocks = (double) grid * W * 64 * NB * ITER;
    unsigned long long h[2048];
    (void) hipMemcpy(h, clk, 2 * grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double cs = 0, ws = 0;
    for (int i = 0; i < grid; i++) { cs += h[2 * i]; ws += h[2 * i + 1]; }
    const double mhz = cs / ws * 100.0;   /* wall_clock64 ticks at 100 MHz */
    printf("MEM=%d W=%2d NB=%d grid=%d  %8.3f ms  %.1f GB/s  shader clock %.0f MHz  %.2f cycles/block/CU\n", MEM, W, NB, grid,
           ms, blocks * 16 / ms / 1e6, mhz, ms * 1e-3 * mhz * 1e6 * 256 / blocks);
}

int main()
{
    uint32_t *rk;
    uint4 *out;
    (void) hipMalloc(&rk, 256);
    (void) hipMemset(rk, 0x5a, 256);
    (void) hipMalloc(&out, 1024 * 1024 * 16);
    unsigned long long *clk;
    (void) hipMalloc(&clk, 2048 * sizeof(unsigned long long));
    uint4 *src, *dst;
    const size_t recs = (size_t) 1024 * 16 * 8;          /* grid x W(max 16) x 8 records */
    (void) hipMalloc(&src, recs * 16384);
    (void) hipMalloc(&dst, recs * 16384);
    (void) hipMemset(src, 0x33, recs * 16384);
    run<16, 1, 0>(rk, out, clk, src, dst, 1024);
    run<16, 1, 0>(rk, out, clk, src, dst, 1024);
    run<16, 1, 1>(rk, out, clk, src, dst, 1024);
    run<12, 1, 1>(rk, out, clk, src, dst, 1024);
    run<16, 2, 1>(rk, out, clk, src, dst, 1024);
    run<12, 2, 1>(rk, out, clk, src, dst, 1024);
    return 0;
}
