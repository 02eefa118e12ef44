// Throughput probe for the bitsliced AES counter mode (tlsrec_bitslice.h):
// every lane makes ITER x 32 keystream blocks; mode 1 also writes the first
// 32 blocks of every lane for a CPU check.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Itools -Imbedtls_amd/csrc tools/bs_probe.hip -o tools_bin/bs_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "tlsrec_device.h"
#include "tlsrec_bitslice.h"

using namespace tlsrec;
constexpr int ITER = 32;

template <int W>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(2))) void bsp(const uint32_t *rk_g, uint32_t *out, unsigned long long *clk, int check)
{
    const unsigned long long c0c = clock64(), w0 = wall_clock64();
    const kconst_u32 *rk = (const kconst_u32 *) (uintptr_t) rk_g;
    const uint32_t gid = blockIdx.x * W * 64 + threadIdx.x;
    uint32_t sink = 0;
    for (int it = 0; it < ITER; it++) {
        uint32_t ks[4][32];
        bs::ctr32<14>(rk, 0, gid, 0x12345678u, 0x9abcdef0u, (uint32_t) it * 32, ks);
        if (check && it == 0) {
            for (int c = 0; c < 4; c++)
                for (int j = 0; j < 32; j++) out[(size_t) gid * 128 + 4 * j + c] = ks[c][j];
        }
        for (int c = 0; c < 4; c++)
            for (int j = 0; j < 32; j++) sink ^= ks[c][j] + j;
    }
    if (sink == 0x5a5a5a5au) out[0] = sink;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = clock64() - c0c;
        clk[2 * blockIdx.x + 1] = wall_clock64() - w0;
    }
}

int main(int argc, char **argv)
{
    const int grid = argc > 1 ? atoi(argv[1]) : 1024;
    uint32_t rk[60];
    for (int i = 0; i < 60; i++) rk[i] = 0x01020304u * (i + 1) ^ (0x9e3779b9u * i);
    uint32_t *d_rk, *d_out; unsigned long long *d_clk;
    hipMalloc(&d_rk, sizeof rk); hipMemcpy(d_rk, rk, sizeof rk, hipMemcpyHostToDevice);
    const size_t nl = (size_t) grid * 256;
    hipMalloc(&d_out, nl * 128 * 4);
    hipMalloc(&d_clk, grid * 16);
    bsp<4><<<grid, 256>>>(d_rk, d_out, d_clk, 1);
    hipDeviceSynchronize();
    /* dump first lanes for the CPU check */
    uint32_t *h = (uint32_t *) malloc(4 * 128 * 4);
    hipMemcpy(h, d_out + 0, 4 * 128 * 4, hipMemcpyDeviceToHost);
    /* host run of the same header (checked against FIPS-197 by bs_check) */
    int bad = 0;
    for (int l = 0; l < 4; l++) {
        uint32_t ks[4][32];
        bs::ctr32<14>(rk, 0, (uint32_t) l, 0x12345678u, 0x9abcdef0u, 0u, ks);
        for (int c = 0; c < 4; c++)
            for (int j = 0; j < 32; j++) bad += h[l * 128 + 4 * j + c] != ks[c][j];
    }
    printf("device vs host keystream mismatches: %d\n", bad);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    bsp<4><<<grid, 256>>>(d_rk, d_out, d_clk, 0);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    unsigned long long *hc = (unsigned long long *) malloc(grid * 16);
    hipMemcpy(hc, d_clk, grid * 16, hipMemcpyDeviceToHost);
    double cs = 0, ws = 0;
    for (int i = 0; i < grid; i++) { cs += hc[2 * i]; ws += hc[2 * i + 1]; }
    const double mhz = cs / ws * 100.0;
    const double blocks = (double) nl * ITER * 32;
    printf("grid=%d  %.3f ms  %.1f Gblocks/s = %.1f GB/s keystream, clock %.0f MHz, %.2f cycles/block/CU\n", grid, ms,
           blocks / ms / 1e6, blocks * 16 / ms / 1e6, mhz, ms * 1e-3 * mhz * 1e6 * 256 / blocks);
    return 0;
}
