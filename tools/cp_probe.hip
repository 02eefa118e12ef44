// ChaCha20 block vs Poly1305 work per 64-B chunk (4 x p_mul), as used by
// tlsrec_chachapoly_kernel; 16 waves/CU, one workgroup per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Imbedtls_amd/csrc tools/cp_probe.hip -o tools_bin/cp_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "tlsrec_device.h"

using namespace tlsrec;
constexpr int ITER = 256;

template <int V>
__global__ __launch_bounds__(1024) void cp(uint32_t *out, unsigned long long *clk)
{
    const unsigned long long c0 = clock64(), w0 = wall_clock64();
    uint32_t key[8], nw[3] = { threadIdx.x, blockIdx.x, 7 };
    for (int i = 0; i < 8; i++) key[i] = threadIdx.x * (i + 1) + blockIdx.x;
    P5 acc = p_zero(), r = p_from_r(threadIdx.x, 5, 6, 7), r4 = p_mul(r, r);
    uint32_t sink = 0;
    for (int it = 0; it < ITER; it++) {
        if (V == 0 || V == 2) {
            uint32_t ks[16];
            chacha_block(key, (uint32_t) it + 1, nw, ks);
            for (int i = 0; i < 16; i++) sink += ks[i];
            key[it & 7] ^= ks[3];
        }
        if (V == 1 || V == 2) {
            P5 x = p_block(make_uint4(it, sink, 3, 4));
            for (int t = 1; t < 4; t++) x = p_add(p_mul(x, r), p_block(make_uint4(t, it, sink, 9)));
            acc = p_add(p_mul(acc, r4), x);
        }
    }
    for (int i = 0; i < 5; i++) sink += acc.v[i];
    out[blockIdx.x * 1024 + threadIdx.x] = sink;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = clock64() - c0;
        clk[2 * blockIdx.x + 1] = wall_clock64() - w0;
    }
}

template <int V>
static void run(const char *name, uint32_t *out, unsigned long long *clk)
{
    cp<V><<<256, 1024>>>(out, clk);
    (void) hipDeviceSynchronize();
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    (void) hipEventRecord(a);
    cp<V><<<1024, 1024>>>(out, clk);
    (void) hipEventRecord(b);
    (void) hipEventSynchronize(b);
    float ms = 0;
    (void) hipEventElapsedTime(&ms, a, b);
    unsigned long long h[2048];
    (void) hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
    double cs = 0, ws = 0;
    for (int i = 0; i < 1024; i++) { cs += h[2 * i]; ws += h[2 * i + 1]; }
    const double mhz = cs / ws * 100.0;
    const double chunks = 1024.0 * 1024 * ITER;   /* 64-B chunks */
    printf("%-24s %8.3f ms  %.1f GB/s of 64-B chunks  clock %.0f MHz  %.1f CU-cycles per chunk\n", name, ms,
           chunks * 64 / ms / 1e6, mhz, ms * 1e-3 * mhz * 1e6 * 256 / chunks);
}

int main()
{
    uint32_t *out;
    unsigned long long *clk;
    (void) hipMalloc(&out, 1024 * 1024 * 4);
    (void) hipMalloc(&clk, 2048 * 8);
    run<0>("chacha20 block", out, clk);
    run<1>("poly1305 4 blocks", out, clk);
    run<2>("both", out, clk);
    return 0;
}
