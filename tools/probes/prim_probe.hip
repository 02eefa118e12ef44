// Probe the real device primitives of tlsrec_device.h in isolation:
// aes_encrypt<14> and gmul<PI> loops, timed with events; run under
// rocprofv3 --pmc to read their LDS counters.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Imbedtls_amd/csrc tools/prim_probe.hip -o build/prim_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "tlsrec_device.h"

using namespace tlsrec;
constexpr int AESOFF = 32768;
constexpr int ITER = 256;

template <int V>
__global__ __launch_bounds__(1024) void prim(const uint32_t *rk_g, uint4 *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[32768 + 65536 + 256];
    const int tid = threadIdx.x;
    aes_fill_tables(lds + AESOFF, tid, 1024);
    for (int i = tid; i < 2048; i += 1024) reinterpret_cast<uint4 *>(lds)[i] = make_uint4(i, 3 * i, 5 * i, 7 * i);
    uint32_t *rkl = reinterpret_cast<uint32_t *>(lds + AESOFF + 65536);
    if (tid < 60) rkl[tid] = rk_g[tid];
    __syncthreads();
    const uint32_t lb = (uint32_t) (tid & 31) << 2;
    uint4 s = make_uint4(tid, blockIdx.x, 7, 9);
    for (int it = 0; it < ITER; it++) {
        if (V == 0) s = aes_encrypt<14, AESOFF>(lds, lb, rkl, s);                  // rk from LDS
        if (V == 1) s = aes_encrypt<14, AESOFF>(lds, lb, rk_g, s);                 // rk from global (uniform)
        if (V == 2) s = xor4(gmul<3>(lds, s), make_uint4(it, 1, 2, 3));
        if (V == 3) {   // decrypt-like: GHASH input independent of the AES output
            uint4 k = aes_encrypt<14, AESOFF>(lds, lb, rk_g, make_uint4(it, 5, 6, 7));
            s = xor4(gmul<3>(lds, s), k);
        }
        if (V == 4) {
            uint4 k = aes_encrypt<14, AESOFF>(lds, lb, rk_g, make_uint4(it, 5, 6, 7));
            s = xor4(gmul<3, 2, true>(lds, s), k);
        }
        if (V == 5) {
            uint4 k = aes_encrypt<14, AESOFF>(lds, lb, rk_g, make_uint4(it, 5, 6, 7));
            s = xor4(gmul<3, 4, false>(lds, s), k);
        }
        if (V == 6) {
            uint4 k = aes_encrypt<14, AESOFF>(lds, lb, rk_g, make_uint4(it, 5, 6, 7));
            s = xor4(gmul<3, 1, false>(lds, s), k);
        }
        if (V == 8) {   // fused, groups after rounds 1,4,7,10
            uint4 k, pr;
            aes_ghash<14, AESOFF, 3>(lds, lb, rk_g, make_uint4(it, 5, 6, 7), s, k, pr);
            s = xor4(pr, k);
        }
        if (V == 9) {   // fused, groups after rounds 2,5,8,11
            uint4 k, pr;
            aes_ghash<14, AESOFF, 3, 2, 1>(lds, lb, rk_g, make_uint4(it, 5, 6, 7), s, k, pr);
            s = xor4(pr, k);
        }
        if (V == 10) {  // fused, groups after rounds 1,2,3,4
            uint4 k, pr;
            aes_ghash<14, AESOFF, 3, 1, 1>(lds, lb, (const kconst_u32 *) (uintptr_t) rk_g, make_uint4(it, 5, 6, 7), s, k, pr);
            s = xor4(pr, k);
        }
        if (V == 7) {
            uint4 k = aes_encrypt<14, AESOFF>(lds, lb, rk_g, make_uint4(it, 5, 6, 7));
            s = xor4(gmul<3, 2, false>(lds, s), k);
        }
    }
    out[blockIdx.x * 1024 + tid] = s;
}

template <int V>
static float run(const uint32_t *rk, uint4 *out)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    prim<V><<<512, 1024>>>(rk, out);
    (void) hipEventRecord(a);
    prim<V><<<512, 1024>>>(rk, out);
    (void) hipEventRecord(b);
    (void) hipEventSynchronize(b);
    float ms = 0;
    (void) hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main()
{
    uint32_t *rk;
    uint4 *out;
    (void) hipMalloc(&rk, 256);
    (void) hipMemset(rk, 0x5a, 256);
    (void) hipMalloc(&out, 512 * 1024 * 16);
    const double blocks = 512.0 * 1024 * ITER;
    const char *nm[11] = {"aes256 rk in LDS", "aes256 rk global", "gmul<3>", "aes+gmul G4 mem",
                         "aes+gmul G2 mem", "aes+gmul G4 nomem", "aes+gmul G1 nomem", "aes+gmul G2 nomem",
                         "fused R0=1 RS=1", "fused R0=2 RS=1", "fused R0=1 kconst"};
    float t[11] = {run<0>(rk, out), run<1>(rk, out), run<2>(rk, out), run<3>(rk, out),
                   run<4>(rk, out), run<5>(rk, out), run<6>(rk, out), run<7>(rk, out),
                   run<8>(rk, out), run<9>(rk, out), run<10>(rk, out)};
    for (int v = 0; v < 11; v++)
        printf("P%d %-20s %8.3f ms  %.1f GB/s (16 B per block-op)\n", v, nm[v], t[v], blocks * 16 / t[v] / 1e6);
    return 0;
}
