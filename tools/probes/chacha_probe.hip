// ChaCha20 block throughput on gfx950 vs waves per SIMD: each lane runs ITER
// dependent blocks (the output feeds the next key, nothing folds), one
// workgroup of 256*W threads per CU = W waves per SIMD.  Wall time (HIP
// events) only: a wave's own s_memtime span is not the kernel's (the SQ
// issues oldest-first, so wave 0 finishes early).  The block is ~990 VALU
// instructions (320 v_add_u32, 320 v_xor_b32, 320 v_alignbit_b32, ...).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Imbedtls_amd/csrc tools/chacha_probe.hip -o varlib/chacha_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "tlsrec_device.h"

using namespace tlsrec;
constexpr int ITER = 64;

template <int W, int NB>
__global__ __launch_bounds__(256 * W) void blocks(uint32_t *out)
{
    uint32_t key[NB][8], nw[3] = { threadIdx.x, blockIdx.x, 7 };
    for (int b = 0; b < NB; b++)
        for (int i = 0; i < 8; i++) key[b][i] = threadIdx.x * (i + 1) + blockIdx.x + b;
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int b = 0; b < NB; b++) {
            uint32_t ks[16];
            chacha_block(key[b], (uint32_t) it + 1, nw, ks);
#pragma unroll
            for (int i = 0; i < 8; i++) key[b][i] ^= ks[i] + ks[8 + i];
        }
    }
    uint32_t s = 0;
    for (int b = 0; b < NB; b++)
        for (int i = 0; i < 8; i++) s += key[b][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int W, int NB>
static void run(uint32_t *out)
{
    blocks<W, NB><<<256, 256 * W>>>(out);
    (void) hipDeviceSynchronize();
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    (void) hipEventRecord(a);
    blocks<W, NB><<<256, 256 * W>>>(out);
    (void) hipEventRecord(b);
    (void) hipEventSynchronize(b);
    float ms;
    (void) hipEventElapsedTime(&ms, a, b);
    /* lane-blocks per second per SIMD (1024 SIMDs) */
    const double lane_blocks = 256.0 * 256 * W * ITER * NB;
    printf("W=%d waves/SIMD, %d blocks/lane in flight: %.3f ms, %.1f GB/s keystream, "
           "%.1f ns per wave-block per SIMD\n",
           W, NB, ms, lane_blocks * 64 / ms / 1e6, ms * 1e6 / (lane_blocks / 64 / 1024));
}

int main()
{
    uint32_t *out;
    (void) hipMalloc(&out, 256 * 1024 * 4);
    run<1, 1>(out);
    run<1, 2>(out);
    run<2, 1>(out);
    run<2, 2>(out);
    run<3, 1>(out);
    run<4, 1>(out);
    run<4, 2>(out);
    return 0;
}
