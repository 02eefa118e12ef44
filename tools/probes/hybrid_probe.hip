// Does bitsliced AES on the VALU add throughput beside T-table AES on the LDS?
// One kernel, WT table waves + WB bitsliced waves per workgroup (one workgroup
// per CU, 256 VGPRs per wave), both pulling 32-KiB units (2048 counter blocks
// + GHASH + load/store) from one atomic counter until the buffer is done.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Itools -Imbedtls_amd/csrc tools/hybrid_probe.hip -o tools_bin/hybrid_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "tlsrec_device.h"
#include "tlsrec_bitslice.h"

using namespace tlsrec;
constexpr int AESOFF = 40960;   /* after 5 GHASH tables */

template <int WT, int WB, int NBT, int PRIO>
__device__ __forceinline__ void hyb_body(const uint32_t *rk_g, const uint32_t *rkr_g, const uint4 *src, uint4 *dst,
                                         uint32_t *ctr, uint32_t units, uint4 *sinkp, uint32_t *cnt)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[AESOFF + 65536];
    __shared__ uint32_t unit_sh[WT + WB];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    aes_fill_tables(lds + AESOFF, tid, (WT + WB) * 64);
    for (int i = tid; i < AESOFF / 16; i += (WT + WB) * 64) reinterpret_cast<uint4 *>(lds)[i] = make_uint4(i, 3 * i, 5 * i, 7 * i);
    __syncthreads();
    const uint32_t lb = (uint32_t) (lane & 31) << 2;
    /* table waves first at the VALU arbiter: their address ops feed the LDS */
    if (PRIO && (WB == 0 || wave < WT)) __builtin_amdgcn_s_setprio(3);
    uint4 sink = make_uint4(0, 0, 0, 0);
    uint32_t done = 0;
    for (;;) {
        if (lane == 0) unit_sh[wave] = atomicAdd(ctr, 1u);
        const uint32_t u = __builtin_amdgcn_readfirstlane(unit_sh[wave]);
        if (u >= units) break;
        done++;
        const uint4 *s = src + (size_t) u * 2048 + lane;
        uint4 *d = dst + (size_t) u * 2048 + lane;
        uint4 z = make_uint4(lane, u, 1, 2), xp = make_uint4(0, 0, 0, 0);
        if (WB == 0 || wave < WT) {
            const kconst_u32 *rk = (const kconst_u32 *) (uintptr_t) rkr_g;
            CtrCache cc = ctr_cache<AESOFF>(lds, lb, rk, lane, u, 7);
            uint4 zz[NBT], xx[NBT];
            for (int b = 0; b < NBT; b++) { zz[b] = z; xx[b] = xp; }
            for (int it = 0; it < 32 / NBT; it++) {
                uint32_t ctrw[NBT];
                uint4 y[NBT], ks[NBT], pr[NBT], blk[NBT];
#pragma unroll
                for (int b = 0; b < NBT; b++) {
                    ctrw[b] = bswap32(it * NBT + b + 2);
                    y[b] = xor4(zz[b], xx[b]);
                    blk[b] = gload16(reinterpret_cast<const uint8_t *>(s + (it * NBT + b) * 64));
                }
                aes_ghash_n<14, AESOFF, 4, NBT>(lds, lb, rk, cc, ctrw, y, ks, pr);
#pragma unroll
                for (int b = 0; b < NBT; b++) {
                    zz[b] = pr[b];
                    gstore16(reinterpret_cast<uint8_t *>(d + (it * NBT + b) * 64), xor4(blk[b], ks[b]));
                    xx[b] = blk[b];
                }
            }
            for (int b = 0; b < NBT; b++) sink = xor4(sink, xor4(zz[b], xx[b]));
        } else if constexpr (WB > 0) {
            const kconst_u32 *rk = (const kconst_u32 *) (uintptr_t) rk_g;
            uint32_t ks[4][32];
            bs::ctr32<14>(rk, 0, lane, u, 7, 0, ks);
#pragma unroll
            for (int j = 0; j < 32; j++) {
                const uint4 blk = gload16(reinterpret_cast<const uint8_t *>(s + j * 64));
                const uint4 o = make_uint4(blk.x ^ ks[0][j], blk.y ^ ks[1][j], blk.z ^ ks[2][j], blk.w ^ ks[3][j]);
                gstore16(reinterpret_cast<uint8_t *>(d + j * 64), o);
                z = gmul<4>(lds, xor4(z, xp));
                xp = blk;
            }
            sink = xor4(sink, xor4(z, xp));
        }
    }
    sinkp[blockIdx.x * (WT + WB) * 64 + tid] = sink;
    if (lane == 0) cnt[blockIdx.x * (WT + WB) + wave] = done;
}

template <int WT, int WB, int NBT, int PRIO>
__global__ __launch_bounds__((WT + WB) * 64) __attribute__((amdgpu_waves_per_eu(2))) void
hyb(const uint32_t *rk_g, const uint32_t *rkr_g, const uint4 *src, uint4 *dst, uint32_t *ctr, uint32_t units,
    uint4 *sinkp, uint32_t *cnt)
{
    hyb_body<WT, WB, NBT, PRIO>(rk_g, rkr_g, src, dst, ctr, units, sinkp, cnt);
}

template <int WT, int NBT>
__global__ __launch_bounds__(WT * 64) void tab(const uint32_t *rk_g, const uint32_t *rkr_g, const uint4 *src,
                                                uint4 *dst, uint32_t *ctr, uint32_t units, uint4 *sinkp, uint32_t *cnt)
{
    hyb_body<WT, 0, NBT, 0>(rk_g, rkr_g, src, dst, ctr, units, sinkp, cnt);
}

template <int WT, int WB, int NBT, int PRIO = 0>
static void run(const uint32_t *rk, const uint32_t *rkr, const uint4 *src, uint4 *dst, uint32_t *ctr, uint32_t units,
                uint4 *sink, uint32_t *cnt)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    float best = 1e9;
    for (int rep = 0; rep < 3; rep++) {
        (void) hipMemset(ctr, 0, 4);
        (void) hipEventRecord(a);
        if (WT + WB > 8)
            tab<WT + WB, NBT><<<256, (WT + WB) * 64>>>(rk, rkr, src, dst, ctr, units, sink, cnt);
        else
            hyb<WT, WB, NBT, PRIO><<<256, (WT + WB) * 64>>>(rk, rkr, src, dst, ctr, units, sink, cnt);
        (void) hipEventRecord(b);
        (void) hipEventSynchronize(b);
        float ms = 0;
        (void) hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    static uint32_t h[256 * 16];
    (void) hipMemcpy(h, cnt, 256 * (WT + WB) * 4, hipMemcpyDeviceToHost);
    double ut = 0, ub = 0;
    for (int g = 0; g < 256; g++)
        for (int w = 0; w < WT + WB; w++) (w < WT ? ut : ub) += h[g * (WT + WB) + w];
    const double blocks = (double) units * 2048;
    printf("PRIO=%d WT=%d WB=%d NBT=%d  %8.3f ms  %7.1f GB/s  units table %.0f%% bitsliced %.0f%%\n", PRIO, WT, WB, NBT, best,
           blocks * 16 / best / 1e6, 100 * ut / units, 100 * ub / units);
}

int main()
{
    uint32_t *rk, *rkr, *ctr, *cnt;
    uint4 *src, *dst, *sink;
    const uint32_t units = 65536;   /* x 32 KiB = 2 GiB */
    (void) hipMalloc(&rk, 256);
    (void) hipMemset(rk, 0x5a, 256);
    (void) hipMalloc(&rkr, 256);
    (void) hipMemset(rkr, 0x3c, 256);
    (void) hipMalloc(&ctr, 4);
    (void) hipMalloc(&cnt, 256 * 16 * 4);
    (void) hipMalloc(&sink, 256 * 1024 * 16);
    (void) hipMalloc(&src, (size_t) units * 32768);
    (void) hipMalloc(&dst, (size_t) units * 32768);
    (void) hipMemset(src, 0x33, (size_t) units * 32768);
    run<16, 0, 1>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<8, 0, 4>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<0, 8, 2>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<7, 1, 4, 1>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<6, 2, 4, 1>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<5, 3, 4, 1>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<4, 4, 4, 1>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<6, 2, 2, 1>(rk, rkr, src, dst, ctr, units, sink, cnt);
    run<4, 4, 2, 1>(rk, rkr, src, dst, ctr, units, sink, cnt);
    return 0;
}
