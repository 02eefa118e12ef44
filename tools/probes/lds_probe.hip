// LDS access-pattern probe for the AES T-table / GHASH table layouts.
// Each variant does ITER x 16 dependent-free LDS lookups per lane with the
// address pattern named below; run under rocprofv3 --pmc SQ_LDS_BANK_CONFLICT.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o build/lds_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITER 4096

template <int V>
__global__ __launch_bounds__(1024) void probe(const uint32_t *seed, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[131072];
    for (int i = threadIdx.x; i < 131072 / 16; i += 1024)
        reinterpret_cast<uint4 *>(lds)[i] = make_uint4(i, i * 3, i * 5, i * 7);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t x = seed[blockIdx.x * 1024 + threadIdx.x];
    const uint32_t lb = (lane & 31) << 2;
    uint32_t acc = 0;
    uint4 acc4 = make_uint4(0, 0, 0, 0);
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            uint32_t byte = (x >> ((k & 3) * 8)) & 0xff;
            const uint32_t kofs = (uint32_t) k * 2048;   /* distinct table per k, same banks */
            if (V == 0) {        // current: 32 copies, row stride 256 B, copy = lane&31
                acc ^= *reinterpret_cast<const uint32_t *>(lds + kofs + (byte << 8) + lb + (k & 1) * 128);
            } else if (V == 1) { // 32 copies, row stride 128 B
                acc ^= *reinterpret_cast<const uint32_t *>(lds + kofs + (byte << 7) + lb);
            } else if (V == 2) { // no data dependence: lane-distinct fixed addresses
                acc ^= *reinterpret_cast<const uint32_t *>(lds + kofs + lb + (k << 8));
            } else if (V == 3) { // 64 copies, copy = lane
                acc ^= *reinterpret_cast<const uint32_t *>(lds + (kofs & 0x3fff) + (byte << 8) + (lane << 2));
            } else if (V == 4) { // GHASH: 16-entry x 16 B windows, random nibble
                uint32_t n = (x >> (k * 2)) & 0xf0;
                uint4 t = *reinterpret_cast<const uint4 *>(lds + n + k * 256);
                acc4.x ^= t.x; acc4.y ^= t.y; acc4.z ^= t.z; acc4.w ^= t.w;
            } else if (V == 5) { // broadcast b128
                uint4 t = *reinterpret_cast<const uint4 *>(lds + k * 16);
                acc4.x ^= t.x; acc4.y ^= t.y; acc4.z ^= t.z; acc4.w ^= t.w;
            } else if (V == 6) { // unreplicated 1 KiB table
                acc ^= *reinterpret_cast<const uint32_t *>(lds + kofs + (byte << 2));
            } else if (V == 8) { // plain ds_read_b32 (distinct bytes -> no read2 pairing), copy = lane&31
                uint32_t b2 = (x >> k) & 0xff;
                acc ^= *reinterpret_cast<const uint32_t *>(lds + (b2 << 8) + lb + (k & 1) * 128);
            } else if (V == 9) { // plain ds_read_b32, 64 copies, copy = lane
                uint32_t b2 = (x >> k) & 0xff;
                acc += *reinterpret_cast<const uint32_t *>(lds + (b2 << 8) + (lane << 2));
            } else if (V == 10) { // plain b32, copy = lane&31, lanes 32-63 shifted to other half-row
                uint32_t b2 = (x >> k) & 0xff;
                acc += *reinterpret_cast<const uint32_t *>(lds + (b2 << 8) + lb + ((lane >> 5) << 7));
            } else if (V == 7) { // 32 copies, but copy = lane>>1 (pairs share)
                acc ^= *reinterpret_cast<const uint32_t *>(lds + kofs + (byte << 8) + ((lane >> 1) << 2));
            }
        }
        x = x * 1664525u + 1013904223u + acc;
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc ^ acc4.x ^ acc4.y ^ acc4.z ^ acc4.w;
}

template <int V>
static float run(const uint32_t *seed, uint32_t *out, int grid)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    probe<V><<<grid, 1024>>>(seed, out);
    hipEventRecord(a);
    probe<V><<<grid, 1024>>>(seed, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main()
{
    const int grid = 256;
    uint32_t *seed, *out;
    hipMalloc(&seed, grid * 1024 * 4);
    hipMalloc(&out, grid * 1024 * 4);
    uint32_t *h = (uint32_t *) malloc(grid * 1024 * 4);
    for (int i = 0; i < grid * 1024; i++) h[i] = i * 2654435761u;
    hipMemcpy(seed, h, grid * 1024 * 4, hipMemcpyHostToDevice);
    const double lookups = (double) grid * 1024 * ITER * 16;
    float t[11];
    t[0] = run<0>(seed, out, grid);
    t[1] = run<1>(seed, out, grid);
    t[2] = run<2>(seed, out, grid);
    t[3] = run<3>(seed, out, grid);
    t[4] = run<4>(seed, out, grid);
    t[5] = run<5>(seed, out, grid);
    t[6] = run<6>(seed, out, grid);
    t[7] = run<7>(seed, out, grid);
    t[8] = run<8>(seed, out, grid);
    t[9] = run<9>(seed, out, grid);
    t[10] = run<10>(seed, out, grid);
    const char *names[11] = {"b32 32copies stride256 (current AES)", "b32 32copies stride128",
                            "b32 fixed lane-distinct", "b32 64copies lane", "b128 ghash window",
                            "b128 broadcast", "b32 unreplicated 1KiB", "b32 lane-pairs share copy",
                            "plain b32 copy=lane&31", "plain b32 64 copies copy=lane", "plain b32 lane&31 + half-row by lane>>5"};
    for (int v = 0; v < 11; v++)
        printf("V%d %-40s %8.3f ms  %.2f Glookups/s  %.3f lookups/clk/CU@2.4GHz\n", v, names[v], t[v],
               lookups / t[v] / 1e6, lookups / (t[v] * 1e-3) / 256 / 2.4e9);
    return 0;
}
