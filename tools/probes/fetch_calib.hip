// FETCH_SIZE / WRITE_SIZE calibration for the record kernels' access shapes
// (MI355X_MICROARCH.md documents the x2 FETCH_SIZE correction
// only for wide coalesced 16 B/lane streaming reads; "other access widths are
// uncalibrated").  Each kernel below reads (or writes) a known set of 128-B
// lines of a 1 GiB region -- past the 256 MiB Infinity Cache -- in the
// pattern of one of the engine's kernels, and writes 16 B per thread of
// results (reads) or nothing else (writes).  The host prints, per kernel, the
// bytes of the lines it touches; tools/probes/fetch_calib.py divides them by
// the counters of a rocprofv3 --pmc pass.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/fetch_calib tools/probes/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d DIR -o run --output-format csv -- tools/probes/fetch_calib
//
// Shapes (L lanes per record, 16 B per lane per step, lane q takes blocks
// q, q+L, ...; G = steps of a line group loaded together):
//   wide      64 lanes read 1 KiB contiguous per instruction (the guide's case)
//   rec8      c2: L = 8, 16 512-B record stride, one 128-B line per record per step
//   rec2g4    c4s GCM half: L = 2, 1 536-B stride, 4-step line groups (one line per group)
//   rec4g2    L = 4, 2-step line groups
//   rec2g1    L = 2 without groups: 32 B of a line per record per step
//   rec2mis   rec2g4 with records starting 0..127 B into their slot (stream / DTLS)
//   dword     4 B per lane, consecutive lanes consecutive
//   w_wide / w_rec2g4 / w_rec8   the same shapes as 16-B stores
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static constexpr size_t REGION = 1ull << 30;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 glob_u32x4;
typedef __attribute__((address_space(1))) uint32_t glob_u32;

__device__ __forceinline__ uint4 ld16(const uint8_t *p)
{
    const u32x4 v = *(const glob_u32x4 *) (uintptr_t) p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void st16(uint8_t *p, uint4 v)
{
    u32x4 w = { v.x, v.y, v.z, v.w };
    *(glob_u32x4 *) (uintptr_t) p = w;
}

template <int L, int G>
__device__ __forceinline__ void rec_read(const uint8_t *base, uint64_t stride, uint32_t nblk, uint64_t nrec,
                                         const uint32_t *mis, uint4 *out)
{
    const uint64_t tid = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t rec = tid / L;
    const uint32_t q = (uint32_t) (tid % L);
    uint4 acc = make_uint4(0, 0, 0, 0);
    if (rec < nrec) {
        const uint8_t *r = base + rec * stride + (mis ? mis[rec] : 0u);
        for (uint32_t j = q; j < nblk; j += L * G) {
            uint4 v[G];
#pragma unroll
            for (int g = 0; g < G; g++) v[g] = j + g * L < nblk ? ld16(r + 16ull * (j + g * L)) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int g = 0; g < G; g++) {
                acc.x ^= v[g].x; acc.y ^= v[g].y; acc.z ^= v[g].z; acc.w ^= v[g].w;
            }
        }
    }
    out[tid] = acc;
}

template <int L, int G>
__device__ __forceinline__ void rec_write(uint8_t *base, uint64_t stride, uint32_t nblk, uint64_t nrec)
{
    const uint64_t tid = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t rec = tid / L;
    const uint32_t q = (uint32_t) (tid % L);
    if (rec >= nrec) return;
    uint8_t *r = base + rec * stride;
    const uint4 v = make_uint4((uint32_t) tid, q, 0x5a5a5a5au, (uint32_t) rec);
    for (uint32_t j = q; j < nblk; j += L * G) {
#pragma unroll
        for (int g = 0; g < G; g++)
            if (j + g * L < nblk) st16(r + 16ull * (j + g * L), v);
    }
}

__global__ __launch_bounds__(256) void calib_wide(const uint8_t *b, uint64_t n16, uint4 *out)
{
    const uint64_t tid = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nt = (uint64_t) gridDim.x * blockDim.x;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint64_t i = tid; i < n16; i += nt) {
        const uint4 v = ld16(b + 16 * i);
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    out[tid] = acc;
}

__global__ __launch_bounds__(256) void calib_dword(const uint8_t *b, uint64_t n4, uint4 *out)
{
    const uint64_t tid = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nt = (uint64_t) gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t i = tid; i < n4; i += nt)
        acc ^= *(const glob_u32 *) (uintptr_t) (b + 4 * i);
    out[tid] = make_uint4(acc, 0, 0, 0);
}

__global__ __launch_bounds__(256) void calib_rec8(const uint8_t *b, uint64_t s, uint32_t nb, uint64_t nr, uint4 *o)
{ rec_read<8, 1>(b, s, nb, nr, nullptr, o); }
__global__ __launch_bounds__(256) void calib_rec2g4(const uint8_t *b, uint64_t s, uint32_t nb, uint64_t nr, uint4 *o)
{ rec_read<2, 4>(b, s, nb, nr, nullptr, o); }
__global__ __launch_bounds__(256) void calib_rec4g2(const uint8_t *b, uint64_t s, uint32_t nb, uint64_t nr, uint4 *o)
{ rec_read<4, 2>(b, s, nb, nr, nullptr, o); }
__global__ __launch_bounds__(256) void calib_rec2g1(const uint8_t *b, uint64_t s, uint32_t nb, uint64_t nr, uint4 *o)
{ rec_read<2, 1>(b, s, nb, nr, nullptr, o); }
__global__ __launch_bounds__(256) void calib_rec2mis(const uint8_t *b, uint64_t s, uint32_t nb, uint64_t nr,
                                                     const uint32_t *mis, uint4 *o)
{ rec_read<2, 4>(b, s, nb, nr, mis, o); }

__global__ __launch_bounds__(256) void calib_w_wide(uint8_t *b, uint64_t n16)
{
    const uint64_t tid = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nt = (uint64_t) gridDim.x * blockDim.x;
    for (uint64_t i = tid; i < n16; i += nt) st16(b + 16 * i, make_uint4((uint32_t) i, 1, 2, 3));
}
__global__ __launch_bounds__(256) void calib_w_rec2g4(uint8_t *b, uint64_t s, uint32_t nb, uint64_t nr)
{ rec_write<2, 4>(b, s, nb, nr); }
__global__ __launch_bounds__(256) void calib_w_rec8(uint8_t *b, uint64_t s, uint32_t nb, uint64_t nr)
{ rec_write<8, 1>(b, s, nb, nr); }

static uint64_t lines_of(uint64_t start, uint64_t len)
{
    return len ? (start + len - 1) / 128 - start / 128 + 1 : 0;
}

int main()
{
    uint8_t *buf = nullptr;
    uint4 *out = nullptr;
    uint32_t *mis = nullptr;
    CHECK(hipMalloc(&buf, REGION));
    CHECK(hipMemset(buf, 0x3c, REGION));
    const uint32_t grid_wide = 256 * 32;
    CHECK(hipMalloc(&out, (size_t) 64 << 20));      // 16 B per thread of the largest grid
    std::vector<uint32_t> hmis(REGION / 1536);
    for (size_t i = 0; i < hmis.size(); i++) hmis[i] = (uint32_t) ((i * 37 + 11) % 113);
    CHECK(hipMalloc(&mis, hmis.size() * 4));
    CHECK(hipMemcpy(mis, hmis.data(), hmis.size() * 4, hipMemcpyHostToDevice));
    printf("{\"region\": %llu, \"kernels\": {", (unsigned long long) REGION);
    auto report = [](const char *name, uint64_t bytes, uint64_t out_bytes, bool first) {
        printf("%s\"%s\": {\"line_bytes\": %llu, \"result_write_bytes\": %llu}", first ? "" : ", ", name,
               (unsigned long long) bytes, (unsigned long long) out_bytes);
    };
    for (int rep = 0; rep < 2; rep++) {       // two dispatches of each (the summary averages them)
        // wide
        hipLaunchKernelGGL(calib_wide, dim3(grid_wide), dim3(256), 0, 0, buf, REGION / 16, out);
        hipLaunchKernelGGL(calib_dword, dim3(grid_wide), dim3(256), 0, 0, buf, REGION / 4, out);
        // rec8: c2 records (16 400 B of 16 512)
        {
            const uint64_t s = 16512, nr = REGION / s;
            const uint32_t nb = 16400 / 16;
            const uint64_t thr = nr * 8;
            hipLaunchKernelGGL(calib_rec8, dim3((thr + 255) / 256), dim3(256), 0, 0, buf, s, nb, nr, out);
        }
        // small records: 1 424 B of 1 536
        {
            const uint64_t s = 1536, nr = REGION / s;
            const uint32_t nb = 1424 / 16;
            hipLaunchKernelGGL(calib_rec2g4, dim3((nr * 2 + 255) / 256), dim3(256), 0, 0, buf, s, nb, nr, out);
            hipLaunchKernelGGL(calib_rec4g2, dim3((nr * 4 + 255) / 256), dim3(256), 0, 0, buf, s, nb, nr, out);
            hipLaunchKernelGGL(calib_rec2g1, dim3((nr * 2 + 255) / 256), dim3(256), 0, 0, buf, s, nb, nr, out);
            hipLaunchKernelGGL(calib_rec2mis, dim3((nr * 2 + 255) / 256), dim3(256), 0, 0, buf, s, nb, nr - 1, mis, out);
        }
        hipLaunchKernelGGL(calib_w_wide, dim3(grid_wide), dim3(256), 0, 0, buf, REGION / 16);
        {
            const uint64_t s = 1536, nr = REGION / s;
            hipLaunchKernelGGL(calib_w_rec2g4, dim3((nr * 2 + 255) / 256), dim3(256), 0, 0, buf, s, 1424 / 16, nr);
            const uint64_t s8 = 16512, nr8 = REGION / s8;
            hipLaunchKernelGGL(calib_w_rec8, dim3((nr8 * 8 + 255) / 256), dim3(256), 0, 0, buf, s8, 16400 / 16, nr8);
        }
        CHECK(hipDeviceSynchronize());
    }
    // the bytes of the 128-B lines each kernel touches
    report("calib_wide", REGION, (uint64_t) grid_wide * 256 * 16, true);
    report("calib_dword", REGION, (uint64_t) grid_wide * 256 * 16, false);
    {
        const uint64_t s = 16512, nr = REGION / s;
        report("calib_rec8", nr * lines_of(0, 16400) * 128, ((nr * 8 + 255) / 256) * 256 * 16, false);
        report("calib_w_rec8", nr * lines_of(0, 16400) * 128, 0, false);
    }
    {
        const uint64_t s = 1536, nr = REGION / s;
        const uint64_t lines = nr * lines_of(0, 1424) * 128;
        report("calib_rec2g4", lines, ((nr * 2 + 255) / 256) * 256 * 16, false);
        report("calib_rec4g2", lines, ((nr * 4 + 255) / 256) * 256 * 16, false);
        report("calib_rec2g1", lines, ((nr * 2 + 255) / 256) * 256 * 16, false);
        uint64_t ml = 0;
        for (uint64_t i = 0; i + 1 < nr; i++) ml += lines_of(i * s + hmis[i], 1424);
        report("calib_rec2mis", ml * 128, ((nr * 2 + 255) / 256) * 256 * 16, false);
        report("calib_w_rec2g4", lines, 0, false);
    }
    report("calib_w_wide", REGION, 0, false);
    printf("}, \"dispatches_each\": 2}\n");
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    CHECK(hipFree(mis));
    return 0;
}
