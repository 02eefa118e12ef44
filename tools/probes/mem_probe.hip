// HBM rate of the record kernels' access patterns, with no crypto: copy N
// records of REC bytes (slot stride STRIDE) from one arena to another.
//   coalesced : a wave copies 1 KiB contiguous per instruction (ideal)
//   chacha L  : L lanes per record, lane q copies 64-B chunk b = L*j + q
//               as four 16-B accesses (tlsrec_chachapoly_kernel)
//   gcm L     : L lanes per record, lane q copies 16-B block L*j + q
//               (tlsrec_gcm_kernel)
// plus read-only / write-only versions of the coalesced pattern.
//   hipcc --offload-arch=gfx950 -O3 tools/mem_probe.hip -o varlib/mem_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 *gin;
typedef __attribute__((address_space(1))) u32x4 *gout;

__global__ __launch_bounds__(256) void coalesced(const uint4 *in, uint4 *out, size_t n16)
{
    gin s = (gin) (uintptr_t) in;
    gout d = (gout) (uintptr_t) out;
    const size_t stride = (size_t) gridDim.x * 256;
    for (size_t i = (size_t) blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) d[i] = s[i];
}

__global__ __launch_bounds__(256) void readonly(const uint4 *in, uint4 *out, size_t n16)
{
    gin s = (gin) (uintptr_t) in;
    const size_t stride = (size_t) gridDim.x * 256;
    u32x4 a = { 0, 0, 0, 0 };
    for (size_t i = (size_t) blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) a ^= s[i];
    if ((a.x ^ a.y ^ a.z ^ a.w) == 0x12345678u) out[threadIdx.x] = make_uint4(a.x, a.y, a.z, a.w);
}

__global__ __launch_bounds__(256) void writeonly(const uint4 *in, uint4 *out, size_t n16)
{
    gout d = (gout) (uintptr_t) out;
    const size_t stride = (size_t) gridDim.x * 256;
    for (size_t i = (size_t) blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
        d[i] = u32x4{ (uint32_t) i, 1, 2, 3 };
}

/* records per wave processed together: 64 / L; waves walk records grid-stride */
template <int L>
__global__ __launch_bounds__(256) void chacha_pat(const uint8_t *in, uint8_t *out, uint32_t nrec, uint32_t rec,
                                                  uint32_t stride)
{
    const int lane = threadIdx.x & 63, g = lane / L, q = lane % L;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
    const uint32_t chunks = rec / 64;
    for (uint32_t r0 = wave * (64 / L); r0 < nrec; r0 += nwaves * (64 / L)) {
        const uint32_t r = r0 + g;
        if (r >= nrec) continue;
        gin s = (gin) (uintptr_t) (in + (size_t) r * stride);
        gout d = (gout) (uintptr_t) (out + (size_t) r * stride);
        for (uint32_t b = q; b < chunks; b += L) {
            u32x4 c[4];
#pragma unroll
            for (int t = 0; t < 4; t++) c[t] = s[b * 4 + t];
#pragma unroll
            for (int t = 0; t < 4; t++) d[b * 4 + t] = c[t];
        }
    }
}

template <int L>
__global__ __launch_bounds__(1024) void gcm_pat(const uint8_t *in, uint8_t *out, uint32_t nrec, uint32_t rec,
                                                uint32_t stride)
{
    const int lane = threadIdx.x & 63, g = lane / L, q = lane % L;
    const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6), nwaves = gridDim.x * 16;
    const uint32_t blocks = rec / 16;
    for (uint32_t r0 = wave * (64 / L); r0 < nrec; r0 += nwaves * (64 / L)) {
        const uint32_t r = r0 + g;
        if (r >= nrec) continue;
        gin s = (gin) (uintptr_t) (in + (size_t) r * stride);
        gout d = (gout) (uintptr_t) (out + (size_t) r * stride);
        for (uint32_t b = q; b < blocks; b += L) d[b] = s[b];
    }
}

static float timeit(void (*launch)(void *), void *ctx)
{
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    launch(ctx);
    (void) hipDeviceSynchronize();
    float best = 1e30f;
    for (int i = 0; i < 5; i++) {
        (void) hipEventRecord(a);
        launch(ctx);
        (void) hipEventRecord(b);
        (void) hipEventSynchronize(b);
        float ms;
        (void) hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

struct Ctx {
    uint8_t *in, *out;
    uint32_t nrec, rec, stride;
    int grid;
};

int main()
{
    const uint32_t nrec = 1u << 20, rec = 16384, stride = 16512;
    const size_t bytes = (size_t) nrec * stride;
    Ctx c;
    (void) hipMalloc(&c.in, bytes);
    (void) hipMalloc(&c.out, bytes);
    (void) hipMemset(c.in, 1, bytes);
    (void) hipMemset(c.out, 0, bytes);
    c.nrec = nrec; c.rec = rec; c.stride = stride;
    const double payload = (double) nrec * rec;
    const size_t n16 = bytes / 16;
    int cus = 256;
    struct Row { const char *name; void (*f)(void *); double bytes; };
    static Ctx *C;
    C = &c;
    auto coal = [](void *p) { Ctx *x = (Ctx *) p; coalesced<<<x->grid, 256>>>((const uint4 *) x->in, (uint4 *) x->out, (size_t) x->nrec * x->stride / 16); };
    auto ro = [](void *p) { Ctx *x = (Ctx *) p; readonly<<<x->grid, 256>>>((const uint4 *) x->in, (uint4 *) x->out, (size_t) x->nrec * x->stride / 16); };
    auto wo = [](void *p) { Ctx *x = (Ctx *) p; writeonly<<<x->grid, 256>>>((const uint4 *) x->in, (uint4 *) x->out, (size_t) x->nrec * x->stride / 16); };
    auto ch2 = [](void *p) { Ctx *x = (Ctx *) p; chacha_pat<2><<<x->grid, 256>>>(x->in, x->out, x->nrec, x->rec, x->stride); };
    auto ch8 = [](void *p) { Ctx *x = (Ctx *) p; chacha_pat<8><<<x->grid, 256>>>(x->in, x->out, x->nrec, x->rec, x->stride); };
    auto gc8 = [](void *p) { Ctx *x = (Ctx *) p; gcm_pat<8><<<x->grid, 1024>>>(x->in, x->out, x->nrec, x->rec, x->stride); };
    auto gc16 = [](void *p) { Ctx *x = (Ctx *) p; gcm_pat<16><<<x->grid, 1024>>>(x->in, x->out, x->nrec, x->rec, x->stride); };
    (void) n16;
    const int grids[3] = { cus * 8, cus * 32, cus * 128 };
    for (int gi = 0; gi < 3; gi++) {
        c.grid = grids[gi];
        printf("grid %d\n", c.grid);
        float t;
        t = timeit(coal, &c); printf("  coalesced copy   %7.3f ms  %7.1f GB/s (r+w)\n", t, 2.0 * bytes / t / 1e6);
        t = timeit(ro, &c);   printf("  coalesced read   %7.3f ms  %7.1f GB/s\n", t, 1.0 * bytes / t / 1e6);
        t = timeit(wo, &c);   printf("  coalesced write  %7.3f ms  %7.1f GB/s\n", t, 1.0 * bytes / t / 1e6);
        t = timeit(ch2, &c);  printf("  chacha L=2 copy  %7.3f ms  %7.1f GB/s (r+w payload)\n", t, 2.0 * payload / t / 1e6);
        t = timeit(ch8, &c);  printf("  chacha L=8 copy  %7.3f ms  %7.1f GB/s (r+w payload)\n", t, 2.0 * payload / t / 1e6);
        c.grid = grids[gi] / 4;
        t = timeit(gc8, &c);  printf("  gcm L=8 copy     %7.3f ms  %7.1f GB/s (r+w payload)\n", t, 2.0 * payload / t / 1e6);
        t = timeit(gc16, &c); printf("  gcm L=16 copy    %7.3f ms  %7.1f GB/s (r+w payload)\n", t, 2.0 * payload / t / 1e6);
        c.grid = grids[gi];
    }
    return 0;
}
