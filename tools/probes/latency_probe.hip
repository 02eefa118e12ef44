/*
 * latency_probe.hip -- what a single small record costs on the launch path
 * (DESIGN.md 5.2): p50 / p99 in microseconds of
 *   launch    empty kernel + hipStreamSynchronize
 *   h2d       1536-B hipMemcpyAsync from pinned memory + sync
 *   d2h       1536-B hipMemcpyAsync to pinned memory + sync
 *   zc_in     one wave copies 1536 B host-mapped -> device, + sync
 *   zc_out    one wave copies 1536 B device -> host-mapped, + sync
 *   zc_both   one wave: host-mapped -> device -> host-mapped, + sync
 *   flag      zc_both, completion seen by spinning on a host-mapped word the
 *             kernel writes last (no hipStreamSynchronize)
 * hipcc --offload-arch=gfx950 -O2 latency_probe.hip -o latency_probe
 */
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <stdio.h>
#include <vector>

__global__ void empty_k() {}

__global__ void copy_k(const uint4 *src, uint4 *dst, int n16)
{
    for (int i = threadIdx.x; i < n16; i += 64) dst[i] = src[i];
}

__global__ void both_k(const uint4 *hin, uint4 *dev, uint4 *hout, int n16, volatile uint32_t *flag, uint32_t tag)
{
    for (int i = threadIdx.x; i < n16; i += 64) dev[i] = hin[i];
    __syncthreads();
    for (int i = threadIdx.x; i < n16; i += 64) hout[i] = dev[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0 && flag) *flag = tag;
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
static void run(const char *name, F f)
{
    std::vector<double> t;
    for (int i = 0; i < 200; i++) f();
    for (int i = 0; i < 2000; i++) {
        const double a = now_us();
        f();
        t.push_back(now_us() - a);
    }
    std::sort(t.begin(), t.end());
    printf("{\"probe\": \"%s\", \"p50_us\": %.2f, \"p99_us\": %.2f}\n", name, t[t.size() / 2], t[t.size() * 99 / 100]);
}

int main()
{
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const int N = 1536;
    uint8_t *h, *h2, *d;
    hipHostMalloc((void **) &h, N, hipHostMallocMapped);
    hipHostMalloc((void **) &h2, N, hipHostMallocMapped);
    hipMalloc((void **) &d, N);
    uint32_t *flag;
    hipHostMalloc((void **) &flag, 64, hipHostMallocMapped);
    uint8_t *dh, *dh2;
    uint32_t *dflag;
    hipHostGetDevicePointer((void **) &dh, h, 0);
    hipHostGetDevicePointer((void **) &dh2, h2, 0);
    hipHostGetDevicePointer((void **) &dflag, flag, 0);
    run("launch", [&] { hipLaunchKernelGGL(empty_k, 1, 64, 0, st); hipStreamSynchronize(st); });
    run("h2d", [&] { hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, st); hipStreamSynchronize(st); });
    run("d2h", [&] { hipMemcpyAsync(h, d, N, hipMemcpyDeviceToHost, st); hipStreamSynchronize(st); });
    run("zc_in", [&] { hipLaunchKernelGGL(copy_k, 1, 64, 0, st, (const uint4 *) dh, (uint4 *) d, N / 16); hipStreamSynchronize(st); });
    run("zc_out", [&] { hipLaunchKernelGGL(copy_k, 1, 64, 0, st, (const uint4 *) d, (uint4 *) dh2, N / 16); hipStreamSynchronize(st); });
    run("zc_both", [&] { hipLaunchKernelGGL(both_k, 1, 64, 0, st, (const uint4 *) dh, (uint4 *) d, (uint4 *) dh2, N / 16, (volatile uint32_t *) nullptr, 0u); hipStreamSynchronize(st); });
    uint32_t tag = 1;
    run("flag", [&] {
        tag++;
        hipLaunchKernelGGL(both_k, 1, 64, 0, st, (const uint4 *) dh, (uint4 *) d, (uint4 *) dh2, N / 16, (volatile uint32_t *) dflag, tag);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != tag) {}
    });
    hipStreamSynchronize(st);
    return 0;
}
