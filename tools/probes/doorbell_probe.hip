/*
 * doorbell_probe.hip -- what the record server's request path costs on this
 * box: a resident one-wave kernel answers host "doorbells"; the host times
 * post -> answer round trips (p50 / p99, microseconds) for
 *   host     doorbell + 1.5 KiB payload in pinned host memory (the GPU polls
 *            and reads over PCIe), answer flag in host memory
 *   dev      doorbell + payload in fine-grained device memory that the CPU
 *            writes directly (large BAR), answer flag in host memory
 * plus whether fine-grained device memory is CPU-writable at all.
 * Every loop is bounded (the kernel leaves after `max_polls` polls or when
 * the host sets the stop word).
 *   hipcc --offload-arch=gfx950 -O2 doorbell_probe.hip -o doorbell_probe
 */
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <stdio.h>
#include <string.h>
#include <vector>

struct Bell {
    uint64_t seq;           /* host -> device */
    uint64_t stop;
    uint8_t pad[48];
    uint8_t payload[1536];
};

__global__ void server(Bell *b, uint32_t *answer, uint32_t max_polls, int sleep)
{
    const int lane = threadIdx.x;
    uint64_t served = 0;
    for (uint32_t it = 0; it < max_polls; it++) {
        const uint64_t s = __hip_atomic_load(&b->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t st = __hip_atomic_load(&b->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (st) break;
        if (s != served) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            /* touch the payload: 1.5 KiB, 24 B per lane */
            uint32_t acc = 0;
            for (int i = lane; i < 1536 / 16; i += 64) {
                const uint4 v = reinterpret_cast<const uint4 *>(b->payload)[i];
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (lane == 0) __hip_atomic_store(answer, (uint32_t) s + (acc == 0x9e3779b9u ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            served = s;
            continue;
        }
        if (sleep) __builtin_amdgcn_s_sleep(8);
    }
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void pingpong(const char *name, Bell *hb, Bell *db, uint32_t *ans_h, uint32_t *ans_d, int sleep)
{
    hipStream_t st;
    (void) hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    __atomic_store_n(&hb->stop, 0ull, __ATOMIC_RELEASE);
    __atomic_store_n(&hb->seq, 0ull, __ATOMIC_RELEASE);
    *ans_h = 0;
    hipLaunchKernelGGL(server, 1, 64, 0, st, db, ans_d, 5000000u, sleep);
    std::vector<double> t;
    bool ok = true;
    for (uint64_t i = 1; i <= 3000 && ok; i++) {
        memset(hb->payload, (int) i, sizeof(hb->payload));
        const double a = now_us();
        __atomic_store_n(&hb->seq, i, __ATOMIC_RELEASE);
        for (uint64_t spin = 0;; spin++) {
            if (__atomic_load_n(ans_h, __ATOMIC_ACQUIRE) == (uint32_t) i) break;
            if (spin > 20000000ull) { ok = false; break; }
        }
        if (i > 200) t.push_back(now_us() - a);
    }
    __atomic_store_n(&hb->stop, 1ull, __ATOMIC_RELEASE);
    const hipError_t e = hipStreamSynchronize(st);
    std::sort(t.begin(), t.end());
    if (!ok || t.empty())
        printf("{\"probe\": \"%s\", \"sleep\": %d, \"ok\": false, \"err\": \"%s\"}\n", name, sleep, hipGetErrorString(e));
    else
        printf("{\"probe\": \"%s\", \"sleep\": %d, \"p50_us\": %.2f, \"p99_us\": %.2f, \"err\": \"%s\"}\n", name, sleep,
               t[t.size() / 2], t[t.size() * 99 / 100], hipGetErrorString(e));
    fflush(stdout);
    (void) hipStreamDestroy(st);
}

int main()
{
    uint32_t *ans_h = nullptr, *ans_d = nullptr;
    (void) hipHostMalloc((void **) &ans_h, 64, hipHostMallocMapped | hipHostMallocCoherent);
    (void) hipHostGetDevicePointer((void **) &ans_d, ans_h, 0);
    Bell *hb = nullptr, *hbd = nullptr;
    (void) hipHostMalloc((void **) &hb, sizeof(Bell), hipHostMallocMapped | hipHostMallocCoherent);
    (void) hipHostGetDevicePointer((void **) &hbd, hb, 0);
    pingpong("host", hb, hbd, ans_h, ans_d, 1);
    pingpong("host", hb, hbd, ans_h, ans_d, 0);
    /* fine-grained device memory: is it CPU-addressable here? */
    Bell *db = nullptr;
    hipError_t e = hipExtMallocWithFlags((void **) &db, sizeof(Bell), hipDeviceMallocFinegrained);
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof(at));
    const hipError_t ea = db ? hipPointerGetAttributes(&at, db) : hipErrorInvalidValue;
    printf("{\"finegrained_alloc\": \"%s\", \"ptr\": \"%p\", \"attr\": \"%s\", \"type\": %d, \"host_ptr\": \"%p\", "
           "\"dev_ptr\": \"%p\"}\n",
           hipGetErrorString(e), (void *) db, hipGetErrorString(ea), (int) at.type, at.hostPointer, at.devicePointer);
    fflush(stdout);
    if (e == hipSuccess && db && at.hostPointer) {
        Bell *hp = (Bell *) at.hostPointer;
        pingpong("dev", hp, db, ans_h, ans_d, 1);
        pingpong("dev", hp, db, ans_h, ans_d, 0);
    }
    return 0;
}
