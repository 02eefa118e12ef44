/* Where the HIP runtime places device and pinned-host allocations (the record
 * server packs device addresses into 48 bits). gcc ptr_probe.c -lamdhip64 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdio.h>
int main(void)
{
    void *d = 0, *d2 = 0, *h = 0, *hd = 0;
    (void) hipMalloc(&d, 1 << 20);
    (void) hipMalloc(&d2, 256 << 20);
    (void) hipHostMalloc(&h, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent);
    (void) hipHostGetDevicePointer(&hd, h, 0);
    printf("{\"dev\": \"%p\", \"dev2\": \"%p\", \"host\": \"%p\", \"host_dev\": \"%p\"}\n", d, d2, h, hd);
    return 0;
}
