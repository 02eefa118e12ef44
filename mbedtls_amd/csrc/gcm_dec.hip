/*
 * gcm_dec.hip -- instantiations of the GCM record kernel, AES-GCM decrypt
 * (tlsrec_gcm.h).
 */
#include "tlsrec_gcm.h"

using namespace tlsrec;

extern "C" hipError_t tlsrec__launch_gcm_dec(const GcmArgs *a, int lanes, int nr, int waves, uint32_t grid, hipStream_t st)
{
    return gcm_dispatch<true>(*a, lanes, nr, waves, grid, st);
}
