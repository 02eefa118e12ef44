/*
 * gcm_enc.hip -- instantiations of the GCM record kernel, AES-GCM encrypt
 * (tlsrec_gcm.h).
 */
#include "tlsrec_gcm.h"

using namespace tlsrec;

extern "C" hipError_t tlsrec__launch_gcm_enc(const GcmArgs *a, int lanes, int nr, int waves, uint32_t grid, hipStream_t st)
{
    return gcm_dispatch<false>(*a, lanes, nr, waves, grid, st);
}
