/*
 * gcm_alt_dec.hip -- instantiations of the GCM record kernel, ARIA-/Camellia-GCM decrypt
 * (tlsrec_gcm.h).
 */
#include "tlsrec_gcm.h"

using namespace tlsrec;

extern "C" hipError_t tlsrec__launch_gcm_alt_dec(const GcmArgs *a, int nr, int cid, uint32_t grid, hipStream_t st)
{
    return gcm_alt_dispatch<true>(*a, nr, cid, grid, st);
}
