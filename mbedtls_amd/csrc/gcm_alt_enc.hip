/*
 * gcm_alt_enc.hip -- instantiations of the GCM record kernel, ARIA-/Camellia-GCM encrypt
 * (tlsrec_gcm.h).
 */
#include "tlsrec_gcm.h"

using namespace tlsrec;

extern "C" hipError_t tlsrec__launch_gcm_alt_enc(const GcmArgs *a, int nr, int cid, uint32_t grid, hipStream_t st)
{
    return gcm_alt_dispatch<false>(*a, nr, cid, grid, st);
}
