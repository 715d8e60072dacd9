// mmv_fused_q80.hip -- the k_mmv_stream instances of one weight format (mmv_fused_impl.h),
// compiled as a translation unit of their own so that the formats build in parallel
#include "mmv_fused_impl.h"

void mi_mmv_launch_q80(const mi_mmv_group & g, int variant, hipStream_t s) {
    // tree order on the repacked 16-byte-aligned copy when the backend handed one over (g.q0r)
    if (g.q0r) launch_stream_nc<FmtQ8R, false>(g, variant, s);
    else launch_stream_ord<FmtQ0<true>>(g, variant, s);
}
