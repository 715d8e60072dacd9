// mmv_fused_q40.hip -- the k_mmv_stream instances of one weight format (mmv_fused_impl.h),
// compiled as a translation unit of their own so that the formats build in parallel
#include "mmv_fused_impl.h"

void mi_mmv_launch_q40(const mi_mmv_group & g, int variant, hipStream_t s) {
    // tree order: pairs of blocks per item (variant % 10 == 1: single blocks), on the repacked
    // 16-byte-aligned copy when the backend handed one over (g.q0r)
    if (g.q0r) launch_stream_nc<FmtQ0R, false>(g, variant, s);
    else if (!mi_mmv_order() && variant % 10 != 1) launch_stream_nc<FmtQ0Pair, false>(g, variant, s);
    else launch_stream_ord<FmtQ0<false>>(g, variant, s);
}
