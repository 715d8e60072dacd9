// mmv_fused_q80.hip -- the k_mmv_stream instances of one weight format (mmv_fused_impl.h),
// compiled as a translation unit of their own so that the formats build in parallel
#include "mmv_fused_impl.h"

void mi_mmv_launch_q80(const mi_mmv_group & g, int variant, hipStream_t s) {
    launch_stream_ord<FmtQ0<true>>(g, variant, s);
}
