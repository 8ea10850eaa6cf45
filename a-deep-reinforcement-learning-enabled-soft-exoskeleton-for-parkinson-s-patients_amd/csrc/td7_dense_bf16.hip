// PREC_BF16 instantiation of the TD7 dense-layer launchers (td7_dense_kernels.h).
#include "td7_dense_kernels.h"

namespace td7dense {
template void launch_gemm_p<PREC_BF16>(const GemmArgs &, dim3, int, hipStream_t);
template void launch_wgrad_p<PREC_BF16, false>(const WgradArgs &, dim3, int, int, int, hipStream_t);
template void launch_fwd_p<PREC_BF16, false>(const GemmArgs &, dim3, int, int, int, int, hipStream_t);
template void launch_wgrad_p<PREC_BF16, true>(const WgradArgs &, dim3, int, int, int, hipStream_t);
template void launch_fwd_p<PREC_BF16, true>(const GemmArgs &, dim3, int, int, int, int, hipStream_t);
template void launch_fwd_p<PREC_BF16, false, true>(const GemmArgs &, dim3, int, int, int, int, hipStream_t);
template void launch_fwd_norm_p<PREC_BF16, false>(const GemmArgs &, dim3, float *, float *, float, hipStream_t);
template void launch_fwd_norm_p<PREC_BF16, true>(const GemmArgs &, dim3, float *, float *, float, hipStream_t);
template void launch_fwd_lds_p<PREC_BF16, false>(const GemmArgs &, dim3, int, hipStream_t);
template void launch_fwd_lds_p<PREC_BF16, true>(const GemmArgs &, dim3, int, hipStream_t);
template void launch_fwd_big_p<PREC_BF16, false>(const GemmArgs &, dim3, int, hipStream_t);
template void launch_fwd_big_p<PREC_BF16, true>(const GemmArgs &, dim3, int, hipStream_t);
template void launch_fwd_xl_p<PREC_BF16, false>(const GemmArgs &, dim3, int, hipStream_t);
template void launch_fwd_xl_p<PREC_BF16, true>(const GemmArgs &, dim3, int, hipStream_t);
} // namespace td7dense
