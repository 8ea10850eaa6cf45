// td7_ops.hip -- fused elementwise pieces of the TD7 nets (gfx950).
//
// AvgL1Norm (Agent/TD7_multi_agent.py:53-54):  y = x / max(mean|x|, eps)
// row-wise.  In PyTorch it is abs -> mean -> clamp -> div forward and five more
// kernels backward; here it is one kernel each way, one wavefront per row
// (rows are <= 1024 wide in every TD7 configuration).
//
//   forward : s_r = max(mean_j |x_rj|, eps);  y_rj = x_rj / s_r
//   backward: m_r = mean_j |x_rj|;  if m_r >= eps:
//               gx_rk = gy_rk / s_r - sign(x_rk) / (n s_r^2) * sum_j gy_rj x_rj
//             else gx_rk = gy_rk / eps            (torch.clamp passes no gradient)
#include <hip/hip_runtime.h>

#include "exo_amd.h"

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

constexpr int ROWS_PER_BLOCK = 4; // 4 wavefronts of 64 lanes

__global__ __launch_bounds__(256) void avgl1_fwd_kernel(const float *__restrict__ x, float *__restrict__ y,
                                                        float *__restrict__ s_out, int rows, int cols, float eps) {
    const int r = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const float *xr = x + (size_t)r * cols;
    float acc = 0.f;
    for (int j = lane; j < cols; j += 64) acc += fabsf(xr[j]);
    const float m = wave_sum(acc) / cols;
    const float s = fmaxf(m, eps);
    float *yr = y + (size_t)r * cols;
    for (int j = lane; j < cols; j += 64) yr[j] = xr[j] / s;
    if (lane == 0) s_out[r] = m;
}

__global__ __launch_bounds__(256) void avgl1_bwd_kernel(const float *__restrict__ x, const float *__restrict__ m_in,
                                                        const float *__restrict__ gy, float *__restrict__ gx,
                                                        int rows, int cols, float eps) {
    const int r = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const float *xr = x + (size_t)r * cols, *gr = gy + (size_t)r * cols;
    float *o = gx + (size_t)r * cols;
    const float m = m_in[r];
    if (m >= eps) {
        float dot = 0.f;
        for (int j = lane; j < cols; j += 64) dot += gr[j] * xr[j];
        dot = wave_sum(dot);
        const float inv = 1.0f / m, c = dot * inv * inv / cols;
        for (int j = lane; j < cols; j += 64) {
            const float xv = xr[j];
            const float sg = (xv > 0.f) ? 1.f : ((xv < 0.f) ? -1.f : 0.f);
            o[j] = gr[j] * inv - sg * c;
        }
    } else {
        for (int j = lane; j < cols; j += 64) o[j] = gr[j] / eps;
    }
}

} // namespace

extern "C" {

/* AvgL1Norm forward over `rows` rows of `cols` fp32 values; mean_out[rows]
 * receives mean|x| for the backward pass. */
int td7_avgl1norm_fwd(const float *x, float *y, float *mean_out, int32_t rows, int32_t cols, float eps,
                      void *stream) {
    if (!x || !y || !mean_out || rows < 0 || cols <= 0) return EXO_EINVAL;
    if (rows == 0) return EXO_OK;
    hipLaunchKernelGGL(avgl1_fwd_kernel, dim3((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK), dim3(256), 0,
                       (hipStream_t)stream, x, y, mean_out, rows, cols, eps);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7_avgl1norm_bwd(const float *x, const float *mean_in, const float *gy, float *gx, int32_t rows, int32_t cols,
                      float eps, void *stream) {
    if (!x || !mean_in || !gy || !gx || rows < 0 || cols <= 0) return EXO_EINVAL;
    if (rows == 0) return EXO_OK;
    hipLaunchKernelGGL(avgl1_bwd_kernel, dim3((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK), dim3(256), 0,
                       (hipStream_t)stream, x, mean_in, gy, gx, rows, cols, eps);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

} // extern "C"
