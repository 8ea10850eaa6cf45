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

#include <cstdlib>

#include <algorithm>

#include "adam_math.h"
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

// The same per-row sums with the row kept in registers (cols <= 64 MAXJ): every
// load of a row in flight at once and no second read for the division (r03d:
// the wide configuration's 65,536 x 1,024 norms).  Lane l still adds
// |x[l]|, |x[l + 64]|, ... in that order: bit-identical to avgl1_fwd_kernel.
// OUT = 1 / 2 (td7_avgl1norm_fwd_h): y written as bf16 / fp16 bits (RNE), the
// values an MFMA consumer rounds it to; s_out may then be null.
template <int OUT>
__device__ __forceinline__ void avgl1_store(float *y, long i, float v) {
    if constexpr (OUT == 0) y[i] = v;
    else if constexpr (OUT == 1) reinterpret_cast<uint16_t *>(y)[i] = __builtin_bit_cast(uint16_t, (__bf16)v);
    else reinterpret_cast<uint16_t *>(y)[i] = __builtin_bit_cast(uint16_t, (_Float16)v);
}
template <int MAXJ, int OUT = 0>
__global__ __launch_bounds__(256) void avgl1_fwd_reg_kernel(const float *__restrict__ x, float *__restrict__ y,
                                                            float *__restrict__ s_out, int rows, int cols, float eps) {
    const int r = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const float *xr = x + (size_t)r * cols;
    float v[MAXJ];
#pragma unroll
    for (int i = 0; i < MAXJ; ++i) v[i] = lane + 64 * i < cols ? xr[lane + 64 * i] : 0.f;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < MAXJ; ++i)
        if (lane + 64 * i < cols) acc += fabsf(v[i]);
    const float m = wave_sum(acc) / cols;
    const float s = fmaxf(m, eps);
#pragma unroll
    for (int i = 0; i < MAXJ; ++i)
        if (lane + 64 * i < cols) avgl1_store<OUT>(y, (long)r * cols + lane + 64 * i, v[i] / s);
    if (lane == 0 && s_out) s_out[r] = m;
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


// Adam (torch.optim.Adam semantics, Agent/TD7_multi_agent.py:165-170 with
// weight_decay) over one flat parameter buffer: grad += wd * p;
// m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2;  p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
// The step count lives on the device: every workgroup reads it, the last one
// to finish (ticket counter) stores step + 1 and rearms the ticket, so one
// launch is the whole optimiser step (HIP-graph safe, no host value).
constexpr int ADAM_THREADS = 256, ADAM_BLOCKS = 256, ADAM_MULTI_BLOCKS = 256;

// grid-stride over float4 groups (a fixed 512-workgroup grid: few ticket
// atomics), scalar tail for n % 4
__global__ __launch_bounds__(ADAM_THREADS) void adam_kernel(float *__restrict__ p, const float *__restrict__ g,
                                                           float *__restrict__ m, float *__restrict__ v,
                                                           float *step, uint32_t *ticket, long n, float lr, float b1,
                                                           float b2, float eps, float wd, float gscale) {
    __shared__ float coef[2];
    if (threadIdx.x == 0) { // bias corrections once per workgroup
        const float t = *step + 1.0f;
        coef[0] = lr / (1.0f - powf(b1, t));        // step_size
        coef[1] = sqrtf(1.0f - powf(b2, t));        // sqrt(bias_correction2)
    }
    __syncthreads();
    const float step_size = coef[0], bc2s = coef[1];
    const long n4 = n >> 2, stride = (long)gridDim.x * ADAM_THREADS;
    const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                       reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
    const long start = (long)blockIdx.x * ADAM_THREADS + threadIdx.x;
    if (vec) {
        float4 *p4 = reinterpret_cast<float4 *>(p), *m4 = reinterpret_cast<float4 *>(m), *v4 = reinterpret_cast<float4 *>(v);
        const float4 *g4 = reinterpret_cast<const float4 *>(g);
        for (long i = start; i < n4; i += stride) {
            float4 pp = p4[i], mm = m4[i], vv = v4[i];
            const float4 gg = g4[i];
            adam_one(pp.x, gg.x, mm.x, vv.x, step_size, bc2s, b1, b2, eps, wd, gscale);
            adam_one(pp.y, gg.y, mm.y, vv.y, step_size, bc2s, b1, b2, eps, wd, gscale);
            adam_one(pp.z, gg.z, mm.z, vv.z, step_size, bc2s, b1, b2, eps, wd, gscale);
            adam_one(pp.w, gg.w, mm.w, vv.w, step_size, bc2s, b1, b2, eps, wd, gscale);
            p4[i] = pp;
            m4[i] = mm;
            v4[i] = vv;
        }
    }
    for (long i = (vec ? 4 * n4 : 0) + start; i < n; i += stride)
        adam_one(p[i], g[i], m[i], v[i], step_size, bc2s, b1, b2, eps, wd, gscale);
    // the last workgroup out advances the device step count (every workgroup
    // has read it: its read precedes its ticket in program order)
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = atomicAdd(ticket, 1u);
        if (done == gridDim.x - 1) {
            *step = *step + 1.0f;
            *ticket = 0u;
        }
    }
}

// Several FlatAdam steps in one launch, the gradients read where autograd left
// them (one tensor per parameter: no concatenation into a flat buffer).
struct AdamOpt {
    float *p, *m, *v, *step;
    float lr, b1, b2, eps, wd;
};
struct AdamSeg {
    const float *g;
    long off; // into the optimiser's flat p / m / v
    int n, opt;
};
struct AdamMulti {
    AdamOpt o[TD7_ADAM_MAX_OPT];
    AdamSeg s[TD7_ADAM_MAX_SEG];
    int q0[TD7_ADAM_MAX_SEG + 1]; // segment k owns the 4-element groups [q0[k], q0[k+1])
    int nopt, nseg;
    uint32_t *ticket;
};

// Threads stride over the 4-element groups of the concatenated segments (every
// segment padded to whole groups), so all segments are updated in one pass.
__global__ __launch_bounds__(ADAM_THREADS) void adam_multi_kernel(AdamMulti a) {
    __shared__ float coef[TD7_ADAM_MAX_OPT][2];
    __shared__ AdamSeg segs[TD7_ADAM_MAX_SEG];
    __shared__ AdamOpt opts[TD7_ADAM_MAX_OPT];
    __shared__ int q0[TD7_ADAM_MAX_SEG + 1];
    // the descriptors staged in LDS (per-lane indexed reads of the kernel
    // arguments would be dependent global loads ahead of the data loads)
    if (threadIdx.x < a.nseg) segs[threadIdx.x] = a.s[threadIdx.x];
    if (threadIdx.x <= a.nseg) q0[threadIdx.x] = a.q0[threadIdx.x];
    if (threadIdx.x < a.nopt) {
        const AdamOpt o = a.o[threadIdx.x];
        opts[threadIdx.x] = o;
        const float t = *o.step + 1.0f;
        coef[threadIdx.x][0] = o.lr / (1.0f - powf(o.b1, t));
        coef[threadIdx.x][1] = sqrtf(1.0f - powf(o.b2, t));
    }
    __syncthreads();
    // grid-stride over the groups: a bounded grid keeps the ticket atomics
    // (one per workgroup, serialised on one address) few
    for (int gi = blockIdx.x * ADAM_THREADS + threadIdx.x; gi < a.q0[a.nseg]; gi += gridDim.x * ADAM_THREADS) {
        // the segment owning group gi: binary search of the group offsets (a
        // linear scan cost 2 VALU per segment per 4 elements, ~10 us at 40 segments)
        int lo = 0, hi = a.nseg - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (gi >= q0[mid]) lo = mid;
            else hi = mid - 1;
        }
        const int k = lo;
        const AdamSeg sg = segs[k];
        const AdamOpt o = opts[sg.opt];
        const float step_size = coef[sg.opt][0], bc2s = coef[sg.opt][1];
        const long e0 = 4L * (gi - q0[k]);
        float *p = o.p + sg.off + e0, *m = o.m + sg.off + e0, *v = o.v + sg.off + e0;
        const float *g = sg.g + e0;
        const bool vec = e0 + 4 <= sg.n && ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                                              reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0;
        if (vec) {
            float4 pp = *reinterpret_cast<float4 *>(p), mm = *reinterpret_cast<float4 *>(m),
                   vv = *reinterpret_cast<float4 *>(v);
            const float4 gg = *reinterpret_cast<const float4 *>(g);
            adam_one(pp.x, gg.x, mm.x, vv.x, step_size, bc2s, o.b1, o.b2, o.eps, o.wd, 1.0f);
            adam_one(pp.y, gg.y, mm.y, vv.y, step_size, bc2s, o.b1, o.b2, o.eps, o.wd, 1.0f);
            adam_one(pp.z, gg.z, mm.z, vv.z, step_size, bc2s, o.b1, o.b2, o.eps, o.wd, 1.0f);
            adam_one(pp.w, gg.w, mm.w, vv.w, step_size, bc2s, o.b1, o.b2, o.eps, o.wd, 1.0f);
            *reinterpret_cast<float4 *>(p) = pp;
            *reinterpret_cast<float4 *>(m) = mm;
            *reinterpret_cast<float4 *>(v) = vv;
        } else {
            const int ne = (int)min(4L, (long)sg.n - e0);
            for (int e = 0; e < ne; ++e) adam_one(p[e], g[e], m[e], v[e], step_size, bc2s, o.b1, o.b2, o.eps, o.wd, 1.0f);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = atomicAdd(a.ticket, 1u);
        if (done == gridDim.x - 1) {
            for (int k = 0; k < a.nopt; ++k) *a.o[k].step = *a.o[k].step + 1.0f;
            *a.ticket = 0u;
        }
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
    const dim3 grid((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
    const char *reg_env = getenv("EXO_AVGL1_REG");  // read per call: the bit-identity test switches it
    if (cols > 256 && cols <= 1024 && !(reg_env && reg_env[0] == '0'))
        hipLaunchKernelGGL(avgl1_fwd_reg_kernel<16>, grid, dim3(256), 0, (hipStream_t)stream, x, y, mean_out, rows,
                           cols, eps);
    else
        hipLaunchKernelGGL(avgl1_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, y, mean_out, rows, cols, eps);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

/* td7_avgl1norm_fwd writing y as 16-bit values (prec 1 = bf16, 2 = fp16 bits,
 * round to nearest even) for an inference chain whose next layer rounds its
 * input to that type anyway (bit-identical results, half the bytes);
 * mean_out may be null.  256 < cols <= 1,024 (else EXO_ERANGE: use fp32). */
int td7_avgl1norm_fwd_h(const float *x, uint16_t *y16, float *mean_out, int32_t rows, int32_t cols, float eps,
                        int32_t prec, void *stream) {
    if (!x || !y16 || rows < 0 || cols <= 0 || prec < 1 || prec > 2) return EXO_EINVAL;
    if (cols <= 256 || cols > 1024) return EXO_ERANGE;
    if (rows == 0) return EXO_OK;
    const dim3 grid((rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
    float *y = reinterpret_cast<float *>(y16);
    if (prec == 1)
        hipLaunchKernelGGL((avgl1_fwd_reg_kernel<16, 1>), grid, dim3(256), 0, (hipStream_t)stream, x, y, mean_out, rows,
                           cols, eps);
    else
        hipLaunchKernelGGL((avgl1_fwd_reg_kernel<16, 2>), grid, dim3(256), 0, (hipStream_t)stream, x, y, mean_out, rows,
                           cols, eps);
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

/* nopt FlatAdam steps in one launch (see include/exo_amd.h). */
int td7_adam_step_multi(int32_t nopt, float *const *p, float *const *m, float *const *v, float *const *step,
                        const float *lr, const float *beta1, const float *beta2, const float *eps,
                        const float *weight_decay, int32_t nseg, const float *const *g, const int64_t *off,
                        const int32_t *n, const int32_t *opt, uint32_t *ticket, void *stream) {
    if (nopt <= 0 || nopt > TD7_ADAM_MAX_OPT || nseg <= 0 || nseg > TD7_ADAM_MAX_SEG || !ticket) return EXO_EINVAL;
    AdamMulti a{};
    a.nopt = nopt;
    a.nseg = nseg;
    a.ticket = ticket;
    for (int k = 0; k < nopt; ++k) {
        if (!p[k] || !m[k] || !v[k] || !step[k]) return EXO_EINVAL;
        a.o[k] = AdamOpt{p[k], m[k], v[k], step[k], lr[k], beta1[k], beta2[k], eps[k], weight_decay[k]};
    }
    long groups = 0;
    for (int k = 0; k < nseg; ++k) {
        if (!g[k] || n[k] <= 0 || off[k] < 0 || opt[k] < 0 || opt[k] >= nopt) return EXO_EINVAL;
        a.s[k] = AdamSeg{g[k], (long)off[k], n[k], opt[k]};
        a.q0[k] = (int)groups;
        groups += (n[k] + 3) / 4;
    }
    if (groups >= (1L << 30)) return EXO_ERANGE;
    a.q0[nseg] = (int)groups;
    const long blocks = std::min<long>(ADAM_MULTI_BLOCKS, (groups + ADAM_THREADS - 1) / ADAM_THREADS);
    hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks), dim3(ADAM_THREADS), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

/* One Adam step over a flat fp32 buffer of n parameters (see adam_kernel). */
int td7_adam_step(float *p, const float *g, float *m, float *v, float *step, uint32_t *ticket, int64_t n, float lr,
                  float beta1, float beta2, float eps, float weight_decay, float grad_scale, void *stream) {
    if (!p || !g || !m || !v || !step || !ticket || n <= 0) return EXO_EINVAL;
    const long blocks = std::min<long>(ADAM_BLOCKS, (n / 4 + ADAM_THREADS - 1) / ADAM_THREADS + 1);
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(ADAM_THREADS), 0, (hipStream_t)stream, p, g, m, v,
                       step, ticket, (long)n, lr, beta1, beta2, eps, weight_decay, grad_scale);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

} // extern "C"
