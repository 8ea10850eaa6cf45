// td7_loss.hip -- the scalar tail of the TD7 critic update (gfx950).
//
// Agent/TD7_multi_agent.py:240-262, per row b of a batch of B (<= 65536):
//   Q_target = reward + not_done * discount * clamp(min_h Qt[b][h], min_target, max_target)
//   running max / min of Q_target                                    (:245-246)
//   td = |Q[b][h] - Q_target[b]|;  loss = mean_b sum_h LAP_huber(td)  (:257-259, :57-58)
//   priority = max_h(td).clamp(min = min_priority) ** alpha          (:262)
// PyTorch spends ~25 elementwise/reduction launches on these (and as many on
// the loss backward); here it is one workgroup per call: q_target, and
// critic_loss which also leaves dloss/dQ per element for the backward.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "philox.h"
#include "exo_amd.h"

namespace {

constexpr int T = 1024;

__device__ float block_reduce(float v, int op, float *sh) { // op 0 sum, 1 max, 2 min
    for (int o = 32; o > 0; o >>= 1) {
        const float u = __shfl_xor(v, o, 64);
        v = op == 0 ? v + u : (op == 1 ? fmaxf(v, u) : fminf(v, u));
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < T / 64; ++k) v = op == 0 ? v + sh[k] : (op == 1 ? fmaxf(v, sh[k]) : fminf(v, sh[k]));
        sh[0] = v;
    }
    __syncthreads();
    return sh[0];
}

__global__ __launch_bounds__(T) void q_target_kernel(const float *qt, long qs_b, long qs_h, const float *reward,
                                                     const float *not_done, float discount, const float *lo,
                                                     const float *hi, float *run_max, float *run_min, float *out,
                                                     int B) {
    __shared__ float sh[T / 64];
    const float l = *lo, h = *hi;
    float mx = -INFINITY, mn = INFINITY;
    for (int b = threadIdx.x; b < B; b += T) {
        const float q = fminf(qt[b * qs_b], qt[b * qs_b + qs_h]);
        const float c = fminf(fmaxf(q, l), h);                 // torch.clamp(min=l, max=h)
        const float v = reward[b] + (not_done[b] * discount) * c;
        out[b] = v;
        mx = fmaxf(mx, v);
        mn = fminf(mn, v);
    }
    mx = block_reduce(mx, 1, sh);
    mn = block_reduce(mn, 2, sh);
    if (threadIdx.x == 0) {
        *run_max = fmaxf(*run_max, mx);
        *run_min = fminf(*run_min, mn);
    }
}

__global__ __launch_bounds__(T) void critic_loss_kernel(const float *q, long qs_b, long qs_h, const float *qtarget,
                                                        float *loss, float *priority, float *dq, long dqs_b,
                                                        long dqs_h, float alpha, float min_priority, int B) {
    __shared__ float sh[T / 64];
    float acc = 0.f;
    const float inv_b = 1.0f / (float)B;
    for (int b = threadIdx.x; b < B; b += T) {
        const float t = qtarget[b];
        float tdmax = 0.f;
        for (int hd = 0; hd < 2; ++hd) {
            const float d = q[b * qs_b + hd * qs_h] - t;
            const float x = fabsf(d);
            acc += x < 1.0f ? 0.5f * x * x : x;               // LAP_huber, min_priority = 1 (:259)
            const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
            dq[b * dqs_b + hd * dqs_h] = inv_b * (x < 1.0f ? x : 1.0f) * sg;
            tdmax = fmaxf(tdmax, x);
        }
        priority[b] = powf(fmaxf(tdmax, min_priority), alpha);
    }
    acc = block_reduce(acc, 0, sh);
    if (threadIdx.x == 0) *loss = acc * inv_b;
}


// Exploration / target-policy noise on an action batch (one workgroup):
//   out = clamp(a + c(noise * sigma), -1, 1) * scale,  c = clamp(+-clip) if clip > 0
//   sigma -= sigma_dec (after every element has used the old value)
// select_action (TD7_multi_agent_Pink_noise.py:209-228 batched; clip 0) and the
// critic target's smoothed next action (TD7_multi_agent.py:236-238).
__global__ __launch_bounds__(T) void noisy_action_kernel(const float *a, const float *noise, float *sigma,
                                                         float sigma_dec, float clip, float scale, float *out, int n) {
    const float sg = *sigma;
    for (int i = threadIdx.x; i < n; i += T) {
        float e = noise[i] * sg;
        if (clip > 0.f) e = fminf(fmaxf(e, -clip), clip);
        out[i] = fminf(fmaxf(a[i] + e, -1.0f), 1.0f) * scale;
    }
    __syncthreads();
    if (threadIdx.x == 0) *sigma = sg - sigma_dec;
}

// noisy_action_kernel with the noise drawn in the kernel: element 2j+t is
// normal t of Philox block j of this call (Box-Muller); the device call
// counter advances by one per launch (no host value: graph-replay safe).
__global__ __launch_bounds__(T) void noisy_action_rng_kernel(const float *a, uint64_t seed, uint32_t tag,
                                                             unsigned long long *counter, uint32_t *ticket,
                                                             float *sigma, float sigma_dec, float clip, float scale,
                                                             float *out, int n, const int32_t *dec_count) {
    const float sg = *sigma;
    const unsigned long long call = *counter;
    for (int j = blockIdx.x * T + threadIdx.x; 2 * j < n; j += gridDim.x * T) {
        uint32_t r[4];
        philox_block(seed, tag, call, (uint32_t)j, r);
        float z[2];
        box_muller(r, z[0], z[1]);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int i = 2 * j + t;
            if (i >= n) break;
            float e = z[t] * sg;
            if (clip > 0.f) e = fminf(fmaxf(e, -clip), clip);
            out[i] = fminf(fmaxf(a[i] + e, -1.0f), 1.0f) * scale;
        }
    }
    // every workgroup has read sigma and the call number: the last one out
    // advances both
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(ticket, 1u) == gridDim.x - 1) {
            *sigma = sg - (dec_count ? sigma_dec * (float)*dec_count : sigma_dec);
            *counter = call + 1ull;
            *ticket = 0u;
        }
    }
}

// F.mse_loss(pred, target) forward (mean of squared differences over n) and
// its backward d/dpred = 2 (pred - target) / n * g.
constexpr int MSE_BLOCKS = 256; // == TD7_MSE_WS - 1
__global__ __launch_bounds__(256) void mse_fwd_kernel(const float *x, const float *y, long n, float *loss, float *ws) {
    __shared__ float sh[256 / 64];
    __shared__ bool last;
    float acc = 0.f;
    const long stride = (long)gridDim.x * 256;
    if ((n & 3) == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0) {
        const float4 *x4 = reinterpret_cast<const float4 *>(x), *y4 = reinterpret_cast<const float4 *>(y);
        for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n / 4; i += stride) {
            const float4 a = x4[i], b = y4[i];
            const float d0 = a.x - b.x, d1 = a.y - b.y, d2 = a.z - b.z, d3 = a.w - b.w;
            acc += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
        }
    } else {
        for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
            const float d = x[i] - y[i];
            acc += d * d;
        }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    // block partials -> ws[b]; the last block to finish sums them in block
    // order (deterministic) and re-arms the ticket (ws[MSE_BLOCKS]) to zero
    unsigned *ticket = reinterpret_cast<unsigned *>(ws + MSE_BLOCKS);
    if (threadIdx.x == 0) {
        ws[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
        __threadfence();
        last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last || threadIdx.x >= 64) return;
    __threadfence();
    float v = 0.f;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += 64) v += __builtin_nontemporal_load(ws + b);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (threadIdx.x == 0) {
        *loss = v / (float)n;
        *ticket = 0u;
    }
}

__global__ __launch_bounds__(256) void mse_bwd_kernel(const float *x, const float *y, const float *g, long n,
                                                      float *dx) {
    const float c = 2.0f * *g / (float)n;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dx[i] = c * (x[i] - y[i]);
}

} // namespace

extern "C" {

int td7_q_target(const float *qt, long qs_b, long qs_h, const float *reward, const float *not_done, float discount,
                 const float *min_target, const float *max_target, float *run_max, float *run_min, float *out,
                 int32_t batch, void *stream) {
    if (!qt || !reward || !not_done || !min_target || !max_target || !run_max || !run_min || !out || batch <= 0)
        return EXO_EINVAL;
    hipLaunchKernelGGL(q_target_kernel, dim3(1), dim3(T), 0, (hipStream_t)stream, qt, qs_b, qs_h, reward, not_done,
                       discount, min_target, max_target, run_max, run_min, out, batch);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7_critic_loss(const float *q, long qs_b, long qs_h, const float *q_target, float *loss, float *priority,
                    float *dq, float alpha, float min_priority, int32_t batch, void *stream) {
    return td7_critic_loss_strided(q, qs_b, qs_h, q_target, loss, priority, dq, 2, 1, alpha, min_priority, batch,
                                   stream);
}

int td7_critic_loss_strided(const float *q, long qs_b, long qs_h, const float *q_target, float *loss,
                            float *priority, float *dq, long dqs_b, long dqs_h, float alpha, float min_priority,
                            int32_t batch, void *stream) {
    if (!q || !q_target || !loss || !priority || !dq || batch <= 0) return EXO_EINVAL;
    hipLaunchKernelGGL(critic_loss_kernel, dim3(1), dim3(T), 0, (hipStream_t)stream, q, qs_b, qs_h, q_target, loss,
                       priority, dq, dqs_b, dqs_h, alpha, min_priority, batch);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7_noisy_action(const float *a, const float *noise, float *sigma, float sigma_dec, float clip, float scale,
                     float *out, int32_t n, void *stream) {
    if (!a || !noise || !sigma || !out || n < 0) return EXO_EINVAL;
    if (n == 0) return EXO_OK;
    hipLaunchKernelGGL(noisy_action_kernel, dim3(1), dim3(T), 0, (hipStream_t)stream, a, noise, sigma, sigma_dec, clip,
                       scale, out, n);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7_noisy_action_rng(const float *a, uint64_t seed, uint32_t tag, unsigned long long *counter,
                         uint32_t *ticket, float *sigma, float sigma_dec, float clip, float scale, float *out,
                         int32_t n, const int32_t *dec_count, void *stream) {
    if (!a || !counter || !ticket || !sigma || !out || n < 0) return EXO_EINVAL;
    const int blocks = std::max(1, std::min(256, (n / 2 + T - 1) / T));
    hipLaunchKernelGGL(noisy_action_rng_kernel, dim3(blocks), dim3(T), 0, (hipStream_t)stream, a, seed, tag, counter,
                       ticket, sigma, sigma_dec, clip, scale, out, n, dec_count);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7_mse_fwd(const float *x, const float *y, int64_t n, float *loss, float *ws, void *stream) {
    if (!x || !y || !loss || !ws || n <= 0) return EXO_EINVAL;
    const long blocks = std::min<long>(MSE_BLOCKS, (n / 4 + 255) / 256 + 1);
    hipLaunchKernelGGL(mse_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, y, (long)n, loss,
                       ws);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7_mse_bwd(const float *x, const float *y, const float *g, int64_t n, float *dx, void *stream) {
    if (!x || !y || !g || !dx || n <= 0) return EXO_EINVAL;
    const long blocks = std::min<long>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(mse_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, y, g, (long)n, dx);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

} // extern "C"
