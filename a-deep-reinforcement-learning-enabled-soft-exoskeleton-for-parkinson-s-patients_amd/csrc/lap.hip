// lap.hip -- LAP prioritised replay (Agent/TD7_buffer_multi_agent.py) as
// per-stratum binary sum trees on gfx950.
//
// The reference keeps one priority row per env ("stratum", :41) and samples
// batch_size indices from every row with torch.cumsum + torch.searchsorted
// (:75-78): O(size) work and a host sync per row per training step.  Here
// every stratum owns a complete binary tree over `cap` (power of two) leaves,
// tree[s][1] is the row total and leaf i lives at tree[s][cap + i].  The
// caller owns the memory (torch tensors) and describes it with lap_tree_desc:
//   sample : one lane per draw descends log2(cap) levels,
//   update : leaves are written (last duplicate wins, like the reference's CPU
//            index_put at :115), then the touched ancestors are recomputed
//            level by level inside one workgroup per stratum (deterministic:
//            a parent is always left + right of final children),
//   max    : max_priority lives in device memory (no host sync, :116, :120).
// For integer-valued priorities the descent returns exactly
// searchsorted_left(cumsum(p), u * sum(p)).
#include <hip/hip_runtime.h>

#include <string>

#include "exo_amd.h"

namespace {

constexpr int UPD_THREADS = 1024;

__device__ __forceinline__ float *stratum_tree(float *tree, int s, int cap) { return tree + (size_t)s * 2 * cap; }

// Recompute the ancestors of the n leaves slot[0..n) of one stratum, bottom-up.
__device__ void propagate(float *T, int cap, int levels, const int32_t *slot, int n) {
    for (int lv = 1; lv <= levels; ++lv) {
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const int node = (cap + slot[k]) >> lv;
            T[node] = T[2 * node] + T[2 * node + 1];
        }
    }
    __syncthreads();
}

// LAP.add: new items get max_priority (:56-57).  The items of this block's
// stratum are gathered in chunks of ADD_CHUNK into LDS, their leaves written,
// then their ancestors recomputed.
constexpr int ADD_CHUNK = 4096;
__global__ __launch_bounds__(UPD_THREADS) void lap_add_kernel(float *tree, const float *maxp, int cap, int levels,
                                                              int capacity, const int32_t *stratum,
                                                              const int32_t *slot, int n) {
    const int s = blockIdx.x;
    float *T = stratum_tree(tree, s, cap);
    __shared__ int32_t mine[ADD_CHUNK];
    __shared__ int count;
    const float p = *maxp;
    for (int base = 0; base < n; base += ADD_CHUNK) {
        if (threadIdx.x == 0) count = 0;
        __syncthreads();
        const int end = min(n, base + ADD_CHUNK);
        for (int k = base + threadIdx.x; k < end; k += blockDim.x) {
            if (stratum[k] != s) continue;
            const int sl = slot[k];
            if (sl < 0 || sl >= capacity) continue;
            T[cap + sl] = p;
            mine[atomicAdd(&count, 1)] = sl;
        }
        __syncthreads();
        propagate(T, cap, levels, mine, count);
    }
}

// LAP.sample (:75-78): idx = searchsorted_left(cumsum(p[:size]), u * total)
__global__ void lap_sample_kernel(const float *tree, int cap, int levels, const float *u, const int32_t *size,
                                  int batch, int32_t *idx) {
    const int s = blockIdx.y;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const float *T = tree + (size_t)s * 2 * cap;
    float val = u[(size_t)s * batch + b] * T[1];
    int node = 1;
    for (int lv = 0; lv < levels; ++lv) {
        const float left = T[2 * node], right = T[2 * node + 1];
        if (val <= left || right <= 0.0f) {
            node = 2 * node;
        } else {
            val -= left;
            node = 2 * node + 1;
        }
    }
    int i = node - cap;
    const int sz = size[s];
    if (i >= sz) i = sz > 0 ? sz - 1 : 0;
    idx[(size_t)s * batch + b] = i;
}

// LAP.update_priority (:113-117)
__global__ __launch_bounds__(UPD_THREADS) void lap_update_kernel(float *tree, float *maxp, int cap, int levels,
                                                                 const int32_t *idx, const float *prio,
                                                                 int batch) {
    const int s = blockIdx.x;
    float *T = stratum_tree(tree, s, cap);
    const int32_t *I = idx + (size_t)s * batch;
    const float *P = prio + (size_t)s * batch;
    __shared__ float red[UPD_THREADS / 64];
    float mx = 0.0f;
    for (int b = threadIdx.x; b < batch; b += blockDim.x) {
        bool last = true; // a later duplicate overwrites this one
        for (int b2 = b + 1; b2 < batch; ++b2) last &= (I[b2] != I[b]);
        if (last) T[cap + I[b]] = P[b];
        mx = fmaxf(mx, P[b]);
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    propagate(T, cap, levels, I, batch);
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) mx = fmaxf(mx, red[w]);
        // priorities are >= min_priority^alpha > 0: int order == float order
        atomicMax(reinterpret_cast<int *>(maxp), __float_as_int(mx));
    }
}

// LAP.reset_max_priority (:119-120): max over every leaf of every stratum.
// maxp is zeroed by the launcher first; leaves are >= 0 so int order works.
__global__ void lap_reset_max_kernel(const float *tree, float *maxp, int cap, int n_strata) {
    __shared__ float red[16];
    float mx = 0.0f;
    const size_t total = (size_t)n_strata * cap;
    for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += (size_t)gridDim.x * blockDim.x) {
        const size_t s = k / cap, i = k % cap;
        mx = fmaxf(mx, tree[s * 2 * cap + cap + i]);
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) mx = fmaxf(mx, red[w]);
        atomicMax(reinterpret_cast<int *>(maxp), __float_as_int(mx));
    }
}

__global__ void lap_totals_kernel(const float *tree, int cap, int n_strata, float *out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n_strata) out[s] = tree[(size_t)s * 2 * cap + 1];
}

__global__ void lap_init_kernel(float *maxp) { *maxp = 1.0f; } // max_priority = 1 (:42)

int rc(hipError_t e) { return e == hipSuccess ? EXO_OK : EXO_EDEVICE; }

int levels_of(const lap_tree_desc *t) {
    int lv = 0;
    while ((1 << lv) < t->cap) ++lv;
    return lv;
}

bool valid(const lap_tree_desc *t) {
    return t && t->tree && t->max_priority && t->n_strata > 0 && t->capacity > 0 && t->cap >= t->capacity &&
           (t->cap & (t->cap - 1)) == 0;
}

} // namespace

extern "C" {

int32_t lap_tree_floats(int32_t n_strata, int32_t capacity) {
    int cap = 1;
    while (cap < capacity) cap <<= 1;
    return n_strata * 2 * cap;
}

int lap_init(const lap_tree_desc *t, void *stream) {
    if (!valid(t)) return EXO_EINVAL;
    hipError_t e = hipMemsetAsync(t->tree, 0, (size_t)t->n_strata * 2 * t->cap * sizeof(float), (hipStream_t)stream);
    if (e != hipSuccess) return EXO_EDEVICE;
    hipLaunchKernelGGL(lap_init_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, t->max_priority);
    return rc(hipGetLastError());
}

int lap_add(const lap_tree_desc *t, const int32_t *stratum, const int32_t *slot, int32_t n, void *stream) {
    if (!valid(t) || !stratum || !slot || n < 0) return EXO_EINVAL;
    if (n == 0) return EXO_OK;
    hipLaunchKernelGGL(lap_add_kernel, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream, t->tree,
                       t->max_priority, t->cap, levels_of(t), t->capacity, stratum, slot, n);
    return rc(hipGetLastError());
}

int lap_sample(const lap_tree_desc *t, const float *u, const int32_t *size, int32_t batch, int32_t *idx, void *stream) {
    if (!valid(t) || !u || !size || !idx || batch <= 0) return EXO_EINVAL;
    const int th = 128;
    hipLaunchKernelGGL(lap_sample_kernel, dim3((batch + th - 1) / th, t->n_strata), dim3(th), 0, (hipStream_t)stream,
                       t->tree, t->cap, levels_of(t), u, size, batch, idx);
    return rc(hipGetLastError());
}

int lap_update(const lap_tree_desc *t, const int32_t *idx, const float *prio, int32_t batch, void *stream) {
    if (!valid(t) || !idx || !prio || batch <= 0) return EXO_EINVAL;
    hipLaunchKernelGGL(lap_update_kernel, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream, t->tree,
                       t->max_priority, t->cap, levels_of(t), idx, prio, batch);
    return rc(hipGetLastError());
}

int lap_reset_max(const lap_tree_desc *t, void *stream) {
    if (!valid(t)) return EXO_EINVAL;
    hipError_t e = hipMemsetAsync(t->max_priority, 0, sizeof(float), (hipStream_t)stream);
    if (e != hipSuccess) return EXO_EDEVICE;
    hipLaunchKernelGGL(lap_reset_max_kernel, dim3(256), dim3(1024), 0, (hipStream_t)stream, t->tree, t->max_priority,
                       t->cap, t->n_strata);
    return rc(hipGetLastError());
}

int lap_totals(const lap_tree_desc *t, float *out, void *stream) {
    if (!valid(t) || !out) return EXO_EINVAL;
    hipLaunchKernelGGL(lap_totals_kernel, dim3((t->n_strata + 63) / 64), dim3(64), 0, (hipStream_t)stream, t->tree,
                       t->cap, t->n_strata, out);
    return rc(hipGetLastError());
}

} // extern "C"
