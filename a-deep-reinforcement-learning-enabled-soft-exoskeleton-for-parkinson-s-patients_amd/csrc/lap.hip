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

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "philox.h"
#include "exo_amd.h"

namespace {

constexpr int UPD_THREADS = 1024;

__device__ __forceinline__ float *stratum_tree(float *tree, int s, int cap) { return tree + (size_t)s * 2 * cap; }

// Recompute the ancestors of the n leaves slot[0..n) of one stratum, bottom-up,
// one level per barrier.  The lower levels work in global memory; once every
// parent of a level is below TOPN/2 the top of the tree (nodes [1, TOPN), the
// parents and their children) is staged in LDS and the remaining levels (12 of
// the 18 of a 250k-slot stratum) run there -- one L2 round trip per level
// fewer -- and the recomputed nodes [1, TOPN/2) are written back.  The same
// additions in the same order: the sums are bit-identical.
constexpr int TOPN = 8192;
// top: the caller's LDS array of NTOP floats; on return (true) it holds the
// final nodes [1, min(NTOP, 2 cap)) (false: no level was staged, T holds them).
// The staging loads are all issued before their LDS stores (one round trip).
template <int NTOP = TOPN>
__device__ bool propagate_top(float *T, int cap, int levels, const int32_t *slot, int n, float *top) {
    int lv = 1;
    for (; lv <= levels && ((2 * cap) >> lv) > NTOP / 2; ++lv) {
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const int node = (cap + slot[k]) >> lv;
            T[node] = T[2 * node] + T[2 * node + 1];
        }
    }
    __syncthreads();
    if (lv > levels) return false;
    const int lim = min(NTOP, 2 * cap);
    if (blockDim.x == UPD_THREADS) {
        constexpr int PER = NTOP / UPD_THREADS;
        float v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = threadIdx.x + j * UPD_THREADS;
            v[j] = i < lim ? T[i] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = threadIdx.x + j * UPD_THREADS;
            if (i < lim) top[i] = v[j];
        }
    } else {
        for (int i = threadIdx.x; i < lim; i += blockDim.x) top[i] = T[i];
    }
    for (; lv <= levels; ++lv) {
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const int node = (cap + slot[k]) >> lv;
            top[node] = top[2 * node] + top[2 * node + 1];
        }
    }
    __syncthreads();
    const int wb = min(NTOP / 2, cap);
    for (int i = 1 + threadIdx.x; i < wb; i += blockDim.x) T[i] = top[i];
    __syncthreads();
    return true;
}
__device__ void propagate(float *T, int cap, int levels, const int32_t *slot, int n) {
    __shared__ float top[TOPN];
    propagate_top(T, cap, levels, slot, n, top);
}

// The same recomputation for the leaves of a ring span: `count` consecutive
// slots from `first`, wrapping at `capacity` (all of them once count reaches
// it).  The ancestors of a contiguous leaf range at one level are a contiguous
// node range, so each level is a loop over (at most two) node ranges instead
// of a per-slot list; the nodes recomputed, and every sum, are the ones
// propagate computes for the same slots.
__device__ void propagate_span(float *T, int cap, int levels, int capacity, int first, int count) {
    __shared__ float top[TOPN];
    if (count <= 0) return;
    int a0 = first, e0 = first + count, a1 = 0, e1 = 0;  // [a0, e0) and [a1, e1)
    if (count >= capacity) {
        a0 = 0;
        e0 = capacity;
    } else if (e0 > capacity) {
        e1 = e0 - capacity;
        e0 = capacity;
    }
    int lv = 1;
    for (; lv <= levels && ((2 * cap) >> lv) > TOPN / 2; ++lv) {
        __syncthreads();
        const int lo0 = (cap + a0) >> lv, n0 = ((cap + e0 - 1) >> lv) - lo0 + 1;
        const int lo1 = (cap + a1) >> lv, n1 = e1 > a1 ? ((cap + e1 - 1) >> lv) - lo1 + 1 : 0;
        for (int k = threadIdx.x; k < n0 + n1; k += blockDim.x) {
            const int node = k < n0 ? lo0 + k : lo1 + k - n0;
            T[node] = T[2 * node] + T[2 * node + 1];
        }
    }
    __syncthreads();
    if (lv > levels) return;
    const int lim = min(TOPN, 2 * cap);
    for (int i = threadIdx.x; i < lim; i += blockDim.x) top[i] = T[i];
    for (; lv <= levels; ++lv) {
        __syncthreads();
        const int lo0 = (cap + a0) >> lv, n0 = ((cap + e0 - 1) >> lv) - lo0 + 1;
        const int lo1 = (cap + a1) >> lv, n1 = e1 > a1 ? ((cap + e1 - 1) >> lv) - lo1 + 1 : 0;
        for (int k = threadIdx.x; k < n0 + n1; k += blockDim.x) {
            const int node = k < n0 ? lo0 + k : lo1 + k - n0;
            top[node] = top[2 * node] + top[2 * node + 1];
        }
    }
    __syncthreads();
    const int wb = min(TOPN / 2, cap);
    for (int i = 1 + threadIdx.x; i < wb; i += blockDim.x) T[i] = top[i];
    __syncthreads();
}

// propagate_span for a span that does not wrap and holds at most SPAN_LDS - 2
// leaves, every level in LDS: the span's nodes of one level are a contiguous
// range [lo, hi] whose children are [lo & ~1, hi | 1] of the level below --
// the span's own recomputed nodes plus at most one unchanged sibling at each
// end.  The siblings of every level are outside the span, so nothing in this
// launch writes them: all of them are loaded up front (one round trip), the
// span's leaves once, and then each level is one barrier of LDS work whose
// results also go to the tree (stores nothing waits for).  The same operands
// in the same order as propagate_span: bit-identical.  Returns false (nothing
// done) when the span does not qualify.
constexpr int SPAN_LDS = 4096;
constexpr int SPAN_LEVELS = 32;
__device__ bool propagate_span_lds(float *T, int cap, int levels, int capacity, int first, int count,
                                   float *buf /* 2 SPAN_LDS */, float *edge /* 2 SPAN_LEVELS */) {
    const int a = cap + first, e = cap + first + count - 1;  // leaf nodes [a, e]
    if (count <= 0 || first + count > capacity || count > SPAN_LDS - 2 || levels >= SPAN_LEVELS) return false;
    // edge[2 lv], edge[2 lv + 1]: the unchanged left / right sibling at level lv
    // (the children of level lv + 1's range), when that range needs one
    const int t = threadIdx.x;
    if (t < 2 * levels) {
        const int lv = t >> 1, right = t & 1;
        const int lo = a >> lv, hi = e >> lv;
        if (!right && (lo & 1)) edge[t] = T[lo - 1];
        if (right && !(hi & 1)) edge[t] = T[hi + 1];
    }
    float *A = buf, *B = buf + SPAN_LDS;
    // level 0: A[c - (a & ~1)] for c in [a & ~1, e | 1]
    {
        const int base = a & ~1;
        for (int c = a + t; c <= e; c += blockDim.x) A[c - base] = T[c];
    }
    __syncthreads();
    if (t == 0) {
        if (a & 1) A[0] = edge[0];
        if (!(e & 1)) A[(e | 1) - (a & ~1)] = edge[1];
    }
    for (int lv = 1; lv <= levels; ++lv) {
        __syncthreads();
        const int lo = a >> lv, hi = e >> lv, cbase = (a >> (lv - 1)) & ~1, nbase = lo & ~1;
        for (int node = lo + t; node <= hi; node += blockDim.x) {
            const int c = 2 * node - cbase;
            const float v = A[c] + A[c + 1];
            T[node] = v;
            B[node - nbase] = v;
        }
        if (t == 0 && lv < levels) {
            if (lo & 1) B[0] = edge[2 * lv];
            if (!(hi & 1)) B[(hi | 1) - nbase] = edge[2 * lv + 1];
        }
        float *tmp = A;
        A = B;
        B = tmp;
    }
    __syncthreads();
    return true;
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

// Sum of the leaves [0, sz) of one stratum's tree: the reference samples
// against cumsum(priority[i, :size]) (:76-77), and with its single-add pointer
// quirk (:59-61) strata 1..E-1 hold their newest transition at slot == size,
// outside that prefix -- so the draw is scaled by the prefix total, not the
// root.  One root-to-leaf walk towards leaf sz adding every left sibling.
// The walk's nodes depend on sz alone (step j visits (1 << j) | sz >> (levels
// - j)): every addend is loaded first, independently, and then added in the
// walk's order (an unset bit adds +0: the same sum) -- one memory round trip
// instead of one per level.  at(node): the tree accessor.
constexpr int MAXLV = 24;  // levels of a stratum tree (capacity <= 2^24)
template <class At>
__device__ __forceinline__ float prefix_sum(At at, int cap, int levels, int sz) {
    if (sz >= cap) return at(1);
    float v[MAXLV];
#pragma unroll
    for (int j = 0; j < MAXLV; ++j) {
        v[j] = 0.0f;
        if (j < levels) {
            const int lv = levels - 1 - j;
            const float x = at(2 * ((1 << j) | (sz >> (lv + 1))));
            v[j] = ((sz >> lv) & 1) ? x : 0.0f;
        }
    }
    float acc = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXLV; ++j)
        if (j < levels) acc += v[j];
    return acc;
}
__device__ __forceinline__ float prefix_total(const float *T, int cap, int levels, int sz) {
    return prefix_sum([T](int n) { return T[n]; }, cap, levels, sz);
}

__device__ __forceinline__ float sel4(int r, float a, float b, float c, float d) {
    return r == 0 ? a : r == 1 ? b : r == 2 ? c : d;
}

// The descent from `node` at level lv to a leaf: at every level go left when
// val <= left (or the right subtree is empty), else subtract left and go
// right.  The children of the next (up to) three levels are read together --
// 2 + 4 + 8 nodes at 2n, 4n, 8n -- and the three choices made from registers:
// the same comparisons and subtractions as the one-level walk, a third of its
// dependent memory round trips.  Returns the leaf node.
template <class At>
__device__ __forceinline__ int descend_from(At at, float val, int node, int lv, int levels) {
    while (lv < levels) {
        const int k = levels - lv >= 3 ? 3 : levels - lv;
        const int n1 = 2 * node, n2 = 4 * node, n3 = 8 * node;
        const float a0 = at(n1), a1 = at(n1 + 1);
        float b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
        float c4 = 0.f, c5 = 0.f, c6 = 0.f, c7 = 0.f;
        if (k >= 2) b0 = at(n2), b1 = at(n2 + 1), b2 = at(n2 + 2), b3 = at(n2 + 3);
        if (k >= 3) {
            c0 = at(n3), c1 = at(n3 + 1), c2 = at(n3 + 2), c3 = at(n3 + 3);
            c4 = at(n3 + 4), c5 = at(n3 + 5), c6 = at(n3 + 6), c7 = at(n3 + 7);
        }
        int r;
        if (val <= a0 || a1 <= 0.0f) {
            r = 0;
        } else {
            val -= a0;
            r = 1;
        }
        if (k >= 2) {
            const float l = r ? b2 : b0, rt = r ? b3 : b1;
            if (val <= l || rt <= 0.0f) {
                r = 2 * r;
            } else {
                val -= l;
                r = 2 * r + 1;
            }
            if (k >= 3) {
                const float l3 = sel4(r, c0, c2, c4, c6), r3 = sel4(r, c1, c3, c5, c7);
                if (val <= l3 || r3 <= 0.0f) {
                    r = 2 * r;
                } else {
                    val -= l3;
                    r = 2 * r + 1;
                }
            }
        }
        node = (node << k) + r;
        lv += k;
    }
    return node;
}

// LAP.sample (:75-78): idx = searchsorted_left(cumsum(p[:size]), u * total)
__global__ void lap_sample_kernel(const float *tree, int cap, int levels, const float *u, const int32_t *size,
                                  int batch, int32_t *idx) {
    const int s = blockIdx.y;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const float *T = tree + (size_t)s * 2 * cap;
    const int sz = size[s];
    const float val = u[(size_t)s * batch + b] * prefix_total(T, cap, levels, sz);
    const int node = descend_from([T](int n) { return T[n]; }, val, 1, 0, levels);
    int i = node - cap;
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
    __shared__ int32_t li[UPD_THREADS];
    float mx = 0.0f;
    for (int b0 = 0; b0 < batch; b0 += UPD_THREADS) { // the batch's indices staged in LDS
        const int nb = min(UPD_THREADS, batch - b0);
        __syncthreads();
        if ((int)threadIdx.x < nb) li[threadIdx.x] = I[b0 + threadIdx.x];
        __syncthreads();
        const int b = b0 + threadIdx.x;
        if (b < batch) {
            const int me = li[threadIdx.x];
            bool last = true; // a later duplicate overwrites this one
            for (int k = threadIdx.x + 1; k < nb; ++k) last &= (li[k] != me);
            for (int b2 = b0 + nb; b2 < batch; ++b2) last &= (I[b2] != me);
            if (last) T[cap + me] = P[b];
            mx = fmaxf(mx, P[b]);
        }
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


// ---------------------------------------------------------------- batched store
// LAP.add for every env of one vectorised step (:49-63 per row): the rows of
// stratum s go to consecutive ring slots starting at ptr[s], in env order.
// Phase 1 (one workgroup per stratum): block scan of "row i is active and in
// stratum s" -> slot of every row (the trash row `capacity` for inactive ones),
// new leaves = max_priority, ring pointer and size; the stratum's new slots are
// one ring span, whose ancestors are recomputed once after the last chunk
// (propagate_span; r03d: a propagate per 4,096-row chunk made the 65,536-env
// store 158 us).
// Phase 2 (many workgroups): one wavefront per row copies its transition.
constexpr int STORE_CHUNK = UPD_THREADS * 4;

template <int RANK_RPT>
__global__ __launch_bounds__(UPD_THREADS) void lap_store_rank_kernel(float *tree, const float *maxp, int cap,
                                                                     int levels, int capacity, int32_t *ring_ptr,
                                                                     int32_t *ring_size, const int32_t *strata,
                                                                     const uint8_t *active, int n, int32_t *row_of) {
    const int s = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    float *T = stratum_tree(tree, s, cap);
    __shared__ int wsum[UPD_THREADS / 64];
    __shared__ int chunk_total;
    const float p = *maxp;
    const int ptr0 = ring_ptr[s];
    const int row0 = s * (capacity + 1);
    int offset = 0; // rows of this stratum placed by earlier chunks
    // RANK_RPT consecutive rows per thread (their strata kept in registers):
    // 16 above 16,384 envs -- 4 chunks of 16,384 rows at 65,536 envs instead of
    // 16 of 4,096, each chunk paying a load latency and two barriers -- and 4
    // below (one chunk at 4,096 envs either way; 16 serial rows per thread
    // measured 16.2 vs 15.0 us there, profiles/r03d_raw/lap2)
    for (int base = 0; base < n; base += RANK_RPT * UPD_THREADS) {
        int st[RANK_RPT], cnt = 0;
        bool f[RANK_RPT];
#pragma unroll
        for (int k = 0; k < RANK_RPT; ++k) {
            const int i = base + RANK_RPT * t + k;
            st[k] = i < n ? strata[i] : -1;
            f[k] = i < n && (!active || active[i]);
        }
#pragma unroll
        for (int k = 0; k < RANK_RPT; ++k) {
            f[k] = f[k] && st[k] == s;
            cnt += f[k];
        }
        // block-wide exclusive scan of cnt
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        if (t == 0) {
            int acc = 0;
            for (int k = 0; k < UPD_THREADS / 64; ++k) {
                const int v = wsum[k];
                wsum[k] = acc;
                acc += v;
            }
            chunk_total = acc;
        }
        __syncthreads();
        int rank = offset + wsum[wv] + incl - cnt;
#pragma unroll
        for (int k = 0; k < RANK_RPT; ++k) {
            const int i = base + RANK_RPT * t + k;
            if (i >= n) continue;
            if (s == 0 && (st[k] < 0 || st[k] >= (int)gridDim.x)) row_of[i] = -1; // no stratum
            if (st[k] != s) continue;
            if (f[k]) {
                const int slot = (ptr0 + rank) % capacity;
                row_of[i] = row0 + slot;
                T[cap + slot] = p;
                ++rank;
            } else {
                row_of[i] = row0 + capacity; // inactive env: the trash row
            }
        }
        const int total = chunk_total;
        __syncthreads();
        offset += total;
    }
    propagate_span(T, cap, levels, capacity, ptr0, offset);
    if (t == 0) {
        ring_ptr[s] = (ptr0 + offset) % capacity;
        ring_size[s] = min(ring_size[s] + offset, capacity);
    }
}

// LAP.add with the reference's SHARED pointer (:49-63), called for every
// active env of one vectorised step in env order -- what the training script's
// per-env loop does (Exoskeleton_agent_train.py:139-142).  The c-th add writes
// slot ptr0 + #{multiples of E in [count0, c)} of its stratum (the pointer
// advances after an add whose count is a multiple of E = num_envs, :59-61), so
// env 0's first transition sits one slot behind the others and, when envs are
// done, two adds of one stratum can land in the same slot -- the later one
// wins, as the reference's overwrite.  One workgroup: a block scan ranks the
// active rows (rank_row[r] = the stratum of rank r), every active row checks
// the next E-1 ranks for a same-stratum, same-slot successor (two counts share
// a slot only if no multiple of E lies between them), winners get slot_of /
// row_of, losers and inactive rows -1.  ref = {ptr, count, size}; every
// stratum's size = size (the reference samples every row against the one
// shared size, :76).
__device__ __forceinline__ long long mult_below(long long x, int E) { return (x + E - 1) / E; }

__global__ __launch_bounds__(UPD_THREADS) void lap_store_ref_slots_kernel(int capacity, int E, long long *ref,
                                                                          int32_t *ring_size,
                                                                          const int32_t *strata,
                                                                          const uint8_t *active, int n,
                                                                          int32_t *rank_row, int32_t *slot_of,
                                                                          int32_t *row_of) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    __shared__ int wsum[UPD_THREADS / 64];
    __shared__ int chunk_total;
    const long long ptr0 = ref[0], count0 = ref[1], size0 = ref[2];
    const long long m0 = mult_below(count0, E);
    int offset = 0;
    for (int base = 0; base < n; base += STORE_CHUNK) {
        int f[4], cnt = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = base + 4 * t + k;
            f[k] = (i < n && strata[i] >= 0 && strata[i] < E && (!active || active[i])) ? 1 : 0;
            cnt += f[k];
        }
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        if (t == 0) {
            int acc = 0;
            for (int k = 0; k < UPD_THREADS / 64; ++k) {
                const int v = wsum[k];
                wsum[k] = acc;
                acc += v;
            }
            chunk_total = acc;
        }
        __syncthreads();
        int rank = offset + wsum[wv] + incl - cnt;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = base + 4 * t + k;
            if (i >= n) continue;
            if (f[k]) {
                rank_row[rank] = strata[i]; // the stratum of each rank (the winner pass reads it)
                row_of[i] = rank;           // the rank, until the winner pass below
                ++rank;
            } else {
                row_of[i] = -1;
                slot_of[i] = -1;
            }
        }
        offset += chunk_total;
        __syncthreads();
    }
    __threadfence_block();
    __syncthreads();
    const int n_act = offset;
    for (int i = t; i < n; i += blockDim.x) {
        const int r = row_of[i];
        if (r < 0) continue;
        const long long mr = mult_below(count0 + r, E);
        const int s = strata[i];
        bool win = true;
        // ranks r < q share r's slot while count0 + q <= mr E (ceil((count0 + q) / E) == mr):
        // one 64-bit product instead of a 64-bit division per candidate, and the
        // candidate's stratum read directly (one load, not rank -> row -> stratum)
        const long long qend = mr * E - count0;
        const int qmax = (int)min((long long)min(r + E, n_act) - 1, qend);
        for (int q = r + 1; q <= qmax; ++q) win &= rank_row[q] != s;
        long long v = ptr0 + (mr - m0); // ptr0 < capacity, mr - m0 <= n / E + 1
        if (v >= capacity) v -= capacity;
        if (v >= capacity) v %= capacity;
        const int slot = (int)v;
        slot_of[i] = win ? slot : -1;
        row_of[i] = win ? s * (capacity + 1) + slot : -1;
    }
    __syncthreads();
    const long long adv = mult_below(count0 + n_act, E) - m0;
    const long long size = min(size0 + adv, (long long)capacity);
    for (int s = t; s < E; s += blockDim.x) ring_size[s] = (int32_t)size;
    if (t == 0) {
        ref[0] = (ptr0 + adv) % capacity;
        ref[1] = count0 + n_act;
        ref[2] = size;
    }
}

// r04: lap_store_batch_ref as ONE launch (the three
// launches above cost ~28 us per 4,096-env step of the reference schedule).
// Grid (E strata) x (K copy parts), 1024 threads.  Every workgroup ranks the
// active rows (the same block scan, chunks of STORE_CHUNK rows) and keeps, for
// ITS stratum, the rows in rank order (LDS).  The winner test needs no rank ->
// stratum table: a row loses iff the next active row of the SAME stratum
// shares its slot (the c-th add's slot depends only on ceil((count0 + c) / E),
// so same-slot ranks are consecutive and all lie within [r, mr E - count0]).
// Part 0 writes the winners' leaves (max_priority) and recomputes the span
// [ptr0, last slot] of its stratum (propagate_span: nodes whose children did
// not change are recomputed to the same sum); every part copies the winners
// with stratum-row index = part (mod K).  The last workgroup out (ticket
// ws[0]) advances the shared pointer and the strata's sampling size.
// Bit-identical to the three launches (tests/test_lap_gpu.py).
__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

template <bool VEC>
__device__ __forceinline__ void copy_rows(const lap_storage_desc &st, const float *state, const float *action,
                                          const float *next_state, const float *reward, const uint8_t *done,
                                          float action_scale, const int32_t *ri, const int32_t *sl, int s,
                                          int capacity, int j0, int step, int m, int t, int nt) {
    const int sd = st.state_dim, ad = st.action_dim;
    const int sdv = VEC ? sd / 4 : sd;        // state items per row (float4 or float)
    const int per = 2 * sdv + ad + 2;         // state, next_state, action, reward, not_done
    const int nrows = j0 < m ? (m - j0 + step - 1) / step : 0;
    const int items = nrows * per;
    constexpr int U = 4;  // items in flight per thread: loads first, then stores
    for (int it0 = t; it0 < items; it0 += U * nt) {
        float4 v[U];
        long dst[U];
        int kind[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int it = it0 + u * nt;
            kind[u] = -1;
            if (it >= items) continue;
            const int q = it / per, c = it - q * per, j = j0 + q * step;
            const int slot = sl[j];
            if (slot < 0) continue;
            const long r = (long)s * (capacity + 1) + slot;
            const long i = ri[j];
            if (c < 2 * sdv) {
                const bool nx = c >= sdv;
                const int e = nx ? c - sdv : c;
                const float *src = (nx ? next_state : state) + i * sd;
                if (VEC) {
                    v[u] = ld4(src + 4 * e);
                    dst[u] = r * sd + 4 * e;
                } else {
                    v[u].x = src[e];
                    dst[u] = r * sd + e;
                }
                kind[u] = nx ? 1 : 0;
            } else if (c < 2 * sdv + ad) {
                const int e = c - 2 * sdv;
                v[u].x = action[i * ad + e] / action_scale;
                dst[u] = r * ad + e;
                kind[u] = 2;
            } else if (c == 2 * sdv + ad) {
                v[u].x = reward[i];
                dst[u] = r;
                kind[u] = 3;
            } else {
                v[u].x = 1.0f - (done[i] ? 1.0f : 0.0f);
                dst[u] = r;
                kind[u] = 4;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            switch (kind[u]) {
            case 0:
                if (VEC) st4(st.state + dst[u], v[u]); else st.state[dst[u]] = v[u].x;
                break;
            case 1:
                if (VEC) st4(st.next_state + dst[u], v[u]); else st.next_state[dst[u]] = v[u].x;
                break;
            case 2: st.action[dst[u]] = v[u].x; break;
            case 3: st.reward[dst[u]] = v[u].x; break;
            case 4: st.not_done[dst[u]] = v[u].x; break;
            default: break;
            }
        }
    }
}

// The vectorised insert as ONE launch (r05, opt-in: EXO_LAP_STORE_FUSED=1,
// measured slower in the loop; lap_store_batch at n <= 8,192):
// lap_store_rank_kernel's scan, leaves and span propagation, and the copy of
// the stratum's rows by the same workgroup -- the scan leaves each rank's env
// and slot in LDS, the workgroup's 1,024 threads copy the rows (8 items in
// flight per thread, float4 state rows where aligned).  One workgroup per
// stratum reads and writes its own ring pointer, so no other workgroup needs
// it.  The same rows, slots, leaves and sums as the two launches (an inactive
// row's copy to the trash row is skipped: nothing reads that row).
constexpr int STORE_FUSED_MAX = 8192;

template <bool VEC>
__global__ __launch_bounds__(UPD_THREADS) void lap_store_fused_kernel(
    float *tree, const float *maxp, int cap, int levels, int capacity, int32_t *ring_ptr, int32_t *ring_size,
    const int32_t *strata, const uint8_t *active, int n, int32_t *row_of, lap_storage_desc st, const float *state,
    const float *action, const float *next_state, const float *reward, const uint8_t *done, float action_scale) {
    constexpr int RPT = 4;
    const int s = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    float *T = stratum_tree(tree, s, cap);
    __shared__ int wsum[UPD_THREADS / 64];
    __shared__ int chunk_total;
    __shared__ int32_t ri[STORE_FUSED_MAX];
    const float p = *maxp;
    const int ptr0 = ring_ptr[s];
    const int row0 = s * (capacity + 1);
    int offset = 0;
    for (int base = 0; base < n; base += RPT * UPD_THREADS) {
        int stk[RPT], cnt = 0;
        bool f[RPT];
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int i = base + RPT * t + k;
            stk[k] = i < n ? strata[i] : -1;
            f[k] = i < n && (!active || active[i]) && stk[k] == s;
            cnt += f[k];
        }
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        if (t == 0) {
            int acc = 0;
            for (int k = 0; k < UPD_THREADS / 64; ++k) {
                const int v = wsum[k];
                wsum[k] = acc;
                acc += v;
            }
            chunk_total = acc;
        }
        __syncthreads();
        int rank = offset + wsum[wv] + incl - cnt;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int i = base + RPT * t + k;
            if (i >= n) continue;
            if (s == 0 && (stk[k] < 0 || stk[k] >= (int)gridDim.x)) row_of[i] = -1;
            if (stk[k] != s) continue;
            if (f[k]) {
                const int slot = (ptr0 + rank) % capacity;
                row_of[i] = row0 + slot;
                T[cap + slot] = p;
                ri[rank] = i;
                ++rank;
            } else {
                row_of[i] = row0 + capacity;
            }
        }
        const int total = chunk_total;
        __syncthreads();
        offset += total;
    }
    // the stratum's rows: rank q -> slot (ptr0 + q) % capacity
    {
        const int sd = st.state_dim, ad = st.action_dim;
        const int sdv = VEC ? sd / 4 : sd;
        const int per = 2 * sdv + ad + 2;
        const int items = offset * per;
        constexpr int U = 8;
        for (int it0 = t; it0 < items; it0 += U * UPD_THREADS) {
            float4 v[U];
            long dst[U];
            int kind[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int it = it0 + u * UPD_THREADS;
                kind[u] = -1;
                if (it >= items) continue;
                const int q = it / per, c = it - q * per;
                const long r = (long)row0 + (ptr0 + q) % capacity;
                const long i = ri[q];
                if (c < 2 * sdv) {
                    const bool nx = c >= sdv;
                    const int e = nx ? c - sdv : c;
                    const float *src = (nx ? next_state : state) + i * sd;
                    if (VEC) {
                        v[u] = ld4(src + 4 * e);
                        dst[u] = r * sd + 4 * e;
                    } else {
                        v[u].x = src[e];
                        dst[u] = r * sd + e;
                    }
                    kind[u] = nx ? 1 : 0;
                } else if (c < 2 * sdv + ad) {
                    const int e = c - 2 * sdv;
                    v[u].x = action[i * ad + e] / action_scale;
                    dst[u] = r * ad + e;
                    kind[u] = 2;
                } else if (c == 2 * sdv + ad) {
                    v[u].x = reward[i];
                    dst[u] = r;
                    kind[u] = 3;
                } else {
                    v[u].x = 1.0f - (done[i] ? 1.0f : 0.0f);
                    dst[u] = r;
                    kind[u] = 4;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                switch (kind[u]) {
                case 0:
                    if (VEC) st4(st.state + dst[u], v[u]); else st.state[dst[u]] = v[u].x;
                    break;
                case 1:
                    if (VEC) st4(st.next_state + dst[u], v[u]); else st.next_state[dst[u]] = v[u].x;
                    break;
                case 2: st.action[dst[u]] = v[u].x; break;
                case 3: st.reward[dst[u]] = v[u].x; break;
                case 4: st.not_done[dst[u]] = v[u].x; break;
                default: break;
                }
            }
        }
    }
    propagate_span(T, cap, levels, capacity, ptr0, offset);
    if (t == 0) {
        ring_ptr[s] = (ptr0 + offset) % capacity;
        ring_size[s] = min(ring_size[s] + offset, capacity);
    }
}

// The training loop's per-step mask advance, optionally done by the insert's
// last workgroup out (lap_store_batch_ref_fused_adv): every workgroup has read
// the step's mask by then.  exo_active_advance_score's arithmetic: score +=
// reward where the step's mask is set, k = min(k + 1, rows - 1), mask = table
// row k, count = its population.
struct MaskAdvance {
    const uint8_t *table;  // nullptr: no advance
    int rows;
    long long *k;
    uint8_t *active;
    int32_t *count;
    double *score;         // nullptr: no score
};

template <bool VEC>
__global__ __launch_bounds__(UPD_THREADS) void lap_store_ref_fused_kernel(
    float *tree, const float *maxp, int cap, int levels, int capacity, int E, long long *ref, int32_t *ring_size,
    lap_storage_desc st, const float *state, const float *action, const float *next_state, const float *reward,
    const uint8_t *done, float action_scale, const int32_t *strata, const uint8_t *active, int n,
    uint32_t *ticket, MaskAdvance adv) {
    const int s = blockIdx.x, part = blockIdx.y, K = gridDim.y;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    __shared__ int wsum[UPD_THREADS / 64];
    __shared__ int chunk_tot, chunk_m;
    __shared__ int32_t rk[STORE_CHUNK], ri[STORE_CHUNK], sl[STORE_CHUNK];
    __shared__ int carry_r, carry_i, carry_J, carry_slot;  // the chunk's last row of stratum s, decided later
    float *T = stratum_tree(tree, s, cap);
    // K > 1: part 0 writes the leaves and propagates, parts 1..K-1 copy the rows
    // (copy part of stratum-row j: 1 + j mod (K - 1)); K == 1: part 0 does both
    const int KC = K > 1 ? K - 1 : 1, cpart = K > 1 ? part - 1 : 0;
    const long long ptr0 = ref[0], count0 = ref[1], size0 = ref[2];
    const long long m0 = mult_below(count0, E);
    const float p = *maxp;
    auto slot_of = [&](long long r) -> int {
        long long v = ptr0 + (mult_below(count0 + r, E) - m0);
        if (v >= capacity) v -= capacity;
        if (v >= capacity) v %= capacity;
        return (int)v;
    };
    if (t == 0) carry_r = -1;
    int offset = 0, soff = 0;  // active rows / stratum-s rows before this chunk
    for (int base = 0; base < n; base += STORE_CHUNK) {
        int cnt = 0, gcnt = 0;
        bool f[4], g[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = base + 4 * t + k;
            const int sk = i < n ? strata[i] : -1;
            f[k] = i < n && sk >= 0 && sk < E && (!active || active[i]);
            g[k] = f[k] && sk == s;
            cnt += f[k];
            gcnt += g[k];
        }
        // block-wide exclusive scan of (cnt, gcnt) packed in one int (each <= STORE_CHUNK < 2^16)
        int incl = cnt | (gcnt << 16);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        if (t == 0) {
            int acc = 0;
            for (int k = 0; k < UPD_THREADS / 64; ++k) {
                const int v = wsum[k];
                wsum[k] = acc;
                acc += v;
            }
            chunk_tot = acc & 0xFFFF;
            chunk_m = acc >> 16;
        }
        __syncthreads();
        const int ex = wsum[wv] + incl - (cnt | (gcnt << 16));
        int rank = offset + (ex & 0xFFFF), j = ex >> 16;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (g[k]) {
                rk[j] = rank;
                ri[j] = base + 4 * t + k;
                ++j;
            }
            rank += f[k];
        }
        __syncthreads();
        const int m = chunk_m;
        // the previous chunk's last row of stratum s: its successor is rk[0]
        if (t == 0) {
            carry_slot = -1;
            if (carry_r >= 0 && m > 0) {
                const long long mr = mult_below(count0 + carry_r, E);
                if ((long long)rk[0] > mr * E - count0) {  // no same-slot successor: a winner
                    carry_slot = slot_of(carry_r);
                    if (part == 0) T[cap + carry_slot] = p;
                }
                carry_r = -1;
            }
        }
        __syncthreads();
        if (carry_slot >= 0 && wv == 0 && carry_J % KC == cpart)
            copy_rows<VEC>(st, state, action, next_state, reward, done, action_scale, &carry_i, &carry_slot, s,
                           capacity, 0, 1, 1, lane, 64);
        __syncthreads();  // the loop below sets the next carry: wave 0 must be done reading this one
        for (int jj = t; jj < m; jj += UPD_THREADS) {
            const int r = rk[jj];
            if (jj + 1 == m) {  // successor unknown until a later chunk (or none: a winner)
                carry_r = r;
                carry_i = ri[jj];
                carry_J = soff + jj;
                sl[jj] = -1;
                continue;
            }
            const long long mr = mult_below(count0 + r, E);
            const bool win = (long long)rk[jj + 1] > mr * E - count0;
            const int slot = win ? slot_of(r) : -1;
            sl[jj] = slot;
            if (win && part == 0) T[cap + slot] = p;
        }
        __syncthreads();
        // this part's share of the chunk's winners: stratum-row index = cpart (mod KC)
        if (cpart >= 0) {
            const int j0 = ((cpart - soff) % KC + KC) % KC;
            copy_rows<VEC>(st, state, action, next_state, reward, done, action_scale, ri, sl, s, capacity, j0, KC, m,
                           t, UPD_THREADS);
        }
        offset += chunk_tot;
        soff += m;
        __syncthreads();
    }
    // the last row of stratum s has no successor: a winner
    if (t == 0) {
        carry_slot = -1;
        if (carry_r >= 0) {
            carry_slot = slot_of(carry_r);
            if (part == 0) T[cap + carry_slot] = p;
        }
    }
    __syncthreads();
    if (carry_slot >= 0 && wv == 0 && carry_J % KC == cpart)
        copy_rows<VEC>(st, state, action, next_state, reward, done, action_scale, &carry_i, &carry_slot, s, capacity,
                       0, 1, 1, lane, 64);
    const int n_act = offset;
    if (part == 0 && n_act > 0) {
        __shared__ float span_buf[2 * SPAN_LDS], span_edge[2 * SPAN_LEVELS];
        __syncthreads();
        const long long last = mult_below(count0 + n_act - 1, E) - m0;  // slots ptr0 .. ptr0 + last
        const int cnt = (int)min(last + 1, (long long)capacity);
        if (!propagate_span_lds(T, cap, levels, capacity, (int)ptr0, cnt, span_buf, span_edge))
            propagate_span(T, cap, levels, capacity, (int)ptr0, cnt);
    }
    __syncthreads();
    __shared__ int last;
    if (t == 0) {  // ref and the mask were read (and used) before this add: no fence needed
        last = atomicAdd(ticket, 1u) == (uint32_t)(E * K - 1);  // every workgroup has read them
        if (last) {
            const long long na = mult_below(count0 + n_act, E) - m0;
            const long long size = min(size0 + na, (long long)capacity);
            for (int q = 0; q < E; ++q) ring_size[q] = (int32_t)size;
            ref[0] = (ptr0 + na) % capacity;
            ref[1] = count0 + n_act;
            ref[2] = size;
            *ticket = 0u;
        }
    }
    __syncthreads();
    if (!last || !adv.table) return;
    const long long k0 = *adv.k;
    const long long kk = k0 + 1 < adv.rows ? k0 + 1 : adv.rows - 1;
    int c = 0;
    for (int e = t; e < n; e += UPD_THREADS) {
        const uint8_t v = adv.table[(size_t)kk * n + e];
        if (adv.score) adv.score[e] += adv.active[e] ? (double)reward[e] : 0.0;
        adv.active[e] = v;
        c += v != 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ int wc[UPD_THREADS / 64];
    if (lane == 0) wc[wv] = c;
    __syncthreads();
    if (t == 0) {
        *adv.k = kk;
        if (adv.count) {
            int tot = 0;
            for (int w = 0; w < UPD_THREADS / 64; ++w) tot += wc[w];
            *adv.count = tot;
        }
    }
}

__global__ __launch_bounds__(256) void lap_store_copy_kernel(lap_storage_desc st, const float *state,
                                                             const float *action, const float *next_state,
                                                             const float *reward, const uint8_t *done,
                                                             float action_scale, int n, const int32_t *row_of) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= n) return;
    const long r = row_of[i];
    if (r < 0) return;
    const int sd = st.state_dim, ad = st.action_dim;
    for (int k = lane; k < sd; k += 64) {
        st.state[r * sd + k] = state[(long)i * sd + k];
        st.next_state[r * sd + k] = next_state[(long)i * sd + k];
    }
    for (int k = lane; k < ad; k += 64) st.action[r * ad + k] = action[(long)i * ad + k] / action_scale;
    if (lane == 0) {
        st.reward[r] = reward[i];
        st.not_done[r] = 1.0f - (done[i] ? 1.0f : 0.0f);
    }
}

// LAP.sample (:65-111) with the gather: one wavefront per draw descends the
// tree (every lane the same path, reads broadcast) and copies the row.
__device__ __forceinline__ void sample_descend(const float *tree, int cap, int levels, int capacity, float ud,
                                               const int32_t *size, int batch, int d, int lane, int32_t *idx,
                                               const lap_storage_desc &st, float *o_state, float *o_action,
                                               float *o_next, float *o_reward, float *o_not_done) {
    const int s = d / batch;
    const float *T = tree + (size_t)s * 2 * cap;
    const int sz = size[s];
    const float val = ud * prefix_total(T, cap, levels, sz);
    const int node = descend_from([T](int n) { return T[n]; }, val, 1, 0, levels);
    int i = node - cap;
    if (i >= sz) i = sz > 0 ? sz - 1 : 0;
    if (lane == 0) idx[d] = i;
    const long r = (long)s * (capacity + 1) + i;
    const int sd = st.state_dim, ad = st.action_dim;
    for (int k = lane; k < sd; k += 64) {
        o_state[(long)d * sd + k] = st.state[r * sd + k];
        o_next[(long)d * sd + k] = st.next_state[r * sd + k];
    }
    for (int k = lane; k < ad; k += 64) o_action[(long)d * ad + k] = st.action[r * ad + k];
    if (lane == 0) {
        o_reward[d] = st.reward[r];
        o_not_done[d] = st.not_done[r];
    }
}

// rng != nullptr: u[d] is drawn in the kernel (Philox block d of this call,
// word 0 -> [0, 1)); the device call counter advances once per launch (the
// last workgroup out, as td7_adam_step's step count).
struct SampleRng {
    uint64_t seed;
    uint32_t tag;
    unsigned long long *counter;
    uint32_t *ticket;
};

__global__ __launch_bounds__(256) void lap_sample_gather_kernel(const float *tree, int cap, int levels, int capacity,
                                                                const float *u, const int32_t *size, int batch,
                                                                int total, int32_t *idx, lap_storage_desc st,
                                                                float *o_state, float *o_action, float *o_next,
                                                                float *o_reward, float *o_not_done, SampleRng rng) {
    const int d = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (rng.counter) {
        const unsigned long long call = *rng.counter;
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(rng.ticket, 1u) == gridDim.x - 1) {
                *rng.counter = call + 1ull;
                *rng.ticket = 0u;
            }
        }
        if (d >= total) return;
        uint32_t r[4];
        philox_block(rng.seed, rng.tag, call, (uint32_t)d, r);
        sample_descend(tree, cap, levels, capacity, u01_open_hi(r[0]), size, batch, d, lane, idx, st, o_state,
                       o_action, o_next, o_reward, o_not_done);
        return;
    }
    if (d >= total) return;
    sample_descend(tree, cap, levels, capacity, u[d], size, batch, d, lane, idx, st, o_state, o_action, o_next,
                   o_reward, o_not_done);
}


// The top of a stratum tree lap_update_sample stages in LDS (r05 A/B at the
// bench's shape, tools/lap_bench.py: 32,768 nodes -- 128 KB, 3 global levels
// left instead of 6 -- 23.9 us per launch against 21.8 with 8,192: staging
// 128 KB costs more than the three level sweeps it saves)
#ifndef LAP_TOPN_US
#define LAP_TOPN_US 8192
#endif
constexpr int TOPN_US = LAP_TOPN_US;

// ---------------------------------------------------------------- planned reference inserts
// The reference schedule's rollout inserts (lap_store_batch_ref_fused_adv per
// step: 18.5 us of its ~80 us per 4,096-env step, r05 lap_bench) planned for
// a whole episode round at its start (r05).  Which envs run at each step of
// a synchronous round is fixed by the motion lengths (the trainer's mask
// table), so the shared pointer's slot of every add of the round -- and
// which adds a later same-slot add of the same stratum overwrites -- follow
// from the pointer at the round start alone: lap_ref_plan writes
// plan[k][e] = the slot env e's step-k transition lands in (-1: inactive or
// overwritten).  A step is then one elementwise launch (lap_ref_step: the
// row copies, the scores, the next mask) with no scan, ticket or tree work,
// and lap_ref_commit writes the round's leaves (max_priority: constant over a
// rollout, nothing trains during it), recomputes the round's ring span once
// and advances the pointer and sizes.  The same rows, leaves, sums, pointer
// and sizes as the per-step inserts: a slot written twice in a round is
// written by the later add either way, an ancestor's last recomputation sees
// its children's final values either way.

// pass 1: rank of every active env within its step (block scan per step row),
// add index c = offs[k] + rank, stratum_of_add[c]; plan[k][e] = c or -1
__global__ __launch_bounds__(UPD_THREADS) void lap_ref_plan_scan_kernel(const uint8_t *table, int n,
                                                                        const int32_t *strata, int E,
                                                                        const long long *offs, int32_t *add_s,
                                                                        int32_t *plan) {
    const int k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    __shared__ int wsum[UPD_THREADS / 64];
    __shared__ int chunk_total;
    const uint8_t *A = table + (size_t)k * n;
    int32_t *P = plan + (size_t)k * n;
    long long offset = offs[k];
    for (int base = 0; base < n; base += STORE_CHUNK) {
        int f[4], sk[4], cnt = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = base + 4 * t + j;
            sk[j] = i < n ? strata[i] : -1;
            f[j] = (i < n && sk[j] >= 0 && sk[j] < E && A[i]) ? 1 : 0;
            cnt += f[j];
        }
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        if (t == 0) {
            int acc = 0;
            for (int q = 0; q < UPD_THREADS / 64; ++q) {
                const int v = wsum[q];
                wsum[q] = acc;
                acc += v;
            }
            chunk_total = acc;
        }
        __syncthreads();
        long long c = offset + wsum[wv] + incl - cnt;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = base + 4 * t + j;
            if (i >= n) continue;
            if (f[j]) {
                add_s[c] = sk[j];
                P[i] = (int32_t)c;
                ++c;
            } else {
                P[i] = -1;
            }
        }
        offset += chunk_total;
        __syncthreads();
    }
}

// pass 2: add c -> its slot, or -1 when a later add of its slot group (the
// adds sharing ceil((count0 + c) / E)) has the same stratum
__global__ __launch_bounds__(256) void lap_ref_plan_slots_kernel(int32_t *plan, long long entries,
                                                                 const int32_t *add_s, long long total,
                                                                 const long long *ref, int E, int capacity) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= entries) return;
    const int c = plan[i];
    if (c < 0) return;
    const long long ptr0 = ref[0], count0 = ref[1];
    const long long m0 = mult_below(count0, E), mr = mult_below(count0 + c, E);
    const long long qend = min(mr * E - count0, total - 1);
    const int s = add_s[c];
    bool win = true;
    for (long long q = c + 1; q <= qend; ++q) win &= add_s[q] != s;
    long long v = ptr0 + (mr - m0);
    if (v >= capacity) v -= capacity;
    if (v >= capacity) v %= capacity;
    plan[i] = win ? (int32_t)v : -1;
}

// one step of the planned round: env e's transition to its slot, the episode
// score (:144) and the next mask -- one wavefront per env, 4 per workgroup.
// The step index lives in kk[par] (the trainers' observation parity); the
// launch writes k + 1 to kk[par ^ 1] (and *k_dev), so no workgroup reads a
// counter another one advances.
__global__ __launch_bounds__(256) void lap_ref_step_kernel(lap_storage_desc st, const int32_t *plan, int rows, int n,
                                                           long long *kk, int par, long long *k_dev,
                                                           const int32_t *strata, int capacity, const float *state,
                                                           const float *action, const float *next_state,
                                                           const float *reward, const uint8_t *done,
                                                           float action_scale, const uint8_t *table,
                                                           uint8_t *active, int32_t *count,
                                                           const int32_t *counts_table, double *score) {
    const long long k = kk[par];
    const long long k1 = k + 1 < rows ? k + 1 : rows - 1;
    const int e = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        kk[par ^ 1] = k1;
        if (k_dev) *k_dev = k1;
        if (count) *count = counts_table[k1];
    }
    if (e >= n) return;
    const int slot = k < rows ? plan[(size_t)k * n + e] : -1;
    if (slot >= 0) {
        const long r = (long)strata[e] * (capacity + 1) + slot;
        const int sd = st.state_dim, ad = st.action_dim;
        for (int q = lane; q < sd; q += 64) {
            st.state[r * sd + q] = state[(long)e * sd + q];
            st.next_state[r * sd + q] = next_state[(long)e * sd + q];
        }
        for (int q = lane; q < ad; q += 64) st.action[r * ad + q] = action[(long)e * ad + q] / action_scale;
        if (lane == 0) {
            st.reward[r] = reward[e];
            st.not_done[r] = 1.0f - (done[e] ? 1.0f : 0.0f);
        }
    }
    if (lane == 0) {
        if (score) score[e] += active[e] ? (double)reward[e] : 0.0;
        active[e] = table[(size_t)k1 * n + e];
    }
}

// the round's leaves (max_priority) at every planned slot
__global__ __launch_bounds__(256) void lap_ref_commit_leaves_kernel(const int32_t *plan, long long entries, int n,
                                                                    const int32_t *strata, float *tree, int cap,
                                                                    const float *maxp) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= entries) return;
    const int slot = plan[i];
    if (slot < 0) return;
    stratum_tree(tree, strata[i % n], cap)[cap + slot] = *maxp;
}

// the round's ring span recomputed per stratum (one workgroup each)
__global__ __launch_bounds__(UPD_THREADS) void lap_ref_commit_tree_kernel(float *tree, int cap, int levels,
                                                                          int capacity, const long long *ref,
                                                                          long long total, int E) {
    const long long ptr0 = ref[0], count0 = ref[1];
    if (total <= 0) return;
    // the round's adds land in slots ptr0 .. ptr0 + last: the last add's slot
    // is ptr0 + adv (not ptr0 + adv - 1) unless count0 + total - 1 is a
    // multiple of E -- the same span as the per-step insert's (:959)
    const long long last = mult_below(count0 + total - 1, E) - mult_below(count0, E);
    propagate_span(stratum_tree(tree, blockIdx.x, cap), cap, levels, capacity, (int)ptr0,
                   (int)min(last + 1, (long long)capacity));
}

// the pointer and sizes after the round
__global__ void lap_ref_commit_ref_kernel(long long *ref, long long total, int E, int capacity, int32_t *ring_size) {
    const long long ptr0 = ref[0], count0 = ref[1], size0 = ref[2];
    const long long adv = mult_below(count0 + total, E) - mult_below(count0, E);
    const long long size = min(size0 + adv, (long long)capacity);
    for (int s = 0; s < E; ++s) ring_size[s] = (int32_t)size;
    ref[0] = (ptr0 + adv) % capacity;
    ref[1] = count0 + total;
    ref[2] = size;
}

// The sampled rows gathered by their own launch (r05): lap_update_sample's
// stratum workgroups stop at the indices, and DRAWS draws per 256-thread
// workgroup here copy state, next_state (float4 where aligned), action,
// reward and not_done -- 64 workgroups for the bench's 8 x 128 batch instead
// of the 8 that ran the update (9.7 of its 24.7 us, r05g).
constexpr int GATHER_DRAWS = 16;
__global__ __launch_bounds__(256) void lap_gather_kernel(lap_storage_desc st, int capacity, const int32_t *idx,
                                                         int batch, int total, float *o_state, float *o_action,
                                                         float *o_next, float *o_reward, float *o_not_done) {
    const int sd = st.state_dim, ad = st.action_dim;
    const bool v4 = (sd & 3) == 0 && ((reinterpret_cast<uintptr_t>(st.state) | reinterpret_cast<uintptr_t>(st.next_state) |
                                       reinterpret_cast<uintptr_t>(o_state) | reinterpret_cast<uintptr_t>(o_next)) & 15) == 0;
    const int sv = v4 ? sd / 4 : sd, per = 2 * sv + ad + 2;
    const int d0 = blockIdx.x * GATHER_DRAWS;
    const int nd = min(GATHER_DRAWS, total - d0);
    const int items = nd * per;
    constexpr int GU = 4;
    for (int it0 = threadIdx.x; it0 < items; it0 += GU * 256) {
        float4 v[GU];
        float *dst[GU];
        bool wide[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            const int it = it0 + u * 256;
            dst[u] = nullptr;
            wide[u] = false;
            if (it >= items) continue;
            const int q = it / per, c = it - q * per;
            const long d = d0 + q;
            const long row = (long)(d / batch) * (capacity + 1) + idx[d];
            if (c < 2 * sv) {
                const bool nx = c >= sv;
                const int e = nx ? c - sv : c;
                const float *src = (nx ? st.next_state : st.state) + row * sd;
                float *o = (nx ? o_next : o_state) + d * sd;
                if (v4) {
                    v[u] = ld4(src + 4 * e);
                    dst[u] = o + 4 * e;
                    wide[u] = true;
                } else {
                    v[u].x = src[e];
                    dst[u] = o + e;
                }
            } else if (c < 2 * sv + ad) {
                const int e = c - 2 * sv;
                v[u].x = st.action[row * ad + e];
                dst[u] = o_action + d * ad + e;
            } else if (c == 2 * sv + ad) {
                v[u].x = st.reward[row];
                dst[u] = o_reward + d;
            } else {
                v[u].x = st.not_done[row];
                dst[u] = o_not_done + d;
            }
        }
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            if (!dst[u]) continue;
            if (wide[u]) st4(dst[u], v[u]);
            else *dst[u] = v[u].x;
        }
    }
}

// LAP.update_priority (:113-117) and the NEXT LAP.sample (:65-111) as ONE
// launch (r04: lap_update_kernel + lap_sample_gather_kernel were 32 us plus a
// queue hand-off at the end of every critic-only iteration).  One workgroup
// per stratum: the update exactly as lap_update_kernel (last duplicate wins,
// level-synchronous ancestors, the max_priority atomic), whose staged top
// levels stay in LDS; then the stratum's `batch` draws (Philox block d =
// s * batch + b of call *counter, as lap_sample_gather_kernel) descend with
// the nodes below TOPN read from LDS, and the workgroup gathers their rows.
// The same sums and comparisons: bit-identical to the two launches.
// TdPrio (lap_update_sample_td): the priorities computed here from the critic
// pass's |td| of both heads, prio = max(|td0|, |td1|, min_priority)^alpha
// (TD7_multi_agent.py:259, the expression td7f_wgrad evaluates), so the update
// need not wait for the weight-gradient launch; written to `out` if non-null.
struct TdPrio {
    const float *td;  // [B][2]; nullptr: the priorities are given (prio)
    float alpha, minp;
    float *out;
};

__global__ __launch_bounds__(UPD_THREADS) void lap_update_sample_kernel(float *tree, float *maxp, int cap, int levels,
                                                                        int capacity, const int32_t *idx_in,
                                                                        const float *prio, int batch,
                                                                        const int32_t *size, lap_storage_desc st,
                                                                        SampleRng rng, int32_t *idx_out,
                                                                        float *o_state, float *o_action, float *o_next,
                                                                        float *o_reward, float *o_not_done,
                                                                        TdPrio tp, bool gather) {
    const int s = blockIdx.x;
    float *T = stratum_tree(tree, s, cap);
    const int32_t *I = idx_in + (size_t)s * batch;
    const float *P = prio + (size_t)s * batch;
    __shared__ float red[UPD_THREADS / 64];
    __shared__ int32_t li[UPD_THREADS];
    __shared__ float top[TOPN_US];
    __shared__ int32_t pick[UPD_THREADS];
    const unsigned long long call = *rng.counter;  // read before any workgroup can take the ticket
    float mx = 0.0f;
    for (int b0 = 0; b0 < batch; b0 += UPD_THREADS) {
        const int nb = min(UPD_THREADS, batch - b0);
        __syncthreads();
        if ((int)threadIdx.x < nb) li[threadIdx.x] = I[b0 + threadIdx.x];
        __syncthreads();
        const int b = b0 + threadIdx.x;
        if (b < batch) {
            const int me = li[threadIdx.x];
            bool last = true;
            for (int k = threadIdx.x + 1; k < nb; ++k) last &= (li[k] != me);
            for (int b2 = b0 + nb; b2 < batch; ++b2) last &= (I[b2] != me);
            float pb;
            if (tp.td) {
                const long d = (long)s * batch + b;
                pb = powf(fmaxf(fmaxf(tp.td[2 * d], tp.td[2 * d + 1]), tp.minp), tp.alpha);
                if (tp.out) tp.out[d] = pb;
            } else {
                pb = P[b];
            }
            if (last) T[cap + me] = pb;
            mx = fmaxf(mx, pb);
        }
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    const bool staged = propagate_top<TOPN_US>(T, cap, levels, I, batch, top);
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) mx = fmaxf(mx, red[w]);
        atomicMax(reinterpret_cast<int *>(maxp), __float_as_int(mx));
    }
    // ---- the next batch of this stratum
    const int lim = staged ? min(TOPN_US, 2 * cap) : 0;
    auto node_at = [&](int node) { return node < lim ? top[node] : T[node]; };
    const int sz = size[s];
    const float tot = prefix_sum(node_at, cap, levels, sz);
    for (int b = threadIdx.x; b < batch; b += UPD_THREADS) {
        const int d = s * batch + b;
        uint32_t r[4];
        philox_block(rng.seed, rng.tag, call, (uint32_t)d, r);
        float val = u01_open_hi(r[0]) * tot;
        // the staged top levels from LDS one level at a time, the rest (below
        // TOPN) three levels per round trip
        int node = 1, lv = 0;
        for (; lv < levels && 2 * node + 1 < lim; ++lv) {
            const float left = top[2 * node], right = top[2 * node + 1];
            if (val <= left || right <= 0.0f) {
                node = 2 * node;
            } else {
                val -= left;
                node = 2 * node + 1;
            }
        }
        node = descend_from([T](int n) { return T[n]; }, val, node, lv, levels);
        int i = node - cap;
        if (i >= sz) i = sz > 0 ? sz - 1 : 0;
        idx_out[d] = i;
        if (b < UPD_THREADS) pick[b] = i;
    }
    __syncthreads();
    if (!gather) {  // the rows follow in lap_gather_kernel; the call counter's ticket below
        if (threadIdx.x == 0 && atomicAdd(rng.ticket, 1u) == gridDim.x - 1) {
            *rng.counter = call + 1ull;
            *rng.ticket = 0u;
        }
        return;
    }
    // gather: (draw, item) over the workgroup, items = state, next_state (float4
    // where the rows are 16-byte aligned), action, reward, not_done; GU items
    // per thread loaded before any is stored (the stores may alias the loads as
    // far as the compiler knows: item by item, every load would wait for the
    // previous store -- r04 first cut, 54 us per launch)
    const int sd = st.state_dim, ad = st.action_dim;
    const bool v4 = (sd & 3) == 0 && ((reinterpret_cast<uintptr_t>(st.state) | reinterpret_cast<uintptr_t>(st.next_state) |
                                       reinterpret_cast<uintptr_t>(o_state) | reinterpret_cast<uintptr_t>(o_next)) & 15) == 0;
    const int sv = v4 ? sd / 4 : sd, per = 2 * sv + ad + 2;
    const int items = min(batch, UPD_THREADS) * per;
    constexpr int GU = 8;
    for (int it0 = threadIdx.x; it0 < items; it0 += GU * UPD_THREADS) {
        float4 v[GU];
        float *dst[GU];
        bool wide[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            const int it = it0 + u * UPD_THREADS;
            dst[u] = nullptr;
            wide[u] = false;
            if (it >= items) continue;
            const int b = it / per, c = it - b * per;
            const long d = (long)s * batch + b;
            const long row = (long)s * (capacity + 1) + pick[b];
            if (c < 2 * sv) {
                const bool nx = c >= sv;
                const int e = nx ? c - sv : c;
                const float *src = (nx ? st.next_state : st.state) + row * sd;
                float *o = (nx ? o_next : o_state) + d * sd;
                if (v4) {
                    v[u] = ld4(src + 4 * e);
                    dst[u] = o + 4 * e;
                    wide[u] = true;
                } else {
                    v[u].x = src[e];
                    dst[u] = o + e;
                }
            } else if (c < 2 * sv + ad) {
                const int e = c - 2 * sv;
                v[u].x = st.action[row * ad + e];
                dst[u] = o_action + d * ad + e;
            } else if (c == 2 * sv + ad) {
                v[u].x = st.reward[row];
                dst[u] = o_reward + d;
            } else {
                v[u].x = st.not_done[row];
                dst[u] = o_not_done + d;
            }
        }
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            if (!dst[u]) continue;
            if (wide[u]) st4(dst[u], v[u]);
            else *dst[u] = v[u].x;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // `call` was read (and used) before this add: no fence needed
        if (atomicAdd(rng.ticket, 1u) == gridDim.x - 1) {
            *rng.counter = call + 1ull;
            *rng.ticket = 0u;
        }
    }
}

int rc(hipError_t e) { return e == hipSuccess ? EXO_OK : EXO_EDEVICE; }

int levels_of(const lap_tree_desc *t) {
    int lv = 0;
    while ((1 << lv) < t->cap) ++lv;
    return lv;
}

// lap_update_sample's rows gathered by lap_gather_kernel (EXO_LAP_GATHER_SPLIT=0:
// by the update's own stratum workgroups, the r04 layout)
bool gather_split() {
    static const bool on = [] {
        const char *e = getenv("EXO_LAP_GATHER_SPLIT");
        return !(e && e[0] == '0');
    }();
    return on;
}

int gather_after(const lap_tree_desc *t, const lap_storage_desc *st, int batch, const int32_t *idx, float *o_state,
                 float *o_action, float *o_next, float *o_reward, float *o_not_done, void *stream) {
    if (hipGetLastError() != hipSuccess) return EXO_EDEVICE;
    if (!gather_split()) return EXO_OK;
    const int total = t->n_strata * batch;
    hipLaunchKernelGGL(lap_gather_kernel, dim3((total + GATHER_DRAWS - 1) / GATHER_DRAWS), dim3(256), 0,
                       (hipStream_t)stream, *st, t->capacity, idx, batch, total, o_state, o_action, o_next, o_reward,
                       o_not_done);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

bool valid(const lap_tree_desc *t) {
    // cap <= 2^MAXLV: prefix_sum unrolls MAXLV levels
    return t && t->tree && t->max_priority && t->n_strata > 0 && t->capacity > 0 && t->cap >= t->capacity &&
           (t->cap & (t->cap - 1)) == 0 && t->cap <= (1 << MAXLV);
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

int lap_store_batch(const lap_tree_desc *t, const lap_storage_desc *st, const float *state, const float *action,
                    const float *next_state, const float *reward, const uint8_t *done, const int32_t *strata,
                    const uint8_t *active, float action_scale, int32_t n, int32_t *row_ws, void *stream) {
    if (!valid(t) || !st || !st->state || !st->action || !st->next_state || !st->reward || !st->not_done ||
        !st->ptr || !st->size || st->state_dim <= 0 || st->action_dim <= 0 || !state || !action || !next_state ||
        !reward || !done || !strata || !row_ws || n < 0 || action_scale == 0.0f)
        return EXO_EINVAL;
    if (n == 0) return EXO_OK;
    // the one-launch insert (lap_store_fused_kernel) measured slower inside the
    // training loop -- 0.2767-0.2771 vs 0.2522-0.2529 ms per iteration
    // (profiles/r05_sched/r05s2): one workgroup per stratum copying its rows is
    // slower than 1,024 copy workgroups -- so EXO_LAP_STORE_FUSED=1 opts in
    // (read per call: the parity test switches it)
    const char *fused_var = getenv("EXO_LAP_STORE_FUSED");
    const bool fused_env = fused_var && fused_var[0] == '1';
    if (fused_env && n <= STORE_FUSED_MAX && n <= t->capacity) {  // (no ring wrap inside one call)
        const bool vec = (st->state_dim & 3) == 0 &&
                         ((reinterpret_cast<uintptr_t>(state) | reinterpret_cast<uintptr_t>(next_state) |
                           reinterpret_cast<uintptr_t>(st->state) | reinterpret_cast<uintptr_t>(st->next_state)) &
                          15) == 0;
        if (vec)
            hipLaunchKernelGGL(lap_store_fused_kernel<true>, dim3(t->n_strata), dim3(UPD_THREADS), 0,
                               (hipStream_t)stream, t->tree, t->max_priority, t->cap, levels_of(t), t->capacity,
                               st->ptr, st->size, strata, active, n, row_ws, *st, state, action, next_state, reward,
                               done, action_scale);
        else
            hipLaunchKernelGGL(lap_store_fused_kernel<false>, dim3(t->n_strata), dim3(UPD_THREADS), 0,
                               (hipStream_t)stream, t->tree, t->max_priority, t->cap, levels_of(t), t->capacity,
                               st->ptr, st->size, strata, active, n, row_ws, *st, state, action, next_state, reward,
                               done, action_scale);
        return rc(hipGetLastError());
    }
    if (n > 4 * STORE_CHUNK)
        hipLaunchKernelGGL(lap_store_rank_kernel<16>, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream,
                           t->tree, t->max_priority, t->cap, levels_of(t), t->capacity, st->ptr, st->size, strata,
                           active, n, row_ws);
    else
        hipLaunchKernelGGL(lap_store_rank_kernel<4>, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream,
                           t->tree, t->max_priority, t->cap, levels_of(t), t->capacity, st->ptr, st->size, strata,
                           active, n, row_ws);
    if (hipGetLastError() != hipSuccess) return EXO_EDEVICE;
    hipLaunchKernelGGL(lap_store_copy_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, *st, state,
                       action, next_state, reward, done, action_scale, n, row_ws);
    return rc(hipGetLastError());
}

int lap_store_batch_ref(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev, const float *state,
                        const float *action, const float *next_state, const float *reward, const uint8_t *done,
                        const int32_t *strata, const uint8_t *active, float action_scale, int32_t n,
                        int32_t *ws_dev, void *stream) {
    if (!valid(t) || !st || !st->state || !st->action || !st->next_state || !st->reward || !st->not_done ||
        !st->size || st->state_dim <= 0 || st->action_dim <= 0 || !ref_dev || !state || !action || !next_state ||
        !reward || !done || !strata || !ws_dev || n < 0 || action_scale == 0.0f)
        return EXO_EINVAL;
    if (n == 0) return EXO_OK;
    int32_t *rank_row = ws_dev, *slot_of = ws_dev + n, *row_of = ws_dev + 2 * n;
    hipLaunchKernelGGL(lap_store_ref_slots_kernel, dim3(1), dim3(UPD_THREADS), 0, (hipStream_t)stream, t->capacity,
                       t->n_strata, (long long *)ref_dev, st->size, strata, active, n, rank_row, slot_of, row_of);
    if (hipGetLastError() != hipSuccess) return EXO_EDEVICE;
    hipLaunchKernelGGL(lap_add_kernel, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream, t->tree,
                       t->max_priority, t->cap, levels_of(t), t->capacity, strata, slot_of, n);
    if (hipGetLastError() != hipSuccess) return EXO_EDEVICE;
    hipLaunchKernelGGL(lap_store_copy_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, *st, state,
                       action, next_state, reward, done, action_scale, n, row_of);
    return rc(hipGetLastError());
}

static int store_ref_fused(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev,
                           const float *state, const float *action, const float *next_state, const float *reward,
                           const uint8_t *done, const int32_t *strata, const uint8_t *active, float action_scale,
                           int32_t n, uint32_t *ticket_dev, const MaskAdvance &adv, void *stream) {
    if (!valid(t) || !st || !st->state || !st->action || !st->next_state || !st->reward || !st->not_done ||
        !st->size || st->state_dim <= 0 || st->action_dim <= 0 || !ref_dev || !state || !action || !next_state ||
        !reward || !done || !strata || !ticket_dev || n < 0 || action_scale == 0.0f)
        return EXO_EINVAL;
    if (n == 0) return EXO_OK;
    const int E = t->n_strata;
    // part 0 of a stratum: leaves + ancestors; parts 1..K-1: ~64 rows of the copy each
    const int K = 1 + std::max(1, std::min(15, (n + E * 64 - 1) / (E * 64)));
    auto al16 = [](const void *p) { return ((uintptr_t)p & 15u) == 0; };
    const bool vec = st->state_dim % 4 == 0 && al16(state) && al16(next_state) && al16(st->state) &&
                     al16(st->next_state);
    if (vec)
        hipLaunchKernelGGL(lap_store_ref_fused_kernel<true>, dim3(E, K), dim3(UPD_THREADS), 0, (hipStream_t)stream,
                           t->tree, t->max_priority, t->cap, levels_of(t), t->capacity, E, (long long *)ref_dev,
                           st->size, *st, state, action, next_state, reward, done, action_scale, strata, active, n,
                           ticket_dev, adv);
    else
        hipLaunchKernelGGL(lap_store_ref_fused_kernel<false>, dim3(E, K), dim3(UPD_THREADS), 0, (hipStream_t)stream,
                           t->tree, t->max_priority, t->cap, levels_of(t), t->capacity, E, (long long *)ref_dev,
                           st->size, *st, state, action, next_state, reward, done, action_scale, strata, active, n,
                           ticket_dev, adv);
    return rc(hipGetLastError());
}

int lap_store_batch_ref_fused(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev,
                              const float *state, const float *action, const float *next_state, const float *reward,
                              const uint8_t *done, const int32_t *strata, const uint8_t *active, float action_scale,
                              int32_t n, uint32_t *ticket_dev, void *stream) {
    return store_ref_fused(t, st, ref_dev, state, action, next_state, reward, done, strata, active, action_scale, n,
                           ticket_dev, MaskAdvance{}, stream);
}

int lap_store_batch_ref_fused_adv(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev,
                                  const float *state, const float *action, const float *next_state,
                                  const float *reward, const uint8_t *done, const int32_t *strata, uint8_t *active,
                                  float action_scale, int32_t n, uint32_t *ticket_dev, const uint8_t *table,
                                  int32_t rows, int64_t *k_dev, int32_t *count_dev, double *score_dev, void *stream) {
    if (!table || rows <= 0 || !k_dev || !active) return EXO_EINVAL;
    return store_ref_fused(t, st, ref_dev, state, action, next_state, reward, done, strata, active, action_scale, n,
                           ticket_dev, MaskAdvance{table, rows, (long long *)k_dev, active, count_dev, score_dev},
                           stream);
}

int lap_sample_gather(const lap_tree_desc *t, const lap_storage_desc *st, const float *u, int32_t batch,
                      int32_t *idx, float *out_state, float *out_action, float *out_next_state, float *out_reward,
                      float *out_not_done, void *stream) {
    if (!valid(t) || !st || !st->size || !u || !idx || batch <= 0 || !out_state || !out_action ||
        !out_next_state || !out_reward || !out_not_done)
        return EXO_EINVAL;
    const int total = t->n_strata * batch;
    hipLaunchKernelGGL(lap_sample_gather_kernel, dim3((total + 3) / 4), dim3(256), 0, (hipStream_t)stream, t->tree,
                       t->cap, levels_of(t), t->capacity, u, st->size, batch, total, idx, *st, out_state, out_action,
                       out_next_state, out_reward, out_not_done, SampleRng{0, 0, nullptr, nullptr});
    return rc(hipGetLastError());
}

int lap_update_sample_rng(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *idx_in,
                          const float *prio, int32_t batch, uint64_t seed, uint32_t tag, unsigned long long *counter,
                          uint32_t *ticket, int32_t *idx_out, float *out_state, float *out_action,
                          float *out_next_state, float *out_reward, float *out_not_done, void *stream) {
    if (!valid(t) || !st || !st->size || !idx_in || !prio || !counter || !ticket || !idx_out || batch <= 0 ||
        batch > UPD_THREADS || !out_state || !out_action || !out_next_state || !out_reward || !out_not_done)
        return EXO_EINVAL;
    hipLaunchKernelGGL(lap_update_sample_kernel, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream,
                       t->tree, t->max_priority, t->cap, levels_of(t), t->capacity, idx_in, prio, batch, st->size,
                       *st, SampleRng{seed, tag, counter, ticket}, idx_out, out_state, out_action, out_next_state,
                       out_reward, out_not_done, TdPrio{nullptr, 0.f, 0.f, nullptr}, !gather_split());
    return gather_after(t, st, batch, idx_out, out_state, out_action, out_next_state, out_reward, out_not_done, stream);
}

int lap_update_sample_idx(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *idx_in,
                          const float *prio, int32_t batch, uint64_t seed, uint32_t tag, unsigned long long *counter,
                          uint32_t *ticket, int32_t *idx_out, void *stream) {
    if (!valid(t) || !st || !st->size || !idx_in || !prio || !counter || !ticket || !idx_out || batch <= 0 ||
        batch > UPD_THREADS)
        return EXO_EINVAL;
    hipLaunchKernelGGL(lap_update_sample_kernel, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream,
                       t->tree, t->max_priority, t->cap, levels_of(t), t->capacity, idx_in, prio, batch, st->size,
                       *st, SampleRng{seed, tag, counter, ticket}, idx_out, nullptr, nullptr, nullptr, nullptr,
                       nullptr, TdPrio{nullptr, 0.f, 0.f, nullptr}, false);
    return rc(hipGetLastError());
}

int lap_gather_rows(const lap_tree_desc *t, const lap_storage_desc *st, int32_t batch, const int32_t *idx,
                    float *out_state, float *out_action, float *out_next_state, float *out_reward,
                    float *out_not_done, void *stream) {
    if (!valid(t) || !st || !st->state || !st->action || !st->next_state || !st->reward || !st->not_done || !idx ||
        batch <= 0 || !out_state || !out_action || !out_next_state || !out_reward || !out_not_done)
        return EXO_EINVAL;
    const int total = t->n_strata * batch;
    hipLaunchKernelGGL(lap_gather_kernel, dim3((total + GATHER_DRAWS - 1) / GATHER_DRAWS), dim3(256), 0,
                       (hipStream_t)stream, *st, t->capacity, idx, batch, total, out_state, out_action,
                       out_next_state, out_reward, out_not_done);
    return rc(hipGetLastError());
}

int lap_update_sample_td(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *idx_in, const float *td,
                         float alpha, float min_priority, float *prio_out, int32_t batch, uint64_t seed, uint32_t tag,
                         unsigned long long *counter, uint32_t *ticket, int32_t *idx_out, float *out_state,
                         float *out_action, float *out_next_state, float *out_reward, float *out_not_done,
                         void *stream) {
    if (!valid(t) || !st || !st->size || !idx_in || !td || !counter || !ticket || !idx_out || batch <= 0 ||
        batch > UPD_THREADS || !out_state || !out_action || !out_next_state || !out_reward || !out_not_done)
        return EXO_EINVAL;
    hipLaunchKernelGGL(lap_update_sample_kernel, dim3(t->n_strata), dim3(UPD_THREADS), 0, (hipStream_t)stream,
                       t->tree, t->max_priority, t->cap, levels_of(t), t->capacity, idx_in, (const float *)nullptr,
                       batch, st->size, *st, SampleRng{seed, tag, counter, ticket}, idx_out, out_state, out_action,
                       out_next_state, out_reward, out_not_done, TdPrio{td, alpha, min_priority, prio_out},
                       !gather_split());
    return gather_after(t, st, batch, idx_out, out_state, out_action, out_next_state, out_reward, out_not_done, stream);
}

int lap_sample_gather_rng(const lap_tree_desc *t, const lap_storage_desc *st, uint64_t seed, uint32_t tag,
                          unsigned long long *counter, uint32_t *ticket, int32_t batch, int32_t *idx,
                          float *out_state, float *out_action, float *out_next_state, float *out_reward,
                          float *out_not_done, void *stream) {
    if (!valid(t) || !st || !st->size || !counter || !ticket || !idx || batch <= 0 || !out_state || !out_action ||
        !out_next_state || !out_reward || !out_not_done)
        return EXO_EINVAL;
    const int total = t->n_strata * batch;
    hipLaunchKernelGGL(lap_sample_gather_kernel, dim3((total + 3) / 4), dim3(256), 0, (hipStream_t)stream, t->tree,
                       t->cap, levels_of(t), t->capacity, nullptr, st->size, batch, total, idx, *st, out_state,
                       out_action, out_next_state, out_reward, out_not_done, SampleRng{seed, tag, counter, ticket});
    return rc(hipGetLastError());
}


// ---------------------------------------------------------------- planned reference inserts (C ABI)
int lap_ref_plan(const lap_tree_desc *t, const int64_t *ref_dev, const uint8_t *table_dev, int32_t rows, int32_t n,
                 const int32_t *strata_dev, const int64_t *offs_dev, int64_t total, int32_t *add_ws_dev,
                 int32_t *plan_dev, void *stream) {
    if (!valid(t) || !ref_dev || !table_dev || rows <= 0 || n <= 0 || !strata_dev || !offs_dev || total < 0 ||
        (total > 0 && !add_ws_dev) || !plan_dev)
        return EXO_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(lap_ref_plan_scan_kernel, dim3(rows), dim3(UPD_THREADS), 0, s, table_dev, n, strata_dev,
                       t->n_strata, (const long long *)offs_dev, add_ws_dev, plan_dev);
    if (hipGetLastError() != hipSuccess) return EXO_EDEVICE;
    const long long entries = (long long)rows * n;
    hipLaunchKernelGGL(lap_ref_plan_slots_kernel, dim3((unsigned)((entries + 255) / 256)), dim3(256), 0, s, plan_dev,
                       entries, add_ws_dev, (long long)total, (const long long *)ref_dev, t->n_strata, t->capacity);
    return rc(hipGetLastError());
}

int lap_ref_step(const lap_tree_desc *t, const lap_storage_desc *st, const int32_t *plan_dev, int32_t rows,
                 int32_t n, int64_t *kk_dev, int32_t par, int64_t *k_dev, const int32_t *strata_dev,
                 const float *state, const float *action, const float *next_state, const float *reward,
                 const uint8_t *done, float action_scale, const uint8_t *table_dev, uint8_t *active_dev,
                 int32_t *count_dev, const int32_t *counts_table_dev, double *score_dev, void *stream) {
    if (!valid(t) || !st || !st->state || !st->action || !st->next_state || !st->reward || !st->not_done ||
        !plan_dev || rows <= 0 || n <= 0 || !kk_dev || (par != 0 && par != 1) || !strata_dev || !state || !action ||
        !next_state || !reward || !done || action_scale == 0.0f || !table_dev || !active_dev ||
        (count_dev && !counts_table_dev))
        return EXO_EINVAL;
    hipLaunchKernelGGL(lap_ref_step_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, *st, plan_dev,
                       rows, n, (long long *)kk_dev, par, (long long *)k_dev, strata_dev, t->capacity, state, action,
                       next_state, reward, done, action_scale, table_dev, active_dev, count_dev, counts_table_dev,
                       score_dev);
    return rc(hipGetLastError());
}

int lap_ref_commit(const lap_tree_desc *t, const lap_storage_desc *st, int64_t *ref_dev, const int32_t *plan_dev,
                   int32_t rows, int32_t n, const int32_t *strata_dev, int64_t total, void *stream) {
    if (!valid(t) || !st || !st->size || !ref_dev || !plan_dev || rows <= 0 || n <= 0 || !strata_dev || total < 0)
        return EXO_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const long long entries = (long long)rows * n;
    hipLaunchKernelGGL(lap_ref_commit_leaves_kernel, dim3((unsigned)((entries + 255) / 256)), dim3(256), 0, s,
                       plan_dev, entries, n, strata_dev, t->tree, t->cap, t->max_priority);
    hipLaunchKernelGGL(lap_ref_commit_tree_kernel, dim3(t->n_strata), dim3(UPD_THREADS), 0, s, t->tree, t->cap,
                       levels_of(t), t->capacity, (const long long *)ref_dev, (long long)total, t->n_strata);
    hipLaunchKernelGGL(lap_ref_commit_ref_kernel, dim3(1), dim3(1), 0, s, (long long *)ref_dev, (long long)total,
                       t->n_strata, t->capacity, st->size);
    return rc(hipGetLastError());
}

} // extern "C"
