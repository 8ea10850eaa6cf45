// td7_fused_train.hip -- the gradient passes of the TD7 update as row-tile-fused
// launches (see td7_fused.h), Agent/TD7_multi_agent.py:211-293:
//
//   td7f_critic  : one workgroup per (16 rows, Q head): the critic forward on
//                  [s, a] and the fixed embeddings, Q_target from the target
//                  heads (:241-246, running bounds by atomics), the LAP-Huber
//                  gradient (:257-259, |td| kept for the priorities) and the
//                  whole dX chain back to the first layer (:260-262)
//   td7f_encoder : one workgroup per 16 rows: zs(s'), zs(s), zsa(zs, a), the
//                  mse gradient (:219-228) and the dX chain through zsa and zs
//   td7f_actor_a : actor(s, fixed_zs) and fixed_encoder.zsa(fixed_zs, actor) (:268-270)
//   td7f_actor_b : the updated critic on them, d(-mean Q) back to the action
//                  and zsa inputs, one workgroup per (16 rows, head) (:271-273)
//   td7f_actor_c : the fixed encoder's zsa backward to the action, tanh' and the
//                  actor's dX chain
//   td7f_wgrad   : every layer's dW = dP^T X and db of one optimiser phase as
//                  ONE grouped MFMA launch over the transposed 16-bit operands
//                  the passes above leave in HBM.
//
// Each backward GEMM reads a dX-packed weight (td7_fused.h Lin.wb) and applies
// act'(Y) with Y the fp32 activation its forward epilogue stored (read back by
// the same lanes).  Bias gradients come from the unrounded fp32 dP (column
// partials per row tile, summed in td7f_wgrad).
#include "td7_fused.h"
#include "adam_math.h"

#include <algorithm>

namespace td7f {

// Transposed operands of one layer's weight gradient (row stride ld = padded batch).
struct XT {
    void *x;   // X^T  [K][ld] (operand type, fragment blocks: td7_fused.h blk8 / blk4)
    void *dp;  // dP^T [N][ld] (x gs)
    float *part;   // [row tiles][N] fp32 column sums of dP
};

// dX over the window [c0, c1) (c0 % 16 == 0) of layer L from the dP image a;
// act'(Y) from global y (row stride yld) when act != ACT_NONE.  Ends with a barrier.
template <int P, int TH>
__device__ __forceinline__ void layer_bwd(char *lds, u32x4 (&R)[PD][TH], R16 a, const Lin &L, int c0, int c1,
                                          const GDesc *next, int act, const float *y, long yld, R32 o32, float *g,
                                          long gld, R16 o16, float *part, int row0, int nrows, int &si) {
    FSTAMP(si);
    floatx4 acc[1][TH], yv[1][TH];
    const GDesc gd{L.wb, L.ksb, c0 / 16};
    gemm<P, 1, TH>(lds, a.off, a.ld, gd, R, acc, next,
                   EpiSrc{act != ACT_NONE ? y : nullptr, yld, c0, row0, nrows, c1 - c0}, yv);
    FSTAMP(si);
    epi_bwd<P, 1, TH>(lds, acc, c0 / 16, c0, c1, act, yv, o32, g, gld, o16, part, row0, nrows);
    __syncthreads();
}

__device__ __forceinline__ GDesc fwd_of(const Lin &L) { return GDesc{L.wf, L.ksf, 0}; }
__device__ __forceinline__ GDesc bwd_of(const Lin &L, int c0) { return GDesc{L.wb, L.ksb, c0 / 16}; }

__device__ __forceinline__ void atomic_max_f(float *a, float v) {
    if (v >= 0.f) atomicMax((int *)a, __float_as_int(v));
    else atomicMin((unsigned int *)a, __float_as_uint(v));
}
__device__ __forceinline__ void atomic_min_f(float *a, float v) {
    if (v >= 0.f) atomicMin((int *)a, __float_as_int(v));
    else atomicMax((unsigned int *)a, __float_as_uint(v));
}

// ---------------------------------------------------------------- critic
struct CriticArgs {
    Lin cr[8];  // [layer][head]
    int act;
    const float *s, *a, *zs, *zsa, *qt, *reward, *not_done;
    float discount, inv_b;
    const float *lo, *hi;
    float *run_max, *run_min;
    int B, S, A, Z, Hc;
    float *td, *q;     // [B][2]
    float *y1, *y2;    // [2][B][Hc] forward activations for act'
    XT xt[8];          // [layer][head]
    long ld;           // row stride of the transposed operands
    R16 X, CAT, H1, H2, DP0, DP1;
    R32 H0, DY, F, TW;
    int small_off;     // 2 x 16 floats: row means, row dots
    int lds_bytes;
    // phase (td7f_critic_phase): 0 the whole pass; 1 the forward alone, its
    // state for the backward stored -- Q [2][Bp], the pre-norm q0 output H0
    // [2][Bp][Hc] and the row means [2][Bp] (Bp = B padded to 16 rows); 2 the
    // loss and the backward from that state
    int phase;
    float *qs, *h0s, *ms;
};

template <int P, int TH>
__global__ __launch_bounds__(NTH) void critic_kernel(CriticArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int row0 = blockIdx.x * TR, B = a.B, h = blockIdx.y, Hc = a.Hc, Z = a.Z, tile = blockIdx.x;
    const Lin *cr = a.cr + h;  // layer l of head h: cr[2 l]
    const XT *xt = a.xt + h;
    float *mean = (float *)(lds + a.small_off), *dot = mean + TR;
    float *y1 = a.y1 + (long)h * B * Hc, *y2 = a.y2 + (long)h * B * Hc;
    int si = 0;
    FSTAMP(si);
    u32x4 R[PD][TH];
    const long Bp = (long)gridDim.x * TR;
    if (a.phase == 2) {
        // the forward's state back into LDS (the same fp32 values), the ring
        // filled with q3's first backward k-steps as the forward's tail left it
        constexpr int PER = TR * 320 / NTH;  // H0 values per thread (Hc <= 320)
        const float *h0 = a.h0s + ((long)h * Bp + row0) * Hc;
        float v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = threadIdx.x + j * NTH;
            v[j] = i < TR * Hc ? ldg(h0 + i) : 0.f;
        }
        const float qv = threadIdx.x < TR ? ldg(a.qs + h * Bp + row0 + threadIdx.x) : 0.f;
        const float mv = threadIdx.x < TR ? ldg(a.ms + h * Bp + row0 + threadIdx.x) : 0.f;
        ring_fill(R, bwd_of(cr[6], 0));
        zero_lds(lds, a.lds_bytes);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = threadIdx.x + j * NTH;
            if (i < TR * Hc) *p32(lds, a.H0, i / Hc, i % Hc) = v[j];
        }
        if (threadIdx.x < TR) {
            *p32(lds, a.F, threadIdx.x, 0) = qv;
            mean[threadIdx.x] = mv;
        }
        __syncthreads();
    } else {
    RowStage ss, sa, sz, szs;
    ThinStage<1> tw;
    row_issue(ss, a.s, a.S, a.S, row0, B);
    row_issue(sa, a.a, a.A, a.A, row0, B);
    row_issue(sz, a.zsa, Z, Z, row0, B);
    row_issue(szs, a.zs, Z, Z, row0, B);
    thin_issue(tw, cr[6].w, cr[6].ldw, 0, false, 1, cr[6].K);
    ring_fill(R, fwd_of(cr[0]));
    zero_lds(lds, a.lds_bytes);
    __syncthreads();
    row_put16<P>(lds, ss, a.X, 0, a.S, row0, B);
    row_put16<P>(lds, sa, a.X, a.S, a.A, row0, B);
    row_put16<P>(lds, sz, a.CAT, Hc, Z, row0, B);
    row_put16<P>(lds, szs, a.CAT, Hc + Z, Z, row0, B);
    thin_put<P>(lds, tw, a.TW, 1, cr[6].K);
    __syncthreads();
    // forward (:121-126): AvgL1Norm(q0([s, a])) | zsa | zs -> q1 -> q2 -> q3
    layer_fwd<P, 1, TH>(lds, R, a.X, cr[0], &cr[2], ACT_NONE, NO16, 0, a.H0, nullptr, 0, row0, B, si);
    norm_fwd<P>(lds, a.H0, Hc, TR, 1e-8f, a.CAT, 0, NO16, 0, NO32, nullptr, 0, mean, nullptr, row0, B);
    __syncthreads();
    save_xt<P>(lds, a.X, 0, a.S + a.A, xt[0].x, a.ld, TR, row0);
    save_xt<P>(lds, a.CAT, 0, Hc + 2 * Z, xt[2].x, a.ld, TR, row0);
    layer_fwd<P, 1, TH>(lds, R, a.CAT, cr[2], &cr[4], a.act, a.H1, 0, NO32, y1, Hc, row0, B, si);
    const GDesc b3 = bwd_of(cr[6], 0);
    layer_fwd<P, 1, TH>(lds, R, a.H1, cr[4], &b3, a.act, a.H2, 0, NO32, y2, Hc, row0, B, si);
    save_xt<P>(lds, a.H1, 0, Hc, xt[4].x, a.ld, TR, row0);
    save_xt<P>(lds, a.H2, 0, Hc, xt[6].x, a.ld, TR, row0);
    layer_thin_fwd<P, 1>(lds, a.H2, cr[6], a.TW, ACT_NONE, a.F, TR, nullptr, 0, row0, B, si);
    if (a.phase == 1) {  // the state the backward launch needs, then done
        __syncthreads();
        float *h0 = a.h0s + ((long)h * Bp + row0) * Hc;
        for (int i = threadIdx.x; i < TR * Hc; i += NTH) stg(h0 + i, *p32(lds, a.H0, i / Hc, i % Hc));
        if (threadIdx.x < TR) {
            stg(a.qs + h * Bp + row0 + threadIdx.x, *p32(lds, a.F, threadIdx.x, 0));
            stg(a.ms + h * Bp + row0 + threadIdx.x, mean[threadIdx.x]);
        }
        return;
    }
    }
    // Q_target (:241-246) and the LAP-Huber gradient (:257-259) of this head
    if (threadIdx.x < TR) {
        const int r = threadIdx.x, b = row0 + r;
        float dq = 0.f;
        if (b < B) {
            const float qv = *p32(lds, a.F, r, 0);
            const float qm = fminf(ldg(a.qt + 2 * b), ldg(a.qt + 2 * b + 1));
            const float c = fminf(fmaxf(qm, ldg(a.lo)), ldg(a.hi));
            const float t = ldg(a.reward + b) + (ldg(a.not_done + b) * a.discount) * c;
            if (h == 0) {
                atomic_max_f(a.run_max, t);
                atomic_min_f(a.run_min, t);
            }
            const float d = qv - t, x = fabsf(d);
            const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
            dq = a.inv_b * (x < 1.0f ? x : 1.0f) * sg;
            stg(a.td + 2 * b + h, x);
            if (a.q) stg(a.q + 2 * b + h, qv);
        }
        *p32(lds, a.F, r, 0) = dq;
    }
    __syncthreads();
    // backward (:260-262): q3 -> q2 -> q1 (the q window) -> AvgL1Norm -> q0's dP
    make_dp<P>(lds, a.F, 1, ACT_NONE, nullptr, 0, a.DP1, xt[6].part + (long)tile * 1, row0, B);
    __syncthreads();
    save_xt<P>(lds, a.DP1, 0, 1, xt[6].dp, a.ld, TR, row0);
    const GDesc nx1 = bwd_of(cr[4], 0);
    layer_bwd<P, TH>(lds, R, a.DP1, cr[6], 0, Hc, &nx1, a.act, y2, Hc, NO32, nullptr, 0, a.DP0,
                     xt[4].part + (long)tile * Hc, row0, B, si);
    save_xt<P>(lds, a.DP0, 0, Hc, xt[4].dp, a.ld, TR, row0);
    const GDesc nx2 = bwd_of(cr[2], 0);
    layer_bwd<P, TH>(lds, R, a.DP0, cr[4], 0, Hc, &nx2, a.act, y1, Hc, NO32, nullptr, 0, a.DP1,
                     xt[2].part + (long)tile * Hc, row0, B, si);
    save_xt<P>(lds, a.DP1, 0, Hc, xt[2].dp, a.ld, TR, row0);
    layer_bwd<P, TH>(lds, R, a.DP1, cr[2], 0, Hc, nullptr, ACT_NONE, nullptr, 0, a.DY, nullptr, 0, NO16, nullptr,
                     row0, B, si);
    norm_bwd<P>(lds, a.DY, a.H0, mean, Hc, 1e-8f, dot, a.DP0, xt[0].dp, a.ld, xt[0].part + (long)tile * Hc,
                row0, B);
}

// ---------------------------------------------------------------- encoder
struct EncoderArgs {
    Lin e[6];  // zs1 zs2 zs3 zsa1 zsa2 zsa3
    int act;
    const float *s, *a, *ns;
    int B, S, A, Z, He;
    float mse_scale;    // 2 / (B * zs_dim)
    float *y0, *y1, *y2, *y3;  // [B][He]: zs1, zs2, zsa1, zsa2 activations
    XT xt[6];
    long ld;
    R16 X, H1, H2, CATZ, DP0, DP1;
    R32 H3, NZ, DY;
    int small_off;
    int lds_bytes;
    // grid.y == 2 (r04): workgroup row 0 computes next_zs and publishes it
    // here ([row tiles * 16][Z] fp32) with a per-tile flag; row 1 runs the rest
    float *nz;
    int32_t *flag;  // [row tiles]: 1 = published; the consumer clears it
};

// grid.y == 1: one workgroup per 16 rows runs the whole pass (next_zs first).
// grid.y == 2 (r04): the no-grad next_zs chain (3 of the
// pass's ~14 serial layers) runs on its own workgroup row: row 0 computes it
// and publishes it to global memory (agent-scope release of a per-tile flag:
// the two workgroups may sit on different XCDs' L2s), row 1 runs zs(s), zsa
// and the backward and waits for the flag only at the mse gradient.  The
// dispatcher issues the grid in order, so every producer is resident or done
// before any consumer spins: no deadlock.  Same arithmetic in the same order:
// bit-identical to grid.y == 1 (tests/test_fused_gpu.py).
template <int P, int TH>
__global__ __launch_bounds__(NTH) void encoder_kernel(EncoderArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int row0 = blockIdx.x * TR, B = a.B, Z = a.Z, He = a.He, tile = blockIdx.x;
    const long ld = a.ld;
    const bool split = gridDim.y == 2, producer = split && blockIdx.y == 0;
    float *mean = (float *)(lds + a.small_off), *dot = mean + TR;
    int si = 0;
    FSTAMP(si);
    RowStage sns, sa, ss;
    if (!split || producer) row_issue(sns, a.ns, a.S, a.S, row0, B);
    if (!producer) {
        row_issue(sa, a.a, a.A, a.A, row0, B);
        row_issue(ss, a.s, a.S, a.S, row0, B);  // put after the next_zs pass
    }
    u32x4 R[PD][TH];
    ring_fill(R, fwd_of(a.e[0]));
    zero_lds(lds, a.lds_bytes);
    __syncthreads();
    if (!split || producer) {
        row_put16<P>(lds, sns, a.X, 0, a.S, row0, B);
        if (!producer) row_put16<P>(lds, sa, a.CATZ, Z, a.A, row0, B);
        __syncthreads();
        // next_zs = encoder.zs(next_state) under no_grad (:219-220) -> NZ (fp32)
        layer_fwd<P, 1, TH>(lds, R, a.X, a.e[0], &a.e[1], a.act, a.H1, 0, NO32, nullptr, 0, row0, B, si);
        layer_fwd<P, 1, TH>(lds, R, a.H1, a.e[1], &a.e[2], a.act, a.H2, 0, NO32, nullptr, 0, row0, B, si);
        const GDesc z1 = fwd_of(a.e[0]);
        layer_fwd<P, 1, TH>(lds, R, a.H2, a.e[2], producer ? nullptr : &z1, ACT_NONE, NO16, 0, a.H3, nullptr, 0,
                            row0, B, si);
        norm_fwd<P>(lds, a.H3, Z, TR, 1e-8f, NO16, 0, NO16, 0, a.NZ, nullptr, 0, nullptr, nullptr, row0, B);
        __syncthreads();
        if (producer) {
            float *dst = a.nz + (long)row0 * Z;
            for (int k = threadIdx.x; k < TR * Z; k += NTH) {
                const int r = k / Z, c = k - r * Z;
                dst[k] = *p32(lds, a.NZ, r, c);
            }
            __threadfence();  // every thread's rows written back past its XCD's L2
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_store(a.flag + tile, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    } else {
        row_put16<P>(lds, sa, a.CATZ, Z, a.A, row0, B);
    }
    // zs = encoder.zs(state) (:222), pred_zs = encoder.zsa(zs, action) (:223)
    row_put16<P>(lds, ss, a.X, 0, a.S, row0, B);
    __syncthreads();
    save_xt<P>(lds, a.X, 0, a.S, a.xt[0].x, ld, TR, row0);
    layer_fwd<P, 1, TH>(lds, R, a.X, a.e[0], &a.e[1], a.act, a.H1, 0, NO32, a.y0, He, row0, B, si);
    save_xt<P>(lds, a.H1, 0, He, a.xt[1].x, ld, TR, row0);
    layer_fwd<P, 1, TH>(lds, R, a.H1, a.e[1], &a.e[2], a.act, a.H2, 0, NO32, a.y1, He, row0, B, si);
    save_xt<P>(lds, a.H2, 0, He, a.xt[2].x, ld, TR, row0);
    layer_fwd<P, 1, TH>(lds, R, a.H2, a.e[2], &a.e[3], ACT_NONE, NO16, 0, a.H3, nullptr, 0, row0, B, si);
    norm_fwd<P>(lds, a.H3, Z, TR, 1e-8f, a.CATZ, 0, NO16, 0, NO32, nullptr, 0, mean, nullptr, row0, B);
    __syncthreads();
    save_xt<P>(lds, a.CATZ, 0, Z + a.A, a.xt[3].x, ld, TR, row0);
    layer_fwd<P, 1, TH>(lds, R, a.CATZ, a.e[3], &a.e[4], a.act, a.H1, 0, NO32, a.y2, He, row0, B, si);
    save_xt<P>(lds, a.H1, 0, He, a.xt[4].x, ld, TR, row0);
    const GDesc b6 = bwd_of(a.e[5], 0);
    layer_fwd<P, 1, TH>(lds, R, a.H1, a.e[4], &a.e[5], a.act, a.H2, 0, NO32, a.y3, He, row0, B, si);
    save_xt<P>(lds, a.H2, 0, He, a.xt[5].x, ld, TR, row0);
    layer_fwd<P, 1, TH>(lds, R, a.H2, a.e[5], &b6, ACT_NONE, NO16, 0, a.DY, nullptr, 0, row0, B, si);
    if (split) {  // next_zs from this tile's producer
        if (threadIdx.x == 0) {
            while (__hip_atomic_load(a.flag + tile, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0)
                __builtin_amdgcn_s_sleep(2);
            __hip_atomic_store(a.flag + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const float *src = a.nz + (long)row0 * Z;
        for (int k = threadIdx.x; k < TR * Z; k += NTH) {
            const int r = k / Z, c = k - r * Z;
            *p32(lds, a.NZ, r, c) = src[k];
        }
        __syncthreads();
    }
    // d mse(pred, next_zs) / d pred = 2 (pred - next_zs) / (B zs_dim) (:226)
    for (int k = threadIdx.x; k < TR * Z; k += NTH) {
        const int r = k / Z, c = k - r * Z;
        float *d = p32(lds, a.DY, r, c);
        *d = (*d - *p32(lds, a.NZ, r, c)) * a.mse_scale;
    }
    __syncthreads();
    make_dp<P>(lds, a.DY, Z, ACT_NONE, nullptr, 0, a.DP0, a.xt[5].part + (long)tile * Z, row0, B);
    __syncthreads();
    save_xt<P>(lds, a.DP0, 0, Z, a.xt[5].dp, ld, TR, row0);
    const GDesc nx3 = bwd_of(a.e[4], 0);
    layer_bwd<P, TH>(lds, R, a.DP0, a.e[5], 0, He, &nx3, a.act, a.y3, He, NO32, nullptr, 0, a.DP1,
                     a.xt[4].part + (long)tile * He, row0, B, si);
    save_xt<P>(lds, a.DP1, 0, He, a.xt[4].dp, ld, TR, row0);
    const GDesc nx4 = bwd_of(a.e[3], 0);
    layer_bwd<P, TH>(lds, R, a.DP1, a.e[4], 0, He, &nx4, a.act, a.y2, He, NO32, nullptr, 0, a.DP0,
                     a.xt[3].part + (long)tile * He, row0, B, si);
    save_xt<P>(lds, a.DP0, 0, He, a.xt[3].dp, ld, TR, row0);
    const GDesc nx5 = bwd_of(a.e[2], 0);
    // d zs from the zs columns of zsa1's input, then AvgL1Norm backward
    layer_bwd<P, TH>(lds, R, a.DP0, a.e[3], 0, Z, &nx5, ACT_NONE, nullptr, 0, a.NZ, nullptr, 0, NO16, nullptr, row0, B,
                     si);
    norm_bwd<P>(lds, a.NZ, a.H3, mean, Z, 1e-8f, dot, a.DP1, a.xt[2].dp, ld, a.xt[2].part + (long)tile * Z, row0, B);
    __syncthreads();
    const GDesc nx6 = bwd_of(a.e[1], 0);
    layer_bwd<P, TH>(lds, R, a.DP1, a.e[2], 0, He, &nx6, a.act, a.y1, He, NO32, nullptr, 0, a.DP0,
                     a.xt[1].part + (long)tile * He, row0, B, si);
    save_xt<P>(lds, a.DP0, 0, He, a.xt[1].dp, ld, TR, row0);
    layer_bwd<P, TH>(lds, R, a.DP0, a.e[1], 0, He, nullptr, a.act, a.y0, He, NO32, nullptr, 0, a.DP1,
                     a.xt[0].part + (long)tile * He, row0, B, si);
    save_xt<P>(lds, a.DP1, 0, He, a.xt[0].dp, ld, TR, row0);
}

// ---------------------------------------------------------------- actor update
struct ActorArgs {
    Lin ac[4], fe[6], cr[8];
    int act_enc, act_actor, act_critic;
    const float *s, *zs;
    int B, S, A, Z, Ha, He, Hc;
    float dq;                  // d(-mean Q)/dQ = -1 / (2 B)
    float *act_out;            // [B][A] actor(s, zs)
    float *zsa_out;            // [B][Z] fixed_encoder.zsa(zs, actor)
    float *h0, *mean0;         // actor l0 pre-norm [B][Ha], row means [B]
    float *ya[2], *yz[2];      // actor l1/l2 [B][Ha]; zsa1/zsa2 [B][He]
    float *yc[2];              // critic l1/l2 per head [2][B][Hc]
    float *da, *dzsa;          // per head [2][B][A], [2][B][Z]
    XT xt[4];                  // actor layers
    long ld;
    R16 X, CATA, CATZ, CAT, H1, H2, DP0, DP1;
    R32 H0, DY, F, TW, TW2;
    int small_off;
    int lds;
};

template <int P, int TH>
__global__ __launch_bounds__(NTH) void actor_a_kernel(ActorArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int row0 = blockIdx.x * TR, B = a.B, Z = a.Z, Ha = a.Ha, He = a.He;
    const long ld = a.ld;
    int si = 0;
    RowStage ss, szs;
    ThinStage<THIN_NC> tw;
    row_issue(ss, a.s, a.S, a.S, row0, B);
    row_issue(szs, a.zs, Z, Z, row0, B);
    thin_issue(tw, a.ac[3].w, a.ac[3].ldw, 0, false, a.A, a.ac[3].K);
    u32x4 R[PD][TH];
    ring_fill(R, fwd_of(a.ac[0]));
    zero_lds(lds, a.lds);
    __syncthreads();
    row_put16<P>(lds, ss, a.X, 0, a.S, row0, B);
    row_put16<P>(lds, szs, a.CATA, Ha, Z, row0, B);
    row_put16<P>(lds, szs, a.CATZ, 0, Z, row0, B);
    thin_put<P>(lds, tw, a.TW, a.A, a.ac[3].K);
    __syncthreads();
    // actor(state, fixed_zs) (:268, :72-77)
    layer_fwd<P, 1, TH>(lds, R, a.X, a.ac[0], &a.ac[1], ACT_NONE, NO16, 0, a.H0, a.h0, Ha, row0, B, si);
    norm_fwd<P>(lds, a.H0, Ha, TR, 1e-8f, a.CATA, 0, NO16, 0, NO32, nullptr, 0, nullptr, a.mean0, row0, B);
    __syncthreads();
    save_xt<P>(lds, a.X, 0, a.S, a.xt[0].x, ld, TR, row0);
    save_xt<P>(lds, a.CATA, 0, Ha + Z, a.xt[1].x, ld, TR, row0);
    layer_fwd<P, 1, TH>(lds, R, a.CATA, a.ac[1], &a.ac[2], a.act_actor, a.H1, 0, NO32, a.ya[0], Ha, row0, B, si);
    layer_fwd<P, 1, TH>(lds, R, a.H1, a.ac[2], &a.fe[3], a.act_actor, a.H2, 0, NO32, a.ya[1], Ha, row0, B, si);
    save_xt<P>(lds, a.H1, 0, Ha, a.xt[2].x, ld, TR, row0);
    save_xt<P>(lds, a.H2, 0, Ha, a.xt[3].x, ld, TR, row0);
    layer_thin_fwd<P, THIN_NC>(lds, a.H2, a.ac[3], a.TW, ACT_TANH, a.F, TR, a.act_out, a.A, row0, B, si);
    for (int k = threadIdx.x; k < TR * a.A; k += NTH) {
        const int r = k / a.A, c = k - r * a.A;
        *pe<P>(lds, a.CATZ, r, Z + c) = Ty<P>::bits(*p32(lds, a.F, r, c));
    }
    __syncthreads();
    // fixed_encoder.zsa(fixed_zs, actor) (:269)
    layer_fwd<P, 1, TH>(lds, R, a.CATZ, a.fe[3], &a.fe[4], a.act_enc, a.H1, 0, NO32, a.yz[0], He, row0, B, si);
    layer_fwd<P, 1, TH>(lds, R, a.H1, a.fe[4], &a.fe[5], a.act_enc, a.H2, 0, NO32, a.yz[1], He, row0, B, si);
    layer_fwd<P, 1, TH>(lds, R, a.H2, a.fe[5], (const Lin *)nullptr, ACT_NONE, NO16, 0, NO32, a.zsa_out, Z, row0, B, si);
}

template <int P, int TH>
__global__ __launch_bounds__(NTH) void actor_b_kernel(ActorArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int row0 = blockIdx.x * TR, B = a.B, Z = a.Z, h = blockIdx.y, Hc = a.Hc;
    const Lin *cr = a.cr + h;
    float *mean = (float *)(lds + a.small_off), *dot = mean + TR;
    float *y1 = a.yc[0] + (long)h * B * Hc, *y2 = a.yc[1] + (long)h * B * Hc;
    int si = 0;
    FSTAMP(si);
    RowStage ss, sa, sz, szs;
    ThinStage<THIN_NC> tw;
    row_issue(ss, a.s, a.S, a.S, row0, B);
    row_issue(sa, a.act_out, a.A, a.A, row0, B);
    row_issue(sz, a.zsa_out, Z, Z, row0, B);
    row_issue(szs, a.zs, Z, Z, row0, B);
    thin_issue(tw, cr[0].w, cr[0].ldw, a.S, true, a.A, Hc);
    u32x4 R[PD][TH];
    ring_fill(R, fwd_of(cr[0]));
    zero_lds(lds, a.lds);
    __syncthreads();
    row_put16<P>(lds, ss, a.X, 0, a.S, row0, B);
    row_put16<P>(lds, sa, a.X, a.S, a.A, row0, B);
    row_put16<P>(lds, sz, a.CAT, Hc, Z, row0, B);
    row_put16<P>(lds, szs, a.CAT, Hc + Z, Z, row0, B);
    if constexpr (P != PREC_F32) thin_put<P>(lds, tw, a.TW, a.A, Hc);
    __syncthreads();
    // Q = critic(state, actor, zsa, zs) with the updated critic (:270)
    layer_fwd<P, 1, TH>(lds, R, a.X, cr[0], &cr[2], ACT_NONE, NO16, 0, a.H0, nullptr, 0, row0, B, si);
    norm_fwd<P>(lds, a.H0, Hc, TR, 1e-8f, a.CAT, 0, NO16, 0, NO32, nullptr, 0, mean, nullptr, row0, B);
    __syncthreads();
    layer_fwd<P, 1, TH>(lds, R, a.CAT, cr[2], &cr[4], a.act_critic, a.H1, 0, NO32, y1, Hc, row0, B, si);
    // (fp32: the thin weights' region lies in CAT, dead from here on)
    if constexpr (P == PREC_F32) thin_put<P>(lds, tw, a.TW, a.A, Hc);
    const GDesc b3 = bwd_of(cr[6], 0);
    layer_fwd<P, 1, TH>(lds, R, a.H1, cr[4], &b3, a.act_critic, a.H2, 0, NO32, y2, Hc, row0, B, si);
    // d(-Q.mean())/dQ (:272): the constant -1/(2B) on every live row
    for (int r = threadIdx.x; r < TR; r += NTH) *p32(lds, a.F, r, 0) = a.dq;
    __syncthreads();
    make_dp<P>(lds, a.F, 1, ACT_NONE, nullptr, 0, a.DP1, nullptr, row0, B);
    __syncthreads();
    const GDesc nx7 = bwd_of(cr[4], 0);
    layer_bwd<P, TH>(lds, R, a.DP1, cr[6], 0, Hc, &nx7, a.act_critic, y2, Hc, NO32, nullptr, 0, a.DP0, nullptr, row0,
                     B, si);
    const GDesc nx8 = bwd_of(cr[2], Hc);
    layer_bwd<P, TH>(lds, R, a.DP0, cr[4], 0, Hc, &nx8, a.act_critic, y1, Hc, NO32, nullptr, 0, a.DP1, nullptr, row0,
                     B, si);
    // the zsa columns of q1's input -> d zsa (this head)
    const GDesc nx9 = bwd_of(cr[2], 0);
    layer_bwd<P, TH>(lds, R, a.DP1, cr[2], Hc, Hc + Z, &nx9, ACT_NONE, nullptr, 0, NO32,
                     a.dzsa + (long)h * B * Z, Z, NO16, nullptr, row0, B, si);
    // the q columns -> AvgL1Norm backward -> q0's dP -> its action columns (thin)
    layer_bwd<P, TH>(lds, R, a.DP1, cr[2], 0, Hc, nullptr, ACT_NONE, nullptr, 0, a.DY, nullptr, 0, NO16, nullptr,
                     row0, B, si);
    FSTAMP(si);
    norm_bwd<P>(lds, a.DY, a.H0, mean, Hc, 1e-8f, dot, a.DP0, nullptr, 0, nullptr, row0, B);
    __syncthreads();
    FSTAMP(si);
    thin<P, THIN_NC>(lds, a.DP0, 0, Hc, a.TW, a.A, a.F, 1.f / Ty<P>::gs);
    __syncthreads();
    FSTAMP(si);
    for (int k = threadIdx.x; k < TR * a.A; k += NTH) {
        const int r = k / a.A, c = k - r * a.A;
        if (row0 + r < B) stg(a.da + ((long)h * B + row0 + r) * a.A + c, *p32(lds, a.F, r, c));
    }
}

template <int P, int TH>
__global__ __launch_bounds__(NTH) void actor_c_kernel(ActorArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int row0 = blockIdx.x * TR, B = a.B, Z = a.Z, Ha = a.Ha, He = a.He, A = a.A, tile = blockIdx.x;
    const long ld = a.ld;
    float *mean = (float *)(lds + a.small_off), *dot = mean + TR;
    int si = 0;
    FSTAMP(si);
    // d zsa = sum over the heads -> the fixed encoder's zsa3 dP (no activation)
    RowStage d0, d1, sh;
    ThinStage<THIN_NC> tw;
    row_issue(d0, a.dzsa, Z, Z, row0, B);
    row_issue(d1, a.dzsa + (long)B * Z, Z, Z, row0, B);
    row_issue(sh, a.h0, Ha, Ha, row0, B);
    const float m0 = ldg(a.mean0 + min(row0 + (int)(threadIdx.x % TR), B - 1));
    thin_issue(tw, a.fe[3].w, a.fe[3].ldw, Z, true, A, He);
    u32x4 R[PD][TH];
    ring_fill(R, bwd_of(a.fe[5], 0));
    zero_lds(lds, a.lds);
    __syncthreads();
    row_add(d0, d1);
    row_put16<P>(lds, d0, a.DP0, 0, Z, row0, B, Ty<P>::gs);
    if (threadIdx.x < TR) mean[threadIdx.x] = row0 + (int)threadIdx.x < B ? m0 : 0.f;
    row_put32(lds, sh, a.H0, Ha, row0, B);
    thin_put<P>(lds, tw, a.TW, A, He);
    __syncthreads();
    const GDesc nx10 = bwd_of(a.fe[4], 0);
    layer_bwd<P, TH>(lds, R, a.DP0, a.fe[5], 0, He, &nx10, a.act_enc, a.yz[1], He, NO32, nullptr, 0, a.DP1, nullptr,
                     row0, B, si);
    const GDesc nx11 = bwd_of(a.ac[3], 0);
    layer_bwd<P, TH>(lds, R, a.DP1, a.fe[4], 0, He, &nx11, a.act_enc, a.yz[0], He, NO32, nullptr, 0, a.DP0, nullptr,
                     row0, B, si);
    // the action columns of zsa1's input (thin), + both critic heads' d action, x tanh'
    FSTAMP(si);
    thin<P, THIN_NC>(lds, a.DP0, 0, He, a.TW, A, a.F, 1.f / Ty<P>::gs);
    __syncthreads();
    FSTAMP(si);
    for (int k = threadIdx.x; k < TR * A; k += NTH) {
        const int r = k / A, c = k - r * A, b = row0 + r;
        float v = 0.f;
        if (b < B) {
            const float y = ldg(a.act_out + (long)b * A + c);
            v = (*p32(lds, a.F, r, c) + ldg(a.da + (long)b * A + c) + ldg(a.da + ((long)B + b) * A + c)) * (1.f - y * y);
        }
        *p32(lds, a.F, r, c) = v;
    }
    __syncthreads();
    make_dp<P>(lds, a.F, A, ACT_NONE, nullptr, 0, a.DP1, a.xt[3].part + (long)tile * A, row0, B);
    __syncthreads();
    save_xt<P>(lds, a.DP1, 0, A, a.xt[3].dp, ld, TR, row0);
    const GDesc nx12 = bwd_of(a.ac[2], 0);
    layer_bwd<P, TH>(lds, R, a.DP1, a.ac[3], 0, Ha, &nx12, a.act_actor, a.ya[1], Ha, NO32, nullptr, 0, a.DP0,
                     a.xt[2].part + (long)tile * Ha, row0, B, si);
    save_xt<P>(lds, a.DP0, 0, Ha, a.xt[2].dp, ld, TR, row0);
    const GDesc nx13 = bwd_of(a.ac[1], 0);
    layer_bwd<P, TH>(lds, R, a.DP0, a.ac[2], 0, Ha, &nx13, a.act_actor, a.ya[0], Ha, NO32, nullptr, 0, a.DP1,
                     a.xt[1].part + (long)tile * Ha, row0, B, si);
    save_xt<P>(lds, a.DP1, 0, Ha, a.xt[1].dp, ld, TR, row0);
    layer_bwd<P, TH>(lds, R, a.DP1, a.ac[1], 0, Ha, nullptr, ACT_NONE, nullptr, 0, a.DY, nullptr, 0, NO16, nullptr,
                     row0, B, si);
    FSTAMP(si);
    norm_bwd<P>(lds, a.DY, a.H0, mean, Ha, 1e-8f, dot, a.DP0, a.xt[0].dp, ld, a.xt[0].part + (long)tile * Ha, row0,
                B);
    __syncthreads();
    FSTAMP(si);
}

// ---------------------------------------------------------------- weight gradients
// dW[n][k] = sum_r dP^T[n][r] X^T[k][r] / gs and db[n] = sum over row tiles of
// the fp32 partials, for up to TD7F_MAX_WG layers in one launch.  A workgroup
// (4 waves, 2 x 2 of 32 x 32) owns a 64 x 64 tile of one dW; A and B fragments
// are 16-byte loads of the transposed operands (rows r contiguous), PD2
// k-steps of 32 rows in flight.
struct WgJob {
    const char *dp, *x;  // operand-type fragment blocks (td7_fused.h blk8 / blk4)
    const float *part;
    float *dw, *db;
    int N, K, tiles_k, ntiles_rows;  // tiles_k = ceil(K / 64); row tiles of part
    int first;                        // first workgroup of this job
    // td7f_wgrad_adam: the layer's Adam step and repack (flat offsets of W[0][0]
    // and b[0] in optimiser opt's p / m / v; packed operands as td7f_pack)
    long w_off, b_off;
    u32x4 *wf, *wb;
    int ksf, ksb, opt;
};
struct WgOpt {
    float *p, *m, *v, *step;
    float lr, b1, b2, eps, wd;
};
struct WgArgs {
    int njobs, total;
    long ld;   // row stride of the transposed operands (padded batch)
    int rows;  // reduction length (multiple of 32)
    // LAP priorities of the critic update (:262) by the last workgroup:
    // prio[b] = max(|td_b0|, |td_b1|, min_priority)^alpha
    const float *td;
    float *prio;
    int B;
    float alpha, minp;
    WgJob j[TD7F_MAX_WG];
    WgOpt o[TD7_ADAM_MAX_OPT];
    int nopt;
    uint32_t *ticket;
};

constexpr int PD2 = 8;  // k-steps (32 rows) in flight; the reduction length is a multiple of 32 PD2

// ADAM: the optimiser step of every weight / bias the launch differentiates
// (adam_one, bit-identical to td7_adam_step_multi) and the repack of the
// updated weights (bit-identical to td7f_pack) in the epilogue: the tile's p /
// m / v are loaded before the k-loop (their latency hides under the MFMAs),
// the updated 16-bit weights are staged in LDS and written out as whole forward
// and dX items.  The optimiser step counts advance once (last workgroup out).
template <int P, bool ADAM>
__global__ __launch_bounds__(256) void wgrad_kernel(WgArgs a) {
    if ((int)blockIdx.x == a.total) {
        for (int b = threadIdx.x; b < a.B; b += 256)
            stg(a.prio + b, powf(fmaxf(fmaxf(ldg(a.td + 2 * b), ldg(a.td + 2 * b + 1)), a.minp), a.alpha));
    } else {
    int q = 0;
    while (q + 1 < a.njobs && (int)blockIdx.x >= a.j[q + 1].first) ++q;
    const WgJob &J = a.j[q];
    const int t = blockIdx.x - J.first;
    const int n0 = (t / J.tiles_k) * 64, k0 = (t % J.tiles_k) * 64;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wn = n0 + 32 * (w >> 1), wk = k0 + 32 * (w & 1);
    const long ld = a.ld;
    float ss = 0.f, bc = 1.f;
    float pp[2][2][4], mm[2][2][4], vv[2][2][4], bp = 0.f, bm = 0.f, bv = 0.f;
    if constexpr (ADAM) {
        const WgOpt &o = a.o[J.opt];
        const float st = *o.step + 1.0f;
        ss = o.lr / (1.0f - powf(o.b1, st));
        bc = sqrtf(1.0f - powf(o.b2, st));
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < 2; ++v)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int n = wn + 16 * u + 4 * (lane >> 4) + e, k = wk + 16 * v + (lane & 15);
                    const long i = J.w_off + ((n < J.N && k < J.K) ? (long)n * J.K + k : 0);
                    pp[u][v][e] = ldg(o.p + i), mm[u][v][e] = ldg(o.m + i), vv[u][v][e] = ldg(o.v + i);
                }
        if (k0 == 0 && J.db && w == 0) {
            const long i = J.b_off + (n0 + lane < J.N ? n0 + lane : 0);
            bp = ldg(o.p + i), bm = ldg(o.m + i), bv = ldg(o.v + i);
        }
    }
    // the operands are in fragment blocks (td7_fused.h blk8 / blk4): the
    // fragment of operand rows g*16.. and k-step s (KD batch rows) is the 1 KiB
    // block g * (ld / KD) + s; they are padded to multiples of 64 rows (zeros),
    // so every load is in range
    constexpr int KD = Ty<P>::KD;
    const char *ap[2], *bp2[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        ap[u] = J.dp + ((long)((wn + 16 * u) >> 4) * (ld / KD)) * 1024 + lane * 16;
        bp2[u] = J.x + ((long)((wk + 16 * u) >> 4) * (ld / KD)) * 1024 + lane * 16;
    }
    floatx4 acc[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) acc[u][v] = floatx4{0.f, 0.f, 0.f, 0.f};
    // rows is a multiple of 32 PD2 (the host pads the operands with zero columns):
    // PD2 k-steps of loads in flight, issue order pinned as in gemm
    const int ns = a.rows / KD;
    u32x4 fa[PD2][2], fb[PD2][2];
#pragma unroll
    for (int p = 0; p < PD2; ++p)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            fa[p][u] = ldg((const u32x4 *)(ap[u] + 1024 * p));
            fb[p][u] = ldg((const u32x4 *)(bp2[u] + 1024 * p));
            __builtin_amdgcn_sched_barrier(0);
        }
    int s0 = 0;
    for (; s0 + PD2 < ns; s0 += PD2) {
#pragma unroll
        for (int p = 0; p < PD2; ++p) {
            const int s = s0 + p;
#pragma unroll
            for (int j = 0; j < Ty<P>::SUB; ++j)
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int v = 0; v < 2; ++v) acc[u][v] = Ty<P>::mfma(fa[p][u], fb[p][v], acc[u][v], j);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                fa[p][u] = ldg((const u32x4 *)(ap[u] + 1024L * (s + PD2)));
                fb[p][u] = ldg((const u32x4 *)(bp2[u] + 1024L * (s + PD2)));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < PD2; ++p)
#pragma unroll
        for (int j = 0; j < Ty<P>::SUB; ++j)
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 2; ++v) acc[u][v] = Ty<P>::mfma(fa[p][u], fb[p][v], acc[u][v], j);
    // C[n][k]: lane holds n = 16u + 4(lane >> 4) + e, k = 16v + (lane & 15)
    // the tile's updated weights in the operand type (rows padded to 144 / 272 B)
    __shared__ alignas(16) typename Ty<P>::E T[ADAM ? 64 : 1][Ty<P>::EB == 4 ? 68 : 72];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int k = wk + 16 * v + (lane & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int n = wn + 16 * u + 4 * (lane >> 4) + e;
                const bool ok = n < J.N && k < J.K;
                const float g = acc[u][v][e] * (1.f / Ty<P>::gs);
                if (ok) stg(J.dw + (long)n * J.K + k, g);
                if constexpr (ADAM) {
                    const WgOpt &o = a.o[J.opt];
                    adam_one(pp[u][v][e], g, mm[u][v][e], vv[u][v][e], ss, bc, o.b1, o.b2, o.eps, o.wd, 1.0f);
                    if (ok) {
                        const long i = J.w_off + (long)n * J.K + k;
                        stg(o.p + i, pp[u][v][e]), stg(o.m + i, mm[u][v][e]), stg(o.v + i, vv[u][v][e]);
                    }
                    T[n - n0][k - k0] = Ty<P>::bits(ok ? pp[u][v][e] : 0.f);
                }
            }
        }
    if (k0 == 0 && J.db) {
        // db[n] = sum of the row-tile partials: the 4 waves take every 4th
        // tile (independent loads in flight), then one LDS reduction
        __shared__ float red[4][64];
        const int n = n0 + lane;
        float sacc = 0.f;
        if (n < J.N) {
#pragma unroll 8
            for (int r = w; r < J.ntiles_rows; r += 4) sacc += ldg(J.part + (long)r * J.N + n);
        }
        red[w][lane] = sacc;
        __syncthreads();
        if (w == 0 && n < J.N) {
            const float g = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
            stg(J.db + n, g);
            if constexpr (ADAM) {
                const WgOpt &o = a.o[J.opt];
                adam_one(bp, g, bm, bv, ss, bc, o.b1, o.b2, o.eps, o.wd, 1.0f);
                stg(o.p + J.b_off + n, bp), stg(o.m + J.b_off + n, bm), stg(o.v + J.b_off + n, bv);
            }
        }
    }
    if constexpr (ADAM && P == PREC_F32) {
        __syncthreads();
        // 64 rows x 16 forward items (4 inputs of one output row) and 64 columns
        // x 16 dX items (4 output rows of one input column): four of each per thread
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int i = threadIdx.x + 256 * h;
            const int r = i >> 4, c = 4 * (i & 15);
            const int n = n0 + r, k = k0 + c;
            if (n < J.N && k < J.K)
                stg(J.wf + ((long)(n >> 4) * J.ksf + (k >> 4)) * 64 + (n & 15) + 16 * ((k & 15) >> 2),
                    *(const u32x4 *)&T[r][c]);
        }
        if (J.wb) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int i = threadIdx.x + 256 * h;
                const int c = i & 63, r4 = 4 * (i >> 6);
                const int n = n0 + r4, k = k0 + c;
                if (n < J.N && k < J.K)
                    stg(J.wb + ((long)(k >> 4) * J.ksb + (n >> 4)) * 64 + (k & 15) + 16 * ((n & 15) >> 2),
                        __builtin_bit_cast(u32x4, floatx4{T[r4][c], T[r4 + 1][c], T[r4 + 2][c], T[r4 + 3][c]}));
            }
        }
    } else if constexpr (ADAM) {
        __syncthreads();
        // 64 rows x 8 forward items (8 inputs of one output row) and 64 columns
        // x 8 dX items (8 output rows of one input column): two of each per thread
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = threadIdx.x + 256 * h;
            const int r = i >> 3, c = 8 * (i & 7);
            const int n = n0 + r, k = k0 + c;
            if (n < J.N && k < J.K)
                stg(J.wf + ((long)(n >> 4) * J.ksf + (k >> 5)) * 64 + (n & 15) + 16 * ((k & 31) >> 3),
                    *(const u32x4 *)&T[r][c]);
        }
        if (J.wb) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = threadIdx.x + 256 * h;
                const int c = i & 63, r8 = 8 * (i >> 6);
                const int n = n0 + r8, k = k0 + c;
                if (n < J.N && k < J.K) {
                    uint32_t d[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) d[jj] = (uint32_t)T[r8 + 2 * jj][c] | ((uint32_t)T[r8 + 2 * jj + 1][c] << 16);
                    stg(J.wb + ((long)(k >> 4) * J.ksb + (n >> 5)) * 64 + (k & 15) + 16 * ((n & 31) >> 3),
                        u32x4{d[0], d[1], d[2], d[3]});
                }
            }
        }
    }
    }
    if constexpr (ADAM) {
        // the last workgroup out advances the optimisers' step counts (every
        // workgroup read them before its ticket)
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t done = atomicAdd(a.ticket, 1u);
            if (done == gridDim.x - 1) {
                for (int k = 0; k < a.nopt; ++k) *a.o[k].step = *a.o[k].step + 1.0f;
                *a.ticket = 0u;
            }
        }
    }
}

}  // namespace td7f

using namespace td7f;

static XT xt_of(const td7f_xt &x) { return XT{x.x, x.dp, x.part}; }

static bool prec_ok(int p) { return p == PREC_BF16 || p == PREC_F16 || p == PREC_F32; }
static bool xt_ok(const td7f_xt *xt, int n) {
    for (int i = 0; i < n; ++i)
        if (!xt[i].x || !xt[i].dp || !xt[i].part) return false;
    return true;
}
// fp32 layouts: two 16-row dP images of row stride ld inside the image region r
static bool alias_pair(R16 r, int ld, R16 &d0, R16 &d1) {
    d0 = R16{r.off, ld};
    d1 = R16{r.off + round_up(TR * ld * 2, 16), ld};
    return d1.off + TR * ld * 2 <= r.off + TR * r.ld * 2;
}
// a 16-row fp32 region of n columns over the adjacent images a | b
static bool alias32(R16 a, R16 b, int n, R32 &d) {
    d = R32{a.off, n};
    return a.off + TR * n * 4 <= b.off + TR * b.ld * 2;
}
static bool wb_ok(const td7f_lin *l, int n) {
    for (int i = 0; i < n; ++i)
        if (!l[i].wb || l[i].ksb <= 0 || l[i].ksb % PD) return false;
    return true;
}

extern "C" {

#ifdef EXO_STAMPS
int td7f_train_debug_set_stamps(unsigned long long *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_td7f_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -5;
}
#endif

int td7f_critic(int32_t prec, const int32_t *act, const td7f_lin *critic, const float *s, const float *a,
                const float *zs, const float *zsa, const float *qt, const float *reward, const float *not_done,
                float discount, const float *lo, const float *hi, float *run_max, float *run_min, int32_t B,
                int32_t S, int32_t A, float *td, float *q, float *y1, float *y2, const td7f_xt *xt, int64_t ld,
                void *stream) {
    return td7f_critic_phase(0, prec, act, critic, s, a, zs, zsa, qt, reward, not_done, discount, lo, hi, run_max,
                             run_min, B, S, A, td, q, y1, y2, xt, ld, nullptr, nullptr, nullptr, stream);
}

int td7f_critic_phase(int32_t phase, int32_t prec, const int32_t *act, const td7f_lin *critic, const float *s,
                      const float *a, const float *zs, const float *zsa, const float *qt, const float *reward,
                      const float *not_done, float discount, const float *lo, const float *hi, float *run_max,
                      float *run_min, int32_t B, int32_t S, int32_t A, float *td, float *q, float *y1, float *y2,
                      const td7f_xt *xt, int64_t ld, float *q_ws, float *h0_ws, float *mean_ws, void *stream) {
    if (!prec_ok(prec) || !act || !critic || !s || !a || !zs || !zsa || !qt || !reward || !not_done || !lo || !hi ||
        !run_max || !run_min || !td || !y1 || !y2 || !xt || B <= 0 || S <= 0 || S > NTH || A <= 0 || A > THIN_NC || ld < B || ld % 32)
        return EXO_EINVAL;
    if (phase < 0 || phase > 2 || (phase != 0 && (!q_ws || !h0_ws || !mean_ws))) return EXO_EINVAL;
    const int th = th_of(critic, 8);
    if ((th != 4 && th != 5) || !wb_ok(critic, 8) || !xt_ok(xt, 8)) return EXO_EINVAL;
    CriticArgs g{};
    for (int i = 0; i < 8; ++i) {
        g.cr[i] = lin_of(critic[i]);
        g.xt[i] = xt_of(xt[i]);
    }
    g.act = act[2];
    g.s = s; g.a = a; g.zs = zs; g.zsa = zsa; g.qt = qt; g.reward = reward; g.not_done = not_done;
    g.discount = discount;
    g.inv_b = 1.0f / (float)B;
    g.lo = lo; g.hi = hi; g.run_max = run_max; g.run_min = run_min;
    g.B = B; g.S = S; g.A = A;
    g.Hc = critic[0].n_out;
    g.Z = (critic[2].n_in - g.Hc) / 2;
    if (critic[0].n_in != S + A || critic[4].n_in != g.Hc || critic[6].n_in != g.Hc || critic[6].n_out != 1 ||
        g.Z * 2 + g.Hc != critic[2].n_in || g.Hc % 16 || g.Hc > 320)
        return EXO_EINVAL;
    g.td = td; g.q = q; g.y1 = y1; g.y2 = y2; g.ld = ld;
    g.phase = phase;
    g.qs = q_ws; g.h0s = h0_ws; g.ms = mean_ws;
    const int kd = kd_of(prec);
    Bump b(1);
    g.X = b.r16(TR, ld16(S + A, kd));
    g.CAT = b.r16(TR, ld16(g.Hc + 2 * g.Z, kd));
    g.H1 = b.r16(TR, ld16(g.Hc, kd));
    g.H2 = b.r16(TR, ld16(g.Hc, kd));
    if (prec == PREC_F32) {
        // fp32 images: the backward's dP images overlay CAT and its fp32 dY
        // overlays H1 | H2 -- all four are dead once the forward has read them
        // (act' comes from the fp32 activations in HBM); leftover values in
        // the padding columns are finite and meet zero weights
        if (!alias_pair(g.CAT, ld16(g.Hc, kd), g.DP0, g.DP1) || !alias32(g.H1, g.H2, g.Hc, g.DY)) return EXO_EINVAL;
    } else {
        g.DP0 = b.r16(TR, ld16(g.Hc));
        g.DP1 = b.r16(TR, ld16(g.Hc));
    }
    g.H0 = b.r32(TR, g.Hc);
    if (prec != PREC_F32) g.DY = b.r32(TR, g.Hc);
    g.F = b.r32(TR, 16);
    g.TW = b.r32(1, g.Hc);
    const R32 sm = b.r32(1, 2 * TR);
    g.small_off = sm.off;
    g.lds_bytes = b.off;
    return DISPATCH(prec, th, critic_kernel, dim3((B + TR - 1) / TR, 2), b.off, g, (hipStream_t)stream);
}

int td7f_encoder(int32_t prec, const int32_t *act, const td7f_lin *enc, const float *s, const float *a,
                 const float *ns, int32_t B, float *const *y, const td7f_xt *xt, int64_t ld, float *nz_ws,
                 int32_t *flag_ws, void *stream) {
    if (!prec_ok(prec) || !act || !enc || !s || !a || !ns || !y || !xt || B <= 0 || ld < B || ld % 32 ||
        (!nz_ws) != (!flag_ws))
        return EXO_EINVAL;
    const int th = th_of(enc, 6);
    if ((th != 4 && th != 5) || !wb_ok(enc, 6) || !xt_ok(xt, 6)) return EXO_EINVAL;
    EncoderArgs g{};
    for (int i = 0; i < 6; ++i) {
        g.e[i] = lin_of(enc[i]);
        g.xt[i] = xt_of(xt[i]);
    }
    if (!y[0] || !y[1] || !y[2] || !y[3]) return EXO_EINVAL;
    g.y0 = y[0];
    g.y1 = y[1];
    g.y2 = y[2];
    g.y3 = y[3];
    g.act = act[0];
    g.s = s; g.a = a; g.ns = ns;
    g.B = B;
    g.S = enc[0].n_in;
    g.He = enc[0].n_out;
    g.Z = enc[2].n_out;
    g.A = enc[3].n_in - g.Z;
    if (g.A <= 0 || g.A > THIN_NC || g.S > NTH || enc[1].n_out != g.He || enc[4].n_out != g.He || enc[5].n_out != g.Z || g.Z % 4)
        return EXO_EINVAL;
    g.mse_scale = 2.0f / ((float)B * (float)g.Z);
    g.ld = ld;
    const int w = std::max(g.Z, g.He), kd = kd_of(prec);
    Bump b(1);
    g.X = b.r16(TR, ld16(g.S, kd));
    g.H1 = b.r16(TR, ld16(g.He, kd));
    g.H2 = b.r16(TR, ld16(g.He, kd));
    g.CATZ = b.r16(TR, ld16(g.Z + g.A, kd));
    if (prec == PREC_F32 && ld16(w, kd) <= g.H1.ld) {
        // fp32: the backward's dP images overlay H1 / H2 (dead once zsa3's
        // forward has read H2; act' comes from the activations in HBM)
        g.DP0 = R16{g.H1.off, ld16(w, kd)};
        g.DP1 = R16{g.H2.off, ld16(w, kd)};
    } else {
        g.DP0 = b.r16(TR, ld16(w, kd));
        g.DP1 = b.r16(TR, ld16(w, kd));
    }
    g.H3 = b.r32(TR, g.Z);
    g.NZ = b.r32(TR, w);
    g.DY = b.r32(TR, w);
    const R32 sm = b.r32(1, 2 * TR);
    g.small_off = sm.off;
    g.lds_bytes = b.off;
    g.nz = nz_ws;
    g.flag = flag_ws;
    return DISPATCH(prec, th, encoder_kernel, dim3((B + TR - 1) / TR, nz_ws ? 2 : 1), b.off, g, (hipStream_t)stream);
}

int td7f_actor(int32_t prec, int32_t phase, const int32_t *act, const td7f_lin *actor, const td7f_lin *fenc,
               const td7f_lin *critic, const float *s, const float *zs, int32_t B, const td7f_actor_bufs *bufs,
               const td7f_xt *xt, int64_t ld, void *stream) {
    if (!prec_ok(prec) || phase < 0 || phase > 2 || !act || !actor || !fenc || !critic || !s || !zs || !bufs || !xt ||
        B <= 0 || ld < B || ld % 32)
        return EXO_EINVAL;
    td7f_lin all[18];
    for (int i = 0; i < 4; ++i) all[i] = actor[i];
    for (int i = 0; i < 6; ++i) all[4 + i] = fenc[i];
    for (int i = 0; i < 8; ++i) all[10 + i] = critic[i];
    const int th = th_of(all, 18);
    if ((th != 4 && th != 5) || !xt_ok(xt, 4)) return EXO_EINVAL;
    if (phase == 1 && !wb_ok(critic, 8)) return EXO_EINVAL;
    if (phase == 2 && (!wb_ok(actor, 4) || !wb_ok(fenc + 3, 3))) return EXO_EINVAL;
    const td7f_actor_bufs &u = *bufs;
    if (!u.act_out || !u.zsa_out || !u.h0 || !u.mean0 || !u.ya[0] || !u.ya[1] || !u.yz[0] || !u.yz[1] ||
        !u.yc[0] || !u.yc[1] || !u.da || !u.dzsa)
        return EXO_EINVAL;
    ActorArgs g{};
    for (int i = 0; i < 4; ++i) {
        g.ac[i] = lin_of(actor[i]);
        g.xt[i] = xt_of(xt[i]);
    }
    for (int i = 0; i < 6; ++i) g.fe[i] = lin_of(fenc[i]);
    for (int i = 0; i < 8; ++i) g.cr[i] = lin_of(critic[i]);
    g.act_enc = act[0]; g.act_actor = act[1]; g.act_critic = act[2];
    g.s = s; g.zs = zs; g.B = B;
    g.S = actor[0].n_in;
    g.A = actor[3].n_out;
    g.Ha = actor[0].n_out;
    g.Z = fenc[2].n_out;
    g.He = fenc[3].n_out;
    g.Hc = critic[0].n_out;
    if (actor[1].n_in != g.Ha + g.Z || fenc[3].n_in != g.Z + g.A || critic[0].n_in != g.S + g.A ||
        critic[2].n_in != g.Hc + 2 * g.Z || g.A > THIN_NC || g.S > NTH || g.Hc % 16 || g.Ha % 16)
        return EXO_EINVAL;
    g.dq = -1.0f / (2.0f * (float)B);
    g.act_out = u.act_out; g.zsa_out = u.zsa_out; g.h0 = u.h0; g.mean0 = u.mean0;
    for (int i = 0; i < 2; ++i) {
        g.ya[i] = u.ya[i];
        g.yz[i] = u.yz[i];
        g.yc[i] = u.yc[i];
    }
    g.da = u.da; g.dzsa = u.dzsa; g.ld = ld;
    const int hmax = std::max(g.Ha, std::max(g.He, g.Hc)), kd = kd_of(prec);
    Bump b(1);
    if (phase == 0) {
        g.X = b.r16(TR, ld16(g.S, kd));
        g.CATA = b.r16(TR, ld16(g.Ha + g.Z, kd));
        g.CATZ = b.r16(TR, ld16(g.Z + g.A, kd));
        g.H1 = b.r16(TR, ld16(hmax, kd));
        g.H2 = b.r16(TR, ld16(hmax, kd));
        g.H0 = b.r32(TR, g.Ha);
        g.F = b.r32(TR, 16);
        g.TW = b.r32(THIN_NC, g.Ha);
    } else if (phase == 1) {
        g.X = b.r16(TR, ld16(g.S + g.A, kd));
        g.CAT = b.r16(TR, ld16(g.Hc + 2 * g.Z, kd));
        g.H1 = b.r16(TR, ld16(g.Hc, kd));
        g.H2 = b.r16(TR, ld16(g.Hc, kd));
        if (prec == PREC_F32) {
            // fp32 (as td7f_critic): dP images and the thin weights (staged
            // after q1's forward) in CAT, dY over H1 | H2
            if (!alias_pair(g.CAT, ld16(g.Hc, kd), g.DP0, g.DP1) || !alias32(g.H1, g.H2, g.Hc, g.DY)) return EXO_EINVAL;
            const int tw = g.DP1.off + round_up(TR * g.DP1.ld * 2, 16);
            g.TW = R32{tw, g.Hc};
            if (tw + THIN_NC * g.Hc * 4 > g.CAT.off + TR * g.CAT.ld * 2) return EXO_EINVAL;
        } else {
            g.DP0 = b.r16(TR, ld16(g.Hc));
            g.DP1 = b.r16(TR, ld16(g.Hc));
        }
        g.H0 = b.r32(TR, g.Hc);
        if (prec != PREC_F32) g.DY = b.r32(TR, g.Hc);
        g.F = b.r32(TR, 16);
        if (prec != PREC_F32) g.TW = b.r32(THIN_NC, g.Hc);
    } else {
        g.DP0 = b.r16(TR, ld16(std::max(hmax, g.Z), kd));
        g.DP1 = b.r16(TR, ld16(std::max(hmax, g.Z), kd));
        g.H0 = b.r32(TR, g.Ha);
        g.DY = b.r32(TR, g.Ha);
        g.F = b.r32(TR, 16);
        g.TW = b.r32(THIN_NC, g.He);
    }
    const R32 sm = b.r32(1, 2 * TR);
    g.small_off = sm.off;
    g.lds = b.off;
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid((B + TR - 1) / TR, phase == 1 ? 2 : 1);
    if (phase == 0) return DISPATCH(prec, th, actor_a_kernel, grid, b.off, g, st);
    if (phase == 1) return DISPATCH(prec, th, actor_b_kernel, grid, b.off, g, st);
    return DISPATCH(prec, th, actor_c_kernel, grid, b.off, g, st);
}

static int wgrad_args(int32_t prec, int32_t njobs, const td7f_wg_job *jobs, int64_t ld, int32_t rows,
                      const float *td, float *prio, int32_t B, float alpha, float min_priority, WgArgs &g) {
    if (!prec_ok(prec) || njobs <= 0 || njobs > TD7F_MAX_WG || !jobs || rows <= 0 || rows % (32 * PD2) ||
        ld < rows || ld % 32 || (prio && (!td || B <= 0)))
        return EXO_EINVAL;
    g.njobs = njobs;
    g.ld = ld;
    g.rows = rows;
    int total = 0;
    for (int q = 0; q < njobs; ++q) {
        const td7f_wg_job &J = jobs[q];
        if (!J.dp || !J.x || !J.dw || J.n <= 0 || J.k <= 0 || (J.db && (!J.part || J.row_tiles <= 0))) return EXO_EINVAL;
        WgJob &w = g.j[q];
        w.dp = (const char *)J.dp;
        w.x = (const char *)J.x;
        w.part = J.part;
        w.dw = J.dw;
        w.db = J.db;
        w.N = J.n;
        w.K = J.k;
        w.tiles_k = (J.k + 63) / 64;
        w.ntiles_rows = J.row_tiles;
        w.first = total;
        total += ((J.n + 63) / 64) * w.tiles_k;
    }
    g.total = total;
    g.td = td;
    g.prio = prio;
    g.B = B;
    g.alpha = alpha;
    g.minp = min_priority;
    return EXO_OK;
}

int td7f_wgrad(int32_t prec, int32_t njobs, const td7f_wg_job *jobs, int64_t ld, int32_t rows, const float *td,
               float *prio, int32_t B, float alpha, float min_priority, void *stream) {
    WgArgs g{};
    const int rc = wgrad_args(prec, njobs, jobs, ld, rows, td, prio, B, alpha, min_priority, g);
    if (rc != EXO_OK) return rc;
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid(g.total + (prio ? 1 : 0));
    if (prec == PREC_BF16) hipLaunchKernelGGL((wgrad_kernel<PREC_BF16, false>), grid, dim3(256), 0, st, g);
    else if (prec == PREC_F16) hipLaunchKernelGGL((wgrad_kernel<PREC_F16, false>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((wgrad_kernel<PREC_F32, false>), grid, dim3(256), 0, st, g);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7f_wgrad_adam(int32_t prec, int32_t njobs, const td7f_wg_job *jobs, int64_t ld, int32_t rows, const float *td,
                    float *prio, int32_t B, float alpha, float min_priority, int32_t nopt, float *const *p,
                    float *const *m, float *const *v, float *const *step, const float *lr, const float *beta1,
                    const float *beta2, const float *eps, const float *weight_decay, const td7f_wg_adam *adam,
                    uint32_t *ticket, void *stream) {
    WgArgs g{};
    const int rc = wgrad_args(prec, njobs, jobs, ld, rows, td, prio, B, alpha, min_priority, g);
    if (rc != EXO_OK) return rc;
    if (nopt <= 0 || nopt > TD7_ADAM_MAX_OPT || !adam || !ticket) return EXO_EINVAL;
    g.nopt = nopt;
    g.ticket = ticket;
    for (int k = 0; k < nopt; ++k) {
        if (!p[k] || !m[k] || !v[k] || !step[k]) return EXO_EINVAL;
        g.o[k] = WgOpt{p[k], m[k], v[k], step[k], lr[k], beta1[k], beta2[k], eps[k], weight_decay[k]};
    }
    for (int q = 0; q < njobs; ++q) {
        const td7f_wg_adam &A = adam[q];
        const td7f_wg_job &J = jobs[q];
        // every layer: weight, bias (its gradient db required) and forward operand
        if (A.opt < 0 || A.opt >= nopt || A.w_off < 0 || A.b_off < 0 || !J.db || !A.wf ||
            A.ksf * kd_of(prec) < J.k || (A.wb && A.ksb * kd_of(prec) < J.n))
            return EXO_EINVAL;
        WgJob &w = g.j[q];
        w.w_off = A.w_off;
        w.b_off = A.b_off;
        w.wf = (u32x4 *)A.wf;
        w.wb = (u32x4 *)A.wb;
        w.ksf = A.ksf;
        w.ksb = A.wb ? A.ksb : 0;
        w.opt = A.opt;
    }
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid(g.total + (prio ? 1 : 0));
    if (prec == PREC_BF16) hipLaunchKernelGGL((wgrad_kernel<PREC_BF16, true>), grid, dim3(256), 0, st, g);
    else if (prec == PREC_F16) hipLaunchKernelGGL((wgrad_kernel<PREC_F16, true>), grid, dim3(256), 0, st, g);
    else hipLaunchKernelGGL((wgrad_kernel<PREC_F32, true>), grid, dim3(256), 0, st, g);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

}  // extern "C"
