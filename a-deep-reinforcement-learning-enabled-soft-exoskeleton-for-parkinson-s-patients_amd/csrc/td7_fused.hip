// td7_fused.hip -- row-tile-fused TD7 networks (see td7_fused.h): weight
// packing and the forward passes of the TD7 update and of select_action.
//
//   td7f_select : Agent.select_action over the vectorised envs (Agent/TD7_multi_agent.py:192-209,
//                 batched; the fixed encoder's zs, the actor, Gaussian exploration noise)
//   td7f_target : the critic target chain (:233-241) -- kernel A: fixed_target_zs(s'),
//                 actor_target + clipped noise, fixed_target_zsa; kernel B: both heads of
//                 critic_target, one workgroup per (16 rows, head)
//   td7f_fixed  : fixed_zs / fixed_zsa of the critic update (:248-249)
//
// Every Linear is the gemm of td7_fused.h (16-bit operands from LDS x packed
// weights streamed from L2, fp32 accumulate) with its bias/activation/norm
// fused; one launch per network pass instead of one (or more) per layer.
#include "td7_fused.h"

#include <algorithm>
#include <cstdlib>

#include "adam_math.h"
#include "philox.h"

namespace td7f {

// ---------------------------------------------------------------- packing
struct PackJob {
    const float *w;
    long ld;
    int N, K;
    u32x4 *wf, *wb;
    int ksf, ntf, ksb, ntb;
};
struct PackArgs {
    int njobs;
    long start[TD7F_MAX_PACK + 1];  // prefix sums of the jobs' 16-byte items
    PackJob j[TD7F_MAX_PACK];
};

// One job per grid row (blockIdx.y: the job's descriptor is uniform -- scalar
// loads, no search), one 16-byte item per thread.  A forward item is 8
// consecutive inputs of one output row: two 16-byte loads when they lie inside
// the matrix and the rows are 16-byte aligned; every other load is issued
// unconditionally from a clamped address and masked after (no branch splits
// the batch of loads).
template <int P>
__device__ __forceinline__ float w_at(const PackJob &J, int n, int c) {
    const bool ok = n < J.N && c < J.K;
    const float x = ldg(J.w + (long)(ok ? n : 0) * J.ld + (ok ? c : 0));
    return ok ? x : 0.f;
}
// fp32 (Ty<PREC_F32>: 16-deep k-steps): a forward item is 4 consecutive inputs
// W[16t + (l&15)][16s + 4(l>>4) + j], a dX item W[16s + 4(l>>4) + j][16t + (l&15)], j < 4
__device__ __forceinline__ void pack_item_f32(const PackJob &J, long k, long nf, bool vec) {
    const int l = (int)(k & 63);
    float x[4];
    u32x4 *dst;
    if (k < nf) {
        const long blk = k >> 6;
        const int t = (int)(blk / J.ksf), s = (int)(blk % J.ksf);
        const int n = 16 * t + (l & 15), k0 = 16 * s + 4 * (l >> 4);
        if (vec && n < J.N && k0 + 4 <= J.K) {
            const floatx4 a0 = ldg((const floatx4 *)(J.w + (long)n * J.ld + k0));
            x[0] = a0[0], x[1] = a0[1], x[2] = a0[2], x[3] = a0[3];
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = w_at<PREC_F32>(J, n, k0 + j);
        }
        dst = J.wf + k;
    } else {
        const long blk = (k - nf) >> 6;
        const int t = (int)(blk / J.ksb), s = (int)(blk % J.ksb);
        const int c = 16 * t + (l & 15), n0 = 16 * s + 4 * (l >> 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = w_at<PREC_F32>(J, n0 + j, c);
        dst = J.wb + (k - nf);
    }
    stg(dst, __builtin_bit_cast(u32x4, floatx4{x[0], x[1], x[2], x[3]}));
}

template <int P>
__global__ __launch_bounds__(256) void pack_kernel(PackArgs a) {
    const PackJob J = a.j[blockIdx.y];
    if constexpr (P == PREC_F32) {
        const long nf = (long)J.ntf * J.ksf * 64, total = nf + (long)J.ntb * J.ksb * 64;
        const bool vec = (J.ld % 4) == 0 && (reinterpret_cast<uintptr_t>(J.w) & 15) == 0;
        for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < total; k += (long)gridDim.x * 256)
            pack_item_f32(J, k, nf, vec);
        return;
    }
    const long nf = (long)J.ntf * J.ksf * 64, total = nf + (long)J.ntb * J.ksb * 64;
    const bool vec = (J.ld % 4) == 0 && (reinterpret_cast<uintptr_t>(J.w) & 15) == 0;
    for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < total; k += (long)gridDim.x * 256) {
        const int l = (int)(k & 63);
        float x[8];
        u32x4 *dst;
        if (k < nf) {  // forward: W[16t + (l&15)][32s + 8(l>>4) + j]
            const long blk = k >> 6;
            const int t = (int)(blk / J.ksf), s = (int)(blk % J.ksf);
            const int n = 16 * t + (l & 15), k0 = 32 * s + 8 * (l >> 4);
            if (vec && n < J.N && k0 + 8 <= J.K) {
                const floatx4 a0 = ldg((const floatx4 *)(J.w + (long)n * J.ld + k0));
                const floatx4 a1 = ldg((const floatx4 *)(J.w + (long)n * J.ld + k0 + 4));
                x[0] = a0[0], x[1] = a0[1], x[2] = a0[2], x[3] = a0[3];
                x[4] = a1[0], x[5] = a1[1], x[6] = a1[2], x[7] = a1[3];
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = w_at<P>(J, n, k0 + j);
            }
            dst = J.wf + k;
        } else {  // dX: W[32s + 8(l>>4) + j][16t + (l&15)]
            const long blk = (k - nf) >> 6;
            const int t = (int)(blk / J.ksb), s = (int)(blk % J.ksb);
            const int c = 16 * t + (l & 15), n0 = 32 * s + 8 * (l >> 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = w_at<P>(J, n0 + j, c);
            dst = J.wb + (k - nf);
        }
        uint32_t v[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
            v[jj] = (uint32_t)Ty<P>::bits(x[2 * jj]) | ((uint32_t)Ty<P>::bits(x[2 * jj + 1]) << 16);
        stg(dst, u32x4{v[0], v[1], v[2], v[3]});
    }
}

// ---------------------------------------------------------------- Adam + packing
// td7_adam_step_multi (td7_ops.hip) and pack_kernel of the weights it changes
// in one launch: the thread that updates a weight also writes its packed
// copies, so the optimiser step and the repack are one node of the update's
// dependency chain instead of two.  A packed weight [N][K] is cut into 8 x 8
// tiles; the 8 lanes of a tile update one row's 8 columns each (a forward item
// is exactly those 8 columns of one row), then swap the 16-bit values through
// LDS so lane r writes the dX item of column c0 + r (8 consecutive rows).
// Workgroups [0, jb[njobs]) own the jobs' tiles, the rest stride over the
// unpacked segments (biases) in 4-element groups as adam_multi_kernel does.
struct APOpt {
    float *p, *m, *v, *step;
    float lr, b1, b2, eps, wd;
};
struct APSeg {  // an unpacked segment
    const float *g;
    long off;
    int n, opt;
};
struct APJob {  // pointers at W[0][0]: p / m / v in the optimiser's buffers, g in the gradient
    float *p, *m, *v;
    const float *g;
    u32x4 *wf, *wb;
    int opt, N, K, nch, ksf, ksb, vec;
};
struct AdamPackArgs {
    APOpt o[TD7_ADAM_MAX_OPT];
    APSeg s[TD7_ADAM_MAX_SEG];
    int q0[TD7_ADAM_MAX_SEG + 1];
    APJob j[TD7F_MAX_ADAM_PACK];
    int jb[TD7F_MAX_ADAM_PACK + 1];
    int nopt, nseg, njobs;
    uint32_t *ticket;
};

template <int P>
__global__ __launch_bounds__(256) void adam_pack_kernel(AdamPackArgs a) {
    __shared__ float coef[TD7_ADAM_MAX_OPT][2];
    __shared__ u32x4 tt[32][8];  // 32 tiles x 8 rows of 8 16-bit values
    if ((int)threadIdx.x < a.nopt) {
        const APOpt o = a.o[threadIdx.x];
        const float t = *o.step + 1.0f;
        coef[threadIdx.x][0] = o.lr / (1.0f - powf(o.b1, t));
        coef[threadIdx.x][1] = sqrtf(1.0f - powf(o.b2, t));
    }
    __syncthreads();
    const int b = blockIdx.x;
    if (b < a.jb[a.njobs]) {
        int q = 0;
        while (q + 1 < a.njobs && b >= a.jb[q + 1]) ++q;
        const APJob &J = a.j[q];
        const APOpt &o = a.o[J.opt];
        const float ss = coef[J.opt][0], bc = coef[J.opt][1];
        const int i = (b - a.jb[q]) * 256 + threadIdx.x;
        const int tile = i >> 3, r = i & 7;
        const int G = tile / J.nch, c0 = 8 * (tile - G * J.nch);
        const int n0 = 8 * G, n = n0 + r;
        const bool rv = n < J.N;  // false for the whole tile past the last row group
        float x[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) x[jj] = 0.f;
        if (rv) {
            const long e = (long)n * J.K + c0;
            const int ne = min(8, J.K - c0);
            float pp[8], mm[8], vv[8], gg[8];
            if (J.vec) {  // K % 4 == 0, 16-byte aligned rows: ne is 4 or 8
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const long eh = e + (h < ne / 4 ? 4 * h : 0);
                    const floatx4 p4 = ldg((const floatx4 *)(J.p + eh)), m4 = ldg((const floatx4 *)(J.m + eh));
                    const floatx4 v4 = ldg((const floatx4 *)(J.v + eh)), g4 = ldg((const floatx4 *)(J.g + eh));
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        pp[4 * h + u] = p4[u], mm[4 * h + u] = m4[u], vv[4 * h + u] = v4[u], gg[4 * h + u] = g4[u];
                }
            } else {
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    const long ej = e + (jj < ne ? jj : 0);
                    pp[jj] = ldg(J.p + ej), mm[jj] = ldg(J.m + ej), vv[jj] = ldg(J.v + ej), gg[jj] = ldg(J.g + ej);
                }
            }
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) adam_one(pp[jj], gg[jj], mm[jj], vv[jj], ss, bc, o.b1, o.b2, o.eps, o.wd, 1.0f);
            if (J.vec) {
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    if (h < ne / 4) {
                        stg((floatx4 *)(J.p + e + 4 * h), floatx4{pp[4 * h], pp[4 * h + 1], pp[4 * h + 2], pp[4 * h + 3]});
                        stg((floatx4 *)(J.m + e + 4 * h), floatx4{mm[4 * h], mm[4 * h + 1], mm[4 * h + 2], mm[4 * h + 3]});
                        stg((floatx4 *)(J.v + e + 4 * h), floatx4{vv[4 * h], vv[4 * h + 1], vv[4 * h + 2], vv[4 * h + 3]});
                    }
            } else {
#pragma unroll
                for (int jj = 0; jj < 8; ++jj)
                    if (jj < ne) stg(J.p + e + jj, pp[jj]), stg(J.m + e + jj, mm[jj]), stg(J.v + e + jj, vv[jj]);
            }
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) x[jj] = jj < ne ? pp[jj] : 0.f;
        }
        if constexpr (P == PREC_F32) {
            // two forward items (columns c0.. and c0 + 4..) and, after the
            // exchange, two dX items (rows n0.. and n0 + 4..) per lane
            __shared__ float tf[32][8][8];
            if (rv)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int c = c0 + 4 * h;
                    stg(J.wf + ((long)(n >> 4) * J.ksf + (c >> 4)) * 64 + (n & 15) + 16 * ((c & 15) >> 2),
                        __builtin_bit_cast(u32x4, floatx4{x[4 * h], x[4 * h + 1], x[4 * h + 2], x[4 * h + 3]}));
                }
            const int slot = threadIdx.x >> 3;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) tf[slot][r][jj] = x[jj];
            __syncthreads();
            const int c = c0 + r;
            if (J.wb && n0 < J.N && c < J.K)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int nn = n0 + 4 * h;
                    stg(J.wb + ((long)(c >> 4) * J.ksb + (nn >> 4)) * 64 + (c & 15) + 16 * ((nn & 15) >> 2),
                        __builtin_bit_cast(u32x4, floatx4{tf[slot][4 * h][r], tf[slot][4 * h + 1][r],
                                                          tf[slot][4 * h + 2][r], tf[slot][4 * h + 3][r]}));
                }
        } else {
        uint32_t w[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
            w[jj] = (uint32_t)Ty<P>::bits(x[2 * jj]) | ((uint32_t)Ty<P>::bits(x[2 * jj + 1]) << 16);
        if (rv)  // forward item: W[n][c0 .. c0 + 8) (pack_kernel's forward order)
            stg(J.wf + ((long)(n >> 4) * J.ksf + (c0 >> 5)) * 64 + (n & 15) + 16 * ((c0 & 31) >> 3),
                u32x4{w[0], w[1], w[2], w[3]});
        const int slot = threadIdx.x >> 3;
        tt[slot][r] = u32x4{w[0], w[1], w[2], w[3]};
        __syncthreads();
        const int c = c0 + r;
        if (J.wb && n0 < J.N && c < J.K) {  // dX item: W[n0 .. n0 + 8)[c]
            const uint16_t *T = reinterpret_cast<const uint16_t *>(&tt[slot][0]);
            uint32_t d[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) d[jj] = (uint32_t)T[16 * jj + r] | ((uint32_t)T[16 * jj + 8 + r] << 16);
            stg(J.wb + ((long)(c >> 4) * J.ksb + (n0 >> 5)) * 64 + (c & 15) + 16 * ((n0 & 31) >> 3),
                u32x4{d[0], d[1], d[2], d[3]});
        }
        }
    } else if (a.nseg > 0) {
        const int pb = b - a.jb[a.njobs], npb = gridDim.x - a.jb[a.njobs];
        for (int gi = pb * 256 + threadIdx.x; gi < a.q0[a.nseg]; gi += npb * 256) {
            int lo = 0, hi = a.nseg - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (gi >= a.q0[mid]) lo = mid;
                else hi = mid - 1;
            }
            const APSeg sg = a.s[lo];
            const APOpt o = a.o[sg.opt];
            const float ss = coef[sg.opt][0], bc = coef[sg.opt][1];
            const long e0 = 4L * (gi - a.q0[lo]);
            const int ne = (int)min(4L, (long)sg.n - e0);
            float *p = o.p + sg.off + e0, *m = o.m + sg.off + e0, *v = o.v + sg.off + e0;
            const float *g = sg.g + e0;
            for (int e = 0; e < ne; ++e) adam_one(p[e], g[e], m[e], v[e], ss, bc, o.b1, o.b2, o.eps, o.wd, 1.0f);
        }
    }
    // the last workgroup out advances every optimiser's step count
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = atomicAdd(a.ticket, 1u);
        if (done == gridDim.x - 1) {
            for (int k = 0; k < a.nopt; ++k) *a.o[k].step = *a.o[k].step + 1.0f;
            *a.ticket = 0u;
        }
    }
}

// ---------------------------------------------------------------- select_action
// Rows per workgroup = 16 RT.  RT = 1 gives a 4,096-env call one workgroup per
// CU (fastest alone: the per-CU weight stream bounds the pass); RT = 2 reads
// each weight half as often and leaves half of the CUs to the graph branches
// that run beside select_action (EXO_SELECT_RT).  F (the fp32 norm input)
// overlays H1 | H2, dead whenever F is written.
struct SelectArgs {
    Lin zs[3], ac[4];
    int act_enc, act_actor;
    const float *obs;
    int n, S, A, Z, Ha;
    float *out;
    Noise nz;
    R16 X, H1, H2, CAT;
    R32 F, TW, FT;
    int lds_bytes;
    int tile0, ticket;  // fp32 chunked launches: first row tile; 1 = take the noise ticket
    void *zimg;         // split launches (ZM 1 / 2): the rows' normalised zs in operand type, [n][Z]
};

#define RING_START(first)      \
    u32x4 R[PD][TH];           \
    ring_fill(R, GDesc{(first).wf, (first).ksf, 0})

__device__ __forceinline__ R16 rows_of(R16 r, int t) { return R16{r.off + t * TR * r.ld * 2, r.ld}; }
__device__ __forceinline__ R32 rows_of(R32 r, int t) { return R32{r.off + t * TR * r.ld * 4, r.ld}; }

// Row tiles tile0 + blockIdx.x: td7f_select may cover the tiles with several
// launches of at most its workgroup cap each (the same per-row arithmetic and
// Philox elements); only the last launch takes the noise ticket, so sigma and
// the call counter advance once, after every tile has drawn.
// ZM (r06, td7f_select_part): 0 the whole pass; 1 the fixed encoder's zs only,
// its normalised image stored to a.zimg (no actor, no noise); 2 the actor from
// that image (the zs layers skipped).  zs needs only the fixed encoder, which
// changes at target refreshes alone, so a training loop can run the ZM 1 half
// as soon as the observations exist and only the ZM 2 half after the actor
// step; the image is the operand-type values ZM 0 leaves in CAT, so 1 + 2 ==
// 0 bit for bit (same row tiles).
template <int P, int TH, int RT, int ZM = 0>
__global__ __launch_bounds__(NTH) void select_kernel(SelectArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int rows = RT * TR;
    // (chunked launches for the 16-row kernels only: the 32-row ones keep
    // blockIdx.x -- their register allocation spills otherwise)
    int row0;
    if constexpr (RT == 1) row0 = (a.tile0 + blockIdx.x) * rows;
    else row0 = blockIdx.x * rows;
    int si = 0;
    FSTAMP(si);
    RowStage so[RT];
    ThinStage<THIN_NC> tw;
    using E = typename Ty<P>::E;
    static_assert(RT * TR * (int)sizeof(E) <= 64, "ZM 2 staging: 16 rows x 512 words at most");
#pragma unroll
    for (int t = 0; t < RT; ++t) row_issue(so[t], a.obs, a.S, a.S, row0 + t * TR, a.n);
    if constexpr (ZM != 1) thin_issue(tw, a.ac[3].w, a.ac[3].ldw, 0, false, a.A, a.ac[3].K);
    // ZM 2: this workgroup's zs image rows in 4-byte words (Z * EB % 4 == 0,
    // at most 16 rows x 512 words per 512 threads: checked on the host),
    // loaded with the observations
    const int zw = a.Z * (int)sizeof(E) / 4;
    constexpr int ZPT = ZM == 2 ? (16 * 512 + NTH - 1) / NTH : 1;
    uint32_t zv[ZPT];
    if constexpr (ZM == 2) {
        const uint32_t *zi = (const uint32_t *)a.zimg;
#pragma unroll
        for (int u = 0; u < ZPT; ++u) {
            const int k = threadIdx.x + u * NTH, r = k / zw, c = k - r * zw;
            zv[u] = (r < rows && row0 + r < a.n) ? zi[(long)(row0 + r) * zw + c] : 0u;
        }
    }
    RING_START(ZM == 2 ? a.ac[0] : a.zs[0]);
    zero_lds(lds, a.lds_bytes);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RT; ++t) row_put16<P>(lds, so[t], rows_of(a.X, t), 0, a.S, row0 + t * TR, a.n);
    if constexpr (ZM != 1) thin_put<P>(lds, tw, a.TW, a.A, a.ac[3].K);
    if constexpr (ZM == 2) {
#pragma unroll
        for (int u = 0; u < ZPT; ++u) {
            const int k = threadIdx.x + u * NTH, r = k / zw, c = k - r * zw;
            if (r < rows) *(uint32_t *)(pe<P>(lds, a.CAT, r, a.Ha) + c * (4 / (int)sizeof(E))) = zv[u];
        }
    }
    __syncthreads();
    if constexpr (ZM != 2) {
        // zs = fixed_encoder.zs(obs) (:93-97) -> CAT[:, Ha:Ha+Z]
        layer_fwd<P, RT, TH>(lds, R, a.X, a.zs[0], &a.zs[1], a.act_enc, a.H1, 0, NO32, nullptr, 0, row0, a.n, si);
        layer_fwd<P, RT, TH>(lds, R, a.H1, a.zs[1], &a.zs[2], a.act_enc, a.H2, 0, NO32, nullptr, 0, row0, a.n, si);
        layer_fwd<P, RT, TH>(lds, R, a.H2, a.zs[2], ZM == 1 ? (const Lin *)nullptr : &a.ac[0], ACT_NONE, NO16, 0, a.F,
                             nullptr, 0, row0, a.n, si);
        norm_fwd<P>(lds, a.F, a.Z, rows, 1e-8f, a.CAT, a.Ha, NO16, 0, NO32, nullptr, 0, nullptr, nullptr, row0, a.n);
        __syncthreads();
    }
    if constexpr (ZM == 1) {
        uint32_t *zo = (uint32_t *)a.zimg;
        for (int k = threadIdx.x; k < rows * zw; k += NTH) {
            const int r = k / zw, c = k - r * zw;
            if (row0 + r < a.n)
                zo[(long)(row0 + r) * zw + c] = *(const uint32_t *)(pe<P>(lds, a.CAT, r, a.Ha) + c * (4 / (int)sizeof(E)));
        }
        return;
    }
    // actor (:72-77): AvgL1Norm(l0(s)) | zs -> l1 -> l2 -> tanh(l3)
    layer_fwd<P, RT, TH>(lds, R, a.X, a.ac[0], &a.ac[1], ACT_NONE, NO16, 0, a.F, nullptr, 0, row0, a.n, si);
    norm_fwd<P>(lds, a.F, a.Ha, rows, 1e-8f, a.CAT, 0, NO16, 0, NO32, nullptr, 0, nullptr, nullptr, row0, a.n);
    __syncthreads();
    // F overlaid H1 | H2: their zero padding columns (read by the GEMMs below
    // where the width is not a multiple of 32 PD) are restored before the
    // epilogues write H1 / H2 (those come after each GEMM's exchange barrier)
    if (a.F.off == a.H1.off) zero_lds(lds + a.H1.off, a.H2.off + rows * a.H2.ld * 2 - a.H1.off);
    layer_fwd<P, RT, TH>(lds, R, a.CAT, a.ac[1], &a.ac[2], a.act_actor, a.H1, 0, NO32, nullptr, 0, row0, a.n, si);
    layer_fwd<P, RT, TH>(lds, R, a.H1, a.ac[2], (const Lin *)nullptr, a.act_actor, a.H2, 0, NO32, nullptr, 0, row0, a.n, si);
    if constexpr (RT == 1) {
        layer_thin_fwd<P, THIN_NC>(lds, a.H2, a.ac[3], a.TW, ACT_TANH, a.FT, rows, nullptr, 0, row0, a.n, si);
    } else {  // thin products per 16-row tile, then bias + tanh over all rows
        FSTAMP(si);
#pragma unroll
        for (int t = 0; t < RT; ++t)
            thin<P, THIN_NC>(lds, rows_of(a.H2, t), 0, a.ac[3].K, a.TW, a.A, rows_of(a.FT, t), 1.f);
        __syncthreads();
        for (int k = threadIdx.x; k < rows * a.A; k += NTH) {
            const int row = k / a.A, c = k - row * a.A;
            *p32(lds, a.FT, row, c) = act_fwd(ACT_TANH, *p32(lds, a.FT, row, c) + ldg(a.ac[3].b + c));
        }
        __syncthreads();
    }
    if constexpr (RT == 1) noise_rows<P>(lds, a.FT, a.A, rows, row0, a.n, a.nz, a.out, NO16, 0, NO16, 0, a.ticket != 0);
    else noise_rows<P>(lds, a.FT, a.A, rows, row0, a.n, a.nz, a.out, NO16, 0, NO16, 0);
}

// ---------------------------------------------------------------- critic target chain
struct TargetArgs {
    Lin enc[6], ac[4], cr[8];
    int act_enc, act_actor, act_critic;
    const float *ns;  // next_state [B][S]
    int B, S, A, Z, Ha, Hc;
    Noise nz;
    void *img;      // [B][round_up(2Z + A, 8)] operand type: zsa | zs | next_action
    float *qt;      // [B][2]
    R16 X, H1, H2, CATA, CATZ, OUT, CAT;
    R32 F, TW;
    int lds_a, lds_b;
};

template <int P, int TH>
__global__ __launch_bounds__(NTH) void target_a_kernel(TargetArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int RT = 1, rows = TR;
    const int row0 = blockIdx.x * rows, B = a.B, Z = a.Z;
    int si = 0;
    FSTAMP(si);
    RowStage sn;
    ThinStage<THIN_NC> tw;
    row_issue(sn, a.ns, a.S, a.S, row0, B);
    thin_issue(tw, a.ac[3].w, a.ac[3].ldw, 0, false, a.A, a.ac[3].K);
    RING_START(a.enc[0]);
    zero_lds(lds, a.lds_a);
    __syncthreads();
    row_put16<P>(lds, sn, a.X, 0, a.S, row0, B);
    thin_put<P>(lds, tw, a.TW, a.A, a.ac[3].K);
    __syncthreads();
    // fixed_target_zs = fixed_encoder_target.zs(next_state) (:234)
    layer_fwd<P, RT, TH>(lds, R, a.X, a.enc[0], &a.enc[1], a.act_enc, a.H1, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H1, a.enc[1], &a.enc[2], a.act_enc, a.H2, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H2, a.enc[2], &a.ac[0], ACT_NONE, NO16, 0, a.F, nullptr, 0, row0, B, si);
    norm_fwd<P>(lds, a.F, Z, rows, 1e-8f, a.CATA, a.Ha, a.CATZ, 0, NO32, nullptr, 0, nullptr, nullptr, row0, B);
    __syncthreads();
    // next_action = (actor_target(s', zs) + clip(noise * sigma)).clamp(-1, 1) (:236-238)
    layer_fwd<P, RT, TH>(lds, R, a.X, a.ac[0], &a.ac[1], ACT_NONE, NO16, 0, a.F, nullptr, 0, row0, B, si);
    norm_fwd<P>(lds, a.F, a.Ha, rows, 1e-8f, a.CATA, 0, NO16, 0, NO32, nullptr, 0, nullptr, nullptr, row0, B);
    __syncthreads();
    layer_fwd<P, RT, TH>(lds, R, a.CATA, a.ac[1], &a.ac[2], a.act_actor, a.H1, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H1, a.ac[2], &a.enc[3], a.act_actor, a.H2, 0, NO32, nullptr, 0, row0, B, si);
    layer_thin_fwd<P, THIN_NC>(lds, a.H2, a.ac[3], a.TW, ACT_TANH, a.F, rows, nullptr, 0, row0, B, si);
    noise_rows<P>(lds, a.F, a.A, rows, row0, B, a.nz, nullptr, a.CATZ, Z, a.OUT, 2 * Z);
    __syncthreads();
    // fixed_target_zsa = fixed_encoder_target.zsa(zs, next_action) (:240) -> OUT[:, 0:Z]
    layer_fwd<P, RT, TH>(lds, R, a.CATZ, a.enc[3], &a.enc[4], a.act_enc, a.H1, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H1, a.enc[4], &a.enc[5], a.act_enc, a.H2, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H2, a.enc[5], (const Lin *)nullptr, ACT_NONE, a.OUT, 0, NO32, nullptr, 0, row0, B, si);
    // zs into OUT[:, Z:2Z] (from CATZ[:, 0:Z])
    for (int k = threadIdx.x; k < rows * Z; k += NTH) {
        const int row = k / Z, c = k - row * Z;
        *pe<P>(lds, a.OUT, row, Z + c) = *pe<P>(lds, a.CATZ, row, c);
    }
    __syncthreads();
    // raw 16-bit copy of the image rows (an fp32 element is two 16-bit units)
    constexpr int EH = Ty<P>::EB / 2;
    const int ild = (2 * Z + a.A + 7) / 8 * 8 * EH;
    store_rows16(lds, a.OUT, 0, (uint16_t *)a.img, ild, ild, rows, row0, B);
}

template <int P, int TH>
__global__ __launch_bounds__(NTH) void target_b_kernel(TargetArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int RT = 1, rows = TR;
    const int row0 = blockIdx.x * rows, B = a.B, Z = a.Z, h = blockIdx.y;
    const long ild = (2 * Z + a.A + 7) / 8 * 8;
    const Lin *cr = a.cr + h;  // layer l of head h: cr[2 l]
    int si = 0;
    FSTAMP(si);
    RowStage sn;
    ThinStage<1> tw;
    row_issue(sn, a.ns, a.S, a.S, row0, B);
    // fp32: zsa, zs and the action as three fp32 row stages (column per thread);
    // 16-bit: zsa | zs and the action as column pairs
    [[maybe_unused]] RowStage fa, fz0, fz1;
    [[maybe_unused]] Row16Stage sa, sc;
    if constexpr (P == PREC_F32) {
        const float *img = (const float *)a.img;
        row_issue(fa, img + 2 * Z, ild, a.A, row0, B);
        row_issue(fz0, img, ild, Z, row0, B);
        row_issue(fz1, img + Z, ild, Z, row0, B);
    } else {
        const uint16_t *img = (const uint16_t *)a.img;
        row16_issue(sa, img + 2 * Z, ild, a.A, row0, B);
        row16_issue(sc, img, ild, 2 * Z, row0, B);
    }
    thin_issue(tw, cr[6].w, cr[6].ldw, 0, false, 1, cr[6].K);
    RING_START(cr[0]);
    zero_lds(lds, a.lds_b);
    __syncthreads();
    row_put16<P>(lds, sn, a.X, 0, a.S, row0, B);
    if constexpr (P == PREC_F32) {
        row_put16<P>(lds, fa, a.X, a.S, a.A, row0, B);
        row_put16<P>(lds, fz0, a.CAT, a.Hc, Z, row0, B);
        row_put16<P>(lds, fz1, a.CAT, a.Hc + Z, Z, row0, B);
    } else {
        row16_put(lds, sa, a.X, a.S, a.A, row0, B);
        row16_put(lds, sc, a.CAT, a.Hc, 2 * Z, row0, B);
    }
    thin_put<P>(lds, tw, a.TW, 1, cr[6].K);
    __syncthreads();
    // critic_target(s', a', zsa, zs) head h (:109-140): AvgL1Norm(q0(sa)) | zsa | zs -> q1 -> q2 -> q3
    layer_fwd<P, RT, TH>(lds, R, a.X, cr[0], &cr[2], ACT_NONE, NO16, 0, a.F, nullptr, 0, row0, B, si);
    norm_fwd<P>(lds, a.F, a.Hc, rows, 1e-8f, a.CAT, 0, NO16, 0, NO32, nullptr, 0, nullptr, nullptr, row0, B);
    __syncthreads();
    layer_fwd<P, RT, TH>(lds, R, a.CAT, cr[2], &cr[4], a.act_critic, a.H1, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H1, cr[4], (const Lin *)nullptr, a.act_critic, a.H2, 0, NO32, nullptr, 0, row0, B, si);
    layer_thin_fwd<P, 1>(lds, a.H2, cr[6], a.TW, ACT_NONE, a.F, rows, a.qt + h, 2, row0, B, si);
}

// ---------------------------------------------------------------- fixed embeddings
struct FixedArgs {
    Lin enc[6];
    int act_enc;
    const float *s, *act;
    int B, S, A, Z;
    float *zs, *zsa;
    R16 X, H1, H2, CATZ;
    R32 F;
    int lds_bytes;
};

template <int P, int TH>
__global__ __launch_bounds__(NTH) void fixed_kernel(FixedArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int RT = 1, rows = TR;
    const int row0 = blockIdx.x * rows, B = a.B, Z = a.Z;
    int si = 0;
    FSTAMP(si);
    RowStage ss, sa;
    row_issue(ss, a.s, a.S, a.S, row0, B);
    row_issue(sa, a.act, a.A, a.A, row0, B);
    RING_START(a.enc[0]);
    zero_lds(lds, a.lds_bytes);
    __syncthreads();
    row_put16<P>(lds, ss, a.X, 0, a.S, row0, B);
    row_put16<P>(lds, sa, a.CATZ, Z, a.A, row0, B);
    __syncthreads();
    layer_fwd<P, RT, TH>(lds, R, a.X, a.enc[0], &a.enc[1], a.act_enc, a.H1, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H1, a.enc[1], &a.enc[2], a.act_enc, a.H2, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H2, a.enc[2], &a.enc[3], ACT_NONE, NO16, 0, a.F, nullptr, 0, row0, B, si);
    norm_fwd<P>(lds, a.F, Z, rows, 1e-8f, a.CATZ, 0, NO16, 0, NO32, a.zs, Z, nullptr, nullptr, row0, B);
    __syncthreads();
    layer_fwd<P, RT, TH>(lds, R, a.CATZ, a.enc[3], &a.enc[4], a.act_enc, a.H1, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H1, a.enc[4], &a.enc[5], a.act_enc, a.H2, 0, NO32, nullptr, 0, row0, B, si);
    layer_fwd<P, RT, TH>(lds, R, a.H2, a.enc[5], (const Lin *)nullptr, ACT_NONE, NO16, 0, NO32, a.zsa, Z, row0, B, si);
}

// ---------------------------------------------------------------- host side
thread_local bool td7f_probe_mode = false;
}  // namespace td7f

using namespace td7f;

static bool prec_ok(int p) { return p == PREC_BF16 || p == PREC_F16 || p == PREC_F32; }

extern "C" {

#ifdef EXO_STAMPS
int td7f_debug_set_stamps(unsigned long long *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_td7f_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -5;
}
#endif

int td7f_pack(int32_t prec, int32_t njobs, const td7f_pack_job *jobs, void *stream) {
    if (!prec_ok(prec) || njobs <= 0 || njobs > TD7F_MAX_PACK || !jobs) return EXO_EINVAL;
    const int kd = kd_of(prec);
    PackArgs a{};
    a.njobs = njobs;
    a.start[0] = 0;
    for (int q = 0; q < njobs; ++q) {
        const td7f_pack_job &J = jobs[q];
        if (!J.w || !J.wf || J.n_out <= 0 || J.n_in <= 0 || J.ld < J.n_in || J.ksf * kd < J.n_in ||
            J.ntf * 16 < J.n_out || (J.wb && (J.ksb * kd < J.n_out || J.ntb * 16 < J.n_in)))
            return EXO_EINVAL;
        a.j[q] = PackJob{J.w, (long)J.ld, J.n_out, J.n_in, (u32x4 *)J.wf, (u32x4 *)J.wb, J.ksf, J.ntf,
                         J.wb ? J.ksb : 0, J.wb ? J.ntb : 0};
        a.start[q + 1] = a.start[q] + (long)J.ntf * J.ksf * 64 + (J.wb ? (long)J.ntb * J.ksb * 64 : 0);
    }
    long most = 0;
    for (int q = 0; q < njobs; ++q) most = std::max(most, a.start[q + 1] - a.start[q]);
    const dim3 grid((unsigned)std::min<long>(1024, (most + 255) / 256), (unsigned)njobs);
    if (prec == PREC_BF16)
        hipLaunchKernelGGL(pack_kernel<PREC_BF16>, grid, dim3(256), 0, (hipStream_t)stream, a);
    else if (prec == PREC_F16)
        hipLaunchKernelGGL(pack_kernel<PREC_F16>, grid, dim3(256), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(pack_kernel<PREC_F32>, grid, dim3(256), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7f_adam_pack(int32_t prec, int32_t nopt, float *const *p, float *const *m, float *const *v, float *const *step,
                   const float *lr, const float *beta1, const float *beta2, const float *eps,
                   const float *weight_decay, int32_t nseg, const float *const *g, const int64_t *off, const int32_t *n,
                   const int32_t *opt, int32_t njobs, const td7f_pack_job *jobs, const int32_t *job_seg,
                   uint32_t *ticket, void *stream) {
    if (!prec_ok(prec) || nopt <= 0 || nopt > TD7_ADAM_MAX_OPT || nseg <= 0 ||
        nseg > TD7_ADAM_MAX_SEG || njobs < 0 || njobs > TD7F_MAX_ADAM_PACK || (njobs && (!jobs || !job_seg)) ||
        !ticket)
        return EXO_EINVAL;
    const int kd = kd_of(prec);
    AdamPackArgs a{};
    a.nopt = nopt;
    a.ticket = ticket;
    for (int k = 0; k < nopt; ++k) {
        if (!p[k] || !m[k] || !v[k] || !step[k]) return EXO_EINVAL;
        a.o[k] = APOpt{p[k], m[k], v[k], step[k], lr[k], beta1[k], beta2[k], eps[k], weight_decay[k]};
    }
    for (int k = 0; k < nseg; ++k)
        if (!g[k] || n[k] <= 0 || off[k] < 0 || opt[k] < 0 || opt[k] >= nopt) return EXO_EINVAL;
    // every job: a contiguous [N][K] block inside its segment; a segment is
    // covered by its jobs exactly or not at all
    long covered[TD7_ADAM_MAX_SEG] = {};
    a.jb[0] = 0;
    for (int q = 0; q < njobs; ++q) {
        const td7f_pack_job &J = jobs[q];
        const int k = job_seg[q];
        if (k < 0 || k >= nseg || !J.w || !J.wf || J.n_out <= 0 || J.n_in <= 0 || J.ld != J.n_in ||
            J.ksf * kd < J.n_in || J.ntf * 16 < J.n_out || (J.wb && (J.ksb * kd < J.n_out || J.ntb * 16 < J.n_in)))
            return EXO_EINVAL;
        const int o = opt[k];
        const long e = (long)(J.w - p[o]), sz = (long)J.n_out * J.n_in;
        if (e < off[k] || e + sz > off[k] + n[k]) return EXO_EINVAL;
        covered[k] += sz;
        const float *gq = g[k] + (e - off[k]);
        const bool vec = J.n_in % 4 == 0 &&
                         ((reinterpret_cast<uintptr_t>(J.w) | reinterpret_cast<uintptr_t>(m[o] + e) |
                           reinterpret_cast<uintptr_t>(v[o] + e) | reinterpret_cast<uintptr_t>(gq)) & 15) == 0;
        const int nch = (J.n_in + 7) / 8;
        a.j[q] = APJob{p[o] + e, m[o] + e, v[o] + e, gq, (u32x4 *)J.wf, (u32x4 *)J.wb, o, J.n_out, J.n_in, nch,
                       J.ksf, J.wb ? J.ksb : 0, vec ? 1 : 0};
        const long threads = (long)(J.n_out + 7) / 8 * nch * 8;
        a.jb[q + 1] = a.jb[q] + (int)((threads + 255) / 256);
    }
    a.njobs = njobs;
    long groups = 0;
    for (int k = 0; k < nseg; ++k) {
        if (covered[k] == n[k]) continue;
        if (covered[k] != 0) return EXO_EINVAL;
        a.s[a.nseg] = APSeg{g[k], (long)off[k], n[k], opt[k]};
        a.q0[a.nseg++] = (int)groups;
        groups += (n[k] + 3) / 4;
    }
    if (groups >= (1L << 30)) return EXO_ERANGE;
    a.q0[a.nseg] = (int)groups;
    const long plain = std::min<long>(64, (groups + 255) / 256);
    const unsigned grid = (unsigned)(a.jb[njobs] + plain);
    if (grid == 0) return EXO_OK;
    if (prec == PREC_BF16)
        hipLaunchKernelGGL(adam_pack_kernel<PREC_BF16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    else if (prec == PREC_F16)
        hipLaunchKernelGGL(adam_pack_kernel<PREC_F16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(adam_pack_kernel<PREC_F32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int td7f_probe(int32_t on) {
    td7f::td7f_probe_mode = on != 0;
    return EXO_OK;
}

}  // extern "C"

namespace {
// the select kernel of (precision, weight-tile count, row tiles, split mode)
template <int ZM>
int select_one(int prec, int th, int RT, dim3 g, int lds, const SelectArgs &a, hipStream_t st) {
    using namespace td7f;
    if (prec == PREC_F32)
        return th == 5 ? launch(select_kernel<PREC_F32, 5, 1, ZM>, g, lds, a, st)
                       : launch(select_kernel<PREC_F32, 4, 1, ZM>, g, lds, a, st);
    if (RT == 2)
        return prec == PREC_BF16 ? (th == 5 ? launch(select_kernel<PREC_BF16, 5, 2, ZM>, g, lds, a, st)
                                            : launch(select_kernel<PREC_BF16, 4, 2, ZM>, g, lds, a, st))
                                 : (th == 5 ? launch(select_kernel<PREC_F16, 5, 2, ZM>, g, lds, a, st)
                                            : launch(select_kernel<PREC_F16, 4, 2, ZM>, g, lds, a, st));
    return prec == PREC_BF16 ? (th == 5 ? launch(select_kernel<PREC_BF16, 5, 1, ZM>, g, lds, a, st)
                                        : launch(select_kernel<PREC_BF16, 4, 1, ZM>, g, lds, a, st))
                             : (th == 5 ? launch(select_kernel<PREC_F16, 5, 1, ZM>, g, lds, a, st)
                                        : launch(select_kernel<PREC_F16, 4, 1, ZM>, g, lds, a, st));
}
int select_mode(int zm, int prec, int th, int RT, dim3 g, int lds, const SelectArgs &a, hipStream_t st) {
    return zm == 1 ? select_one<1>(prec, th, RT, g, lds, a, st)
         : zm == 2 ? select_one<2>(prec, th, RT, g, lds, a, st)
                   : select_one<0>(prec, th, RT, g, lds, a, st);
}

int select_impl(int32_t prec, const int32_t *act, const td7f_lin *enc, const td7f_lin *actor, const float *obs,
                int32_t n, const td7f_noise *noise, float *out, int32_t wg_cap, int32_t rt, void *zimg, int zm,
                void *stream) {
    if (!prec_ok(prec) || !act || !enc || !actor || !obs || n <= 0 || wg_cap < 0 || rt < 0 || rt > 2 || zm < 0 ||
        zm > 2 || (zm != 1 && (!noise || !out)) || (zm != 0 && !zimg))
        return EXO_EINVAL;
    const int kd = kd_of(prec);
    td7f_lin all[7] = {enc[0], enc[1], enc[2], actor[0], actor[1], actor[2], actor[3]};
    const int th = th_of(all, 7);
    if (th != 4 && th != 5) return EXO_EINVAL;
    SelectArgs a{};
    for (int i = 0; i < 3; ++i) a.zs[i] = lin_of(enc[i]);
    for (int i = 0; i < 4; ++i) a.ac[i] = lin_of(actor[i]);
    a.act_enc = act[0];
    a.act_actor = act[1];
    a.obs = obs;
    a.n = n;
    a.S = enc[0].n_in;
    a.A = actor[3].n_out;
    a.Z = enc[2].n_out;
    a.Ha = actor[0].n_out;
    if (actor[0].n_in != a.S || actor[1].n_in != a.Ha + a.Z || a.A > THIN_NC || a.S > NTH) return EXO_EINVAL;
    a.out = out;
    if (zm != 1) a.nz = noise_of(*noise);
    a.zimg = zimg;
    if (zm != 0 && (((long)a.Z * (prec == PREC_F32 ? 4 : 2)) % 4 || ((long)a.Ha * (prec == PREC_F32 ? 4 : 2)) % 4 || a.Z > 512))
        return EXO_EINVAL;  // the image moves in 4-byte words, at most 512 per row
    // 32-row tiles above 8,192 envs (more than two 16-row workgroups per CU:
    // the weights are then streamed half as often; configs[3]'s 16,384 envs
    // 0.452 vs 0.494 ms per iteration, profiles/r04q_raw); 16-row tiles below
    // (4,096 envs: one workgroup per CU); `rt` 1 | 2 asks for one (the
    // overlapped training pairs run select_action on their critical chain
    // beside the update's passes: 32-row tiles, half the workgroups and weight
    // bytes, 0.249-0.255 vs 0.259-0.265 ms per iteration, profiles/r05_sched).
    // EXO_SELECT_RT=1|2 overrides (read per call: tests switch it).
    const char *rt_env = getenv("EXO_SELECT_RT");
    // (fp32: 16-row tiles only -- a 32-row tile's fp32 images exceed the LDS)
    const int RT = prec == PREC_F32 ? 1
                   : rt_env && (rt_env[0] == '1' || rt_env[0] == '2') ? rt_env[0] - '0'
                   : rt ? rt : (n > 8192 ? 2 : 1);
    const int rows = RT * TR, hmax = std::max(enc[0].n_out, std::max(enc[1].n_out, std::max(a.Ha, actor[1].n_out)));
    Bump b(RT);
    a.X = b.r16(rows, ld16(a.S, kd));
    a.H1 = b.r16(rows, ld16(hmax, kd));
    a.H2 = b.r16(rows, ld16(hmax, kd));
    const int fld = std::max(std::max(a.Z, a.Ha), 16);
    if (rows * fld * 4 <= a.H2.off + rows * a.H2.ld * 2 - a.H1.off) {
        a.F = R32{a.H1.off, fld};  // overlays H1 | H2 (both dead whenever F is written)
    } else {
        a.F = b.r32(rows, fld);
    }
    a.CAT = b.r16(rows, ld16(a.Ha + a.Z, kd));
    a.TW = b.r32(THIN_NC, actor[3].n_in);
    a.FT = b.r32(rows, 16);
    a.lds_bytes = b.off;
    // workgroup cap (wg_cap; EXO_SELECT_WG_CAP overrides it when set; 0 = all
    // tiles in one launch): the tiles in launches of at most cap workgroups back to
    // back, leaving CUs to the fused passes that run beside select_action in
    // the training loop -- fp32 at 4,096 envs, cap 128: 0.488-0.491 vs
    // 0.493-0.499 ms per iteration (64: 0.525; profiles/r04sc_raw)
    // (16-row tiles only; exo_amd.fused.select's wg_cap, which the training
    // loop passes and the reference schedule's rollout -- select_action on
    // its critical chain -- does not)
    const char *cap_env = getenv("EXO_SELECT_WG_CAP");
    const int ntiles = (n + rows - 1) / rows;
    const int cap = cap_env ? atoi(cap_env) : wg_cap;
    const hipStream_t st = (hipStream_t)stream;
    if (RT == 1 && cap > 0 && cap < ntiles) {
        for (int t0 = 0; t0 < ntiles; t0 += cap) {
            a.tile0 = t0;
            a.ticket = t0 + cap >= ntiles;
            const dim3 g(std::min(cap, ntiles - t0));
            const int rc = select_mode(zm, prec, th, 1, g, b.off, a, st);
            if (rc != EXO_OK) return rc;
        }
        return EXO_OK;
    }
    a.tile0 = 0;
    a.ticket = 1;
    return select_mode(zm, prec, th, RT, dim3(ntiles), b.off, a, st);
}
}  // namespace

extern "C" {

int td7f_select(int32_t prec, const int32_t *act, const td7f_lin *enc, const td7f_lin *actor, const float *obs,
                int32_t n, const td7f_noise *noise, float *out, int32_t wg_cap, int32_t rt, void *stream) {
    return select_impl(prec, act, enc, actor, obs, n, noise, out, wg_cap, rt, nullptr, 0, stream);
}

int td7f_select_part(int32_t prec, const int32_t *act, const td7f_lin *enc, const td7f_lin *actor, const float *obs,
                     int32_t n, const td7f_noise *noise, float *out, int32_t wg_cap, int32_t rt, void *zimg,
                     int32_t mode, void *stream) {
    if (mode != 1 && mode != 2) return EXO_EINVAL;
    return select_impl(prec, act, enc, actor, obs, n, noise, out, wg_cap, rt, zimg, mode, stream);
}

int td7f_target(int32_t prec, const int32_t *act, const td7f_lin *tenc, const td7f_lin *tactor,
                const td7f_lin *tcritic, const float *ns, int32_t B, const td7f_noise *noise, void *img,
                float *qt, void *stream) {
    if (!prec_ok(prec) || !act || !tenc || !tactor || !tcritic || !ns || !noise || !img || !qt || B <= 0)
        return EXO_EINVAL;
    const int kd = kd_of(prec), eh = prec == PREC_F32 ? 2 : 1;
    td7f_lin all[18];
    for (int i = 0; i < 6; ++i) all[i] = tenc[i];
    for (int i = 0; i < 4; ++i) all[6 + i] = tactor[i];
    for (int i = 0; i < 8; ++i) all[10 + i] = tcritic[i];
    const int th = th_of(all, 18);
    if (th != 4 && th != 5) return EXO_EINVAL;
    TargetArgs a{};
    for (int i = 0; i < 6; ++i) a.enc[i] = lin_of(tenc[i]);
    for (int i = 0; i < 4; ++i) a.ac[i] = lin_of(tactor[i]);
    for (int i = 0; i < 8; ++i) a.cr[i] = lin_of(tcritic[i]);
    a.act_enc = act[0];
    a.act_actor = act[1];
    a.act_critic = act[2];
    a.ns = ns;
    a.B = B;
    a.S = tenc[0].n_in;
    a.A = tactor[3].n_out;
    a.Z = tenc[2].n_out;
    a.Ha = tactor[0].n_out;
    a.Hc = tcritic[0].n_out;
    // tcritic is [layer][head]: layer l of head h at 2l + h
    if (tcritic[0].n_in != a.S + a.A || tcritic[2].n_in != a.Hc + 2 * a.Z || tcritic[4].n_in != a.Hc ||
        tenc[3].n_in != a.Z + a.A || a.A > THIN_NC || a.S > NTH)
        return EXO_EINVAL;
    a.nz = noise_of(*noise);
    a.img = img;
    a.qt = qt;
    const int rows = TR;
    int hmax = 0;
    for (int i = 0; i < 18; ++i) hmax = std::max(hmax, all[i].n_out);
    const int old = eh * round_up(2 * a.Z + a.A, 8);  // == the image row (16-byte stores)
    const int fld = std::max(hmax, 16);
    // fp32 with an OUT row wider than CATA's (zs_dim well above actor_hdim):
    // X and CATA side by side, OUT over both (below)
    const bool wide_out = prec == PREC_F32 && old > ld16(a.Ha + a.Z, kd);
    Bump ba(1);
    a.X = ba.r16(rows, ld16(a.S + a.A, kd));
    if (wide_out) a.CATA = ba.r16(rows, ld16(a.Ha + a.Z, kd));
    a.H1 = ba.r16(rows, ld16(hmax, kd));
    a.H2 = ba.r16(rows, ld16(hmax, kd));
    if (!wide_out) a.CATA = ba.r16(rows, ld16(a.Ha + a.Z, kd));
    a.CATZ = ba.r16(rows, ld16(a.Z + a.A, kd));
    if (prec == PREC_F32) {
        // fp32 images: OUT overlays CATA (dead once actor_target's l1 has read
        // it; OUT is first written by the noise after l3) -- or, wider than
        // CATA's rows, X | CATA (X is dead after actor_target's l0, before
        // l1) -- and F overlays H1 | H2 (dead whenever F is written; the thin
        // l3 writes F's first columns only, inside H1, while it reads H2); a
        // region no overlay fits gets its own bytes, as in the 16-bit images
        if (!wide_out) a.OUT = R16{a.CATA.off, old};
        else if (rows * old * 2 <= a.CATA.off + rows * a.CATA.ld * 2 - a.X.off) a.OUT = R16{a.X.off, old};
        else a.OUT = ba.r16(rows, old);
        a.F = rows * fld * 4 <= a.H2.off + rows * a.H2.ld * 2 - a.H1.off ? R32{a.H1.off, fld} : ba.r32(rows, fld);
    } else {
        a.OUT = ba.r16(rows, old);
        a.F = ba.r32(rows, fld);
    }
    a.TW = ba.r32(THIN_NC, tactor[3].n_in);
    a.lds_a = ba.off;
    Bump bb(1);
    const R16 Xb = bb.r16(rows, ld16(a.S + a.A, kd)), H1b = bb.r16(rows, ld16(hmax, kd)), H2b = bb.r16(rows, ld16(hmax, kd));
    const R16 CATb = bb.r16(rows, ld16(a.Hc + 2 * a.Z, kd));
    const R32 Fb = bb.r32(rows, std::max(hmax, 16));
    const R32 TWb = bb.r32(1, tcritic[6].n_in);
    a.lds_b = bb.off;
    const hipStream_t st = (hipStream_t)stream;
    int rc = DISPATCH(prec, th, target_a_kernel, dim3((B + rows - 1) / rows), ba.off, a, st);
    if (rc != EXO_OK) return rc;
    TargetArgs b2 = a;
    b2.X = Xb;
    b2.H1 = H1b;
    b2.H2 = H2b;
    b2.CAT = CATb;
    b2.F = Fb;
    b2.TW = TWb;
    return DISPATCH(prec, th, target_b_kernel, dim3((B + rows - 1) / rows, 2), bb.off, b2, st);
}

int td7f_fixed(int32_t prec, const int32_t *act, const td7f_lin *fenc, const float *s, const float *action,
               int32_t B, float *zs, float *zsa, void *stream) {
    if (!prec_ok(prec) || !act || !fenc || !s || !action || !zs || !zsa || B <= 0) return EXO_EINVAL;
    const int kd = kd_of(prec);
    const int th = th_of(fenc, 6);
    if (th != 4 && th != 5) return EXO_EINVAL;
    FixedArgs a{};
    for (int i = 0; i < 6; ++i) a.enc[i] = lin_of(fenc[i]);
    a.act_enc = act[0];
    a.s = s;
    a.act = action;
    a.B = B;
    a.S = fenc[0].n_in;
    a.Z = fenc[2].n_out;
    a.A = fenc[3].n_in - a.Z;
    if (a.A <= 0 || a.A > THIN_NC || a.S > NTH) return EXO_EINVAL;
    a.zs = zs;
    a.zsa = zsa;
    const int rows = TR;
    int hmax = 0;
    for (int i = 0; i < 6; ++i) hmax = std::max(hmax, fenc[i].n_out);
    Bump b(1);
    a.X = b.r16(rows, ld16(a.S, kd));
    a.H1 = b.r16(rows, ld16(hmax, kd));
    a.H2 = b.r16(rows, ld16(hmax, kd));
    a.CATZ = b.r16(rows, ld16(a.Z + a.A, kd));
    a.F = b.r32(rows, std::max(hmax, 16));
    a.lds_bytes = b.off;
    return DISPATCH(prec, th, fixed_kernel, dim3((B + rows - 1) / rows), b.off, a, (hipStream_t)stream);
}

}  // extern "C"
