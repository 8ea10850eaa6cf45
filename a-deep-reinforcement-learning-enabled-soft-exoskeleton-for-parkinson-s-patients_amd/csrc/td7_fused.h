// td7_fused.h -- building blocks of the row-tile-fused TD7 networks (gfx950).
//
// The TD7 update (Agent/TD7_multi_agent.py:211-293) is a chain of small MLPs
// (encoder zs/zsa, actor, twin critic) over B = 8 x 128 rows whose widths are
// 300-320.  Layer-per-launch, every GEMM is latency bound (M = 1,024, N <= 320)
// and the graph holds ~53 of them.  Here a workgroup owns 16 rows and runs a
// whole network on them: activations stay in LDS (bf16 / fp16 / fp32, the MFMA
// operand format), each wave streams its column tiles of every weight matrix
// straight from L2 into registers in a pre-packed fragment order (one 1 KiB
// contiguous block per 16-column tile and k-step -- 32 16-bit or 16 fp32
// inputs -- written by td7f_pack), and v_mfma_f32_16x16x32_{bf16,f16} (fp32:
// 4 x v_mfma_f32_16x16x4_f32 per k-step) accumulates in fp32.  Bias, activation,
// AvgL1Norm, losses, noise and the backward's act' are fused epilogues; the
// backward chains (dX) run in the same launch and leave the per-layer
// gradient operands dP = dY act'(Y) (and the layer inputs X) transposed in
// HBM for one grouped weight-gradient launch (td7_fused_wgrad).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "exo_amd.h"
#include "philox.h"

namespace td7f {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Global-memory accesses through address-space-1 pointers: pointers read from
// the argument structs are generic, and a generic access compiles to a FLAT
// instruction, which counts against the LDS counter too -- every LDS wait would
// then also wait for every weight load in flight.
template <typename T>
__device__ __forceinline__ T ldg(const T *p) {
    return *(const __attribute__((address_space(1))) T *)p;
}
template <typename T>
__device__ __forceinline__ void stg(T *p, T v) {
    *(__attribute__((address_space(1))) T *)p = v;
}

constexpr int NW = 4;            // waves of one k-group: output tile t goes to wave t % NW
constexpr int NKG = 2;           // k-groups: each gemm's k-steps are split over NKG sets of NW waves
constexpr int NTH = 64 * NW * NKG;  // threads per workgroup (2 waves per SIMD)
constexpr int PD = TD7F_PD;    // k-steps of weight loads in flight per wave (k-steps are padded to multiples)
constexpr int TR = 16;         // rows of one MFMA row tile

enum Prec : int { PREC_BF16 = 1, PREC_F16 = 2, PREC_F32 = 3 };
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2, ACT_TANH = 3 };

// The MFMA operand type.  Every operand -- a packed weight block, a k-step of
// an LDS image row, a weight-gradient fragment -- is 16 bytes per lane and 64
// bytes per row per k-step whatever the type: 32 16-bit values (one
// v_mfma_f32_16x16x32_{bf16,f16}) or 16 fp32 values (SUB = 4 chained
// v_mfma_f32_16x16x4_f32, lane l's k = 4 (l >> 4) + j in sub-step j: the same
// k-permutation on both operands, so the sum is over the same 16 products).
// Image geometry is kept in 16-bit units (R16.ld), an fp32 element being two
// of them, so the GEMM core and the LDS layout code are shared.
template <int P> struct Ty;
struct Ty16 {
    using E = uint16_t;
    static constexpr int EB = 2, KD = 32, SUB = 1;
};
template <> struct Ty<PREC_BF16> : Ty16 {
    static __device__ __forceinline__ floatx4 mfma(u32x4 a, u32x4 b, floatx4 c, int = 0) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
    }
    static __device__ __forceinline__ uint16_t bits(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }
    static __device__ __forceinline__ float val(uint16_t b) { return (float)__builtin_bit_cast(__bf16, b); }
    // gradient operands are rounded unscaled (bf16 has fp32's exponent range)
    static constexpr float gs = 1.f;
};
template <> struct Ty<PREC_F16> : Ty16 {
    static __device__ __forceinline__ floatx4 mfma(u32x4 a, u32x4 b, floatx4 c, int = 0) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8, a), __builtin_bit_cast(halfx8, b), c,
                                                      0, 0, 0);
    }
    static __device__ __forceinline__ uint16_t bits(float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }
    static __device__ __forceinline__ float val(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
    // fp16 gradient operands dP are multiplied by 2^10 before rounding (the
    // td7_dense convention, td7_dense_kernels.h grad_scale) and the
    // accumulators by 2^-10 after: exact, keeps ~1e-6 gradients normal
    static constexpr float gs = 1024.f;
};
// fp32 operands (the reference's precision, Agent/TD7_multi_agent.py:211-293):
// exact products, fp32 accumulation; sub-step j of a 16-deep k-step
template <> struct Ty<PREC_F32> {
    using E = float;
    static constexpr int EB = 4, KD = 16, SUB = 4;
    // (the vectors are bit-cast whole, then indexed: bit_cast(float, a[j]) of a
    // u32x4 element compiled to a[0] for every j -- tools/mfma_f32_probe.hip)
    static __device__ __forceinline__ floatx4 mfma(u32x4 a, u32x4 b, floatx4 c, int j) {
        const floatx4 af = __builtin_bit_cast(floatx4, a), bf = __builtin_bit_cast(floatx4, b);
        return __builtin_amdgcn_mfma_f32_16x16x4f32(af[j], bf[j], c, 0, 0, 0);
    }
    static __device__ __forceinline__ float bits(float v) { return v; }
    static __device__ __forceinline__ float val(float b) { return b; }
    static constexpr float gs = 1.f;
};

// ELU's negative branch as exp(x) - 1 (v_exp_f32): within ~1e-7 of expm1f,
// four orders below the 16-bit rounding every activation then takes; the
// per-element epilogue cost matters here (every layer's epilogue runs it)
__device__ __forceinline__ float act_fwd(int act, float x) {
    if (act == ACT_RELU) return x > 0.f ? x : 0.f;
    if (act == ACT_ELU) return x > 0.f ? x : __expf(x) - 1.0f;
    if (act == ACT_TANH) return tanhf(x);
    return x;
}
// act'(x) through the output y (td7_dense_kernels.h act_grad_t)
__device__ __forceinline__ float act_grad(int act, float y) {
    if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
    if (act == ACT_ELU) return y > 0.f ? 1.f : y + 1.f;
    if (act == ACT_TANH) return 1.f - y * y;
    return 1.f;
}

// One linear layer's packed operands (td7_pack_weights):
//   wf: forward B operand of Y = X W^T, block (t, s) = tile t of 16 output
//       columns, k-step s of 32 inputs: lane l holds W[16t + (l&15)][32s + 8(l>>4) + j], j < 8
//       at wf[(t * ksf + s) * 64 + l]; zero outside [N, K).
//   wb: backward B operand of dX = dP W, block (t, s) = tile t of 16 input
//       columns, k-step s of 32 outputs: lane l holds W[32s + 8(l>>4) + j][16t + (l&15)].
// ksf, ksb are padded to multiples of PD; tiles to multiples of NW (zeros).
struct Lin {
    const u32x4 *wf, *wb;
    const float *b;
    int N, K, ksf, ksb;
    const float *w;  // fp32 master [N][K] (row stride ldw), for the thin products
    long ldw;
};

// ---------------------------------------------------------------- GEMM core
// One MFMA GEMM of a fused layer computes, for the workgroup's rows, the
// TRANSPOSED product  C^T[n][row] = sum_k W'[n][k] X[row][k]  with the packed
// weight fragment as the MFMA's A operand and the 16-bit LDS image of X as B,
// so that a lane ends up with 4 CONSECUTIVE output columns of one row
// (row = (lane & 15) + 16 r, cols 16 t + 4 (lane >> 4) + e): the epilogue
// loads biases / saved activations as 16-byte vectors and writes 8-byte
// (16-bit x 4) or 16-byte (fp32 x 4) LDS stores.
//
// Work split: output tile t (16 columns) of the NW * TH tiles from t0 goes to
// wave t % NW of each k-group; the k-steps are split over the NKG = 2 k-groups
// (multiples of PD each).  After the k-loop the groups exchange partial sums
// through the LDS area at offset 0 so that group 0 finishes tiles i < (TH+1)/2
// of each wave and group 1 the rest -- both halves of the workgroup run the
// epilogue.
//
// Weight stream: each wave keeps PD k-steps x TH tiles of 16-byte loads in
// flight in a register ring that persists across layers: the tail of a GEMM
// refills the ring with the first PD k-steps of the NEXT layer's weights, so
// they load during this layer's epilogue and barrier.  Issue order is pinned
// with scheduling barriers (loads in consumption order keep s_waitcnt at
// vmcnt(20..24)).  The X fragment is read from LDS one k-step ahead.
struct GDesc {
    const u32x4 *wp;  // packed operand (forward wf or dX wb)
    int ks;           // k-steps (multiple of PD)
    int t0;           // first output tile
};

__device__ __forceinline__ void kgroup_range(int ks, int kg, int &kb, int &ke) {
    const int kA = ks >= 2 * PD ? ((ks / 2 + PD - 1) / PD) * PD : ks;
    kb = kg ? kA : 0;
    ke = kg ? ks : kA;
}

template <int TH>
__device__ __forceinline__ void ring_fill(u32x4 (&R)[PD][TH], const GDesc &g) {
    const int wv = threadIdx.x >> 6, w = wv % NW, kg = wv / NW, lane = threadIdx.x & 63;
    int kb, ke;
    kgroup_range(g.ks, kg, kb, ke);
    // a k-group with no k-steps of g reloads the first fragment instead of
    // skipping: the loads stay unconditional, so s_waitcnt counts stay exact for
    // the loads issued before the ring (kernel-start staging)
    const bool live = ke > kb;
#pragma unroll
    for (int p = 0; p < PD; ++p)
#pragma unroll
        for (int i = 0; i < TH; ++i) {
            R[p][i] = ldg(g.wp + (live ? ((size_t)(g.t0 + w + NW * i) * g.ks + kb + p) * 64 : 0) + lane);
            __builtin_amdgcn_sched_barrier(0);
        }
}

// acc[r][i] (tile t0 + w + NW i) over the rows 16r..16r+15 of the image at a_off.
// Every thread of the workgroup calls it (one barrier).  The ring must hold g's
// first PD k-steps (ring_fill or the previous gemm's `next`).
// Epilogue operands loaded BEFORE the k-loop (vmcnt is in issue order: loaded
// after the tail's prefetch of the next layer, they would wait for all of it):
// ep[r][i] = vector at (col of slot i) of the bias (per column, r ignored) or of
// a saved fp32 activation y[(row0 + row) * yld + col - c0] (per row).
struct EpiSrc {
    const float *p;  // null: none
    long ld;         // 0: a bias row (same for every row); else row stride
    int c0, row0, nrows, ncols;
};
template <int RT, int TH>
__device__ __forceinline__ void epi_prefetch(const EpiSrc &e, int t0, floatx4 (&ep)[RT][TH]) {
#pragma unroll
    for (int i = 0; i < TH; ++i) {
        const int wv = threadIdx.x >> 6;
        const int col = 16 * (t0 + wv % NW + NW * i) + 4 * ((threadIdx.x & 63) >> 4) - e.c0;
        const bool mine = (i < (TH + 1) / 2) == (wv < NW);
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = (threadIdx.x & 15) + TR * r;
            const bool ok = e.p && mine && col >= 0 && col < e.ncols && (e.ld == 0 || e.row0 + row < e.nrows);
            ep[r][i] = ok ? ldg((const floatx4 *)(e.p + (e.ld ? (long)(e.row0 + row) * e.ld : 0) + col))
                          : floatx4{0.f, 0.f, 0.f, 0.f};
        }
    }
}

template <int P, int RT, int TH>
__device__ __forceinline__ void gemm(char *lds, int a_off, int lda, const GDesc &g, u32x4 (&R)[PD][TH],
                                     floatx4 (&acc)[RT][TH], const GDesc *next, const EpiSrc &es,
                                     floatx4 (&ep)[RT][TH]) {
    const int wv = threadIdx.x >> 6, w = wv % NW, kg = wv / NW, lane = threadIdx.x & 63;
    int kb, ke, nb = 0, ne = 0;
    kgroup_range(g.ks, kg, kb, ke);
    if (next) kgroup_range(next->ks, kg, nb, ne);
    epi_prefetch(es, g.t0, ep);
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int i = 0; i < TH; ++i) acc[r][i] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (ke > kb) {
        const u32x4 *bp[TH];
#pragma unroll
        for (int i = 0; i < TH; ++i) bp[i] = g.wp + ((size_t)(g.t0 + w + NW * i) * g.ks + kb) * 64 + lane;
        const char *ap = lds + a_off + ((lane & 15) * lda + 8 * (lane >> 4) + 32 * kb) * 2;
        const int n = ke - kb;
        u32x4 an[RT];
#pragma unroll
        for (int r = 0; r < RT; ++r) an[r] = *(const u32x4 *)(ap + r * TR * lda * 2);
        int s0 = 0;
        for (; s0 + PD < n; s0 += PD) {
#pragma unroll
            for (int p = 0; p < PD; ++p) {
                const int s = s0 + p;
                u32x4 x[RT];
#pragma unroll
                for (int r = 0; r < RT; ++r) {
                    x[r] = an[r];
                    an[r] = *(const u32x4 *)(ap + (r * TR * lda + 32 * (s + 1)) * 2);
                }
#pragma unroll
                for (int j = 0; j < Ty<P>::SUB; ++j)
#pragma unroll
                    for (int i = 0; i < TH; ++i) {
#pragma unroll
                        for (int r = 0; r < RT; ++r) acc[r][i] = Ty<P>::mfma(R[p][i], x[r], acc[r][i], j);
                        __builtin_amdgcn_sched_barrier(0);
                    }
#pragma unroll
                for (int i = 0; i < TH; ++i) {
                    R[p][i] = ldg(bp[i] + (s + PD) * 64);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        const u32x4 *np[TH];
        if (ne > nb)
#pragma unroll
            for (int i = 0; i < TH; ++i) np[i] = next->wp + ((size_t)(next->t0 + w + NW * i) * next->ks + nb) * 64 + lane;
#pragma unroll
        for (int p = 0; p < PD; ++p) {
            const int s = s0 + p;
            u32x4 x[RT];
#pragma unroll
            for (int r = 0; r < RT; ++r) {
                x[r] = an[r];
                if (p + 1 < PD) an[r] = *(const u32x4 *)(ap + (r * TR * lda + 32 * (s + 1)) * 2);
            }
#pragma unroll
            for (int j = 0; j < Ty<P>::SUB; ++j)
#pragma unroll
                for (int i = 0; i < TH; ++i) {
#pragma unroll
                    for (int r = 0; r < RT; ++r) acc[r][i] = Ty<P>::mfma(R[p][i], x[r], acc[r][i], j);
                    __builtin_amdgcn_sched_barrier(0);
                }
            if (ne > nb) {
#pragma unroll
                for (int i = 0; i < TH; ++i) {
                    R[p][i] = ldg(np[i] + p * 64);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    } else if (next) {
        ring_fill(R, *next);
    }
    // exchange: group 0 keeps tiles i < h, group 1 tiles i >= h
    constexpr int h = (TH + 1) / 2;
    floatx4 *red = (floatx4 *)lds + ((w * 64 + lane) * RT) * TH;
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int i = 0; i < TH; ++i)
            if ((i < h) != (kg == 0)) red[r * TH + i] = acc[r][i];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int i = 0; i < TH; ++i)
            if ((i < h) == (kg == 0)) acc[r][i] += red[r * TH + i];
}

// bytes of the LDS exchange area gemm uses (offset 0 of every fused kernel)
constexpr int red_bytes(int rt, int tpw) { return NW * 64 * rt * tpw * 16; }

// This wave finishes tile slot i (see gemm); its columns and row.
template <int TH>
__device__ __forceinline__ bool owns(int i) {
    return (i < (TH + 1) / 2) == ((threadIdx.x >> 6) < NW);
}
__device__ __forceinline__ int acc_col(int t0, int i) {
    const int wv = threadIdx.x >> 6;
    return 16 * (t0 + wv % NW + NW * i) + 4 * ((threadIdx.x & 63) >> 4);
}
__device__ __forceinline__ int acc_row(int r) { return (threadIdx.x & 15) + TR * r; }

// LDS regions: 16-bit operand images [rows][ld] and fp32 scratch [rows][ld].
struct R16 {
    int off, ld;
};
struct R32 {
    int off, ld;
};
constexpr R16 NO16{-1, 0};
constexpr R32 NO32{-1, 0};
__device__ __forceinline__ uint16_t *p16(char *lds, R16 r, int row, int col) {
    return (uint16_t *)(lds + r.off) + row * r.ld + col;
}
__device__ __forceinline__ float *p32(char *lds, R32 r, int row, int col) {
    return (float *)(lds + r.off) + row * r.ld + col;
}
template <int P>
__device__ __forceinline__ u32x2 pack4(const float (&v)[4]) {
    return u32x2{(uint32_t)Ty<P>::bits(v[0]) | ((uint32_t)Ty<P>::bits(v[1]) << 16),
                 (uint32_t)Ty<P>::bits(v[2]) | ((uint32_t)Ty<P>::bits(v[3]) << 16)};
}
// element `col` of row `row` of an operand image (R16.ld in 16-bit units)
template <int P>
__device__ __forceinline__ typename Ty<P>::E *pe(char *lds, R16 r, int row, int col) {
    return (typename Ty<P>::E *)(lds + r.off + row * r.ld * 2) + col;
}
// 4 consecutive elements (col % 4 == 0): one 8-byte (16-bit) or 16-byte (fp32) LDS store
template <int P>
__device__ __forceinline__ void put4(char *lds, R16 r, int row, int col, const float (&v)[4]) {
    if constexpr (Ty<P>::EB == 4) *(floatx4 *)pe<P>(lds, r, row, col) = floatx4{v[0], v[1], v[2], v[3]};
    else *(u32x2 *)pe<P>(lds, r, row, col) = pack4<P>(v);
}

// Forward epilogue of an MFMA layer (N % 4 == 0): v = act(acc + b) for the
// owned columns n < N, written to any of: 16-bit LDS image (column col0 + n),
// fp32 LDS region, global fp32 [row0+row][n] (rows < nrows).
template <int P, int RT, int TH>
__device__ __forceinline__ void epi_fwd(char *lds, const floatx4 (&acc)[RT][TH], const floatx4 (&bias)[RT][TH], int N,
                                        int act, R16 o16, int col0, R32 o32, float *g, long gld, int row0,
                                        int nrows) {
#pragma unroll
    for (int i = 0; i < TH; ++i) {
        if (!owns<TH>(i)) continue;
        const int n = acc_col(0, i);
        if (n >= N) continue;
        const floatx4 b = bias[0][i];
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = acc_row(r);
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = act_fwd(act, acc[r][i][e] + b[e]);
            if (o16.off >= 0) put4<P>(lds, o16, row, col0 + n, v);
            if (o32.off >= 0) *(floatx4 *)p32(lds, o32, row, n) = floatx4{v[0], v[1], v[2], v[3]};
            if (g && row0 + row < nrows) stg((floatx4 *)(g + (long)(row0 + row) * gld + n), floatx4{v[0], v[1], v[2], v[3]});
        }
    }
}

// Backward epilogue of dX = dP W' over the input-column window [c0, c1)
// (c0, c1 multiples of 4; output tiles from t0 = c0 / 16): v = acc / gs at
// window column m = col - c0; v *= act'(Y) with Y read as 16-byte vectors from
// global fp32 y[(row0+row) * yld + m] when act != ACT_NONE.  Rows >= nrows give
// 0.  Outputs: fp32 LDS region [row][m], global fp32 [row0+row][m], and for a
// gradient operand dP: the 16-bit LDS image (x gs) and the fp32 column sums of
// the rows (bias-gradient partials part[m], written by lanes 0..3 of a column group).
template <int P, int RT, int TH>
__device__ __forceinline__ void epi_bwd(char *lds, const floatx4 (&acc)[RT][TH], int t0, int c0, int c1, int act,
                                        const floatx4 (&yv_)[RT][TH], R32 o32, float *g, long gld, R16 o16,
                                        float *part, int row0, int nrows) {
#pragma unroll
    for (int i = 0; i < TH; ++i) {
        if (!owns<TH>(i)) continue;
        const int col = acc_col(t0, i);
        const bool in = col >= c0 && col < c1;
        const int m = col - c0;
        float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = acc_row(r);
            const bool live = in && row0 + row < nrows;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = live ? acc[r][i][e] * (1.f / Ty<P>::gs) : 0.f;
            if (live && act != ACT_NONE) {
                const floatx4 yv = yv_[r][i];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] *= act_grad(act, yv[e]);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) cs[e] += v[e];
            if (in) {
                if (o32.off >= 0) *(floatx4 *)p32(lds, o32, row, m) = floatx4{v[0], v[1], v[2], v[3]};
                if (o16.off >= 0) {
                    float s[4] = {v[0] * Ty<P>::gs, v[1] * Ty<P>::gs, v[2] * Ty<P>::gs, v[3] * Ty<P>::gs};
                    put4<P>(lds, o16, row, m, s);
                }
                if (g && row0 + row < nrows) stg((floatx4 *)(g + (long)(row0 + row) * gld + m), floatx4{v[0], v[1], v[2], v[3]});
            }
        }
        if (part) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) cs[e] += __shfl_xor(cs[e], o, 64);
            if (in && (threadIdx.x & 15) == 0) stg((floatx4 *)(part + m), floatx4{cs[0], cs[1], cs[2], cs[3]});
        }
    }
}

// Thin GEMMs on the VALU (an output width or a reduction too narrow for a
// 16-wide MFMA tile: the N = 1 / 7 heads, the 7-wide action windows of the
// backward), their weight slices staged in LDS at kernel start (thin_issue /
// thin_put), rounded to the MFMA operand type.
// out[row][j] = scale * sum_{k < K} X[row][xc0 + k] wl[j][k] for j < ncols <= NC
// (raw sums to the fp32 LDS region out; wl holds NC rows, zero past ncols),
// 16 rows: one pass, a thread per (row, k-slice of NTH / 16) accumulating all
// NC outputs of its row in registers (no per-column branches: every LDS read of
// a step is in flight at once), then reduced over the slices by shuffles.
template <int P, int NC>
__device__ __forceinline__ void thin(char *lds, R16 in, int xc0, int K, R32 wl, int ncols, R32 out, float scale) {
    constexpr int KS = NTH / TR;
    const int row = threadIdx.x / KS, sl = threadIdx.x % KS;
    float acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[j] = 0.f;
#pragma unroll 2
    for (int k = sl; k < K; k += KS) {
        const float x = Ty<P>::val(*pe<P>(lds, in, row, xc0 + k));
#pragma unroll
        for (int j = 0; j < NC; ++j) acc[j] += x * *p32(lds, wl, j, k);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
#pragma unroll
        for (int o = KS / 2; o > 0; o >>= 1) acc[j] += __shfl_xor(acc[j], o, 64);
    }
    if (sl == 0)
#pragma unroll
        for (int j = 0; j < NC; ++j)
            if (j < ncols) *p32(lds, out, row, j) = acc[j] * scale;
}
constexpr int THIN_NC = 8;  // action width <= 8 (7 here); the Q heads use 1

// Gradient operand dP from an fp32 LDS region dy [16][0..N) (thin layers and
// the loss gradients): dP = dy act'(Y) (Y from global fp32 y[(row0+row)*yld + n]
// when act != ACT_NONE), rows >= nrows zero; written as the 16-bit image (x gs,
// columns 0..N), its fp32 column sums part[n] and (fp32) back into dy.
template <int P>
__device__ __forceinline__ void make_dp(char *lds, R32 dy, int N, int act, const float *y, long yld, R16 o16,
                                        float *part, int row0, int nrows) {
    for (int n = threadIdx.x; n < N; n += NTH) {
        float cs = 0.f;
        for (int r = 0; r < TR; ++r) {
            float v = *p32(lds, dy, r, n);
            if (row0 + r >= nrows) v = 0.f;
            else if (act != ACT_NONE) v *= act_grad(act, ldg(y + (long)(row0 + r) * yld + n));
            *p32(lds, dy, r, n) = v;
            *pe<P>(lds, o16, r, n) = Ty<P>::bits(v * Ty<P>::gs);
            cs += v;
        }
        if (part) stg(part + n, cs);
    }
}

// 16-bit LDS image rows -> global [row0+row][c] (same element type)
__device__ __forceinline__ void store_rows16(char *lds, R16 src, int col0, uint16_t *dst, long dld, int ncols,
                                             int rows, int row0, int nrows) {
    if (ncols % 8 == 0 && dld % 8 == 0 && col0 % 8 == 0 && src.ld % 8 == 0) {
        const int nq = ncols / 8;
        for (int k = threadIdx.x; k < rows * nq; k += NTH) {
            const int row = k / nq, c = 8 * (k - row * nq);
            if (row0 + row < nrows) stg((u32x4 *)(dst + (long)(row0 + row) * dld + c), *(const u32x4 *)p16(lds, src, row, col0 + c));
        }
        return;
    }
    for (int k = threadIdx.x; k < rows * ncols; k += NTH) {
        const int row = k / ncols, c = k - row * ncols;
        if (row0 + row < nrows) stg(dst + (long)(row0 + row) * dld + c, *p16(lds, src, row, col0 + c));
    }
}

// ---------------------------------------------------------------- kernel-start staging
// A kernel's inputs go global -> registers -> LDS in two phases, so that every
// load of its start (input rows, thin weights, the first layer's ring) is in
// flight at once: *_issue() loads without a branch (addresses clamped in
// bounds, values masked at the store), *_put() stores after zero_lds's barrier.
// (A load-then-store loop waits one full global latency per element.)
// RowStage: column c = threadIdx.x (< ncols <= NTH) of the 16 rows.
struct RowStage {
    float v[TR];
};
__device__ __forceinline__ void row_issue(RowStage &s, const float *src, long sld, int ncols, int row0, int nrows) {
    const int c = min((int)threadIdx.x, ncols - 1);
#pragma unroll
    for (int r = 0; r < TR; ++r) s.v[r] = ldg(src + (long)(row0 + r < nrows ? row0 + r : row0) * sld + c);
}
__device__ __forceinline__ void row_add(RowStage &s, const RowStage &o) {
#pragma unroll
    for (int r = 0; r < TR; ++r) s.v[r] += o.v[r];
}
// -> 16-bit image dst[row][col0 + c] (x scale), rows >= nrows zero
template <int P>
__device__ __forceinline__ void row_put16(char *lds, const RowStage &s, R16 dst, int col0, int ncols, int row0,
                                          int nrows, float scale = 1.f) {
    if ((int)threadIdx.x < ncols)
#pragma unroll
        for (int r = 0; r < TR; ++r)
            *pe<P>(lds, dst, r, col0 + threadIdx.x) = Ty<P>::bits(row0 + r < nrows ? s.v[r] * scale : 0.f);
}
__device__ __forceinline__ void row_put32(char *lds, const RowStage &s, R32 dst, int ncols, int row0, int nrows) {
    if ((int)threadIdx.x < ncols)
#pragma unroll
        for (int r = 0; r < TR; ++r) *p32(lds, dst, r, threadIdx.x) = row0 + r < nrows ? s.v[r] : 0.f;
}
// 16-bit rows, column pairs c = 2 threadIdx.x, 2 threadIdx.x + 1 (src and sld even)
struct Row16Stage {
    uint32_t v[TR];
};
__device__ __forceinline__ void row16_issue(Row16Stage &s, const uint16_t *src, long sld, int ncols, int row0,
                                            int nrows) {
    const int c = 2 * min((int)threadIdx.x, (ncols - 1) / 2);
#pragma unroll
    for (int r = 0; r < TR; ++r)
        s.v[r] = ldg((const uint32_t *)(src + (long)(row0 + r < nrows ? row0 + r : row0) * sld + c));
}
__device__ __forceinline__ void row16_put(char *lds, const Row16Stage &s, R16 dst, int col0, int ncols, int row0,
                                          int nrows) {
    const int c = 2 * threadIdx.x;
    if (c < ncols)
#pragma unroll
        for (int r = 0; r < TR; ++r) {
            const uint32_t v = row0 + r < nrows ? s.v[r] : 0u;
            *p16(lds, dst, r, col0 + c) = (uint16_t)(v & 0xffffu);
            if (c + 1 < ncols) *p16(lds, dst, r, col0 + c + 1) = (uint16_t)(v >> 16);
        }
}
// the thin weights (stage_thin's slice) for k = threadIdx.x (< K <= NTH)
template <int NC>
struct ThinStage {
    float v[NC];
};
template <int NC>
__device__ __forceinline__ void thin_issue(ThinStage<NC> &s, const float *W, long ldw, int j0, bool trans, int ncols,
                                           int K) {
    const int k = min((int)threadIdx.x, K - 1);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const int jj = min(j, ncols - 1);
        s.v[j] = ldg(trans ? W + (long)k * ldw + j0 + jj : W + (long)(j0 + jj) * ldw + k);
    }
}
template <int P, int NC>
__device__ __forceinline__ void thin_put(char *lds, const ThinStage<NC> &s, R32 wl, int ncols, int K) {
    if ((int)threadIdx.x < K)
#pragma unroll
        for (int j = 0; j < NC; ++j) *p32(lds, wl, j, threadIdx.x) = j < ncols ? Ty<P>::val(Ty<P>::bits(s.v[j])) : 0.f;
}

// The weight-gradient operands (layer inputs X^T, gradient operands dP^T) are
// stored in MFMA-fragment blocks: operand row c (an input column of X or an
// output column of dP), batch row r lives at
//   ((c / 16) * (ld / 32) + r / 32) * 512 + ((c % 16) + 16 ((r % 32) / 8)) * 8 + r % 8
// (16-bit units, ld = padded batch), so that td7f_wgrad's 16 x 32 fragment of a
// k-step is one contiguous 1 KiB block (one full-line 16-byte load per lane).
// blk8 -> the 8 batch rows r..r+7 (r % 8 == 0) of operand row c.
// fp32 operands: k-steps of 16 batch rows, the 4 rows r..r+3 (r % 4 == 0) of
// operand row c at blk4 (the same 1 KiB block per fragment, 16 bytes per lane).
__device__ __forceinline__ uint16_t *blk8(uint16_t *base, long ld, int c, int r) {
    return base + ((long)(c >> 4) * (ld >> 5) + (r >> 5)) * 512 + ((c & 15) + 16 * ((r & 31) >> 3)) * 8;
}
__device__ __forceinline__ float *blk4(float *base, long ld, int c, int r) {
    return base + ((long)(c >> 4) * (ld >> 4) + (r >> 4)) * 256 + ((c & 15) + 16 * ((r & 15) >> 2)) * 4;
}

// The layer input for the weight gradient from the LDS image (columns col0 + c,
// c < ncols), 16 rows per call (row0 % 16 == 0), in the blocked layout above.
template <int P>
__device__ __forceinline__ void save_xt(char *lds, R16 src, int col0, int ncols, void *xt_, long ld, int rows,
                                        int row0) {
    if constexpr (P == PREC_F32) {  // a thread per (column, 16 rows): 4 x 16-byte stores
        float *xt = (float *)xt_;
        for (int k = threadIdx.x; k < ncols * (rows / TR); k += NTH) {
            const int c = k % ncols, rb = (k / ncols) * TR;
            float v[TR];
#pragma unroll
            for (int j = 0; j < TR; ++j) v[j] = *pe<P>(lds, src, rb + j, col0 + c);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                stg((floatx4 *)blk4(xt, ld, c, row0 + rb + 4 * q), floatx4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]});
        }
        return;
    }
    uint16_t *xt = (uint16_t *)xt_;
    if (col0 % 2 == 0 && src.ld % 2 == 0) {  // column pairs: 32-bit LDS reads
        for (int k = threadIdx.x; k < ((ncols + 1) / 2) * (rows / TR); k += NTH) {
            const int c = 2 * (k % ((ncols + 1) / 2)), rb = (k / ((ncols + 1) / 2)) * TR;
            uint32_t lo[8], hi[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t r0 = *(const uint32_t *)p16(lds, src, rb + 2 * j, col0 + c);
                const uint32_t r1 = *(const uint32_t *)p16(lds, src, rb + 2 * j + 1, col0 + c);
                lo[j] = (r0 & 0xffffu) | (r1 << 16);
                hi[j] = (r0 >> 16) | (r1 & 0xffff0000u);
            }
            stg((u32x4 *)blk8(xt, ld, c, row0 + rb), u32x4{lo[0], lo[1], lo[2], lo[3]});
            stg((u32x4 *)blk8(xt, ld, c, row0 + rb + 8), u32x4{lo[4], lo[5], lo[6], lo[7]});
            if (c + 1 < ncols) {
                stg((u32x4 *)blk8(xt, ld, c + 1, row0 + rb), u32x4{hi[0], hi[1], hi[2], hi[3]});
                stg((u32x4 *)blk8(xt, ld, c + 1, row0 + rb + 8), u32x4{hi[4], hi[5], hi[6], hi[7]});
            }
        }
        return;
    }
    for (int k = threadIdx.x; k < ncols * (rows / TR); k += NTH) {
        const int c = k % ncols, rb = (k / ncols) * TR;
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = (uint32_t)*p16(lds, src, rb + 2 * j, col0 + c) |
                   ((uint32_t)*p16(lds, src, rb + 2 * j + 1, col0 + c) << 16);
        stg((u32x4 *)blk8(xt, ld, c, row0 + rb), u32x4{v[0], v[1], v[2], v[3]});
        stg((u32x4 *)blk8(xt, ld, c, row0 + rb + 8), u32x4{v[4], v[5], v[6], v[7]});
    }
}

// AvgL1Norm forward (Agent/TD7_multi_agent.py:53-54) of the fp32 rows h[row][0..N):
// m = mean|h|, y = h / max(m, eps) written as 16-bit at o16 (column col0 + n)
// and at o16b (column col0b + n) when its offset is >= 0, optionally fp32 to
// global g[(row0+row)*gld + n]; the mean to mean_lds[row] (LDS fp32, may be
// null) and to global gmean[row0 + row] (may be null).
template <int P>
__device__ __forceinline__ void norm_fwd(char *lds, R32 h, int N, int rows, float eps, R16 o16, int col0, R16 o16b,
                                         int col0b, R32 o32, float *g, long gld, float *mean_lds, float *gmean,
                                         int row0, int nrows) {
    const int tpr = NTH / rows;  // threads per row (16 at 16 rows, 8 at 32)
    const int row = threadIdx.x / tpr, j0 = threadIdx.x % tpr;
    float acc = 0.f;
    for (int n = j0; n < N; n += tpr) acc += fabsf(*p32(lds, h, row, n));
    for (int o = tpr / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    const float m = acc / N, s = fmaxf(m, eps);
    for (int n = j0; n < N; n += tpr) {
        const float v = *p32(lds, h, row, n) / s;
        const auto b = Ty<P>::bits(v);
        if (o16.off >= 0) *pe<P>(lds, o16, row, col0 + n) = b;
        if (o16b.off >= 0) *pe<P>(lds, o16b, row, col0b + n) = b;
        if (o32.off >= 0) *p32(lds, o32, row, n) = v;
        if (g && row0 + row < nrows) stg(g + (long)(row0 + row) * gld + n, v);
    }
    if (j0 == 0) {
        if (mean_lds) mean_lds[row] = m;
        if (gmean && row0 + row < nrows) stg(gmean + row0 + row, m);
    }
}

// AvgL1Norm backward (td7_ops.hip avgl1_bwd_kernel) of dy (fp32 LDS [16][N])
// given the pre-norm h (fp32 LDS) and the row means; the result is the layer's
// gradient operand dP (no activation before a norm): 16-bit LDS image (x gs),
// dP^T in HBM and the bias-gradient column partials.  16 rows.
template <int P>
__device__ __forceinline__ void norm_bwd(char *lds, R32 dy, R32 h, const float *mean, int N, float eps, float *dot,
                                         R16 o16, void *dpt, long dpt_ld, float *part, int row0, int nrows) {
    {
        constexpr int tpr = NTH / TR;
        const int row = threadIdx.x / tpr, j0 = threadIdx.x % tpr;
        float acc = 0.f;
        for (int n = j0; n < N; n += tpr) acc += *p32(lds, dy, row, n) * *p32(lds, h, row, n);
        for (int o = tpr / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if (j0 == 0) dot[row] = acc;
    }
    __syncthreads();
    for (int n = threadIdx.x; n < N; n += NTH) {
        float csum = 0.f;
        uint32_t v[8];
        float f[TR];
#pragma unroll
        for (int r = 0; r < TR; ++r) {
            const float m = mean[r];
            float gx;
            if (m >= eps) {
                const float inv = 1.0f / m, c = dot[r] * inv * inv / N;
                const float xv = *p32(lds, h, r, n);
                const float sg = (xv > 0.f) ? 1.f : ((xv < 0.f) ? -1.f : 0.f);
                gx = *p32(lds, dy, r, n) * inv - sg * c;
            } else {
                gx = *p32(lds, dy, r, n) / eps;
            }
            if (row0 + r >= nrows) gx = 0.f;
            csum += gx;
            const auto hb = Ty<P>::bits(gx * Ty<P>::gs);
            *pe<P>(lds, o16, r, n) = hb;
            if constexpr (P == PREC_F32) {
                f[r] = hb;
            } else {
                if (r & 1) v[r >> 1] |= (uint32_t)hb << 16;
                else v[r >> 1] = hb;
            }
        }
        if (dpt) {
            if constexpr (P == PREC_F32) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    stg((floatx4 *)blk4((float *)dpt, dpt_ld, n, row0 + 4 * q), floatx4{f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]});
            } else {
                stg((u32x4 *)blk8((uint16_t *)dpt, dpt_ld, n, row0), u32x4{v[0], v[1], v[2], v[3]});
                stg((u32x4 *)blk8((uint16_t *)dpt, dpt_ld, n, row0 + 8), u32x4{v[4], v[5], v[6], v[7]});
            }
        }
        if (part) stg(part + n, csum);
    }
}

// Gaussian noise on the [rows][7] fp32 actions a (td7_loss.hip
// noisy_action_rng_kernel, element-for-element): element i = (row0+row)*A + c
// of the whole [n_rows, A] tensor takes normal i%2 of Philox block i/2 of
// call *counter of the stream (seed, tag); out = clamp(a + c(z sigma), -1, 1) * scale
// with c = clamp(+-clip) when clip > 0.  The last workgroup to pass advances
// sigma by -sigma_dec and the call counter (ticket), as that kernel does.
struct Noise {
    uint64_t seed;
    uint32_t tag;
    unsigned long long *counter;
    uint32_t *ticket;
    float *sigma;
    float sigma_dec, clip, scale;
    const float *z;  // given standard normals (null: Philox)
    const int32_t *dec_count;  // non-null: sigma -= sigma_dec * *dec_count (active envs of the step)
};

// ---------------------------------------------------------------- stamps
// Diagnostic build only (make stamps -> libexo_amd_stamps.so): s_memtime at the
// phase boundaries of every fused layer, wave 0 of each workgroup, into
// g_td7f_stamps[block * 64 + k]; the product build compiles them out.
#ifdef EXO_STAMPS
static __device__ unsigned long long *g_td7f_stamps;  // per translation unit
#define FSTAMP(si)                                                                                 \
    do {                                                                                           \
        unsigned long long _t;                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        if (g_td7f_stamps && threadIdx.x == 0 && (si) < 64)                                        \
            stg(g_td7f_stamps + (size_t)(blockIdx.x + blockIdx.y * gridDim.x) * 64 + (si), _t);    \
        ++(si);                                                                                    \
    } while (0)
#else
#define FSTAMP(si) do {} while (0)
#endif

// ---------------------------------------------------------------- layers

// One forward MFMA Linear: gemm over the image `a` (the ring holds its first
// k-steps) + epilogue; `next` = the next MFMA layer of the pass (its weights
// start loading in this layer's tail).  Ends with a barrier.
template <int P, int RT, int TH>
__device__ __forceinline__ void layer_fwd(char *lds, u32x4 (&R)[PD][TH], R16 a, const Lin &L, const GDesc *next,
                                          int act, R16 o16, int col0, R32 o32, float *g, long gld, int row0,
                                          int nrows, int &si) {
    FSTAMP(si);
    floatx4 acc[RT][TH], bias[RT][TH];
    const GDesc gd{L.wf, L.ksf, 0};
    gemm<P, RT, TH>(lds, a.off, a.ld, gd, R, acc, next, EpiSrc{L.b, 0, 0, 0, 0, L.N}, bias);
    FSTAMP(si);
    epi_fwd<P, RT, TH>(lds, acc, bias, L.N, act, o16, col0, o32, g, gld, row0, nrows);
    __syncthreads();
}
// ... with the next layer's forward operand as `next`
template <int P, int RT, int TH>
__device__ __forceinline__ void layer_fwd(char *lds, u32x4 (&R)[PD][TH], R16 a, const Lin &L, const Lin *next, int act,
                                          R16 o16, int col0, R32 o32, float *g, long gld, int row0, int nrows,
                                          int &si) {
    GDesc gn{nullptr, 0, 0};
    if (next) gn = GDesc{next->wf, next->ksf, 0};
    layer_fwd<P, RT, TH>(lds, R, a, L, next ? &gn : (const GDesc *)nullptr, act, o16, col0, o32, g, gld, row0, nrows,
                         si);
}

// A thin forward Linear (N <= 16) on the VALU: out[row][n] = act(x W^T + b) in
// the fp32 region `out` (and global g when not null).  Ends with a barrier.
template <int P, int NC>
__device__ __forceinline__ void layer_thin_fwd(char *lds, R16 a, const Lin &L, R32 wl, int act, R32 out, int rows,
                                               float *g, long gld, int row0, int nrows, int &si) {
    FSTAMP(si);
    thin<P, NC>(lds, a, 0, L.K, wl, L.N, out, 1.f);
    __syncthreads();
    for (int k = threadIdx.x; k < rows * L.N; k += NTH) {
        const int row = k / L.N, n = k - row * L.N;
        const float v = act_fwd(act, *p32(lds, out, row, n) + ldg(L.b + n));
        *p32(lds, out, row, n) = v;
        if (g && row0 + row < nrows) stg(g + (long)(row0 + row) * gld + n, v);
    }
    __syncthreads();
}

__device__ __forceinline__ void zero_lds(char *lds, int bytes) {
    for (int i = threadIdx.x * 16; i < bytes; i += NTH * 16) *(u32x4 *)(lds + i) = u32x4{0u, 0u, 0u, 0u};
}

// Gaussian noise on the fp32 actions a[row][0..A) (see Noise); results to
// global out[(row0+row)*A + c] (may be null) and 16-bit images o1 / o2 at
// columns c1 / c2 (offsets < 0: none).  Ends with the ticket of the last
// workgroup, which advances sigma and the call counter.
template <int P>
__device__ __forceinline__ void noise_rows(char *lds, R32 a, int A, int rows, int row0, int nrows, const Noise &nz,
                                           float *out, R16 o1, int c1, R16 o2, int c2, bool ticket = true) {
    const float sg = ldg(nz.sigma);
    const unsigned long long call = ldg(nz.counter);
    for (int k = threadIdx.x; k < rows * A; k += NTH) {
        const int row = k / A, c = k - row * A;
        float v = 0.f;
        if (row0 + row < nrows) {
            const uint32_t i = (uint32_t)((row0 + row) * A + c);
            float z;
            if (nz.z) {
                z = ldg(nz.z + i);
            } else {
                uint32_t r[4];
                philox_block(nz.seed, nz.tag, call, i >> 1, r);
                float z0, z1;
                box_muller(r, z0, z1);
                z = (i & 1) ? z1 : z0;
            }
            float e = z * sg;
            if (nz.clip > 0.f) e = fminf(fmaxf(e, -nz.clip), nz.clip);
            v = fminf(fmaxf(*p32(lds, a, row, c) + e, -1.0f), 1.0f) * nz.scale;
            if (out) stg(out + i, v);
        }
        const auto b = Ty<P>::bits(v);
        if (o1.off >= 0) *pe<P>(lds, o1, row, c1 + c) = b;
        if (o2.off >= 0) *pe<P>(lds, o2, row, c2 + c) = b;
    }
    __syncthreads();
    if (ticket && threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(nz.ticket, 1u) == gridDim.x * gridDim.y - 1) {
            *nz.sigma = sg - (nz.dec_count ? nz.sigma_dec * (float)*nz.dec_count : nz.sigma_dec);
            if (!nz.z) *nz.counter = call + 1ull;
            *nz.ticket = 0u;
        }
    }
}

// ---------------------------------------------------------------- host helpers
inline int round_up(int x, int m) { return (x + m - 1) / m * m; }
// k per k-step of the operand type (Ty<P>::KD)
inline int kd_of(int prec) { return prec == PREC_F32 ? 16 : 32; }
inline int ks_of(int k, int kd = 32) { return round_up((k + kd - 1) / kd, PD); }
// operand image of an n-wide input in 16-bit units (64 bytes per k-step the
// gemm reads, +32 bytes of bank spread)
inline int ld16(int n, int kd = 32) { return ks_of(n, kd) * 32 + 16; }

struct Bump {
    int off;
    explicit Bump(int rt) : off(red_bytes(rt, 5)) {}  // gemm's reduction area at offset 0
    R16 r16(int rows, int ld) {
        R16 r{off, ld};
        off += round_up(rows * ld * 2, 16);
        return r;
    }
    R32 r32(int rows, int ld) {
        R32 r{off, ld};
        off += round_up(rows * ld * 4, 16);
        return r;
    }
};

inline Lin lin_of(const td7f_lin &l) {
    return Lin{(const u32x4 *)l.wf, (const u32x4 *)l.wb, l.b, l.n_out, l.n_in, l.ksf, l.ksb, l.w, (long)l.ldw};
}
inline Noise noise_of(const td7f_noise &n) {
    return Noise{n.seed, n.tag, n.counter, n.ticket, n.sigma, n.sigma_dec, n.clip, n.scale, n.z, n.dec_count};
}

// tiles per wave of the MFMA layers: every layer wider than 16 outputs must be
// a multiple of 4 wide with exactly NW * TH (padded) tiles, TH in {4, 5}
// (widths 196..320 at TH 5, 132..256 at TH 4); layers <= 16 wide run thin
// (VALU) and need the fp32 master weight.
inline int th_of(const td7f_lin *ls, int n) {
    int th = 0;
    for (int i = 0; i < n; ++i) {
        if (!ls[i].wf || ls[i].ksf <= 0 || ls[i].ksf % PD || !ls[i].b) return -1;
        if (ls[i].n_out <= 16) {
            if (!ls[i].w || ls[i].ldw < ls[i].n_in) return -1;
            continue;
        }
        if (ls[i].n_out % 4) return -1;
        const int t = round_up((ls[i].n_out + 15) / 16, NW) / NW;
        if (th && t != th) return -1;
        th = t;
    }
    return th ? th : 4;
}

constexpr int LDS_MAX = 160 * 1024;

// Plan-only mode (td7f_probe, per host thread): launch() checks a pass's LDS
// plan and returns without launching, so the host can test a network shape
// once when it builds the fused passes (exo_amd.fused.FusedNets) instead of
// failing at the first call of a pass whose images do not fit.
extern thread_local bool td7f_probe_mode;

template <typename K, typename A>
int launch(K kernel, dim3 grid, int lds, A args, hipStream_t st) {
    if (lds > LDS_MAX) return EXO_EINVAL;
    if (td7f_probe_mode) return EXO_OK;
    if (hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return EXO_EDEVICE;
    hipLaunchKernelGGL(kernel, grid, dim3(NTH), lds, st, args);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

#define DISPATCH(PREC, TH, KERNEL, ...)                                                                 \
    ((PREC) == PREC_BF16  ? ((TH) == 5 ? launch(KERNEL<PREC_BF16, 5>, __VA_ARGS__)                      \
                                       : launch(KERNEL<PREC_BF16, 4>, __VA_ARGS__))                     \
     : (PREC) == PREC_F16 ? ((TH) == 5 ? launch(KERNEL<PREC_F16, 5>, __VA_ARGS__)                       \
                                       : launch(KERNEL<PREC_F16, 4>, __VA_ARGS__))                      \
                          : ((TH) == 5 ? launch(KERNEL<PREC_F32, 5>, __VA_ARGS__)                       \
                                       : launch(KERNEL<PREC_F32, 4>, __VA_ARGS__)))

}  // namespace td7f
