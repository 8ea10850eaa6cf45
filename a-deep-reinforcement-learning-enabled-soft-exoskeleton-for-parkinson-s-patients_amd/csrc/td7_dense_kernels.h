// td7_dense_kernels.h -- the TD7 dense-layer kernels and their per-precision
// launchers (see td7_dense.hip for the design notes).  Each precision's
// launchers are instantiated in their own translation unit
// (td7_dense_{f32,bf16,f16}.hip) so the three compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "exo_amd.h"

namespace td7dense {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
typedef uint32_t uint32_t4 __attribute__((ext_vector_type(4), aligned(4))); // 16-byte global load, dword aligned
typedef const __attribute__((address_space(1))) uint32_t4 *gptr4;

// 16-byte global (not flat) load; lanes with !ok read a valid fallback address
// and return zeros (no exec-mask branch around the load)
__device__ __forceinline__ uint32_t4 gload4(const float *p, const float *fallback, bool ok) {
    const uint32_t4 v = *(gptr4)(ok ? p : fallback);
    return ok ? v : uint32_t4{0u, 0u, 0u, 0u};
}

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2, ACT_TANH = 3 };

// MFMA operand precision.  F32: v_mfma_f32_16x16x4_f32, four per 16-wide
// reduction step (exact f32 fma chains).  BF16 / F16: the same fp32 operands
// rounded to nearest even as they are loaded, one v_mfma_f32_16x16x16_{bf16,f16}
// per step with the step's 4 values per lane as the instruction's 4 k-slots,
// fp32 accumulate; memory, epilogues and bias gradients stay fp32.
enum Prec : int { PREC_F32 = 0, PREC_BF16 = 1, PREC_F16 = 2 };

// fp16 operands of the backward: the gradient operand dP = dY act'(Y) is
// multiplied by 2^10 before it is rounded and the fp32 accumulators by 2^-10
// after (exact: a power of two).  The TD7 gradients are small -- the wide
// encoder's d mse / d pred is 2 (pred - target) / (B zs_dim) ~ 1e-6, the
// critic's dloss/dQ <= 1/B -- and below fp16's 6.1e-5 they would be rounded as
// subnormals (1e-6: ~6 % quantum); scaled, they stay normal down to 6e-8 and
// keep 11 bits, with overflow only above 64.  bf16 has fp32's exponent range.
template <int P>
__device__ __forceinline__ constexpr float grad_scale() { return P == PREC_F16 ? 1024.f : 1.f; }

template <int P>
__device__ __forceinline__ floatx4 mfma_k16(const float (&a)[4], const float (&b)[4], floatx4 c) {
    if constexpr (P == PREC_F16) {
        const halfx4 ha = {(_Float16)a[0], (_Float16)a[1], (_Float16)a[2], (_Float16)a[3]};
        const halfx4 hb = {(_Float16)b[0], (_Float16)b[1], (_Float16)b[2], (_Float16)b[3]};
        return __builtin_amdgcn_mfma_f32_16x16x16f16(ha, hb, c, 0, 0, 0);
    } else {
        const bf16x4 ba = {(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)a[3]};
        const bf16x4 bb = {(__bf16)b[0], (__bf16)b[1], (__bf16)b[2], (__bf16)b[3]};
        return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(shortx4, ba),
                                                         __builtin_bit_cast(shortx4, bb), c, 0, 0, 0);
    }
}

// derivative of the activation expressed through its output y
template <int ACT>
__device__ __forceinline__ float act_grad_t(float y) {
    if (ACT == ACT_RELU) return y > 0.f ? 1.f : 0.f;
    if (ACT == ACT_ELU) return y > 0.f ? 1.f : y + 1.f;
    if (ACT == ACT_TANH) return 1.f - y * y;
    return 1.f;
}
template <int ACT>
__device__ __forceinline__ float act_fwd_t(float x) {
    if (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
    if (ACT == ACT_ELU) return x > 0.f ? x : expm1f(x);
    if (ACT == ACT_TANH) return tanhf(x);
    return x;
}

// An operand element (i, r) of group g lives at p[g*sg + i*si + r*sr].  When
// act >= 0 the operand is dY and is multiplied by act'(Y) read at the same
// (g, i, r) from y (strides ysg/ysi/ysr).
struct Operand {
    const float *p;
    long sg, si, sr;
    const float *y;
    long ysg, ysi, ysr;
    int act; // -1: plain operand
    int ones_col; // >= 0: index i == ones_col reads 1.0 (bias column of bwd-weight)
};

// A concatenated operand X = [X_0 | X_1 | ... ] along its columns (the
// inputs of the TD7 layers that read torch.cat(...) in the reference): segment
// s holds columns [kb[s], kb[s+1]) at p[s] + g*sg[s] + row*ld[s] + (col - kb[s]);
// sg[s] = 0 for a segment shared by the groups.  Interior boundaries are
// multiples of 4 and the last segment is >= 4 wide, so every 4-column chunk a
// lane loads lies in one segment.  Unused entries: kb = INT_MAX.
constexpr int CAT_MAX = 4;
struct CatSeg {
    const float *p[CAT_MAX];
    long sg[CAT_MAX];
    int ld[CAT_MAX];
    int kb[CAT_MAX + 1];
};

// segment of column r (r < total width)
__device__ __forceinline__ int cat_seg(const CatSeg &c, int r) {
    return (r >= c.kb[1]) + (r >= c.kb[2]) + (r >= c.kb[3]);
}

// The b128 chunk X(row, r .. r+3) of a CAT operand from segment sg (wave-
// uniform): one buffer load whose lanes outside the segment (or !ok) read past
// the records, i.e. 0.  Returned unconsumed, so the load stays in flight.
// (uniform branches with constant indices: a dynamic index into the kernel
// arguments would put them in scratch)
__device__ __forceinline__ uint32_t4 cat_load_seg(const CatSeg &c, int sg, int g, int row, int r, bool ok) {
    uint32_t4 v = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < CAT_MAX; ++k) {
        if (sg != k) continue;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(c.p[k] + g * c.sg[k]), 0, 0x7FFFFF00, 0x00020000);
        const bool in = ok & (r >= c.kb[k]) & (r < c.kb[k + 1]);
        v = __builtin_amdgcn_raw_buffer_load_b128(rs, in ? (row * c.ld[k] + (r - c.kb[k])) * 4 : 0x7FFFFF00, 0, 0);
    }
    return v;
}

// ... for a wave-uniform reduction window [w0, w1] (the columns a load
// instruction covers): one load when the window lies in one segment (the
// common case); a window across a boundary ORs its segments' loads.
__device__ __forceinline__ uint32_t4 cat_load(const CatSeg &c, int g, int row, int r, bool ok, int w0, int w1) {
    const int sa = cat_seg(c, w0), sb = cat_seg(c, w1);
    uint32_t4 v = cat_load_seg(c, sa, g, row, r, ok);
    for (int sg = sa + 1; sg <= sb; ++sg) v |= cat_load_seg(c, sg, g, row, r, ok);
    return v;
}

struct GemmArgs {
    CatSeg cat; // forward with CAT: the A operand (X) by segments
    Operand A, B;
    int I, J, R;      // C is I x J, reduction length R
    int groups_red;   // > 1: also reduce over this many groups (bwd-data of a shared input)
    // epilogue
    float *C;
    long csg, csi, csj;
    const float *bias; // forward: + bias[g*bsg + j]
    long bsg;
    int act;           // forward activation
    float *bias_grad;  // bwd-weight: column j == J_bias goes to bias_grad[g*bgsg + i]
    long bgsg;
    int j_bias;        // -1: none
    // forward, dense_fwd_big_kernel: W already rounded to the MFMA operand
    // type, [G][N][K] contiguous 16-bit (null: round the fp32 W as it is loaded)
    const uint16_t *b16;
    // dense_fwd_big_kernel, inference chains (td7_dense_fwd_h): the input X
    // (non-concatenated) and / or the output Y as 16-bit values of the MFMA
    // operand type -- what the consumer rounds its input to anyway (null: fp32)
    const uint16_t *a16;
    uint16_t *c16;
};

// Workgroup tile 32x32 (2x2 v_mfma_f32_16x16x4_f32 tiles per wave, four
// independent accumulators); the NW waves of a workgroup split the reduction
// dimension in 16-wide steps (step s goes to wave s % NW) and their partial
// tiles are summed through LDS at the end.  Operands are loaded straight
// from global memory (L2) into registers -- no LDS staging, no barrier in
// the loop: each wave streams its steps with the next step group's loads in
// flight under the current group's MFMAs.  A lane (c, q) feeds MFMA jj of a
// step with A(i, r0+4q+jj) and B(j, r0+4q+jj) (the same permutation of the
// step's r on both operands).  Per 16-wide step a wave loads 2 A and 2 B
// fragments for 16 MFMAs, half the L2 traffic per MFMA of one 16x16 tile
// per wave, and NW x (I/32)(J/32) waves keep the whole chip busy on these
// small GEMMs (M <= 4096, N, K <= 921).
constexpr int BUF_BYTES = 0x7FFFFF00, BUF_OOB = 0x7FFFFF00; // offset past the records -> the load returns 0
constexpr int SPG = 2;                                      // 16-wide steps per prefetch group

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(p), 0, BUF_BYTES, 0x00020000);
}

__device__ __forceinline__ float ldb(__amdgpu_buffer_rsrc_t r, bool ok, int off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, ok ? off * 4 : BUF_OOB, 0, 0));
}

// one operand's fragments for SPG steps: [step][tile 0/1][jj]
struct Frag {
    float v[SPG][2][4];
};

// element (i, r) with i = i0 + 16*tile + c, r = r0 + 4q + jj.  VEC (contiguous
// along r, the step fully inside R): one 16-byte load; else 4 checked dwords.
template <bool VEC>
__device__ __forceinline__ void load_step(__amdgpu_buffer_rsrc_t rp, int base_g, int si, int sr, int i0, int c, int I,
                                          int r0, int R, int q, float (&f)[2][4], bool full) {
#pragma unroll
    for (int tl = 0; tl < 2; ++tl) {
        const int i = i0 + 16 * tl + c;
        const int r = r0 + 4 * q;
        if (VEC && full) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, i < I ? (base_g + i * si + r) * 4 : BUF_OOB, 0, 0);
            f[tl][0] = __uint_as_float(v[0]);
            f[tl][1] = __uint_as_float(v[1]);
            f[tl][2] = __uint_as_float(v[2]);
            f[tl][3] = __uint_as_float(v[3]);
        } else {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) f[tl][jj] = ldb(rp, (i < I) & (r + jj < R), base_g + i * si + (r + jj) * sr);
        }
    }
}

// Workgroups are dealt round-robin to the 8 XCDs (each with its own L2): the
// linear workgroup id is remapped so that XCD k works a contiguous run of
// (row-major) tiles -- one L2 sees 1/8 of the X rows and all of W instead of
// all of both.  Returns the tile's (x, y, z).
__device__ __forceinline__ int3 xcd_tile() {
    const int gx = gridDim.x, gy = gridDim.y;
    const int T = gx * gy * gridDim.z;
    const int id = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int q8 = T >> 3, r8 = T & 7, x = id & 7, loc = id >> 3;
    const int t = x < r8 ? x * (q8 + 1) + loc : r8 * (q8 + 1) + (x - r8) * q8 + loc;
    return make_int3(t % gx, (t / gx) % gy, t / (gx * gy));
}

template <int AG, int EP, bool AV, bool BV, int NW, int P>
__global__ __launch_bounds__(64 * NW) void dense_gemm_kernel(GemmArgs a) {
    __shared__ __attribute__((aligned(16))) float red[NW > 1 ? NW - 1 : 1][32][33];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, q = lane >> 4, c = lane & 15;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * 32, j0 = tile.x * 32, g = tile.z;
    const __amdgpu_buffer_rsrc_t ra = rsrc(a.A.p), rb = rsrc(a.B.p);
    const __amdgpu_buffer_rsrc_t ry = rsrc(AG >= 0 ? a.A.y : a.A.p);
    const int nsteps_g = (a.R + 15) >> 4;            // 16-wide steps per reduction group
    const int nsteps = nsteps_g * a.groups_red;
    const int full_steps = a.R >> 4;                  // steps entirely inside R
    // this wave's steps: w, w + NW, ...; processed SPG at a time
    const int my = nsteps > w ? (nsteps - w + NW - 1) / NW : 0;
    const int ngrp = (my + SPG - 1) / SPG;

    // epilogue bias fetched up front (its latency hides under the main loop)
    float bias_pre[2];
#pragma unroll
    for (int y = 0; y < 2; ++y) {
        const int col = j0 + 16 * y + c;
        bias_pre[y] = (a.bias && col < a.J) ? a.bias[g * a.bsg + col] : 0.f;
    }
    floatx4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = floatx4{0.f, 0.f, 0.f, 0.f};
    // bwd-weight with 16-bit operands: the bias gradient (the ones column) is
    // summed from the UNROUNDED dP in fp32 here, as the wgrad kernel does, not
    // taken from the rounded MFMA column; bsum[tl] = this lane's part of row
    // i0 + 16 tl + c
    // The loop is compiled twice: the workgroups whose tile holds the ones
    // column (one column of tiles) inject the ones and sum the bias; the rest
    // run a loop without either (the per-element checks cost 60 % on the wide
    // configuration's fp16 weight gradients, profiles/r03_wide_summary.md).
    const bool ones_tile = a.B.ones_col >= j0 && a.B.ones_col < j0 + 32;
    const bool bias_tile = P != PREC_F32 && ones_tile;
    float bsum[2] = {0.f, 0.f};

    auto load = [&](auto ones, int grp, Frag &fa, Frag &fy, Frag &fb) {
        constexpr bool ONES = decltype(ones)::value;
#pragma unroll
        for (int sp = 0; sp < SPG; ++sp) {
            const int k = grp * SPG + sp;           // k-th step of this wave
            const int st = w + k * NW;              // global step index
            const bool live = k < my;
            const int gg = a.groups_red > 1 ? st / nsteps_g : g;
            const int sl = live ? st % nsteps_g : 0;
            const int r0 = live ? sl * 16 : a.R;    // a dead step loads zeros (r >= R)
            const bool full = live && sl < full_steps;
            load_step<AV>(ra, gg * (int)a.A.sg, (int)a.A.si, (int)a.A.sr, i0, c, a.I, r0, a.R, q, fa.v[sp], full);
            if (AG >= 0)
                load_step<AV>(ry, gg * (int)a.A.ysg, (int)a.A.ysi, (int)a.A.ysr, i0, c, a.I, r0, a.R, q, fy.v[sp], full);
            load_step<BV>(rb, gg * (int)a.B.sg, (int)a.B.si, (int)a.B.sr, j0, c, a.J, r0, a.R, q, fb.v[sp], full);
            if constexpr (ONES) { // bwd-weight: column ones_col of B is all ones (-> bias gradient)
#pragma unroll
                for (int tl = 0; tl < 2; ++tl)
                    if (j0 + 16 * tl + c == a.B.ones_col)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) fb.v[sp][tl][jj] = (r0 + 4 * q + jj < a.R) ? 1.f : 0.f;
            }
        }
    };
    auto mma = [&](auto ones, const Frag &fa, const Frag &fy, const Frag &fb) {
        constexpr bool ONES = decltype(ones)::value;
        if constexpr (P != PREC_F32) {
#pragma unroll
            for (int sp = 0; sp < SPG; ++sp) {
                float av[2][4];
#pragma unroll
                for (int tl = 0; tl < 2; ++tl)
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) {
                        if constexpr (ONES) {
                            const float dp = AG >= 0 ? fa.v[sp][tl][jj] * act_grad_t<AG>(fy.v[sp][tl][jj]) : fa.v[sp][tl][jj];
                            bsum[tl] += dp;
                            av[tl][jj] = AG >= 0 ? dp * grad_scale<P>() : dp;
                        } else { // (x g) 2^10 == x (g 2^10): the scale folds into act'
                            av[tl][jj] = AG >= 0 ? fa.v[sp][tl][jj] * (act_grad_t<AG>(fy.v[sp][tl][jj]) * grad_scale<P>())
                                                 : fa.v[sp][tl][jj];
                        }
                    }
#pragma unroll
                for (int x = 0; x < 2; ++x)
#pragma unroll
                    for (int y = 0; y < 2; ++y) acc[x][y] = mfma_k16<P>(av[x], fb.v[sp][y], acc[x][y]);
            }
            return;
        }
#pragma unroll
        for (int sp = 0; sp < SPG; ++sp)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                float av[2];
#pragma unroll
                for (int tl = 0; tl < 2; ++tl)
                    av[tl] = AG >= 0 ? fa.v[sp][tl][jj] * act_grad_t<AG>(fy.v[sp][tl][jj]) : fa.v[sp][tl][jj];
#pragma unroll
                for (int x = 0; x < 2; ++x)
#pragma unroll
                    for (int y = 0; y < 2; ++y)
                        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[x], fb.v[sp][y][jj], acc[x][y], 0, 0, 0);
            }
    };
    auto run = [&](auto ones) {
        Frag a0, y0, b0, a1, y1, b1;
        if (ngrp > 0) load(ones, 0, a0, y0, b0);
        for (int grp = 0; grp < ngrp; grp += 2) {
            if (grp + 1 < ngrp) load(ones, grp + 1, a1, y1, b1);
            mma(ones, a0, y0, b0);
            if (grp + 1 >= ngrp) break;
            if (grp + 2 < ngrp) load(ones, grp + 2, a0, y0, b0);
            mma(ones, a1, y1, b1);
        }
    };
    if (ones_tile) run(std::true_type{});
    else run(std::false_type{});
    if (bias_tile)
#pragma unroll
        for (int tl = 0; tl < 2; ++tl) {
            bsum[tl] += __shfl_xor(bsum[tl], 16);
            bsum[tl] += __shfl_xor(bsum[tl], 32);
        }
    // sum the NW partial tiles: waves 1.. park theirs in LDS, wave 0 adds them
    // acc[x][y][k] is C[i0 + 16x + 4q + k][j0 + 16y + c]; the bias partials go
    // to the padding column 32
    if (NW > 1) {
        if (w > 0) {
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int k = 0; k < 4; ++k) red[w - 1][16 * x + 4 * q + k][16 * y + c] = acc[x][y][k];
            if (bias_tile && q == 0)
#pragma unroll
                for (int tl = 0; tl < 2; ++tl) red[w - 1][16 * tl + c][32] = bsum[tl];
        }
        __syncthreads();
        if (w > 0) return;
#pragma unroll
        for (int ww = 0; ww < NW - 1; ++ww) {
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[x][y][k] += red[ww][16 * x + 4 * q + k][16 * y + c];
            if (bias_tile)
#pragma unroll
                for (int tl = 0; tl < 2; ++tl) bsum[tl] += red[ww][16 * tl + c][32];
        }
    }
    // the bias of row i0 + 16x + 4q + k sits in lane c = 4q + k
    float bias_row[2][4];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int k = 0; k < 4; ++k) bias_row[x][k] = bias_tile ? __shfl(bsum[x], 4 * q + k) : 0.f;
#pragma unroll
    for (int y = 0; y < 2; ++y) {
        const int col = j0 + 16 * y + c;
        const bool is_bias = a.j_bias >= 0 && col == a.j_bias;
        if (!is_bias && col >= a.J) continue;
        const float bias_v = is_bias ? 0.f : bias_pre[y];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int row = i0 + 16 * x + 4 * q + k;
                if (row >= a.I) continue;
                const float v = (is_bias && bias_tile) ? bias_row[x][k]
                                : AG >= 0 ? acc[x][y][k] * (1.f / grad_scale<P>()) : acc[x][y][k];
                if (is_bias) a.bias_grad[g * a.bgsg + row] = v;
                else a.C[g * a.csg + (long)row * a.csi + (long)col * a.csj] = act_fwd_t<EP>(v + bias_v);
            }
    }
}

template <int P>
void launch_gemm_p(const GemmArgs &a, dim3 grid, int nw, hipStream_t s) {
#define DENSE_LAUNCH(AGv, EPv, AVv, BVv)                                                                            \
    do {                                                                                                          \
        if (nw == 8) hipLaunchKernelGGL((dense_gemm_kernel<AGv, EPv, AVv, BVv, 8, P>), grid, dim3(512), 0, s, a);    \
        else if (nw == 4) hipLaunchKernelGGL((dense_gemm_kernel<AGv, EPv, AVv, BVv, 4, P>), grid, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((dense_gemm_kernel<AGv, EPv, AVv, BVv, 2, P>), grid, dim3(128), 0, s, a);           \
    } while (0)
    if (a.A.sr == 1) { // bwd-data: dY rows contiguous, W^T column walk
        switch (a.A.act) {
        case ACT_RELU: DENSE_LAUNCH(ACT_RELU, ACT_NONE, true, false); break;
        case ACT_ELU: DENSE_LAUNCH(ACT_ELU, ACT_NONE, true, false); break;
        case ACT_TANH: DENSE_LAUNCH(ACT_TANH, ACT_NONE, true, false); break;
        default: DENSE_LAUNCH(ACT_NONE, ACT_NONE, true, false); break;
        }
    } else {           // bwd-weight (generic layout): both operands walk rows (contiguous along i)
        switch (a.A.act) {
        case ACT_RELU: DENSE_LAUNCH(ACT_RELU, ACT_NONE, false, false); break;
        case ACT_ELU: DENSE_LAUNCH(ACT_ELU, ACT_NONE, false, false); break;
        case ACT_TANH: DENSE_LAUNCH(ACT_TANH, ACT_NONE, false, false); break;
        default: DENSE_LAUNCH(ACT_NONE, ACT_NONE, false, false); break;
        }
    }
#undef DENSE_LAUNCH
}

// Forward Y = act(X W^T + b): one wavefront per 16x16 output tile, the whole
// reduction loaded up front in groups of GS 16-wide steps (one 16-byte load
// of X and one of W per lane per step) so a wave makes one or two L2 round
// trips instead of one per step; the tail (K % 16) is a range-checked step.
// (2x2 waves per workgroup sharing X / W rows through L1 measured slower than
// one wave per workgroup with this remap.)
// 16-bit X element (the a16 operand) as the float it equals
template <int P>
__device__ __forceinline__ uint32_t half_bits_to_float_bits(uint32_t h) {
    if constexpr (P == PREC_F16) return __float_as_uint((float)__builtin_bit_cast(_Float16, (uint16_t)h));
    else return h << 16;
}

template <int EP, int GS, int TM, int TN, int KW, int P, bool CAT, bool AH = false>
__global__ __launch_bounds__(64 * KW) void dense_fwd_kernel(GemmArgs a) {
    // a (16 TM) x (16 TN) tile per workgroup; per 16-wide step TM + TN b128
    // loads feed 4 TM TN MFMAs.  KW waves split the reduction (halves, summed
    // through LDS at the end).  AH (r05): X is the 16-bit a16 operand (an
    // inference chain's 16-bit activations), 8-byte loads of the same 4
    // values the fp32 path rounds to -- the same MFMA operands in the same
    // order, bit-identical output.
    constexpr bool SPLIT = TM * TN == 1; // 1x1: two accumulators break the MFMA dependency chain
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * 16 * TM, j0 = tile.x * 16 * TN, g = tile.z;
    const __amdgpu_buffer_rsrc_t ra = AH ? rsrc(reinterpret_cast<const float *>(a.a16)) : rsrc(a.A.p),
                                 rb = rsrc(a.B.p);
    int abase[TM], bbase[TN];
    bool arow[TM], bcol[TN];
    int arowi[TM];
#pragma unroll
    for (int x = 0; x < TM; ++x) {
        const int row = i0 + 16 * x + c;
        abase[x] = g * (int)a.A.sg + row * (int)a.A.si;
        arow[x] = row < a.I;
        arowi[x] = arow[x] ? row : 0;
    }
    // CAT: segment bases (wave-uniform: group offset and -kb folded in)
    const float *cb0 = a.cat.p[0] + g * a.cat.sg[0], *cb1 = a.cat.p[1] + g * a.cat.sg[1] - a.cat.kb[1],
                *cb2 = a.cat.p[2] + g * a.cat.sg[2] - a.cat.kb[2], *cb3 = a.cat.p[3] + g * a.cat.sg[3] - a.cat.kb[3];
    // pointer to X(row, r) for a chunk r .. r+3 (one segment)
    const int kb1 = a.cat.kb[1], kb2 = a.cat.kb[2], kb3 = a.cat.kb[3];
    const int cl0 = a.cat.ld[0], dl1 = a.cat.ld[1] - cl0, dl2 = a.cat.ld[2] - a.cat.ld[1], dl3 = a.cat.ld[3] - a.cat.ld[2];
    const long e1 = cb1 - cb0, e2 = cb2 - cb1, e3 = cb3 - cb2; // element distances between segment bases
    // (the segment picked by arithmetic on the monotone flags s1 >= s2 >= s3: a
    // select chain over the bases is turned into an LDS lookup table)
    auto cat_ptr = [=](int row, int r) {
        const int s1 = r >= kb1, s2 = r >= kb2, s3 = r >= kb3;
        const long off = s1 * e1 + s2 * e2 + s3 * e3;
        const int ld = cl0 + s1 * dl1 + s2 * dl2 + s3 * dl3;
        return cb0 + off + (long)row * ld + r;
    };
    // CAT: the 4 A values (r .. r+3) of row tile x as one 16-byte global load
    auto ld_cat = [&](int x, int r, bool ok) { return gload4(cat_ptr(arowi[x], ok ? r : 0), cb0, ok); };
    float bias_v[TN];
#pragma unroll
    for (int y = 0; y < TN; ++y) {
        const int col = j0 + 16 * y + c;
        bbase[y] = g * (int)a.B.sg + col * (int)a.B.si;
        bcol[y] = col < a.J;
        bias_v[y] = (a.bias && bcol[y]) ? a.bias[g * a.bsg + col] : 0.f;
    }
    const int nall = a.R >> 4, per = (nall + KW - 1) / KW;
    const int sbeg = w * per, nfull = min(nall, sbeg + per); // this wave's steps [sbeg, nfull)
    floatx4 acc[TM][TN][SPLIT ? 2 : 1];
#pragma unroll
    for (int x = 0; x < TM; ++x)
#pragma unroll
        for (int y = 0; y < TN; ++y)
#pragma unroll
            for (int h = 0; h < (SPLIT ? 2 : 1); ++h) acc[x][y][h] = floatx4{0.f, 0.f, 0.f, 0.f};
    // groups of GS 16-wide steps, two register buffers: group k+1's loads are
    // in flight while group k's MFMAs run
    auto load = [&](int s0, uint32_t (&av)[GS][TM][4], uint32_t (&bv)[GS][TN][4]) {
#pragma unroll
        for (int s = 0; s < GS; ++s) {
            const int r = 16 * (s0 + s) + 4 * q;
            const bool live = s0 + s < nfull;
#pragma unroll
            for (int x = 0; x < TM; ++x) {
                if constexpr (CAT) {
                    // (16-byte global loads: per-segment buffer loads behind
                    // uniform branches measured slower in this kernel)
                    const auto v = ld_cat(x, r, live & arow[x]);
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) av[s][x][jj] = v[jj];
                } else if constexpr (AH) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b64(ra, (live & arow[x]) ? (abase[x] + r) * 2 : BUF_OOB, 0, 0);
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        av[s][x][jj] = half_bits_to_float_bits<P>((v[jj >> 1] >> (16 * (jj & 1))) & 0xffffu);
                } else {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(ra, (live & arow[x]) ? (abase[x] + r) * 4 : BUF_OOB, 0, 0);
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) av[s][x][jj] = v[jj];
                }
            }
#pragma unroll
            for (int y = 0; y < TN; ++y) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, (live & bcol[y]) ? (bbase[y] + r) * 4 : BUF_OOB, 0, 0);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) bv[s][y][jj] = v[jj];
            }
        }
    };
    auto step = [&](const float (&xa)[TM][4], const float (&xb)[TN][4], int h) {
        if constexpr (P != PREC_F32) {
#pragma unroll
            for (int x = 0; x < TM; ++x)
#pragma unroll
                for (int y = 0; y < TN; ++y) {
                    floatx4 &d = acc[x][y][SPLIT ? (h & 1) : 0];
                    d = mfma_k16<P>(xa[x], xb[y], d);
                }
            return;
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
            for (int x = 0; x < TM; ++x)
#pragma unroll
                for (int y = 0; y < TN; ++y) {
                    floatx4 &d = acc[x][y][SPLIT ? (jj & 1) : 0];
                    d = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[x][jj], xb[y][jj], d, 0, 0, 0);
                }
    };
    auto mma = [&](const uint32_t (&av)[GS][TM][4], const uint32_t (&bv)[GS][TN][4]) {
#pragma unroll
        for (int s = 0; s < GS; ++s) {
            float xa[TM][4], xb[TN][4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
#pragma unroll
                for (int x = 0; x < TM; ++x) xa[x][jj] = __uint_as_float(av[s][x][jj]);
#pragma unroll
                for (int y = 0; y < TN; ++y) xb[y][jj] = __uint_as_float(bv[s][y][jj]);
            }
            step(xa, xb, s);
        }
    };
    if constexpr (GS >= 20) { // the launcher picks GS = 20 only for R < 336: one group
        uint32_t a0[GS][TM][4], b0[GS][TN][4];
        load(sbeg, a0, b0);
        __builtin_amdgcn_sched_barrier(0); // all loads in flight before the first MFMA
        mma(a0, b0);
    } else {
        uint32_t a0[GS][TM][4], b0[GS][TN][4], a1[GS][TM][4], b1[GS][TN][4];
        if (nfull > sbeg) load(sbeg, a0, b0);
        for (int s0 = sbeg; s0 < nfull; s0 += 2 * GS) {
            if (s0 + GS < nfull) load(s0 + GS, a1, b1);
            mma(a0, b0);
            if (s0 + GS >= nfull) break;
            if (s0 + 2 * GS < nfull) load(s0 + 2 * GS, a0, b0);
            mma(a1, b1);
        }
    }
    if ((a.R & 15) && w == KW - 1) { // tail step
        const int r = 16 * nall + 4 * q;
        float xa[TM][4], xb[TN][4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
#pragma unroll
            for (int x = 0; x < TM; ++x) {
                if constexpr (CAT) { // the chunk r .. r+3 lies in one segment
                    xa[x][jj] = (arow[x] & (r + jj < a.R)) ? cat_ptr(arowi[x], r)[jj] : 0.f;
                } else if constexpr (AH) {
                    const bool ok = arow[x] & (r + jj < a.R);
                    xa[x][jj] = __uint_as_float(half_bits_to_float_bits<P>(
                        __builtin_amdgcn_raw_buffer_load_b16(ra, ok ? (abase[x] + r + jj) * 2 : BUF_OOB, 0, 0)));
                } else {
                    xa[x][jj] = ldb(ra, arow[x] & (r + jj < a.R), abase[x] + r + jj);
                }
            }
#pragma unroll
            for (int y = 0; y < TN; ++y) xb[y][jj] = ldb(rb, bcol[y] & (r + jj < a.R), bbase[y] + r + jj);
        }
        step(xa, xb, 0);
    }
    if constexpr (SPLIT)
#pragma unroll
        for (int x = 0; x < TM; ++x)
#pragma unroll
            for (int y = 0; y < TN; ++y) {
                acc[x][y][0] += acc[x][y][SPLIT ? 1 : 0];
                acc[x][y][SPLIT ? 1 : 0] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
    if constexpr (KW > 1) {
        __shared__ floatx4 red[KW - 1][TM * TN][64];
        if (w > 0)
#pragma unroll
            for (int x = 0; x < TM; ++x)
#pragma unroll
                for (int y = 0; y < TN; ++y) red[w - 1][x * TN + y][lane] = acc[x][y][0];
        __syncthreads();
        if (w > 0) return;
#pragma unroll
        for (int ww = 0; ww < KW - 1; ++ww)
#pragma unroll
            for (int x = 0; x < TM; ++x)
#pragma unroll
                for (int y = 0; y < TN; ++y) acc[x][y][0] += red[ww][x * TN + y][lane];
    }
    // acc[x][y][.][k] is C[i0 + 16x + 4q + k][j0 + 16y + c]
#pragma unroll
    for (int y = 0; y < TN; ++y) {
        if (!bcol[y]) continue;
        const int col = j0 + 16 * y + c;
#pragma unroll
        for (int x = 0; x < TM; ++x) {
            const floatx4 v = SPLIT ? acc[x][y][0] + acc[x][y][SPLIT ? 1 : 0] : acc[x][y][0];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int rr = i0 + 16 * x + 4 * q + k;
                if (rr < a.I) a.C[g * a.csg + (long)rr * a.csi + (long)col * a.csj] = act_fwd_t<EP>(v[k] + bias_v[y]);
            }
        }
    }
}

// ---- forward + AvgL1Norm ----------------------------------------------------
// y = h / max(mean_j |h_j|, eps) with h = X W^T + b (no activation): the TD7
// layers followed by AvgL1Norm (Agent/TD7_multi_agent.py:53-54 after :61, :103,
// :126).  One workgroup owns 16 rows and ALL N <= 320 output columns (4 waves x
// NT = 5 16-wide column tiles), so the row mean is a workgroup reduction and
// the separate AvgL1Norm launch disappears.  h and the raw mean are stored when
// hout / mean_out are given (the backward of a trained layer needs them).
// Per 16-wide reduction step a lane loads one A (b128, shared by the 4 waves
// through L1) and NT B fragments; GS steps per prefetch group, two groups in
// flight.
struct CatRows { // segment bases of a CAT A operand for one group (see CatSeg)
    const float *cb0;
    long e1, e2, e3;
    int kb1, kb2, kb3, cl0, dl1, dl2, dl3;
    __device__ __forceinline__ CatRows(const CatSeg &c, int g) {
        const float *b0 = c.p[0] + g * c.sg[0], *b1 = c.p[1] + g * c.sg[1] - c.kb[1],
                    *b2 = c.p[2] + g * c.sg[2] - c.kb[2], *b3 = c.p[3] + g * c.sg[3] - c.kb[3];
        cb0 = b0;
        e1 = b1 - b0;
        e2 = b2 - b1;
        e3 = b3 - b2;
        kb1 = c.kb[1];
        kb2 = c.kb[2];
        kb3 = c.kb[3];
        cl0 = c.ld[0];
        dl1 = c.ld[1] - c.ld[0];
        dl2 = c.ld[2] - c.ld[1];
        dl3 = c.ld[3] - c.ld[2];
    }
    __device__ __forceinline__ const float *ptr(int row, int r) const {
        const int s1 = r >= kb1, s2 = r >= kb2, s3 = r >= kb3;
        return cb0 + (s1 * e1 + s2 * e2 + s3 * e3) + (long)row * (cl0 + s1 * dl1 + s2 * dl2 + s3 * dl3) + r;
    }
};

template <int P, bool CAT>
__global__ __launch_bounds__(256) void dense_fwd_norm_kernel(GemmArgs a, float *hout, float *mean_out, float eps) {
    constexpr int NT = 5, GS = 2;
    __shared__ float red[4][16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
    const int i0 = blockIdx.x * 16, g = blockIdx.y, j0 = w * 16 * NT;
    const __amdgpu_buffer_rsrc_t ra = rsrc(a.A.p), rb = rsrc(a.B.p);
    const int row = i0 + c;
    const bool arow = row < a.I;
    const int abase = g * (int)a.A.sg + row * (int)a.A.si;
    const CatRows cr(a.cat, CAT ? g : 0);
    int bbase[NT];
    bool bcol[NT];
#pragma unroll
    for (int y = 0; y < NT; ++y) {
        const int col = j0 + 16 * y + c;
        bbase[y] = g * (int)a.B.sg + col * (int)a.B.si;
        bcol[y] = col < a.J;
    }
    floatx4 acc[NT];
#pragma unroll
    for (int y = 0; y < NT; ++y) acc[y] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int nall = a.R >> 4;
    auto load = [&](int s0, uint32_t (&av)[GS][4], uint32_t (&bv)[GS][NT][4]) {
#pragma unroll
        for (int s = 0; s < GS; ++s) {
            const int r = 16 * (s0 + s) + 4 * q;
            const bool live = s0 + s < nall;
            if constexpr (CAT) {
                const auto v = gload4(cr.ptr(arow ? row : 0, live ? r : 0), cr.cb0, live & arow);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) av[s][jj] = v[jj];
            } else {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(ra, (live & arow) ? (abase + r) * 4 : BUF_OOB, 0, 0);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) av[s][jj] = v[jj];
            }
#pragma unroll
            for (int y = 0; y < NT; ++y) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, (live & bcol[y]) ? (bbase[y] + r) * 4 : BUF_OOB, 0, 0);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) bv[s][y][jj] = v[jj];
            }
        }
    };
    auto step = [&](const float (&xa)[4], const float (&xb)[NT][4]) {
        if constexpr (P != PREC_F32) {
#pragma unroll
            for (int y = 0; y < NT; ++y) acc[y] = mfma_k16<P>(xa, xb[y], acc[y]);
        } else {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int y = 0; y < NT; ++y) acc[y] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[jj], xb[y][jj], acc[y], 0, 0, 0);
        }
    };
    auto mma = [&](const uint32_t (&av)[GS][4], const uint32_t (&bv)[GS][NT][4]) {
#pragma unroll
        for (int s = 0; s < GS; ++s) {
            float xa[4], xb[NT][4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                xa[jj] = __uint_as_float(av[s][jj]);
#pragma unroll
                for (int y = 0; y < NT; ++y) xb[y][jj] = __uint_as_float(bv[s][y][jj]);
            }
            step(xa, xb);
        }
    };
    {
        uint32_t a0[GS][4], b0[GS][NT][4], a1[GS][4], b1[GS][NT][4];
        if (nall > 0) load(0, a0, b0);
        for (int s0 = 0; s0 < nall; s0 += 2 * GS) {
            if (s0 + GS < nall) load(s0 + GS, a1, b1);
            mma(a0, b0);
            if (s0 + GS >= nall) break;
            if (s0 + 2 * GS < nall) load(s0 + 2 * GS, a0, b0);
            mma(a1, b1);
        }
    }
    if (a.R & 15) { // tail step
        const int r = 16 * nall + 4 * q;
        float xa[4], xb[NT][4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            if constexpr (CAT)
                xa[jj] = (arow & (r + jj < a.R)) ? cr.ptr(row, r)[jj] : 0.f;
            else
                xa[jj] = ldb(ra, arow & (r + jj < a.R), abase + r + jj);
#pragma unroll
            for (int y = 0; y < NT; ++y) xb[y][jj] = ldb(rb, bcol[y] & (r + jj < a.R), bbase[y] + r + jj);
        }
        step(xa, xb);
    }
    // acc[y][k] is h[i0 + 4q + k][j0 + 16y + c] (before the bias)
    float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int y = 0; y < NT; ++y) {
        const float bv = (a.bias && bcol[y]) ? a.bias[g * a.bsg + j0 + 16 * y + c] : 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            acc[y][k] = bcol[y] ? acc[y][k] + bv : 0.f;
            part[k] += fabsf(acc[y][k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) part[k] += __shfl_xor(part[k], o, 64);
    if (c == 0)
#pragma unroll
        for (int k = 0; k < 4; ++k) red[w][4 * q + k] = part[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rr = i0 + 4 * q + k;
        // the same summation order for every lane of the row
        const float m = (red[0][4 * q + k] + red[1][4 * q + k] + red[2][4 * q + k] + red[3][4 * q + k]) / a.J;
        const float sc = fmaxf(m, eps);
        if (rr >= a.I) continue;
        if (mean_out && w == 0 && c == 0) mean_out[(long)g * a.I + rr] = m;
#pragma unroll
        for (int y = 0; y < NT; ++y) {
            if (!bcol[y]) continue;
            const long o = g * a.csg + (long)rr * a.csi + (j0 + 16 * y + c);
            a.C[o] = acc[y][k] / sc;
            if (hout) hout[o] = acc[y][k];
        }
    }
}

template <int P, bool CAT>
void launch_fwd_norm_p(const GemmArgs &a, dim3 grid, float *hout, float *mean_out, float eps, hipStream_t s) {
    hipLaunchKernelGGL((dense_fwd_norm_kernel<P, CAT>), grid, dim3(256), 0, s, a, hout, mean_out, eps);
}

// ---- forward of the large layers: LDS-tiled ---------------------------------
// Y = act(X W^T + b) for the big GEMMs (the batched policy over thousands of
// envs, the 1024-wide configuration), bf16 / fp16 operands only.  A workgroup
// (4 waves as 2 x 2) owns a BM x BN output tile; per 32-deep K slice every
// thread loads (BM + BN) x 32 / 256 fp32 values with 16-byte buffer loads,
// rounds them to 16-bit and stores them to LDS (double-buffered, rows padded
// to 40 halves against bank conflicts); each wave then runs (BM/32) x (BN/32)
// 16x16x16 MFMAs per 16-deep step from LDS fragments.  The next slice's global
// loads are in flight while the current one is multiplied.  Compared with the
// register-streaming kernel above, each global byte feeds BM/16 (resp. BN/16)
// MFMA tiles instead of 1-2.
template <int P>
__device__ __forceinline__ uint16_t to_half_bits(float v) {
    if constexpr (P == PREC_F16) return __builtin_bit_cast(uint16_t, (_Float16)v);
    else return __builtin_bit_cast(uint16_t, (__bf16)v);
}

template <int EP, int P, int BM, int BN, bool CAT, bool CHF = false>
__global__ __launch_bounds__(256) void dense_fwd_lds_kernel(GemmArgs a) {
    constexpr int BK = 32, LDK = 40;                 // halves per LDS row (32 + 8 pad)
    constexpr int AL = BM * BK / 256 / 4, BL = BN * BK / 256 / 4;  // 16-byte loads per thread per slice
    constexpr int TM = BM / 32, TN = BN / 32;        // 16x16 MFMA tiles per wave
    __shared__ __attribute__((aligned(16))) uint16_t As[2][BM][LDK];
    __shared__ __attribute__((aligned(16))) uint16_t Bs[2][BN][LDK];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, q = lane >> 4, c = lane & 15;
    const int wm = w >> 1, wn = w & 1;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * BM, j0 = tile.x * BN, g = tile.z;
    const __amdgpu_buffer_rsrc_t ra = rsrc(a.A.p), rb = rsrc(a.B.p);
    const int K = a.R, nk = (K + BK - 1) / BK;
    // this thread's load slots: row (t >> 3) + 32 l, k chunk 4 (t & 7)
    const int lr = t >> 3, lk = 4 * (t & 7);
    const CatRows cr(a.cat, CAT ? g : 0);
    float ra_v[AL][4], rb_v[BL][4];
    auto gload = [&](int kt) {
        const int k = kt * BK + lk;
        const bool full = k + 4 <= K;
#pragma unroll
        for (int l = 0; l < AL; ++l) {
            const int row = i0 + lr + 32 * l;
            const bool ok = row < a.I;
            if constexpr (CAT) { // the chunk k .. k+3 lies in one segment
                if (full) {
                    const int w0 = kt * BK;
                    const auto v = cat_load(a.cat, g, ok ? row : 0, k, ok, w0, min(w0 + BK - 1, K - 1));
#pragma unroll
                    for (int e = 0; e < 4; ++e) ra_v[l][e] = __uint_as_float(v[e]);
                } else {
                    const float *p = cr.ptr(ok ? row : 0, (k < K) ? k : 0);
#pragma unroll
                    for (int e = 0; e < 4; ++e) ra_v[l][e] = (ok & (k + e < K)) ? p[e] : 0.f;
                }
                continue;
            }
            const int base = g * (int)a.A.sg + row * (int)a.A.si + k;
            if (full) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? base * 4 : BUF_OOB, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e) ra_v[l][e] = __uint_as_float(v[e]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) ra_v[l][e] = ldb(ra, ok & (k + e < K), base + e);
            }
        }
#pragma unroll
        for (int l = 0; l < BL; ++l) {
            const int col = j0 + lr + 32 * l;
            const bool ok = col < a.J;
            const int base = g * (int)a.B.sg + col * (int)a.B.si + k;
            if (full) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, ok ? base * 4 : BUF_OOB, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e) rb_v[l][e] = __uint_as_float(v[e]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) rb_v[l][e] = ldb(rb, ok & (k + e < K), base + e);
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int l = 0; l < AL; ++l) {
            uint16_t h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) h[e] = to_half_bits<P>(ra_v[l][e]);
            *reinterpret_cast<uint2 *>(&As[buf][lr + 32 * l][lk]) = __builtin_bit_cast(uint2, h);
        }
#pragma unroll
        for (int l = 0; l < BL; ++l) {
            uint16_t h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) h[e] = to_half_bits<P>(rb_v[l][e]);
            *reinterpret_cast<uint2 *>(&Bs[buf][lr + 32 * l][lk]) = __builtin_bit_cast(uint2, h);
        }
    };
    floatx4 acc[TM][TN];
#pragma unroll
    for (int x = 0; x < TM; ++x)
#pragma unroll
        for (int y = 0; y < TN; ++y) acc[x][y] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < BK; ks += 16) {
            shortx4 af[TM], bf[TN];
#pragma unroll
            for (int x = 0; x < TM; ++x)
                af[x] = *reinterpret_cast<const shortx4 *>(&As[buf][wm * (BM / 2) + 16 * x + c][ks + 4 * q]);
#pragma unroll
            for (int y = 0; y < TN; ++y)
                bf[y] = *reinterpret_cast<const shortx4 *>(&Bs[buf][wn * (BN / 2) + 16 * y + c][ks + 4 * q]);
#pragma unroll
            for (int x = 0; x < TM; ++x)
#pragma unroll
                for (int y = 0; y < TN; ++y) {
                    if constexpr (P == PREC_F16)
                        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(halfx4, af[x]),
                                                                          __builtin_bit_cast(halfx4, bf[y]), acc[x][y],
                                                                          0, 0, 0);
                    else
                        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af[x], bf[y], acc[x][y], 0, 0, 0);
                }
        }
    };
    gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload(kt + 1);
        compute(buf);
        if (kt + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }
    // acc[x][y][k] is C[i0 + wm BM/2 + 16x + 4q + k][j0 + wn BN/2 + 16y + c]
#pragma unroll
    for (int y = 0; y < TN; ++y) {
        const int col = j0 + wn * (BN / 2) + 16 * y + c;
        if (col >= a.J) continue;
        const float bv = a.bias ? a.bias[g * a.bsg + col] : 0.f;
#pragma unroll
        for (int x = 0; x < TM; ++x)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int row = i0 + wm * (BM / 2) + 16 * x + 4 * q + k;
                if (row < a.I) {
                    const float v = act_fwd_t<EP>(acc[x][y][k] + bv);
                    const long at = g * a.csg + (long)row * a.csi + (long)col * a.csj;
                    if constexpr (CHF) a.c16[at] = to_half_bits<P>(v);  // td7_dense_fwd_h's 16-bit Y
                    else a.C[at] = v;
                }
            }
    }
}

template <int P, bool CAT>
void launch_fwd_lds_p(const GemmArgs &a, dim3 grid, int bm, hipStream_t s) {
#define FWD_LDS(EPv)                                                                                    \
    do {                                                                                              \
        if (bm == 128 && a.c16)                                                                        \
            hipLaunchKernelGGL((dense_fwd_lds_kernel<EPv, P, 128, 128, CAT, true>), grid, dim3(256), 0, s, a); \
        else if (bm == 128) hipLaunchKernelGGL((dense_fwd_lds_kernel<EPv, P, 128, 128, CAT>), grid, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((dense_fwd_lds_kernel<EPv, P, 64, 64, CAT>), grid, dim3(256), 0, s, a);          \
    } while (0)
    switch (a.act) {
    case ACT_RELU: FWD_LDS(ACT_RELU); break;
    case ACT_ELU: FWD_LDS(ACT_ELU); break;
    case ACT_TANH: FWD_LDS(ACT_TANH); break;
    default: FWD_LDS(ACT_NONE); break;
    }
#undef FWD_LDS
}

// ---- forward of the largest layers: 128 x 256 tiles, 16x16x32 MFMA ----------
// Y = act(X W^T + b) where the output tiles number >= 256 and K is a multiple
// of 8 (the wide configuration's update at 8 x 1,024 rows and its policy over
// 65,536 envs: M = 8,192-65,536, N = 1,024, K = 1,024-3,072).
// dense_fwd_lds_kernel above stages 32-deep slices for 16x16x16 MFMAs from
// 8-byte LDS reads; here a 512-thread workgroup (8 waves, each a 64 x 64
// sub-tile of 4 x 4 accumulators) stages 64-deep slices: every thread loads 6
// chunks of 8 consecutive fp32 (two 16-byte buffer loads each) of the tile's
// X and W rows, rounds them to 16-bit and writes one 16-byte LDS store per
// chunk; each wave reads its A and B fragments as ds_read_b128 (4 + 4 per
// 32-deep step) for 16 v_mfma_f32_16x16x32 (twice the K of the 16x16x16 form).
// The chunk column of row r is stored at (chunk ^ ((r >> 1) & 7)): the
// fragment reads of every ds_read_b128 lane group (MI355X_MICROARCH.md, LDS
// table) then hit 16 distinct 16-byte bank quads.  The next slice's global
// loads are in flight under the current slice's MFMAs (two LDS buffers, one
// barrier per slice); workgroups go to the XCDs in runs of consecutive tiles
// (xcd_tile), so the column tiles of one row block of X share an L2.  CAT
// operands need segment boundaries at multiples of 64 (a slice then lies in
// one segment).  Same products and fp32 accumulation as the other forward
// kernels; the summation order differs (K in 32-steps).  Measured
// (profiles/r03_big_raw): 1.1-1.6x the LDS kernel on the concatenated
// layers, level at 65,536 x 1,024 x 1,024 -- ~390-500 TF/s.  r03d: slices
// two ahead (the next slice rounded to 16-bit early, freeing its fp32
// registers): 691 -> 623 us on [a | zs], 205 -> 182 on the wide critic's
// concatenated layer; neither operand's footprint bounds the 1,024 x 1,024
// layers (profiles/r03d_raw).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8_t __attribute__((ext_vector_type(8)));

template <int P>
__device__ __forceinline__ uint32_t pack_h2(float lo, float hi) {
    return (uint32_t)to_half_bits<P>(lo) | ((uint32_t)to_half_bits<P>(hi) << 16);
}

template <int P>
__device__ __forceinline__ floatx4 mfma_k32(uint32_t4 a, uint32_t4 b, floatx4 c) {
    if constexpr (P == PREC_F16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8_t, a), __builtin_bit_cast(halfx8_t, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                       c, 0, 0, 0);
}

constexpr int BIG_BK = 64, BIG_CH = BIG_BK / 8;

template <int EP, int P, bool CAT, int BM, int BN, bool BH = false, bool AH = false, bool CHF = false>
__global__ __launch_bounds__(512) void dense_fwd_big_kernel(GemmArgs a) {
    constexpr int BK = BIG_BK, CH = BIG_CH, WN = BN / 64;
    constexpr int AC = BM * CH / 512, BC = BN * CH / 512; // chunks per thread per slice
    __shared__ uint32_t4 As[2][BM * CH];
    __shared__ uint32_t4 Bs[2][BN * CH];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, q = lane >> 4, c = lane & 15;
    const int wm = w / WN, wn = w % WN;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * BM, j0 = tile.x * BN, g = tile.z;
    const int K = a.R, nk = (K + BK - 1) / BK;
    const int lr = t >> 3, lc = t & 7; // this thread's chunks: rows lr + 64 j, chunk column lc
    const __amdgpu_buffer_rsrc_t rb =
        BH ? rsrc(reinterpret_cast<const float *>(a.b16 + (long)g * a.J * a.R)) : rsrc(a.B.p + g * a.B.sg);
    // AH with CAT: the segments' pointers hold 16-bit values (non-grouped only)
    __amdgpu_buffer_rsrc_t ra = CAT  ? rsrc(a.cat.p[0])
                                : AH ? rsrc(reinterpret_cast<const float *>(a.a16 + g * a.A.sg))
                                     : rsrc(a.A.p + g * a.A.sg);
    int lda = CAT ? a.cat.ld[0] : (int)a.A.si, kbase = 0, seg = 0;
    uint32_t4 xa[AC][2], xb[BC][2];
    auto gload = [&](int kt) {
        const int k0 = kt * BK;
        if constexpr (CAT) { // the slice's segment (boundaries are multiples of BK)
            const int s = cat_seg(a.cat, k0);
            if (s != seg || kt == 0) {
                seg = s;
                const float *p = a.cat.p[0];
                long gs = a.cat.sg[0];
                int ld = a.cat.ld[0], kb = 0;
#pragma unroll
                for (int m = 1; m < CAT_MAX; ++m)
                    if (s == m) p = a.cat.p[m], gs = a.cat.sg[m], ld = a.cat.ld[m], kb = a.cat.kb[m];
                ra = AH ? rsrc(reinterpret_cast<const float *>(reinterpret_cast<const uint16_t *>(p) + g * gs))
                        : rsrc(p + g * gs);
                lda = ld;
                kbase = kb;
            }
        }
        const int k = k0 + 8 * lc;
        const bool kin = k < K;
#pragma unroll
        for (int j = 0; j < AC; ++j) {
            const int row = i0 + lr + 64 * j;
            const bool ok = kin & (row < a.I);
            if constexpr (AH) {  // 8 consecutive 16-bit inputs: one load, no rounding
                xa[j][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? (row * lda + k - kbase) * 2 : BUF_OOB, 0, 0);
            } else {
                const int off = (row * lda + k - kbase) * 4;
                xa[j][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? off : BUF_OOB, 0, 0);
                xa[j][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? off + 16 : BUF_OOB, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < BC; ++j) {
            const int col = j0 + lr + 64 * j;
            const bool ok = kin & (col < a.J);
            if constexpr (BH) {  // 8 consecutive 16-bit weights: one load, no rounding
                xb[j][0] = __builtin_amdgcn_raw_buffer_load_b128(rb, ok ? (col * a.R + k) * 2 : BUF_OOB, 0, 0);
            } else {
                const int off = (col * (int)a.B.si + k) * 4;
                xb[j][0] = __builtin_amdgcn_raw_buffer_load_b128(rb, ok ? off : BUF_OOB, 0, 0);
                xb[j][1] = __builtin_amdgcn_raw_buffer_load_b128(rb, ok ? off + 16 : BUF_OOB, 0, 0);
            }
        }
    };
    auto cvt = [&](const uint32_t4 (&v)[2]) {
        uint32_t4 h;
        h[0] = pack_h2<P>(__uint_as_float(v[0][0]), __uint_as_float(v[0][1]));
        h[1] = pack_h2<P>(__uint_as_float(v[0][2]), __uint_as_float(v[0][3]));
        h[2] = pack_h2<P>(__uint_as_float(v[1][0]), __uint_as_float(v[1][1]));
        h[3] = pack_h2<P>(__uint_as_float(v[1][2]), __uint_as_float(v[1][3]));
        return h;
    };
    auto lwrite = [&](int buf) {
#pragma unroll
        for (int j = 0; j < AC; ++j) {
            const int r = lr + 64 * j;
            As[buf][r * CH + (lc ^ ((r >> 1) & 7))] = AH ? xa[j][0] : cvt(xa[j]);
        }
#pragma unroll
        for (int j = 0; j < BC; ++j) {
            const int r = lr + 64 * j;
            Bs[buf][r * CH + (lc ^ ((r >> 1) & 7))] = BH ? xb[j][0] : cvt(xb[j]);
        }
    };
    floatx4 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int buf) {
#pragma unroll
        for (int s = 0; s < BK / 32; ++s) {
            const int kc = 4 * s + q;
            uint32_t4 af[4], bf[4];
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const int r = wm * 64 + 16 * x + c;
                af[x] = As[buf][r * CH + (kc ^ ((r >> 1) & 7))];
            }
#pragma unroll
            for (int y = 0; y < 4; ++y) {
                const int r = wn * 64 + 16 * y + c;
                bf[y] = Bs[buf][r * CH + (kc ^ ((r >> 1) & 7))];
            }
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) acc[x][y] = mfma_k32<P>(af[x], bf[y], acc[x][y]);
        }
    };
    gload(0);
    lwrite(0);
    __syncthreads();
    // two slices ahead (nk >= 4): slice kt+1's fp32 registers (loaded during
    // the previous iteration) are rounded to 16-bit at the top of iteration
    // kt, which frees them for slice kt+2's loads -- a whole iteration of
    // cover for every load at 24 more VGPRs than one slice ahead (r03d:
    // 211 VGPRs, no spill; the concatenated layers 1.1x, 65,536 x 1,024 x
    // 1,024 level; profiles/r03d_raw/big_fwd_pipe2.txt)
    auto lwrite16 = [&](int buf, const uint32_t4 (&ha)[AC], const uint32_t4 (&hb)[BC]) {
#pragma unroll
        for (int j = 0; j < AC; ++j) {
            const int r = lr + 64 * j;
            As[buf][r * CH + (lc ^ ((r >> 1) & 7))] = ha[j];
        }
#pragma unroll
        for (int j = 0; j < BC; ++j) {
            const int r = lr + 64 * j;
            Bs[buf][r * CH + (lc ^ ((r >> 1) & 7))] = hb[j];
        }
    };
    gload(1);
    int kt = 0;
    for (; kt + 2 < nk; ++kt) {
        uint32_t4 ha[AC], hb[BC];
#pragma unroll
        for (int j = 0; j < AC; ++j) ha[j] = AH ? xa[j][0] : cvt(xa[j]);
#pragma unroll
        for (int j = 0; j < BC; ++j) hb[j] = BH ? xb[j][0] : cvt(xb[j]);
        gload(kt + 2);
        compute(kt & 1);
        lwrite16((kt + 1) & 1, ha, hb);
        __syncthreads();
    }
    {
        uint32_t4 ha[AC], hb[BC];
#pragma unroll
        for (int j = 0; j < AC; ++j) ha[j] = AH ? xa[j][0] : cvt(xa[j]);
#pragma unroll
        for (int j = 0; j < BC; ++j) hb[j] = BH ? xb[j][0] : cvt(xb[j]);
        compute(kt & 1);
        lwrite16((kt + 1) & 1, ha, hb);
        __syncthreads();
        ++kt;
    }
    compute(kt & 1);
    // acc[x][y][i] is C[i0 + 64 wm + 16x + 4q + i][j0 + 64 wn + 16y + c]
#pragma unroll
    for (int y = 0; y < 4; ++y) {
        const int col = j0 + wn * 64 + 16 * y + c;
        if (col >= a.J) continue;
        const float bv = a.bias ? a.bias[g * a.bsg + col] : 0.f;
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = i0 + wm * 64 + 16 * x + 4 * q + i;
                if (row < a.I) {
                    const float v = act_fwd_t<EP>(acc[x][y][i] + bv);
                    const long at = g * a.csg + (long)row * a.csi + (long)col * a.csj;
                    if constexpr (CHF) a.c16[at] = to_half_bits<P>(v);
                    else a.C[at] = v;
                }
            }
    }
}

// ---- forward, 256 x 256 tiles on 32x32x16 MFMAs (r05) --------------------
// The wide configuration's inference chain (16-bit X, W and Y: the a16 / b16
// / c16 operands of td7_dense_fwd_h) at 65,536 rows, where
// dense_fwd_big_kernel ran at 380-520 TFLOP/s (65,536 x 1,024 x 1,024 /
// 2,048; tools/wide_gemm_compare.py).  Two kernels:
//  - dense_fwd_xl8_kernel (K % 64 == 0, the default): 8 waves of 128 x 64,
//    LDS-DMA staging, below;
//  - dense_fwd_xl_kernel (any K % 8 == 0): 4 waves each owning a 128 x 128
//    tile as 4 x 4 accumulators (all 256 accumulator registers, one wave per
//    SIMD), register-staged slices software pipelined into the MFMA bursts.
// Both: slices of BK = 64 through a double-buffered LDS stage (128 KB,
// dynamic), 16-byte chunks of a row XOR-swizzled, the output tile staged
// through the same LDS so the 16-bit stores are whole 16-byte rows.  Lane l of
// a 32x32x16 MFMA holds A[row l & 31][k = 8 (l >> 5) + j] and B[k = 8 (l >> 5)
// + j][col l & 31]; C[row (r & 3) + 8 (r >> 2) + 4 (l >> 5)][col l & 31] in
// accumulator register r.  Measured (r05, profiles/r05_xl): at 65,536 x
// 1,024 x 1,024 dense_fwd_big_kernel 289 us per call (ops.dense, 16-bit in
// and out), dense_fwd_xl_kernel 252, dense_fwd_xl8_kernel 194; the first
// xl cut (no software pipelining) 269, xl8 with a 4-stage ring of 32-deep
// halves 203, s_setprio around the MFMA bursts +-0 -- not kept.
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int XL_BM = 256, XL_BN = 256, XL_BK = 64, XL_CH = XL_BK / 8;
constexpr int XL_LDS = 2 * (XL_BM + XL_BN) * XL_CH * 16;  // 128 KB

template <int P>
__device__ __forceinline__ floatx16 mfma32_k16(uint32_t4 a, uint32_t4 b, floatx16 c) {
    if constexpr (P == PREC_F16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8_t, a), __builtin_bit_cast(halfx8_t, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                       __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

template <int EP, int P, bool CAT, bool CHF>
__global__ __launch_bounds__(256) void dense_fwd_xl_kernel(GemmArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t4 xl_smem[];
    constexpr int BM = XL_BM, BN = XL_BN, BK = XL_BK, CH = XL_CH;
    uint32_t4 *const As = xl_smem, *const Bs = xl_smem + 2 * BM * CH;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
    const int l31 = lane & 31, lh = lane >> 5;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * BM, j0 = tile.x * BN, g = tile.z;
    const int K = a.R, nk = (K + BK - 1) / BK;
    const int lr = t >> 3, lc = t & 7;  // this thread's chunks: rows lr + 32 j, chunk column lc
    const int wsw = lr * CH + (lc ^ (lr & 7));  // its LDS chunk in row lr (rows lr + 32 j: + 32 j CH)
    const __amdgpu_buffer_rsrc_t rb = rsrc(reinterpret_cast<const float *>(a.b16 + (long)g * a.J * a.R));
    __amdgpu_buffer_rsrc_t ra = CAT ? rsrc(a.cat.p[0]) : rsrc(reinterpret_cast<const float *>(a.a16 + g * a.A.sg));
    int lda = CAT ? a.cat.ld[0] : (int)a.A.si, kbase = 0, seg = 0;
    uint32_t4 xa[8], xb[8];
    auto gseg = [&](int kt) {
        if constexpr (CAT) {  // the slice's segment (boundaries are multiples of BK)
            const int s = cat_seg(a.cat, kt * BK);
            if (s != seg || kt == 0) {
                seg = s;
                const float *p = a.cat.p[0];
                long gs = a.cat.sg[0];
                int ld = a.cat.ld[0], kb = 0;
#pragma unroll
                for (int m = 1; m < CAT_MAX; ++m)
                    if (s == m) p = a.cat.p[m], gs = a.cat.sg[m], ld = a.cat.ld[m], kb = a.cat.kb[m];
                ra = rsrc(reinterpret_cast<const float *>(reinterpret_cast<const uint16_t *>(p) + g * gs));
                lda = ld;
                kbase = kb;
            }
        }
    };
    // chunk j of slice kt (past the last slice: zeros, no access)
    auto ga = [&](int kt, int j) {
        const int k = kt * BK + 8 * lc, row = i0 + lr + 32 * j;
        xa[j] = __builtin_amdgcn_raw_buffer_load_b128(ra, (k < K && row < a.I) ? (row * lda + k - kbase) * 2 : BUF_OOB,
                                                      0, 0);
    };
    auto gb = [&](int kt, int j) {
        const int k = kt * BK + 8 * lc, col = j0 + lr + 32 * j;
        xb[j] = __builtin_amdgcn_raw_buffer_load_b128(rb, (k < K && col < a.J) ? (col * a.R + k) * 2 : BUF_OOB, 0, 0);
    };
    auto gload = [&](int kt) {
        gseg(kt);
#pragma unroll
        for (int j = 0; j < 8; ++j) ga(kt, j);
#pragma unroll
        for (int j = 0; j < 8; ++j) gb(kt, j);
    };
    auto lwrite = [&](int buf) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            As[buf * BM * CH + wsw + 32 * j * CH] = xa[j];
            Bs[buf * BN * CH + wsw + 32 * j * CH] = xb[j];
        }
    };
    floatx16 acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;
    // this lane's fragments of k-step ks (16 columns) of an LDS slice
    auto frag = [&](const uint32_t4 *A, const uint32_t4 *B, int ks, uint32_t4 (&af)[4], uint32_t4 (&bf)[4]) {
        const int ch = 2 * ks + lh;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            const int r = wm * 128 + 32 * x + l31;
            af[x] = A[r * CH + (ch ^ (r & 7))];
        }
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const int r = wn * 128 + 32 * y + l31;
            bf[y] = B[r * CH + (ch ^ (r & 7))];
        }
    };
    auto mma = [&](const uint32_t4 (&af)[4], const uint32_t4 (&bf)[4]) {
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) acc[x][y] = mfma32_k16<P>(af[x], bf[y], acc[x][y]);
    };
    gload(0);
    lwrite(0);
    if (nk > 1) gload(1);
    __syncthreads();
    // software pipelined: k-step ks + 1's fragments are read while ks's 16
    // MFMAs run, and the next slice's chunks (loaded a slice earlier) go
    // to the other LDS buffer between them, each register reloaded with
    // slice kt + 2 as soon as it is written -- branch-free (past the last
    // slice the loads return zeros and the writes land in the idle
    // buffer), so the schedule hints below see the whole slice
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1, nxt = cur ^ 1;
        const uint32_t4 *A = As + cur * BM * CH, *B = Bs + cur * BN * CH;
        uint32_t4 *An = As + nxt * BM * CH + wsw, *Bn = Bs + nxt * BN * CH + wsw;
        gseg(kt + 2);
        uint32_t4 f[2][2][4];
        frag(A, B, 0, f[0][0], f[0][1]);
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            if (ks + 1 < BK / 16) frag(A, B, ks + 1, f[(ks + 1) & 1][0], f[(ks + 1) & 1][1]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int j = 2 * ks + h;
                An[32 * j * CH] = xa[j];
                Bn[32 * j * CH] = xb[j];
                ga(kt + 2, j);
                gb(kt + 2, j);
            }
            mma(f[ks & 1][0], f[ks & 1][1]);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // LDS read
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // LDS write
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // global load
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
        }
        __syncthreads();
    }
    // epilogue: bias + activation
    if constexpr (CHF) {
        // the 256 x 256 tile of 16-bit values through the LDS stage ([row][256],
        // 512-byte rows), then whole 16-byte chunks out
        uint16_t *Cs = reinterpret_cast<uint16_t *>(xl_smem);
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const int cl = wn * 128 + 32 * y + l31, col = j0 + cl;
            const float bv = (a.bias && col < a.J) ? a.bias[g * a.bsg + col] : 0.f;
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int rl = wm * 128 + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * lh;
                    Cs[rl * BN + cl] = to_half_bits<P>(act_fwd_t<EP>(acc[x][y][e] + bv));
                }
        }
        __syncthreads();
        const uint32_t4 *C4 = reinterpret_cast<const uint32_t4 *>(Cs);
        for (int q = t; q < BM * (BN / 8); q += 256) {
            const int rl = q / (BN / 8), cc = q - rl * (BN / 8);
            const int row = i0 + rl, col = j0 + 8 * cc;
            if (row >= a.I || col >= a.J) continue;
            const long at = g * a.csg + (long)row * a.csi + col;  // (csj == 1: rows contiguous)
            if (col + 8 <= a.J) {
                *reinterpret_cast<uint32_t4 *>(a.c16 + at) = C4[q];
            } else {
                for (int e = 0; e < a.J - col; ++e) a.c16[at + e] = Cs[rl * BN + 8 * cc + e];
            }
        }
    } else {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const int col = j0 + wn * 128 + 32 * y + l31;
            if (col >= a.J) continue;
            const float bv = a.bias ? a.bias[g * a.bsg + col] : 0.f;
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = i0 + wm * 128 + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * lh;
                    if (row < a.I) a.C[g * a.csg + (long)row * a.csi + (long)col * a.csj] = act_fwd_t<EP>(acc[x][y][e] + bv);
                }
        }
    }
}

// bias + activation of the 8 waves' 128 x 64 accumulators (4 x 2 of 32x32);
// a 16-bit output through the LDS stage as whole 16-byte rows (the stage
// must be idle: every wave past its last fragment read, no DMA in flight)
template <int EP, int P, bool CHF>
__device__ __forceinline__ void xl8_epilogue(const GemmArgs &a, floatx16 (&acc)[4][2], int i0, int j0, int g) {
    extern __shared__ __attribute__((aligned(16))) uint32_t4 xl_smem[];
    constexpr int BM = XL_BM, BN = XL_BN;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 2, wn = w & 3;
    const int l31 = lane & 31, lh = lane >> 5;
    if constexpr (CHF) {
        uint16_t *Cs = reinterpret_cast<uint16_t *>(xl_smem);
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int cl = wn * 64 + 32 * y + l31, col = j0 + cl;
            const float bv = (a.bias && col < a.J) ? a.bias[g * a.bsg + col] : 0.f;
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int rl = wm * 128 + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * lh;
                    Cs[rl * BN + cl] = to_half_bits<P>(act_fwd_t<EP>(acc[x][y][e] + bv));
                }
        }
        __syncthreads();
        const uint32_t4 *C4 = reinterpret_cast<const uint32_t4 *>(Cs);
        for (int q = t; q < BM * (BN / 8); q += 512) {
            const int rl = q / (BN / 8), cc = q - rl * (BN / 8);
            const int row = i0 + rl, col = j0 + 8 * cc;
            if (row >= a.I || col >= a.J) continue;
            const long at = g * a.csg + (long)row * a.csi + col;  // (csj == 1: rows contiguous)
            if (col + 8 <= a.J) {
                *reinterpret_cast<uint32_t4 *>(a.c16 + at) = C4[q];
            } else {
                for (int e = 0; e < a.J - col; ++e) a.c16[at + e] = Cs[rl * BN + 8 * cc + e];
            }
        }
    } else {
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int col = j0 + wn * 64 + 32 * y + l31;
            if (col >= a.J) continue;
            const float bv = a.bias ? a.bias[g * a.bsg + col] : 0.f;
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int row = i0 + wm * 128 + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * lh;
                    if (row < a.I) a.C[g * a.csg + (long)row * a.csi + (long)col * a.csj] = act_fwd_t<EP>(acc[x][y][e] + bv);
                }
        }
    }
}

// The same 256 x 256 tile with 8 waves (2 per SIMD: one wave's LDS reads
// hide behind the other's MFMAs) of 128 x 64 each (4 x 2 accumulators of
// 32x32x16, 128 accumulator registers), and LDS-DMA staging: every slice
// goes global -> LDS by buffer_load ... lds (no VGPR round trip, no
// ds_write pass), 8 pieces of 8 rows x 128 B per wave and slice.  A piece's
// LDS image is lane-linear, so the XOR swizzle of dense_fwd_xl_kernel is
// applied on the SOURCE side (lane l of a piece loads chunk (l & 7) ^ (row &
// 7) into slot l & 7); the fragment reads are the same.  Two LDS buffers:
// slice kt + 1 is in flight while slice kt is multiplied; the barrier at the
// end of a slice waits for it (the only vmcnt(0) of the loop).
template <int EP, int P, bool CAT, bool CHF>
__global__ __launch_bounds__(512) void dense_fwd_xl8_kernel(GemmArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t4 xl_smem[];
    constexpr int BM = XL_BM, BN = XL_BN, BK = XL_BK, CH = XL_CH;
    uint32_t4 *const As = xl_smem, *const Bs = xl_smem + 2 * BM * CH;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 2, wn = w & 3;
    const int l31 = lane & 31, lh = lane >> 5;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * BM, j0 = tile.x * BN, g = tile.z;
    const int K = a.R, nk = (K + BK - 1) / BK;
    // this lane's piece geometry: row 8 p + pr of the tile; its slot lane & 7
    // holds chunk (lane & 7) ^ (((8 p + pr) >> 1) & 7) = (lane & 7) ^ (4 (p & 1) +
    // (pr >> 1)) -- rows of one parity get 8 distinct slots, so the 16 lanes of
    // a fragment read's pass (16 consecutive rows, one chunk) hit 16 distinct
    // 16-byte bank groups (a (r & 7) swizzle pairs rows r and r + 8: 2-way)
    const int pr = lane >> 3;
    auto pcol = [&](int p) { return (lane & 7) ^ (((p & 1) << 2) | (pr >> 1)); };
    const __amdgpu_buffer_rsrc_t rb = rsrc(reinterpret_cast<const float *>(a.b16 + (long)g * a.J * a.R));
    __amdgpu_buffer_rsrc_t ra = CAT ? rsrc(a.cat.p[0]) : rsrc(reinterpret_cast<const float *>(a.a16 + g * a.A.sg));
    int lda = CAT ? a.cat.ld[0] : (int)a.A.si, kbase = 0, seg = 0;
    auto gseg = [&](int kt) {
        if constexpr (CAT) {  // the slice's segment (boundaries are multiples of BK)
            const int s = cat_seg(a.cat, kt * BK);
            if (s != seg || kt == 0) {
                seg = s;
                const float *p = a.cat.p[0];
                long gs = a.cat.sg[0];
                int ld = a.cat.ld[0], kb = 0;
#pragma unroll
                for (int m = 1; m < CAT_MAX; ++m)
                    if (s == m) p = a.cat.p[m], gs = a.cat.sg[m], ld = a.cat.ld[m], kb = a.cat.kb[m];
                ra = rsrc(reinterpret_cast<const float *>(reinterpret_cast<const uint16_t *>(p) + g * gs));
                lda = ld;
                kbase = kb;
            }
        }
    };
    // slice kt into LDS buffer buf: this wave's pieces p = 4 w + i of A and B.
    // K % 64 == 0 (the launcher's condition), so every chunk is inside K; a
    // row past I or a column past J starts at BUF_OOB (unsigned offsets: the
    // load returns zeros), no per-load select
    uint32_t brow[4], bcol[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 8 * (4 * w + i) + pr;
        bcol[i] = j0 + r < a.J ? (uint32_t)((j0 + r) * a.R + 8 * pcol(4 * w + i)) * 2u : (uint32_t)BUF_OOB;
    }
    auto rows = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 8 * (4 * w + i) + pr;
            brow[i] = i0 + r < a.I ? (uint32_t)((i0 + r) * lda + 8 * pcol(4 * w + i) - kbase) * 2u : (uint32_t)BUF_OOB;
        }
    };
    rows();
    auto issue = [&](int kt, int buf) {
        if constexpr (CAT) {
            const int s0 = seg;
            gseg(kt);
            if (seg != s0) rows();
        }
        const uint32_t kb = (uint32_t)kt * BK * 2u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = 4 * w + i;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                ra, (__attribute__((address_space(3))) void *)(As + buf * BM * CH + p * 64), 16, brow[i] + kb, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rb, (__attribute__((address_space(3))) void *)(Bs + buf * BN * CH + p * 64), 16, bcol[i] + kb, 0, 0, 0);
        }
    };
    floatx16 acc[4][2];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;
    auto frag = [&](const uint32_t4 *A, const uint32_t4 *B, int ks, uint32_t4 (&af)[4], uint32_t4 (&bf)[2]) {
        const int ch = 2 * ks + lh;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            const int r = wm * 128 + 32 * x + l31;
            af[x] = A[r * CH + (ch ^ ((r >> 1) & 7))];
        }
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int r = wn * 64 + 32 * y + l31;
            bf[y] = B[r * CH + (ch ^ ((r >> 1) & 7))];
        }
    };
    if constexpr (CAT) gseg(0), rows();
    issue(0, 0);
    // the LDS-DMA's completion is this wave's vmcnt; __syncthreads() alone
    // does not wait for it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
        const uint32_t4 *A = As + cur * BM * CH, *B = Bs + cur * BN * CH;
        uint32_t4 fa[2][4], fb[2][2];
        frag(A, B, 0, fa[0], fb[0]);
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            if (ks + 1 < BK / 16) frag(A, B, ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y) acc[x][y] = mfma32_k16<P>(fa[ks & 1][x], fb[ks & 1][y], acc[x][y]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    xl8_epilogue<EP, P, CHF>(a, acc, i0, j0, g);
}

template <int EP, int P, bool CAT, bool CHF>
void launch_fwd_xl_one(const GemmArgs &a, dim3 grid, int variant, hipStream_t s) {
    if (variant == 2) {
        (void)hipFuncSetAttribute((const void *)dense_fwd_xl8_kernel<EP, P, CAT, CHF>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, XL_LDS);
        hipLaunchKernelGGL((dense_fwd_xl8_kernel<EP, P, CAT, CHF>), grid, dim3(512), XL_LDS, s, a);
    } else {
        (void)hipFuncSetAttribute((const void *)dense_fwd_xl_kernel<EP, P, CAT, CHF>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, XL_LDS);
        hipLaunchKernelGGL((dense_fwd_xl_kernel<EP, P, CAT, CHF>), grid, dim3(256), XL_LDS, s, a);
    }
}

// variant 2: dense_fwd_xl8_kernel (K % 64 == 0), else dense_fwd_xl_kernel
template <int P, bool CAT>
void launch_fwd_xl_p(const GemmArgs &a, dim3 grid, int variant, hipStream_t s) {
#define FWD_XL(EPv)                                                                                                \
    (a.c16 ? launch_fwd_xl_one<EPv, P, CAT, true>(a, grid, variant, s)                                             \
           : launch_fwd_xl_one<EPv, P, CAT, false>(a, grid, variant, s))
    switch (a.act) {
    case ACT_RELU: FWD_XL(ACT_RELU); break;
    case ACT_ELU: FWD_XL(ACT_ELU); break;
    case ACT_TANH: FWD_XL(ACT_TANH); break;
    default: FWD_XL(ACT_NONE); break;
    }
#undef FWD_XL
}

template <int P, bool CAT>
void launch_fwd_big_p(const GemmArgs &a, dim3 grid, int bm, hipStream_t s) {
#define FWD_BIG(EPv)                                                                                               \
    do {                                                                                                         \
        if (bm == 256) hipLaunchKernelGGL((dense_fwd_big_kernel<EPv, P, CAT, 256, 128>), grid, dim3(512), 0, s, a); \
        else if (a.b16 && a.c16 && a.a16)                                                                        \
            hipLaunchKernelGGL((dense_fwd_big_kernel<EPv, P, CAT, 128, 256, true, true, true>), grid, dim3(512), 0, s, a); \
        else if (a.b16 && a.a16 && !CAT)                                                                         \
            hipLaunchKernelGGL((dense_fwd_big_kernel<EPv, P, CAT, 128, 256, true, true, false>), grid, dim3(512), 0, s, a); \
        else if (a.b16 && a.c16)                                                                                 \
            hipLaunchKernelGGL((dense_fwd_big_kernel<EPv, P, CAT, 128, 256, true, false, true>), grid, dim3(512), 0, s, a); \
        else if (a.b16)                                                                                          \
            hipLaunchKernelGGL((dense_fwd_big_kernel<EPv, P, CAT, 128, 256, true>), grid, dim3(512), 0, s, a);     \
        else hipLaunchKernelGGL((dense_fwd_big_kernel<EPv, P, CAT, 128, 256>), grid, dim3(512), 0, s, a);           \
    } while (0)
    switch (a.act) {
    case ACT_RELU: FWD_BIG(ACT_RELU); break;
    case ACT_ELU: FWD_BIG(ACT_ELU); break;
    case ACT_TANH: FWD_BIG(ACT_TANH); break;
    default: FWD_BIG(ACT_NONE); break;
    }
#undef FWD_BIG
}

// ---- bwd-weight on the output-contiguous layout ------------------------------
// dW[g][i][j] = sum_m dP[m][i] X[m][j], dP = dY * act'(Y), db[g][i] = sum_m dP[m][i].
// Both operands are contiguous along the OUTPUT dimensions (i resp. j) and
// strided along the reduction m, so the k-permutation of the forward kernel
// is applied to the output dimensions instead: in a 4-row step (rows m0..m0+3)
// lane (c, q) loads VA consecutive i of row m0+q (one b32/b64/b128) and 4
// consecutive j of that row (one b128).  MFMA (s, t) of the step multiplies A
// row r <-> i = i0 + VA*r + s with B column c <-> j = j0 + 4c + t: VA*4 MFMAs
// per 2-3 vector loads, a (16 VA) x 64 tile per workgroup.  The NW waves of a
// workgroup take the steps round-robin and are summed through LDS.
//
// Lanes past the edge load the last VA (4) in-range elements of the row and
// shift them into place; what they deliver for rows i >= I / columns j >= J
// only reaches accumulator elements that are never stored.  Rows m >= M load 0.
struct WgradArgs {
    CatSeg cat; // CAT: X by segments (along j)
    const float *dy, *y, *x;
    int dysg, lddy, ysg, ldy, xsg, ldx;
    float *dw, *db;
    int I, J, M;
};

template <int VA>
__device__ __forceinline__ void ld_vec(__amdgpu_buffer_rsrc_t r, int byte_off, float (&v)[VA]) {
    if (VA == 4) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = __uint_as_float(x[e]);
    } else if (VA == 2) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0);
        v[0] = __uint_as_float(x[0]);
        v[VA - 1] = __uint_as_float(x[1]);
    } else {
        v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
    }
}

// out[e] = v[min(e + sh, VA - 1)]  (sh > 0 only on the edge lanes)
// (written as a select on sh with constant indices: a compare against e + sh
// lets the compiler fold the chain into a dynamic index -> scratch)
template <int VA>
__device__ __forceinline__ float shifted(const float (&v)[VA], int sh, int e) {
    float o = v[VA - 1];
#pragma unroll
    for (int d = VA - 2; d >= 0; --d) o = (sh == d) ? v[e + d < VA ? e + d : VA - 1] : o;
    return o;
}

template <int AG, int VA, int NW, int P, bool CAT>
__global__ __launch_bounds__(64 * NW) void dense_wgrad_kernel(WgradArgs a) {
    constexpr int KS = VA == 1 ? 8 : 4; // 4-row steps per prefetch group (two groups in flight)
    constexpr int NACC = VA * 4;
    __shared__ float red[NW > 1 ? NW / 2 : 1][NACC * 4 + VA][64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, q = lane >> 4, c = lane & 15;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * 16 * VA, j0 = tile.x * 64, g = tile.z;
    const int ia = i0 + VA * c, ib = min(ia, a.I - VA), shi = ia - ib;
    const int ja = j0 + 4 * c, jb = min(ja, a.J - 4), shj = ja - jb;
    const __amdgpu_buffer_rsrc_t rdy = rsrc(a.dy), ry = rsrc(AG > 0 ? a.y : a.dy), rx = rsrc(a.x);
    const int dyb = g * a.dysg + ib, yb = g * a.ysg + ib, xb = g * a.xsg + jb;
    const float *xcat = nullptr; // CAT: this lane's 4 columns jb .. jb+3 (one segment)
    int xld = 0;
    if constexpr (CAT) {
        const int sg = cat_seg(a.cat, jb);
        const float *p = a.cat.p[0];
        long gs = a.cat.sg[0];
        int ld = a.cat.ld[0], kb = a.cat.kb[0];
#pragma unroll
        for (int k = 1; k < CAT_MAX; ++k)
            if (sg == k) p = a.cat.p[k], gs = a.cat.sg[k], ld = a.cat.ld[k], kb = a.cat.kb[k];
        xcat = p + g * gs + (jb - kb);
        xld = ld;
    }
    const int nks = (a.M + 3) >> 2;
    const int my = nks > w ? (nks - w + NW - 1) / NW : 0;
    const int ngrp = (my + KS - 1) / KS;

    struct Buf {
        float a[KS][VA], y[KS][VA], b[KS][4];
        bool lv[CAT ? KS : 1]; // CAT: row m in range (the X load is masked where consumed)
    };
    floatx4 acc[VA][4];
    float bsum[VA];
#pragma unroll
    for (int s = 0; s < VA; ++s) {
        bsum[s] = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[s][u] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    auto load = [&](int grp, Buf &f) {
#pragma unroll
        for (int sp = 0; sp < KS; ++sp) {
            const int k = grp * KS + sp;
            const int m = 4 * (w + k * NW) + q;
            const bool live = (k < my) & (m < a.M);
            ld_vec<VA>(rdy, live ? (dyb + m * a.lddy) * 4 : BUF_OOB, f.a[sp]);
            if (AG > 0) ld_vec<VA>(ry, live ? (yb + m * a.ldy) * 4 : BUF_OOB, f.y[sp]);
            if constexpr (CAT) {
                // a valid address for dead rows, zeroed at the MFMA (no wait here)
                const uint32_t4 v = *(gptr4)(live ? xcat + (long)m * xld : xcat);
                f.lv[CAT ? sp : 0] = live;
#pragma unroll
                for (int e = 0; e < 4; ++e) f.b[sp][e] = __uint_as_float(v[e]);
            } else {
                ld_vec<4>(rx, live ? (xb + m * a.ldx) * 4 : BUF_OOB, f.b[sp]);
            }
        }
    };
    auto mma = [&](const Buf &f) {
        if constexpr (P != PREC_F32) {
            // four 4-row steps form one 16-deep MFMA: k-slot 4q + e of lane
            // (c, q) is row m of step e (the same m on both operands)
#pragma unroll
            for (int s4 = 0; s4 < KS; s4 += 4) {
                float fa[VA][4], fb[4][4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
#pragma unroll
                    for (int s = 0; s < VA; ++s) {
                        float v = shifted<VA>(f.a[s4 + e], shi, s);
                        if (AG > 0) v *= act_grad_t<AG>(shifted<VA>(f.y[s4 + e], shi, s));
                        bsum[s] += v;
                        fa[s][e] = v * grad_scale<P>();
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        fb[u][e] = shifted<4>(f.b[s4 + e], shj, u);
                        if constexpr (CAT) fb[u][e] = f.lv[CAT ? s4 + e : 0] ? fb[u][e] : 0.f;
                    }
                }
#pragma unroll
                for (int s = 0; s < VA; ++s)
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc[s][u] = mfma_k16<P>(fa[s], fb[u], acc[s][u]);
            }
            return;
        }
#pragma unroll
        for (int sp = 0; sp < KS; ++sp) {
            float fa[VA], fb[4];
#pragma unroll
            for (int s = 0; s < VA; ++s) {
                fa[s] = shifted<VA>(f.a[sp], shi, s);
                if (AG > 0) fa[s] *= act_grad_t<AG>(shifted<VA>(f.y[sp], shi, s));
                bsum[s] += fa[s];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                fb[u] = shifted<4>(f.b[sp], shj, u);
                if constexpr (CAT) fb[u] = f.lv[CAT ? sp : 0] ? fb[u] : 0.f;
            }
#pragma unroll
            for (int s = 0; s < VA; ++s)
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[s][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[s], fb[u], acc[s][u], 0, 0, 0);
        }
    };
    Buf b0, b1;
    if (ngrp > 0) load(0, b0);
    for (int grp = 0; grp < ngrp; grp += 2) {
        if (grp + 1 < ngrp) load(grp + 1, b1);
        mma(b0);
        if (grp + 1 >= ngrp) break;
        if (grp + 2 < ngrp) load(grp + 2, b0);
        mma(b1);
    }
    // tree-sum the NW partial tiles through LDS (lane-major: conflict free)
#pragma unroll
    for (int half = NW / 2; half >= 1; half >>= 1) {
        if (w >= half && w < 2 * half) {
#pragma unroll
            for (int s = 0; s < VA; ++s) {
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < 4; ++k) red[w - half][(s * 4 + u) * 4 + k][lane] = acc[s][u][k];
                red[w - half][NACC * 4 + s][lane] = bsum[s];
            }
        }
        __syncthreads();
        if (w < half) {
#pragma unroll
            for (int s = 0; s < VA; ++s) {
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[s][u][k] += red[w][(s * 4 + u) * 4 + k][lane];
                bsum[s] += red[w][NACC * 4 + s][lane];
            }
        }
        __syncthreads();
    }
    if (w > 0) return;
    // acc[s][u][k] is dW[i0 + VA*(4q + k) + s][j0 + 4c + u]
    float *dwg = a.dw + (long)g * a.I * a.J;
#pragma unroll
    for (int s = 0; s < VA; ++s)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = i0 + VA * (4 * q + k) + s;
            if (i >= a.I) continue;
            float *row = dwg + (long)i * a.J;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (ja + u < a.J) row[ja + u] = acc[s][u][k] * (1.f / grad_scale<P>());
        }
    if (a.db && tile.x == 0) {
#pragma unroll
        for (int s = 0; s < VA; ++s) {
            float v = bsum[s];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (q == 0 && ia + s < a.I) a.db[(long)g * a.I + ia + s] = v;
        }
    }
}

template <int P, bool CAT>
void launch_wgrad_p(const WgradArgs &a, dim3 grid, int va, int nw, int act, hipStream_t s) {
#define WG_NW(AGv, VAv)                                                                              \
    do {                                                                                           \
        if (nw == 8) hipLaunchKernelGGL((dense_wgrad_kernel<AGv, VAv, 8, P, CAT>), grid, dim3(512), 0, s, a); \
        else if (nw == 4) hipLaunchKernelGGL((dense_wgrad_kernel<AGv, VAv, 4, P, CAT>), grid, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((dense_wgrad_kernel<AGv, VAv, 2, P, CAT>), grid, dim3(128), 0, s, a);       \
    } while (0)
#define WG_VA(AGv)                      \
    do {                              \
        if (va == 4) WG_NW(AGv, 4);   \
        else if (va == 2) WG_NW(AGv, 2); \
        else WG_NW(AGv, 1);           \
    } while (0)
    switch (act) {
    case ACT_RELU: WG_VA(ACT_RELU); break;
    case ACT_ELU: WG_VA(ACT_ELU); break;
    case ACT_TANH: WG_VA(ACT_TANH); break;
    default: WG_VA(ACT_NONE); break;
    }
#undef WG_VA
#undef WG_NW
}

template <int P, bool CAT, bool AH = false>
void launch_fwd_p(const GemmArgs &a, dim3 grid, int tm, int tn, int kw, int wsteps, hipStream_t s) {
#define FWD_GS(EPv, TMv, TNv, KWv)                                                                              \
    do {                                                                                                      \
        const dim3 blk(64 * KWv);                                                                             \
        if (wsteps <= 5) hipLaunchKernelGGL((dense_fwd_kernel<EPv, 5, TMv, TNv, KWv, P, CAT, AH>), grid, blk, 0, s, a); \
        else if (TMv * TNv == 1 && wsteps <= 20)                                                              \
            hipLaunchKernelGGL((dense_fwd_kernel<EPv, 20, TMv, TNv, KWv, P, CAT, AH>), grid, blk, 0, s, a);        \
        else if (TMv * TNv == 1)                                                                              \
            hipLaunchKernelGGL((dense_fwd_kernel<EPv, 10, TMv, TNv, KWv, P, CAT, AH>), grid, blk, 0, s, a);        \
        else hipLaunchKernelGGL((dense_fwd_kernel<EPv, 5, TMv, TNv, KWv, P, CAT, AH>), grid, blk, 0, s, a);         \
    } while (0)
#define FWD_LAUNCH(EPv)                                                                 \
    do {                                                                                \
        if (tm == 2 && tn == 2) FWD_GS(EPv, 2, 2, 1);                                   \
        else if (kw == 2) FWD_GS(EPv, 1, 1, 2);                                         \
        else FWD_GS(EPv, 1, 1, 1);                                                      \
    } while (0)
    switch (a.act) {
    case ACT_RELU: FWD_LAUNCH(ACT_RELU); break;
    case ACT_ELU: FWD_LAUNCH(ACT_ELU); break;
    case ACT_TANH: FWD_LAUNCH(ACT_TANH); break;
    default: FWD_LAUNCH(ACT_NONE); break;
    }
#undef FWD_LAUNCH
#undef FWD_GS
}


} // namespace td7dense
