// td7_dense.hip -- fused dense layers of the TD7 nets on fp32 MFMA (gfx950).
//
// Every Linear of Agent/TD7_multi_agent.py:61-140 is followed by an
// activation (ELU / ReLU / tanh / none).  In PyTorch one layer is a
// hipBLASLt GEMM plus an elementwise kernel forward and elementwise-backward,
// two GEMMs, a column reduction and a fill backward.  Here:
//
//   forward      Y  = act(X W^T + b)                      1 kernel
//   bwd-data     dX = (dY * act'(Y)) W                    1 kernel  (act' in the A prologue)
//   bwd-weight   dW = (dY * act'(Y))^T X,  db = colsum    1 kernel  (db = the GEMM against a ones column)
//
// act'(pre) is recovered from the saved output Y: ELU 1|Y+1, ReLU 1|0,
// tanh 1-Y^2 -- nothing but Y, X and W is kept for backward.
//
// All three are one GEMM core: C[i][j] = sum_r A(i,r) B(j,r) with arbitrary
// element strides on v_mfma_f32_16x16x4_f32 (layout notes at the kernel).
// Groups (the critic's two Q heads) are the grid's z dimension; an input
// shared by the groups (stride 0) has its bwd-data reduced over the groups
// inside the kernel.  fp32 in, fp32 accumulate: exact f32 fma chains.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "exo_amd.h"

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2, ACT_TANH = 3 };

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

struct GemmArgs {
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

template <int AG, int EP, bool AV, bool BV, int NW>
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

    auto load = [&](int grp, Frag &fa, Frag &fy, Frag &fb) {
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
            if (a.B.ones_col >= 0) { // bwd-weight: column ones_col of B is all ones (-> bias gradient)
#pragma unroll
                for (int tl = 0; tl < 2; ++tl)
                    if (j0 + 16 * tl + c == a.B.ones_col)
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) fb.v[sp][tl][jj] = (r0 + 4 * q + jj < a.R) ? 1.f : 0.f;
            }
        }
    };
    auto mma = [&](const Frag &fa, const Frag &fy, const Frag &fb) {
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
    Frag a0, y0, b0, a1, y1, b1;
    if (ngrp > 0) load(0, a0, y0, b0);
    for (int grp = 0; grp < ngrp; grp += 2) {
        if (grp + 1 < ngrp) load(grp + 1, a1, y1, b1);
        mma(a0, y0, b0);
        if (grp + 1 >= ngrp) break;
        if (grp + 2 < ngrp) load(grp + 2, a0, y0, b0);
        mma(a1, y1, b1);
    }
    // sum the NW partial tiles: waves 1.. park theirs in LDS, wave 0 adds them
    // acc[x][y][k] is C[i0 + 16x + 4q + k][j0 + 16y + c]
    if (NW > 1) {
        if (w > 0)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int k = 0; k < 4; ++k) red[w - 1][16 * x + 4 * q + k][16 * y + c] = acc[x][y][k];
        __syncthreads();
        if (w > 0) return;
#pragma unroll
        for (int ww = 0; ww < NW - 1; ++ww)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[x][y][k] += red[ww][16 * x + 4 * q + k][16 * y + c];
    }
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
                const float v = acc[x][y][k];
                if (is_bias) a.bias_grad[g * a.bgsg + row] = v;
                else a.C[g * a.csg + (long)row * a.csi + (long)col * a.csj] = act_fwd_t<EP>(v + bias_v);
            }
    }
}

int launch(const GemmArgs &a, int groups_grid, hipStream_t s) {
    const int Jt = a.J + (a.j_bias >= 0 ? 1 : 0);
    dim3 grid((Jt + 31) / 32, (a.I + 31) / 32, groups_grid);
    // 32-bit element offsets inside the kernel (byte offsets below BUF_BYTES)
    const int gmax = a.groups_red > 1 ? a.groups_red : groups_grid;
    const long span_a = (long)gmax * a.A.sg + (long)a.I * a.A.si + (long)a.R * a.A.sr;
    const long span_b = (long)gmax * a.B.sg + (long)(a.J + 1) * a.B.si + (long)a.R * a.B.sr;
    if (span_a >= (1L << 29) || span_b >= (1L << 29)) return EXO_ERANGE;
    // split the reduction over more waves when the tile grid alone is small
    const long tiles = (long)grid.x * grid.y * grid.z;
    const long steps = (long)((a.R + 15) / 16) * a.groups_red;
    // waves per workgroup: about one wave per SIMD of the chip (1024), at
    // least 4 reduction steps per wave
    int nw = 2;
    while (nw < 8 && tiles * nw * 2 <= 1024 && steps >= 4L * nw * 2) nw *= 2;
#define DENSE_LAUNCH(AGv, EPv, AVv, BVv)                                                                         \
    do {                                                                                                       \
        if (nw == 8) hipLaunchKernelGGL((dense_gemm_kernel<AGv, EPv, AVv, BVv, 8>), grid, dim3(512), 0, s, a); \
        else if (nw == 4) hipLaunchKernelGGL((dense_gemm_kernel<AGv, EPv, AVv, BVv, 4>), grid, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((dense_gemm_kernel<AGv, EPv, AVv, BVv, 2>), grid, dim3(128), 0, s, a);        \
    } while (0)
    const bool av = a.A.sr == 1, bv = a.B.sr == 1;
    if (a.A.act < 0) { // forward: both operands contiguous along the reduction
        if (!(av && bv)) return EXO_EINVAL;
        switch (a.act) {
        case ACT_RELU: DENSE_LAUNCH(-1, ACT_RELU, true, true); break;
        case ACT_ELU: DENSE_LAUNCH(-1, ACT_ELU, true, true); break;
        case ACT_TANH: DENSE_LAUNCH(-1, ACT_TANH, true, true); break;
        default: DENSE_LAUNCH(-1, ACT_NONE, true, true); break;
        }
    } else if (av) {   // bwd-data: dY rows contiguous, W^T column walk
        switch (a.A.act) {
        case ACT_RELU: DENSE_LAUNCH(ACT_RELU, ACT_NONE, true, false); break;
        case ACT_ELU: DENSE_LAUNCH(ACT_ELU, ACT_NONE, true, false); break;
        case ACT_TANH: DENSE_LAUNCH(ACT_TANH, ACT_NONE, true, false); break;
        default: DENSE_LAUNCH(ACT_NONE, ACT_NONE, true, false); break;
        }
    } else {           // bwd-weight: both operands walk rows (contiguous along i)
        switch (a.A.act) {
        case ACT_RELU: DENSE_LAUNCH(ACT_RELU, ACT_NONE, false, false); break;
        case ACT_ELU: DENSE_LAUNCH(ACT_ELU, ACT_NONE, false, false); break;
        case ACT_TANH: DENSE_LAUNCH(ACT_TANH, ACT_NONE, false, false); break;
        default: DENSE_LAUNCH(ACT_NONE, ACT_NONE, false, false); break;
        }
    }
#undef DENSE_LAUNCH
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}


// Forward Y = act(X W^T + b): one wavefront per 16x16 output tile, the whole
// reduction loaded up front in groups of GS 16-wide steps (one 16-byte load
// of X and one of W per lane per step) so a wave makes one or two L2 round
// trips instead of one per step; the tail (K % 16) is a range-checked step.
// (2x2 waves per workgroup sharing X / W rows through L1 measured slower than
// one wave per workgroup with this remap.)
template <int EP, int GS, int TM, int TN, int KW>
__global__ __launch_bounds__(64 * KW) void dense_fwd_kernel(GemmArgs a) {
    // a (16 TM) x (16 TN) tile per workgroup; per 16-wide step TM + TN b128
    // loads feed 4 TM TN MFMAs.  KW waves split the reduction (halves, summed
    // through LDS at the end).
    constexpr bool SPLIT = TM * TN == 1; // 1x1: two accumulators break the MFMA dependency chain
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
    const int3 tile = xcd_tile();
    const int i0 = tile.y * 16 * TM, j0 = tile.x * 16 * TN, g = tile.z;
    const __amdgpu_buffer_rsrc_t ra = rsrc(a.A.p), rb = rsrc(a.B.p);
    int abase[TM], bbase[TN];
    bool arow[TM], bcol[TN];
#pragma unroll
    for (int x = 0; x < TM; ++x) {
        const int row = i0 + 16 * x + c;
        abase[x] = g * (int)a.A.sg + row * (int)a.A.si;
        arow[x] = row < a.I;
    }
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
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(ra, (live & arow[x]) ? (abase[x] + r) * 4 : BUF_OOB, 0, 0);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) av[s][x][jj] = v[jj];
            }
#pragma unroll
            for (int y = 0; y < TN; ++y) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, (live & bcol[y]) ? (bbase[y] + r) * 4 : BUF_OOB, 0, 0);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) bv[s][y][jj] = v[jj];
            }
        }
    };
    auto step = [&](const float (&xa)[TM][4], const float (&xb)[TN][4]) {
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
            step(xa, xb);
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
            for (int x = 0; x < TM; ++x) xa[x][jj] = ldb(ra, arow[x] & (r + jj < a.R), abase[x] + r + jj);
#pragma unroll
            for (int y = 0; y < TN; ++y) xb[y][jj] = ldb(rb, bcol[y] & (r + jj < a.R), bbase[y] + r + jj);
        }
        step(xa, xb);
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

template <int AG, int VA, int NW>
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
    const int nks = (a.M + 3) >> 2;
    const int my = nks > w ? (nks - w + NW - 1) / NW : 0;
    const int ngrp = (my + KS - 1) / KS;

    struct Buf {
        float a[KS][VA], y[KS][VA], b[KS][4];
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
            ld_vec<4>(rx, live ? (xb + m * a.ldx) * 4 : BUF_OOB, f.b[sp]);
        }
    };
    auto mma = [&](const Buf &f) {
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
            for (int u = 0; u < 4; ++u) fb[u] = shifted<4>(f.b[sp], shj, u);
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
                if (ja + u < a.J) row[ja + u] = acc[s][u][k];
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

int launch_wgrad(const WgradArgs &a, int groups, int act, hipStream_t s) {
    const int jt = (a.J + 63) / 64;
    auto tiles = [&](int va) { return (long)jt * ((a.I + 16 * va - 1) / (16 * va)) * groups; };
    // the widest i-vector that still yields ~1k waves at NW = 8
    int va = 4;
    while (va > 1 && (tiles(va) * 8 < 768 || a.I < va)) va >>= 1;
    const long nks = (a.M + 3) / 4;
    int nw = 2;
    while (nw < 8 && nks >= 8L * nw * 2 && tiles(va) * nw * 2 <= 2048) nw *= 2;
    dim3 grid(jt, (a.I + 16 * va - 1) / (16 * va), groups);
#define WG_NW(AGv, VAv)                                                                              \
    do {                                                                                           \
        if (nw == 8) hipLaunchKernelGGL((dense_wgrad_kernel<AGv, VAv, 8>), grid, dim3(512), 0, s, a); \
        else if (nw == 4) hipLaunchKernelGGL((dense_wgrad_kernel<AGv, VAv, 4>), grid, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((dense_wgrad_kernel<AGv, VAv, 2>), grid, dim3(128), 0, s, a);       \
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
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int launch_fwd(const GemmArgs &a, int groups_grid, hipStream_t s) {
    const long span_a = (long)groups_grid * a.A.sg + (long)a.I * a.A.si + (long)a.R;
    const long span_b = (long)groups_grid * a.B.sg + (long)a.J * a.B.si + (long)a.R;
    if (span_a >= (1L << 29) || span_b >= (1L << 29) || a.A.sr != 1 || a.B.sr != 1) return EXO_ERANGE;
    const int steps = a.R >> 4;
    static const int force = [] {
        const char *e = std::getenv("EXO_FWD_TILE");
        return e ? std::atoi(e) : 0;
    }();
    // 16x16 tiles (one wave each) while they number < ~2 per SIMD; beyond
    // that 32x32 tiles (half the L2 traffic per MFMA).  (Splitting the
    // reduction over 2 waves, EXO_FWD_TILE=xx2, measured slower at every TD7
    // shape.)
    const long t16 = (long)((a.I + 15) / 16) * ((a.J + 15) / 16) * groups_grid;
    int tm = 1, tn = 1, kw = 1;
    if (force) {
        tm = force / 100;
        tn = force / 10 % 10;
        kw = force % 10;
    } else if (t16 >= 2048) {
        tm = tn = 2;
    }
    dim3 grid((a.J + 16 * tn - 1) / (16 * tn), (a.I + 16 * tm - 1) / (16 * tm), groups_grid);
    const int wsteps = (steps + kw - 1) / kw;
#define FWD_GS(EPv, TMv, TNv, KWv)                                                                              \
    do {                                                                                                      \
        const dim3 blk(64 * KWv);                                                                             \
        if (wsteps <= 5) hipLaunchKernelGGL((dense_fwd_kernel<EPv, 5, TMv, TNv, KWv>), grid, blk, 0, s, a);    \
        else if (TMv * TNv == 1 && wsteps <= 20)                                                              \
            hipLaunchKernelGGL((dense_fwd_kernel<EPv, 20, TMv, TNv, KWv>), grid, blk, 0, s, a);               \
        else if (TMv * TNv == 1)                                                                              \
            hipLaunchKernelGGL((dense_fwd_kernel<EPv, 10, TMv, TNv, KWv>), grid, blk, 0, s, a);               \
        else hipLaunchKernelGGL((dense_fwd_kernel<EPv, 5, TMv, TNv, KWv>), grid, blk, 0, s, a);                \
    } while (0)
#define FWD_LAUNCH(EPv)                                            \
    do {                                                           \
        if (tm == 2 && tn == 2 && kw == 2) FWD_GS(EPv, 2, 2, 2);   \
        else if (tm == 2 && tn == 2) FWD_GS(EPv, 2, 2, 1);         \
        else if (kw == 2) FWD_GS(EPv, 1, 1, 2);                    \
        else FWD_GS(EPv, 1, 1, 1);                                 \
    } while (0)
    switch (a.act) {
    case ACT_RELU: FWD_LAUNCH(ACT_RELU); break;
    case ACT_ELU: FWD_LAUNCH(ACT_ELU); break;
    case ACT_TANH: FWD_LAUNCH(ACT_TANH); break;
    default: FWD_LAUNCH(ACT_NONE); break;
    }
#undef FWD_LAUNCH
#undef FWD_GS
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

Operand plain(const float *p, long sg, long si, long sr) {
    Operand o{};
    o.p = p;
    o.sg = sg;
    o.si = si;
    o.sr = sr;
    o.act = -1;
    o.ones_col = -1;
    return o;
}

} // namespace

extern "C" {

/* Forward of G grouped dense layers: Y[g] = act(X[g] W[g]^T + b[g]).
 * X: [G][M][K] with group stride xsg (0 = one X shared by all groups) and row
 * stride ldx; W: [G][N][K] contiguous; b: [G][N] or null; Y: [G][M][N] with
 * group stride ysg and row stride ldy.  act: 0 none, 1 relu, 2 elu, 3 tanh. */
int td7_dense_fwd(const float *x, long xsg, long ldx, const float *w, const float *b, float *y, long ysg, long ldy,
                  int32_t groups, int32_t m, int32_t n, int32_t k, int32_t act, void *stream) {
    if (!x || !w || !y || groups <= 0 || m < 0 || n <= 0 || k <= 0 || act < 0 || act > 3) return EXO_EINVAL;
    if (m == 0) return EXO_OK;
    GemmArgs a{};
    a.A = plain(x, xsg, ldx, 1);
    a.B = plain(w, (long)n * k, k, 1);
    a.I = m;
    a.J = n;
    a.R = k;
    a.groups_red = 1;
    a.C = y;
    a.csg = ysg;
    a.csi = ldy;
    a.csj = 1;
    a.bias = b;
    a.bsg = n;
    a.act = act;
    a.j_bias = -1;
    return launch_fwd(a, groups, (hipStream_t)stream);
}

/* dX = sum over the reduced groups of (dY[g] * act'(Y[g])) W[g].
 * dY, Y: [G][M][N] (group stride dysg / ysg, row strides lddy / ldy);
 * W: [G][N][K]; dX: [M][K] per group (dxsg, lddx).  shared_input != 0: X was
 * one tensor for all groups, dX (a single [M][K]) sums over them. */
int td7_dense_bwd_data(const float *dy, long dysg, long lddy, const float *yv, long ysg, long ldy, const float *w,
                       float *dx, long dxsg, long lddx, int32_t groups, int32_t shared_input, int32_t m, int32_t n,
                       int32_t k, int32_t act, void *stream) {
    if (!dy || !yv || !w || !dx || groups <= 0 || m < 0 || n <= 0 || k <= 0 || act < 0 || act > 3) return EXO_EINVAL;
    if (m == 0) return EXO_OK;
    GemmArgs a{};
    a.A = plain(dy, dysg, lddy, 1);
    a.A.y = yv;
    a.A.ysg = ysg;
    a.A.ysi = ldy;
    a.A.ysr = 1;
    a.A.act = act;
    a.B = plain(w, (long)n * k, 1, k); // B(j = out col k, r = n) = W[n][k]
    a.I = m;
    a.J = k;
    a.R = n;
    a.groups_red = shared_input ? groups : 1;
    a.C = dx;
    a.csg = dxsg;
    a.csi = lddx;
    a.csj = 1;
    a.act = ACT_NONE;
    a.j_bias = -1;
    return launch(a, shared_input ? 1 : groups, (hipStream_t)stream);
}

/* dW[g] = (dY[g] * act'(Y[g]))^T X[g]  ([N][K], contiguous per group) and,
 * when db != null, db[g] = column sums of dY[g] * act'(Y[g])  ([N]). */
int td7_dense_bwd_weight(const float *dy, long dysg, long lddy, const float *yv, long ysg, long ldy, const float *x,
                         long xsg, long ldx, float *dw, float *db, int32_t groups, int32_t m, int32_t n, int32_t k,
                         int32_t act, void *stream) {
    if (!dy || !yv || !x || !dw || groups <= 0 || m < 0 || n <= 0 || k <= 0 || act < 0 || act > 3) return EXO_EINVAL;
    GemmArgs a{};
    a.A = plain(dy, dysg, 1, lddy); // A(i = n, r = m) = dY[m][n]
    a.A.y = yv;
    a.A.ysg = ysg;
    a.A.ysi = 1;
    a.A.ysr = ldy;
    a.A.act = act;
    a.B = plain(x, xsg, 1, ldx);    // B(j = k, r = m) = X[m][k]
    a.B.ones_col = db ? k : -1;     // column K of the product is colsum(dP) = db
    a.I = n;
    a.J = k;
    a.R = m;
    a.groups_red = 1;
    a.C = dw;
    a.csg = (long)n * k;
    a.csi = k;
    a.csj = 1;
    a.act = ACT_NONE;
    a.bias_grad = db;
    a.bgsg = n;
    a.j_bias = db ? k : -1;
    if (m == 0) return EXO_EINVAL;
    if (n >= 4 && k >= 4 && std::getenv("EXO_WGRAD_V3") == nullptr) {
        // output-contiguous wgrad kernel: 32-bit element offsets
        const long span = (long)groups * (dysg > ysg ? (dysg > xsg ? dysg : xsg) : (ysg > xsg ? ysg : xsg)) +
                          (long)m * (lddy > ldy ? (lddy > ldx ? lddy : ldx) : (ldy > ldx ? ldy : ldx)) + n + k;
        if (span < (1L << 29)) {
            WgradArgs w{dy, yv, x, (int)dysg, (int)lddy, (int)ysg, (int)ldy, (int)xsg, (int)ldx, dw, db, n, k, m};
            return launch_wgrad(w, groups, act, (hipStream_t)stream);
        }
    }
    return launch(a, groups, (hipStream_t)stream);
}

} // extern "C"
