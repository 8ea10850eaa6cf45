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
// inside the kernel.  fp32 in memory, fp32 accumulate; the MFMA operands are
// exact f32 (default) or rounded to bf16 / f16 (Prec, bits 8-15 of act).
#include <climits>

#include "td7_dense_kernels.h"

namespace td7dense {

// instantiated in td7_dense_{f32,bf16,f16}.hip
#define TD7_EXTERN(P)                                                                                 \
    extern template void launch_gemm_p<P>(const GemmArgs &, dim3, int, hipStream_t);                  \
    extern template void launch_wgrad_p<P, false>(const WgradArgs &, dim3, int, int, int, hipStream_t); \
    extern template void launch_wgrad_p<P, true>(const WgradArgs &, dim3, int, int, int, hipStream_t);  \
    extern template void launch_fwd_p<P, false>(const GemmArgs &, dim3, int, int, int, int, hipStream_t); \
    extern template void launch_fwd_p<P, true>(const GemmArgs &, dim3, int, int, int, int, hipStream_t); \
    extern template void launch_fwd_norm_p<P, false>(const GemmArgs &, dim3, float *, float *, float, hipStream_t); \
    extern template void launch_fwd_norm_p<P, true>(const GemmArgs &, dim3, float *, float *, float, hipStream_t);
extern template void launch_fwd_lds_p<PREC_BF16, false>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_lds_p<PREC_F16, false>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_lds_p<PREC_BF16, true>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_lds_p<PREC_F16, true>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_big_p<PREC_BF16, false>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_big_p<PREC_F16, false>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_big_p<PREC_BF16, true>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_big_p<PREC_F16, true>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_p<PREC_BF16, false, true>(const GemmArgs &, dim3, int, int, int, int, hipStream_t);
extern template void launch_fwd_p<PREC_F16, false, true>(const GemmArgs &, dim3, int, int, int, int, hipStream_t);
extern template void launch_fwd_xl_p<PREC_BF16, false>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_xl_p<PREC_F16, false>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_xl_p<PREC_BF16, true>(const GemmArgs &, dim3, int, hipStream_t);
extern template void launch_fwd_xl_p<PREC_F16, true>(const GemmArgs &, dim3, int, hipStream_t);
TD7_EXTERN(PREC_F32)
TD7_EXTERN(PREC_BF16)
TD7_EXTERN(PREC_F16)
#undef TD7_EXTERN

// the generic core for bwd-data (and bwd-weight when the output-contiguous
// kernel does not apply); the forward has its own kernel (launch_fwd)
int launch(const GemmArgs &a, int groups_grid, int prec, hipStream_t s) {
    const int Jt = a.J + (a.j_bias >= 0 ? 1 : 0);
    dim3 grid((Jt + 31) / 32, (a.I + 31) / 32, groups_grid);
    // 32-bit element offsets inside the kernel (byte offsets below BUF_BYTES)
    const int gmax = a.groups_red > 1 ? a.groups_red : groups_grid;
    const long span_a = (long)gmax * a.A.sg + (long)a.I * a.A.si + (long)a.R * a.A.sr;
    const long span_b = (long)gmax * a.B.sg + (long)(a.J + 1) * a.B.si + (long)a.R * a.B.sr;
    if (span_a >= (1L << 29) || span_b >= (1L << 29)) return EXO_ERANGE;
    if (a.A.act < 0) return EXO_EINVAL;
    // split the reduction over more waves when the tile grid alone is small
    const long tiles = (long)grid.x * grid.y * grid.z;
    const long steps = (long)((a.R + 15) / 16) * a.groups_red;
    // waves per workgroup: about one wave per SIMD of the chip (1024), at
    // least 4 reduction steps per wave
    int nw = 2;
    while (nw < 8 && tiles * nw * 2 <= 1024 && steps >= 4L * nw * 2) nw *= 2;
    if (prec == PREC_BF16) launch_gemm_p<PREC_BF16>(a, grid, nw, s);
    else if (prec == PREC_F16) launch_gemm_p<PREC_F16>(a, grid, nw, s);
    else launch_gemm_p<PREC_F32>(a, grid, nw, s);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}


int launch_wgrad(const WgradArgs &a, int groups, int act, int prec, hipStream_t s, bool cat = false) {
    const int jt = (a.J + 63) / 64;
    auto tiles = [&](int va) { return (long)jt * ((a.I + 16 * va - 1) / (16 * va)) * groups; };
    // the widest i-vector that still yields ~1k waves at NW = 8
    int va = 4;
    while (va > 1 && (tiles(va) * 8 < 768 || a.I < va)) va >>= 1;
    const long nks = (a.M + 3) / 4;
    int nw = 2;
    while (nw < 8 && nks >= 8L * nw * 2 && tiles(va) * nw * 2 <= 2048) nw *= 2;
    dim3 grid(jt, (a.I + 16 * va - 1) / (16 * va), groups);
    if (cat) {
        if (prec == PREC_BF16) launch_wgrad_p<PREC_BF16, true>(a, grid, va, nw, act, s);
        else if (prec == PREC_F16) launch_wgrad_p<PREC_F16, true>(a, grid, va, nw, act, s);
        else launch_wgrad_p<PREC_F32, true>(a, grid, va, nw, act, s);
    } else {
        if (prec == PREC_BF16) launch_wgrad_p<PREC_BF16, false>(a, grid, va, nw, act, s);
        else if (prec == PREC_F16) launch_wgrad_p<PREC_F16, false>(a, grid, va, nw, act, s);
        else launch_wgrad_p<PREC_F32, false>(a, grid, va, nw, act, s);
    }
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

// the 256 x 256-tile forward's kernel: EXO_FWD_XL (0 dense_fwd_big_kernel,
// 1 dense_fwd_xl_kernel, 2 dense_fwd_xl8_kernel; the K % 64 == 0 kernel
// falls back to 1 elsewhere), td7_dense_set_xl at run time (r06: the A/Bs of
// profiles/r06_xl ran two more 256 x 256 kernels through it)
static int g_fwd_xl = -1;
static int fwd_xl_variant() {
    if (g_fwd_xl < 0) {
        const char *e = std::getenv("EXO_FWD_XL");
        g_fwd_xl = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 2;
    }
    return g_fwd_xl;
}

int launch_fwd(const GemmArgs &a, int groups_grid, int prec, hipStream_t s, bool cat = false) {
    const long span_a = cat ? 0 : (long)groups_grid * a.A.sg + (long)a.I * a.A.si + (long)a.R;
    const long span_b = (long)groups_grid * a.B.sg + (long)a.J * a.B.si + (long)a.R;
    if (span_a >= (1L << 29) || span_b >= (1L << 29) || a.A.sr != 1 || a.B.sr != 1) return EXO_ERANGE;
    const int steps = a.R >> 4;
    // large layers with 16-bit operands: the LDS-tiled kernel when its 64 x 64
    // tiles number >= 256 (one per CU) and K >= 256, or >= 2,048 tiles and K >= 64
    // (profiles/r01e_raw/
    // lds_fwd.txt: 1.3-1.6x at 4,096 rows, 2.8x on the wide critic's
    // 2 x 1,024 x 1,024 x 3,072, 4.7-5.7x at 65,536 rows; with fewer tiles it
    // loses to the register-streaming kernel, cat_bench_lds1024.txt).
    // EXO_FWD_LDS=0 disables it.
    static const bool lds_on = [] {
        const char *e = std::getenv("EXO_FWD_LDS");
        return !(e && e[0] == '0');
    }();
    // the largest layers: 256 x 128 tiles and 16x16x32 MFMAs (dense_fwd_big_kernel)
    // when they number >= 256 and the operands allow 16-byte chunks of 8
    // (K % 8, rows 16-byte aligned; CAT boundaries at multiples of 64);
    // EXO_FWD_BIG=0 disables it
    static const bool big_on = [] {
        const char *e = std::getenv("EXO_FWD_BIG");
        return !(e && e[0] == '0');
    }();
    // tile 128 x 256 (half the re-reads of X of 256 x 128: 419 vs 429 us at
    // 65,536 x 1,024 x 1,024, 692 vs 746 on [a | zs]; EXO_FWD_BIG=2 picks 256 x 128)
    static const int big_bm = [] {
        const char *e = std::getenv("EXO_FWD_BIG");
        return (e && e[0] == '2') ? 256 : 128;
    }();
    const int big_bn = big_bm == 256 ? 128 : 256;
    const long tbig = (long)((a.I + big_bm - 1) / big_bm) * ((a.J + big_bn - 1) / big_bn) * groups_grid;
    auto al16 = [](const void *p) { return ((uintptr_t)p & 15) == 0; };
    bool big = prec != PREC_F32 && big_on && tbig >= 256 && a.R >= 256 && a.R % 8 == 0 && a.J >= 128 &&
               a.B.si % 4 == 0 && a.B.sg % 4 == 0 && al16(a.B.p);
    if (big && cat) {
        for (int sg = 0; sg < CAT_MAX && a.cat.kb[sg] < a.R; ++sg)
            big = big && a.cat.kb[sg] % BIG_BK == 0 && a.cat.ld[sg] % (a.a16 ? 8 : 4) == 0 &&
                  a.cat.sg[sg] % 4 == 0 && al16(a.cat.p[sg]);
    } else if (big && a.a16) {
        big = a.A.si % 8 == 0 && a.A.sg % 8 == 0 && al16(a.a16);
    } else if (big) {
        big = a.A.si % 4 == 0 && a.A.sg % 4 == 0 && al16(a.A.p);
    }
    // 16-bit input / output (td7_dense_fwd_h): the 128 x 256 big kernel with
    // 16-bit weights, or a 16-bit output of the 128 x 128 LDS kernel (fp32 X:
    // the K = 80 first layers); anything else is the caller's fp32 fallback
    if (cat && a.a16 && !a.c16) return EXO_ERANGE;  // 16-bit segments: the CHF variant only
    // 16-bit X into a layer the fp32 path gives dense_fwd_kernel (neither the
    // big nor the LDS-tiled kernel; e.g. the actor's 7-wide tanh head after a
    // 16-bit l2): its AH variant, the same operands and order (r05)
    const long t64x = (long)((a.I + 63) / 64) * ((a.J + 63) / 64) * groups_grid;
    const bool lds_would = prec != PREC_F32 && lds_on && a.J >= 64 &&
                           ((t64x >= 256 && a.R >= 256) || (t64x >= 2048 && a.R >= 64));
    const bool small_h = a.a16 && !a.c16 && !cat && prec != PREC_F32 && !big && !lds_would &&
                         a.A.si % 4 == 0 && a.A.sg % 4 == 0 && ((uintptr_t)a.a16 & 7) == 0;
    if ((a.a16 || a.c16) && !small_h) {
        const long t128 = (long)((a.I + 127) / 128) * ((a.J + 127) / 128) * groups_grid;
        const bool lds128 = !big && !a.a16 && prec != PREC_F32 && lds_on && a.J >= 64 &&
                            ((t64x >= 256 && a.R >= 256) || (t64x >= 2048 && a.R >= 64)) && t128 >= 256;
        if (!(big && big_bm == 128 && a.b16) && !lds128) return EXO_ERANGE;
    }
    // 16-bit X and W at >= 256 tiles of 256 x 256 (r05): dense_fwd_xl8_kernel
    // where K % 64 == 0, else dense_fwd_xl_kernel; EXO_FWD_XL=0 keeps
    // dense_fwd_big_kernel, EXO_FWD_XL=1 dense_fwd_xl_kernel everywhere
    // (td7_dense_set_xl switches it at run time for same-process A/Bs)
    const int xl_v = fwd_xl_variant();
    const bool xl_on = xl_v != 0;
    const int xl_var = (xl_v >= 2 && a.R % XL_BK == 0) ? xl_v : 1;
    const long txl = (long)((a.I + XL_BM - 1) / XL_BM) * ((a.J + XL_BN - 1) / XL_BN) * groups_grid;
    if (big && xl_on && a.a16 && a.b16 && txl >= 256 &&
        (!a.c16 || (a.csj == 1 && a.csi % 8 == 0 && a.csg % 8 == 0 && ((uintptr_t)a.c16 & 15) == 0))) {
        dim3 grid((a.J + XL_BN - 1) / XL_BN, (a.I + XL_BM - 1) / XL_BM, groups_grid);
        if (cat) {
            if (prec == PREC_BF16) launch_fwd_xl_p<PREC_BF16, true>(a, grid, xl_var, s);
            else launch_fwd_xl_p<PREC_F16, true>(a, grid, xl_var, s);
        } else {
            if (prec == PREC_BF16) launch_fwd_xl_p<PREC_BF16, false>(a, grid, xl_var, s);
            else launch_fwd_xl_p<PREC_F16, false>(a, grid, xl_var, s);
        }
        return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
    }
    if (big) {
        dim3 grid((a.J + big_bn - 1) / big_bn, (a.I + big_bm - 1) / big_bm, groups_grid);
        if (cat) {
            if (prec == PREC_BF16) launch_fwd_big_p<PREC_BF16, true>(a, grid, big_bm, s);
            else launch_fwd_big_p<PREC_F16, true>(a, grid, big_bm, s);
        } else {
            if (prec == PREC_BF16) launch_fwd_big_p<PREC_BF16, false>(a, grid, big_bm, s);
            else launch_fwd_big_p<PREC_F16, false>(a, grid, big_bm, s);
        }
        return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
    }
    const long t64 = (long)((a.I + 63) / 64) * ((a.J + 63) / 64) * groups_grid;
    if (prec != PREC_F32 && lds_on && a.J >= 64 && ((t64 >= 256 && a.R >= 256) || (t64 >= 2048 && a.R >= 64))) {
        const long t128 = (long)((a.I + 127) / 128) * ((a.J + 127) / 128) * groups_grid;
        const int bm = t128 >= 256 ? 128 : 64;
        dim3 grid((a.J + bm - 1) / bm, (a.I + bm - 1) / bm, groups_grid);
        if (cat) {
            if (prec == PREC_BF16) launch_fwd_lds_p<PREC_BF16, true>(a, grid, bm, s);
            else launch_fwd_lds_p<PREC_F16, true>(a, grid, bm, s);
        } else {
            if (prec == PREC_BF16) launch_fwd_lds_p<PREC_BF16, false>(a, grid, bm, s);
            else launch_fwd_lds_p<PREC_F16, false>(a, grid, bm, s);
        }
        return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
    }
    static const int force = [] {
        const char *e = std::getenv("EXO_FWD_TILE");
        return e ? std::atoi(e) : 0;
    }();
    // 16x16 tiles (one wave each) while they number < ~2 per SIMD; beyond
    // that 32x32 tiles (half the L2 traffic per MFMA).  (Splitting the
    // reduction over 2 waves, EXO_FWD_TILE=112, measured slower at every TD7
    // shape.)
    const long t16 = (long)((a.I + 15) / 16) * ((a.J + 15) / 16) * groups_grid;
    int tm = 1, tn = 1, kw = 1;
    if (force) {
        tm = force / 100 == 2 ? 2 : 1;
        tn = tm;
        kw = tm == 1 && force % 10 == 2 && prec == PREC_F32 ? 2 : 1;
    } else if (t16 >= 2048) {
        tm = tn = 2;
    }
    dim3 grid((a.J + 16 * tn - 1) / (16 * tn), (a.I + 16 * tm - 1) / (16 * tm), groups_grid);
    const int wsteps = (steps + kw - 1) / kw;
    if (cat) {
        if (prec == PREC_BF16) launch_fwd_p<PREC_BF16, true>(a, grid, tm, tn, kw, wsteps, s);
        else if (prec == PREC_F16) launch_fwd_p<PREC_F16, true>(a, grid, tm, tn, kw, wsteps, s);
        else launch_fwd_p<PREC_F32, true>(a, grid, tm, tn, kw, wsteps, s);
    } else if (small_h) {
        if (prec == PREC_BF16) launch_fwd_p<PREC_BF16, false, true>(a, grid, tm, tn, kw, wsteps, s);
        else launch_fwd_p<PREC_F16, false, true>(a, grid, tm, tn, kw, wsteps, s);
    } else {
        if (prec == PREC_BF16) launch_fwd_p<PREC_BF16, false>(a, grid, tm, tn, kw, wsteps, s);
        else if (prec == PREC_F16) launch_fwd_p<PREC_F16, false>(a, grid, tm, tn, kw, wsteps, s);
        else launch_fwd_p<PREC_F32, false>(a, grid, tm, tn, kw, wsteps, s);
    }
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

// segments of a concatenated input -> CatSeg; the total width, or < 0 when the
// layout breaks the kernels' 4-column chunk rule
static int make_cat(CatSeg &c, int nseg, const float *const *xs, const long *xsg, const long *ldx, const int32_t *widths) {
    if (nseg < 1 || nseg > CAT_MAX || !xs || !xsg || !ldx || !widths) return -1;
    int k = 0;
    for (int s = 0; s < CAT_MAX; ++s) {
        c.p[s] = s < nseg ? xs[s] : xs[0];
        c.sg[s] = s < nseg ? xsg[s] : 0;
        c.ld[s] = s < nseg ? (int)ldx[s] : 0;
        c.kb[s] = s < nseg ? k : INT_MAX;
        if (s < nseg) {
            if (!xs[s] || widths[s] <= 0 || xsg[s] < 0 || ldx[s] < widths[s] || ldx[s] >= (1L << 30)) return -1;
            if (s < nseg - 1 && widths[s] % 4) return -1;
            if (s == nseg - 1 && widths[s] < 4) return -1;
            k += widths[s];
        }
    }
    c.kb[CAT_MAX] = INT_MAX;
    return k;
}

static int launch_fwd_norm(const GemmArgs &a, int groups, int prec, float *h, float *mean, float eps, hipStream_t s, bool cat) {
    if (a.J > 320) return EXO_EINVAL; // 4 waves x 5 column tiles per workgroup
    const long span_a = cat ? 0 : (long)groups * a.A.sg + (long)a.I * a.A.si + (long)a.R;
    const long span_b = (long)groups * a.B.sg + (long)a.J * a.B.si + (long)a.R;
    if (span_a >= (1L << 29) || span_b >= (1L << 29)) return EXO_ERANGE;
    const dim3 grid((a.I + 15) / 16, groups);
    if (cat) {
        if (prec == PREC_BF16) launch_fwd_norm_p<PREC_BF16, true>(a, grid, h, mean, eps, s);
        else if (prec == PREC_F16) launch_fwd_norm_p<PREC_F16, true>(a, grid, h, mean, eps, s);
        else launch_fwd_norm_p<PREC_F32, true>(a, grid, h, mean, eps, s);
    } else {
        if (prec == PREC_BF16) launch_fwd_norm_p<PREC_BF16, false>(a, grid, h, mean, eps, s);
        else if (prec == PREC_F16) launch_fwd_norm_p<PREC_F16, false>(a, grid, h, mean, eps, s);
        else launch_fwd_norm_p<PREC_F32, false>(a, grid, h, mean, eps, s);
    }
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

} // namespace td7dense

using namespace td7dense;

extern "C" {

int td7_dense_set_xl(int32_t variant) {
    const int prev = td7dense::fwd_xl_variant();
    if (variant < 0 || variant > 2) return EXO_EINVAL;
    td7dense::g_fwd_xl = variant;
    return prev;
}

/* Forward of G grouped dense layers: Y[g] = act(X[g] W[g]^T + b[g]).
 * X: [G][M][K] with group stride xsg (0 = one X shared by all groups) and row
 * stride ldx; W: [G][N][K] contiguous; b: [G][N] or null; Y: [G][M][N] with
 * group stride ysg and row stride ldy.  act: bits 0-7 the activation (0 none,
 * 1 relu, 2 elu, 3 tanh), bits 8-15 the MFMA operand precision (Prec). */
int td7_dense_fwd(const float *x, long xsg, long ldx, const float *w, const float *b, float *y, long ysg, long ldy,
                  int32_t groups, int32_t m, int32_t n, int32_t k, int32_t act, void *stream) {
    return td7_dense_fwd_w16(x, xsg, ldx, w, b, y, ysg, ldy, groups, m, n, k, act, nullptr, stream);
}

/* td7_dense_fwd with W also given rounded to the MFMA operand type (bf16 /
 * fp16 bits, [G][N][K] contiguous, w16 = W.to(dtype)): the large-layer kernel
 * then loads 16-bit weights instead of rounding fp32 ones per slice -- the
 * same operand values, bit-identical results; ignored by the other kernels
 * and at fp32.  w16 may be null. */
int td7_dense_fwd_w16(const float *x, long xsg, long ldx, const float *w, const float *b, float *y, long ysg, long ldy,
                      int32_t groups, int32_t m, int32_t n, int32_t k, int32_t act, const uint16_t *w16, void *stream) {
    if (!x || !w || !y || groups <= 0 || m < 0 || n <= 0 || k <= 0) return EXO_EINVAL;
    const int prec = act >> 8;
    act &= 0xFF;
    if (act > 3 || prec > PREC_F16) return EXO_EINVAL;
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
    a.b16 = prec != PREC_F32 ? w16 : nullptr;
    return launch_fwd(a, groups, prec, (hipStream_t)stream);
}

/* td7_dense_fwd of a concatenated input X = [X_0 | ... | X_{nseg-1}] (the
 * reference's Linear(torch.cat(...))) read in place: segment s is
 * xs[s] [G][M][widths[s]] with group stride xsg[s] (0 = shared by the groups)
 * and row stride ldx[s]; K = sum of widths.  nseg <= 4, interior widths
 * multiples of 4, the last >= 4 (else EXO_EINVAL: concatenate instead). */
int td7_dense_fwd_cat(int32_t nseg, const float *const *xs, const long *xsg, const long *ldx, const int32_t *widths,
                      const float *w, const float *b, float *y, long ysg, long ldy, int32_t groups, int32_t m, int32_t n,
                      int32_t act, void *stream) {
    return td7_dense_fwd_cat_w16(nseg, xs, xsg, ldx, widths, w, b, y, ysg, ldy, groups, m, n, act, nullptr, stream);
}

/* td7_dense_fwd_w16 on an inference chain (no backward): X and / or Y as
 * 16-bit values of the MFMA operand type (x16 / y16; the fp32 pointer of the
 * same operand null) -- the values the consumer rounds its operand to, so a
 * chain of layers gives bit-identical results with half the activation
 * bytes.  Only where the large-layer kernel runs (else EXO_ERANGE: fall back to
 * fp32).  w16 required. */
int td7_dense_fwd_h(const float *x, const uint16_t *x16, long xsg, long ldx, const float *w, const float *b,
                    float *y, uint16_t *y16, long ysg, long ldy, int32_t groups, int32_t m, int32_t n, int32_t k,
                    int32_t act, const uint16_t *w16, void *stream) {
    if ((!x == !x16) || (!y == !y16) || !w || !w16 || groups <= 0 || m < 0 || n <= 0 || k <= 0) return EXO_EINVAL;
    const int prec = act >> 8;
    act &= 0xFF;
    if (act > 3 || prec < PREC_BF16 || prec > PREC_F16) return EXO_EINVAL;
    if (m == 0) return EXO_OK;
    GemmArgs a{};
    a.A = plain(x ? x : reinterpret_cast<const float *>(x16), xsg, ldx, 1);
    a.a16 = x16;
    a.B = plain(w, (long)n * k, k, 1);
    a.I = m;
    a.J = n;
    a.R = k;
    a.groups_red = 1;
    a.C = y;
    a.c16 = y16;
    a.csg = ysg;
    a.csi = ldy;
    a.csj = 1;
    a.bias = b;
    a.bsg = n;
    a.act = act;
    a.j_bias = -1;
    a.b16 = w16;
    return launch_fwd(a, groups, prec, (hipStream_t)stream);
}

/* td7_dense_fwd_cat_w16 with a 16-bit output (td7_dense_fwd_h's Y); xs16: the
 * segments are 16-bit values too (the big kernel's 16-bit X, per segment) */
int td7_dense_fwd_cat_h(int32_t nseg, const void *const *xs_, int32_t xs16, const long *xsg, const long *ldx,
                        const int32_t *widths, const float *w, const float *b, uint16_t *y16, long ysg, long ldy,
                        int32_t groups, int32_t m, int32_t n, int32_t act, const uint16_t *w16, void *stream) {
    if (!xs_ || !w || !w16 || !y16 || groups <= 0 || m < 0 || n <= 0 || xs16 < 0 || xs16 > 1) return EXO_EINVAL;
    const float *const *xs = reinterpret_cast<const float *const *>(xs_);
    const int prec = act >> 8;
    act &= 0xFF;
    if (act > 3 || prec < PREC_BF16 || prec > PREC_F16) return EXO_EINVAL;
    if (xs16 && groups != 1) return EXO_ERANGE;
    GemmArgs a{};
    const int k = make_cat(a.cat, nseg, xs, xsg, ldx, widths);
    if (k <= 0) return EXO_EINVAL;
    if (m == 0) return EXO_OK;
    a.A = plain(xs[0], 0, 0, 1);
    if (xs16) a.a16 = reinterpret_cast<const uint16_t *>(xs[0]);  // marks the segments 16-bit
    a.B = plain(w, (long)n * k, k, 1);
    a.I = m;
    a.J = n;
    a.R = k;
    a.groups_red = 1;
    a.c16 = y16;
    a.csg = ysg;
    a.csi = ldy;
    a.csj = 1;
    a.bias = b;
    a.bsg = n;
    a.act = act;
    a.j_bias = -1;
    a.b16 = w16;
    return launch_fwd(a, groups, prec, (hipStream_t)stream, true);
}

/* td7_dense_fwd_cat with W also given rounded to 16 bits (see td7_dense_fwd_w16) */
int td7_dense_fwd_cat_w16(int32_t nseg, const float *const *xs, const long *xsg, const long *ldx,
                          const int32_t *widths, const float *w, const float *b, float *y, long ysg, long ldy,
                          int32_t groups, int32_t m, int32_t n, int32_t act, const uint16_t *w16, void *stream) {
    if (!w || !y || groups <= 0 || m < 0 || n <= 0) return EXO_EINVAL;
    const int prec = act >> 8;
    act &= 0xFF;
    if (act > 3 || prec > PREC_F16) return EXO_EINVAL;
    GemmArgs a{};
    const int k = make_cat(a.cat, nseg, xs, xsg, ldx, widths);
    if (k <= 0) return EXO_EINVAL;
    if (m == 0) return EXO_OK;
    a.A = plain(xs[0], 0, 0, 1);
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
    a.b16 = prec != PREC_F32 ? w16 : nullptr;
    return launch_fwd(a, groups, prec, (hipStream_t)stream, true);
}

/* y = AvgL1Norm(X W^T + b) per output row (no activation), N <= 320: one
 * launch for td7_dense_fwd + td7_avgl1norm_fwd.  Layout as td7_dense_fwd (y:
 * [G][M][N] with group stride ysg, row stride ldy); h (pre-norm, same layout)
 * and mean ([G][M], the raw mean |h|) are written when non-null.  prec: the
 * MFMA operand precision (Prec). */
int td7_dense_fwd_norm(const float *x, long xsg, long ldx, const float *w, const float *b, float *y, float *h,
                       float *mean, long ysg, long ldy, int32_t groups, int32_t m, int32_t n, int32_t k, int32_t prec,
                       float eps, void *stream) {
    if (!x || !w || !y || groups <= 0 || m < 0 || n <= 0 || n > 320 || k <= 0 || prec < 0 || prec > PREC_F16)
        return EXO_EINVAL;
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
    a.act = ACT_NONE;
    a.j_bias = -1;
    return launch_fwd_norm(a, groups, prec, h, mean, eps, (hipStream_t)stream, false);
}

/* td7_dense_fwd_norm of a concatenated input (td7_dense_fwd_cat's segments). */
int td7_dense_fwd_norm_cat(int32_t nseg, const float *const *xs, const long *xsg, const long *ldx,
                           const int32_t *widths, const float *w, const float *b, float *y, float *h, float *mean,
                           long ysg, long ldy, int32_t groups, int32_t m, int32_t n, int32_t prec, float eps,
                           void *stream) {
    if (!w || !y || groups <= 0 || m < 0 || n <= 0 || n > 320 || prec < 0 || prec > PREC_F16) return EXO_EINVAL;
    GemmArgs a{};
    const int k = make_cat(a.cat, nseg, xs, xsg, ldx, widths);
    if (k <= 0) return EXO_EINVAL;
    if (m == 0) return EXO_OK;
    a.A = plain(xs[0], 0, 0, 1);
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
    a.act = ACT_NONE;
    a.j_bias = -1;
    return launch_fwd_norm(a, groups, prec, h, mean, eps, (hipStream_t)stream, true);
}

/* td7_dense_bwd_weight of a layer whose input was given by segments
 * (td7_dense_fwd_cat's layout); N >= 4. */
int td7_dense_bwd_weight_cat(const float *dy, long dysg, long lddy, const float *yv, long ysg, long ldy, int32_t nseg,
                             const float *const *xs, const long *xsg, const long *ldx, const int32_t *widths, float *dw,
                             float *db, int32_t groups, int32_t m, int32_t n, int32_t act, void *stream) {
    if (!dy || !yv || !dw || groups <= 0 || m <= 0 || n < 4) return EXO_EINVAL;
    const int prec = act >> 8;
    act &= 0xFF;
    if (act > 3 || prec > PREC_F16) return EXO_EINVAL;
    WgradArgs w{};
    const int k = make_cat(w.cat, nseg, xs, xsg, ldx, widths);
    if (k <= 0) return EXO_EINVAL;
    const long span = (long)groups * (dysg > ysg ? dysg : ysg) + (long)m * (lddy > ldy ? lddy : ldy) + n;
    if (span >= (1L << 29)) return EXO_ERANGE;
    w.dy = dy;
    w.y = yv;
    w.x = xs[0];
    w.dysg = (int)dysg;
    w.lddy = (int)lddy;
    w.ysg = (int)ysg;
    w.ldy = (int)ldy;
    w.dw = dw;
    w.db = db;
    w.I = n;
    w.J = k;
    w.M = m;
    return launch_wgrad(w, groups, act, prec, (hipStream_t)stream, true);
}

/* dX = sum over the reduced groups of (dY[g] * act'(Y[g])) W[g].
 * dY, Y: [G][M][N] (group stride dysg / ysg, row strides lddy / ldy);
 * W: [G][N][K]; dX: [M][K] per group (dxsg, lddx).  shared_input != 0: X was
 * one tensor for all groups, dX (a single [M][K]) sums over them. */
int td7_dense_bwd_data(const float *dy, long dysg, long lddy, const float *yv, long ysg, long ldy, const float *w,
                       float *dx, long dxsg, long lddx, int32_t groups, int32_t shared_input, int32_t m, int32_t n,
                       int32_t k, int32_t act, void *stream) {
    return td7_dense_bwd_data_cols(dy, dysg, lddy, yv, ysg, ldy, w, dx, dxsg, lddx, groups, shared_input, m, n, k, 0,
                                   k, act, stream);
}

/* td7_dense_bwd_data for the input columns [c0, c1) only: the gradient w.r.t.
 * the slice of a concatenated input that requires it (the rest of dX is left
 * untouched). */
int td7_dense_bwd_data_cols(const float *dy, long dysg, long lddy, const float *yv, long ysg, long ldy,
                            const float *w, float *dx, long dxsg, long lddx, int32_t groups, int32_t shared_input,
                            int32_t m, int32_t n, int32_t k, int32_t c0, int32_t c1, int32_t act, void *stream) {
    if (!dy || !yv || !w || !dx || groups <= 0 || m < 0 || n <= 0 || k <= 0) return EXO_EINVAL;
    if (c0 < 0 || c1 > k || c0 >= c1) return EXO_EINVAL;
    const int prec = act >> 8;
    act &= 0xFF;
    if (act > 3 || prec > PREC_F16) return EXO_EINVAL;
    if (m == 0) return EXO_OK;
    GemmArgs a{};
    a.A = plain(dy, dysg, lddy, 1);
    a.A.y = yv;
    a.A.ysg = ysg;
    a.A.ysi = ldy;
    a.A.ysr = 1;
    a.A.act = act;
    a.B = plain(w + c0, (long)n * k, 1, k); // B(j = out col c0 + j, r = n) = W[n][c0 + j]
    a.I = m;
    a.J = c1 - c0;
    a.R = n;
    a.groups_red = shared_input ? groups : 1;
    a.C = dx + c0;
    a.csg = dxsg;
    a.csi = lddx;
    a.csj = 1;
    a.act = ACT_NONE;
    a.j_bias = -1;
    return launch(a, shared_input ? 1 : groups, prec, (hipStream_t)stream);
}

/* dW[g] = (dY[g] * act'(Y[g]))^T X[g]  ([N][K], contiguous per group) and,
 * when db != null, db[g] = column sums of dY[g] * act'(Y[g])  ([N]). */
int td7_dense_bwd_weight(const float *dy, long dysg, long lddy, const float *yv, long ysg, long ldy, const float *x,
                         long xsg, long ldx, float *dw, float *db, int32_t groups, int32_t m, int32_t n, int32_t k,
                         int32_t act, void *stream) {
    if (!dy || !yv || !x || !dw || groups <= 0 || m < 0 || n <= 0 || k <= 0) return EXO_EINVAL;
    const int prec = act >> 8;
    act &= 0xFF;
    if (act > 3 || prec > PREC_F16) return EXO_EINVAL;
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
            WgradArgs w{{}, dy, yv, x, (int)dysg, (int)lddy, (int)ysg, (int)ldy, (int)xsg, (int)ldx, dw, db, n, k, m};
            return launch_wgrad(w, groups, act, prec, (hipStream_t)stream);
        }
    }
    return launch(a, groups, prec, (hipStream_t)stream);
}

} // extern "C"
