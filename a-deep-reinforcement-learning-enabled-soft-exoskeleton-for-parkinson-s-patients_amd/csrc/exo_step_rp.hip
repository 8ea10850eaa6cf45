// exo_step_rp.hip -- row-parallel variant of the env step for small env counts.
//
// exo_step_kernel (exo_env.hip) gives each ODE solve ONE lane: at 4,096 envs
// that is 128 wavefronts on a 1,024-SIMD chip, so the step is bound by the
// serial latency of ~36 RHS evaluations per lane.  Here every env gets 16
// lanes: lanes 0-7 run the actuated solve, lanes 8-15 the tremor-only solve,
// and lane r of a group owns joint row r of the 7-DOF ODE (row 7 pads).  The
// RHS a = I^-1 (T - D v - K q) needs the other rows' q, v and r: they are
// exchanged through wave-private LDS slots inside the 8-lane group; the
// RK45 error norm is an 8-lane butterfly sum, so every lane of a group takes
// the same step-size decisions.  The arithmetic is the same as the one-lane
// kernel (same per-row summation orders), so the two variants agree to
// rounding of the error-norm sum.
//
// Prologue: all lanes of an env compute the forward kinematics redundantly
// (same instructions, no divergence); lane j < 7 of the actuated group
// evaluates actuator j (force components, position/radius vectors, torque)
// and the torque table is shared by permutes.  Reward, done, observation,
// info and the carried state are written before the solves (none depends on
// the ODE), the joint-target motor update after them.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "exo_amd.h"
#include "exo_model.h"

using namespace exo;

// Diagnostic build only (make STAMPS=1 -> libexo_amd_stamps.so): per-wave
// s_memtime stamps at the phase boundaries of the step; the product build
// compiles them out.
#ifdef EXO_STAMPS
__device__ unsigned long long *g_exo_stamps;
#define STAMP(k)                                                                                                  \
    do {                                                                                                          \
        unsigned long long _t;                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                             \
        __builtin_amdgcn_sched_barrier(0);                                                                        \
        if (g_exo_stamps && (threadIdx.x & 63) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63))               \
            g_exo_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + (k)] = _t;                 \
    } while (0)
// RK45 step attempts (accepted + rejected) of each env's two solves, [2][N]
// (tools/rk45_hist.py: the configs[3] slowest-env histogram)
__device__ int32_t *g_exo_rksteps;
#else
#define STAMP(k) do {} while (0)
#endif

namespace {

__device__ __forceinline__ double cfg(const Dev &S, int k, int e) { return S.cfg[(size_t)k * S.N + e]; }

// Row-r tables of the sparse RHS (padding entries point at row 7 with a zero coefficient).
constexpr int RP_DCOL[8][4] = {{0, 1, 2, 3}, {0, 1, 2, 7}, {0, 1, 2, 7}, {0, 3, 7, 7},
                               {4, 5, 6, 7}, {4, 5, 6, 7}, {4, 5, 6, 7}, {7, 7, 7, 7}};
constexpr int RP_DSYM[8][4] = {{0, 1, 2, 3}, {1, 4, 5, -1}, {2, 5, 6, -1}, {3, 7, -1, -1},
                               {8, 9, 10, -1}, {9, 11, 12, -1}, {10, 12, 13, -1}, {-1, -1, -1, -1}};
constexpr int RP_ICOL[8][4] = {{0, 3, 6, 7}, {1, 2, 4, 5}, {1, 2, 4, 5}, {0, 3, 6, 7},
                               {1, 2, 4, 5}, {1, 2, 4, 5}, {0, 3, 6, 7}, {7, 7, 7, 7}};
constexpr int RP_ISYM[8][4] = {{0, 1, 2, -1}, {6, 7, 8, 9}, {7, 10, 11, 12}, {1, 3, 4, -1},
                               {8, 11, 13, 14}, {9, 12, 14, 15}, {2, 4, 5, -1}, {-1, -1, -1, -1}};

// The tables above indexed by the lane's row r (a runtime value) compile to
// global loads of the table, each followed by a wait for EVERY outstanding
// load (vmcnt(0)) before the dependent load of the matrix entry could issue:
// the kernel-start load burst was drained 4+ times in a row.  Packed into
// 64-bit immediates instead (byte r of column m = entry + 1): pure ALU.
constexpr unsigned long long pack_col(const int (&t)[8][4], int m) {
    unsigned long long v = 0;
    for (int r = 0; r < 8; ++r) v |= (unsigned long long)(t[r][m] + 1) << (8 * r);
    return v;
}
__device__ __forceinline__ int tab_at(unsigned long long k, int r) { return (int)((k >> (8 * r)) & 0xff) - 1; }
// K_LINK[k] (exo_model.h) for a runtime k < 14, likewise
constexpr unsigned long long pack_klink(int k0) {
    unsigned long long v = 0;
    for (int k = k0; k < k0 + 8 && k < 14; ++k) v |= (unsigned long long)K_LINK[k] << (8 * (k - k0));
    return v;
}
__device__ __forceinline__ int klink(int k) {
    constexpr unsigned long long lo = pack_klink(0), hi = pack_klink(8);
    return (int)(((k < 8 ? lo : hi) >> (8 * (k & 7))) & 0xff);
}

struct RowM {
    double d[4], s[4], ii[4];
    int dsrc[4], isrc[4];
};

__device__ __forceinline__ double shfl_d(double x, int src) { return __shfl(x, src, 64); }

// DPP lane moves of a double (two dword moves, VALU only: no LDS round trip)
// (every control used here -- quad_perm, row_half_mirror -- reads a valid lane
// of the same row, so bound_ctrl and the old value never apply: mov_dpp
// without the zeroed old operand the update form materialised per move)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const long long v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(v & 0xffffffffLL), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// sum over the 8-lane group, identical in all lanes: xor-1 and xor-2 inside
// each quad (quad_perm), then the half-row mirror pairs the group's two quads
__device__ __forceinline__ double group_sum(double x) {
    x += dpp_d<0xB1>(x);  // quad_perm [1,0,3,2]
    x += dpp_d<0x4E>(x);  // quad_perm [2,3,0,1]
    x += dpp_d<0x141>(x); // row_half_mirror: lane i <-> 7 - i within each 8 lanes
    return x;
}

// The same RHS with every neighbour pull a DPP lane move (VALU, no LDS round
// trip).  For term m the source column of row r, RP_DCOL[r][m], is one
// quad_perm pattern shared by both quads of the group (pads take any lane:
// their coefficient is 0), so D v and K q need one move per term.  I^-1's
// blocks {0,3,6} and {1,2,4,5} cross the quads: a term's column comes from
// the own quad (quad_perm of r) in one quad and from the other one
// (quad_perm of the half-row mirror of r) in the other, picked by a select.
// Same terms in the same order as row_acc: bit-identical results.
__device__ __forceinline__ double row_acc_dpp(const RowM &M, bool upper, double T, double q, double v) {
    double dq = 0.0, kq = 0.0;
    dq += M.d[0] * dpp_d<0x00>(v); kq += M.s[0] * dpp_d<0x00>(q);  // columns [0,0,0,0] of each quad
    dq += M.d[1] * dpp_d<0xD5>(v); kq += M.s[1] * dpp_d<0xD5>(q);  // [1,1,1,3]
    dq += M.d[2] * dpp_d<0xAA>(v); kq += M.s[2] * dpp_d<0xAA>(q);  // [2,2,2,2]
    dq += M.d[3] * dpp_d<0xFF>(v); kq += M.s[3] * dpp_d<0xFF>(q);  // [3,3,3,3]
    const double r = T - dq - kq;
    const double mr = dpp_d<0x141>(r);  // lane i <- lane 7 - i of the 8
    double a = 0.0;
    a += M.ii[0] * (upper ? dpp_d<0xFA>(mr) : dpp_d<0x14>(r));
    a += M.ii[1] * (upper ? dpp_d<0x05>(mr) : dpp_d<0xEB>(r));
    a += M.ii[2] * (upper ? dpp_d<0xA0>(r) : dpp_d<0x7D>(mr));
    a += M.ii[3] * (upper ? dpp_d<0x55>(r) : dpp_d<0xAA>(mr));
    return a;
}

// selects the pull form (template flag of rk45_rows)
struct RowD {
    RowM m;
    bool upper;
};
__device__ __forceinline__ double row_acc(const RowD &M, double T, double q, double v) {
    return row_acc_dpp(M.m, M.upper, T, q, v);
}

// The same RHS with the neighbour values exchanged through LDS: each lane
// stores its (q, v) as one 16-byte write and reads its 4 source rows' pairs
// as 16-byte reads (5 LDS ops where the permutes take 16 32-bit moves), then
// r the same way (1 + 4 ops instead of 8).  Wave-private slots (one per lane),
// so no workgroup barrier: a wavefront's LDS ops execute in order, and the
// wave_barrier keeps the compiler from moving the reads above the write.
// Same terms in the same order as row_acc: bit-identical results.
struct RowL {
    RowM m;
    double2 *qv;    // [64 x waves] workgroup slots
    double *rr;
    int self, wbase; // this lane's slot, its wavefront's first slot
};
__device__ __forceinline__ double row_acc(const RowL &M, double T, double q, double v) {
    M.qv[M.self] = make_double2(q, v);
    __builtin_amdgcn_wave_barrier();
    double2 p[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) p[m] = M.qv[M.wbase + M.m.dsrc[m]];
    double dq = 0.0, kq = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        dq += M.m.d[m] * p[m].y;
        kq += M.m.s[m] * p[m].x;
    }
    const double r = T - dq - kq;
    M.rr[M.self] = r;
    __builtin_amdgcn_wave_barrier();
    double rs[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) rs[m] = M.rr[M.wbase + M.m.isrc[m]];
    double a = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) a += M.m.ii[m] * rs[m];
    __builtin_amdgcn_wave_barrier();
    return a;
}

// acceleration of row r: I^-1 (T - D v - K q), neighbours pulled from the group
__device__ __forceinline__ double row_acc(const RowM &M, double T, double q, double v) {
    double dq = 0.0, kq = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const double vv = shfl_d(v, M.dsrc[m]), qq = shfl_d(q, M.dsrc[m]);
        dq += M.d[m] * vv;
        kq += M.s[m] * qq;
    }
    const double r = T - dq - kq;
    double a = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) a += M.ii[m] * shfl_d(r, M.isrc[m]);
    return a;
}

// scipy RK45 (common.py select_initial_step, rk.py _step_impl) for the row
// this lane owns; same second-order storage as rk45_solve in exo_model.h.
// The solver's whole state between two step attempts: this row's (q, v) and
// FSAL acceleration a0, and the group-uniform t, h_abs, attempt count and
// "inside a step after a rejection" flags -- a budgeted launch stops between
// two attempts and the next launch continues from exactly this state.
struct RkState {
    double q, v, a0, t, h_abs;
    int guard;
    bool rejected, in_step;
};

template <typename RM>
__device__ __forceinline__ void rk45_begin(const RM &M, double T, RkState &s) {
    const double atol = 1e-6, tb = DT, inv_sqrt14 = 1.0 / 3.7416573867739413;
    s.q = 0.0;
    s.v = 0.0;
    s.a0 = row_acc(M, T, 0.0, 0.0);
    {
        const double x1 = s.a0 / atol;
        const double d1 = sqrt(group_sum(x1 * x1)) * inv_sqrt14;
        const double h0 = 1e-6;
        const double y1v = h0 * s.a0;
        const double a1 = row_acc(M, T, 0.0, y1v);
        const double xq = y1v / atol, xv = (a1 - s.a0) / atol;
        const double d2 = sqrt(group_sum(xq * xq + xv * xv)) * inv_sqrt14 / h0;
        // scipy's (0.01 / max(d1, d2)) ** 0.2 with the library pow (once per solve)
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
        s.h_abs = fmin(fmin(100 * h0, h1), tb);
    }
    s.t = 0.0;
    s.guard = 0;
    s.rejected = s.in_step = false;
}

// Step attempts until t reaches dt: 1 = done, -1 = failed (step too small /
// 4,096 attempts), 0 = `budget` (> 0) attempts used in this call with the
// solve unfinished (the state is left between two attempts).  The attempt
// sequence, and every value, is the one of an uninterrupted solve.
template <typename RM>
__device__ int rk45_advance(const RM &M, double T, RkState &s, int budget) {
    const double rtol = 1e-3, atol = 1e-6, tb = DT, inv_sqrt14 = 1.0 / 3.7416573867739413;
    int used = 0;
    while (s.t != tb) {
        const double min_step = 10 * fabs(nextafter(s.t, INFINITY) - s.t);
        if (!s.in_step) {  // a new step (rk.py _step_impl): h_abs raised to min_step
            if (s.h_abs < min_step) s.h_abs = min_step;
            s.rejected = false;
            s.in_step = true;
        }
        if (budget > 0 && used == budget) return 0;
        if (s.h_abs < min_step || ++s.guard > 4096) return -1;
        ++used;
        const double q = s.q, v = s.v;
        double t_new = s.t + s.h_abs;
        if (t_new - tb > 0) t_new = tb;
        const double h = t_new - s.t, h2 = h * h;
        s.h_abs = fabs(h);
        double A[7];
        A[0] = s.a0;
        double qs = 0.0, vs = 0.0;
#pragma unroll
        for (int st = 1; st < 6; ++st) {
            double dv = 0.0, dq = 0.0;
#pragma unroll
            for (int l = 0; l < st; ++l) { dv += A[l] * RK_A[st][l]; dq += A[l] * RKN.AA[st][l]; }
            vs = v + dv * h;
            qs = q + RKN.C[st] * h * v + dq * h2;
            A[st] = row_acc(M, T, qs, vs);
        }
        {
            double dv = A[0] * RK_B[0], dq = A[0] * RKN.BB[0] + A[1] * RKN.BB[1];
#pragma unroll
            for (int l = 2; l < 5; ++l) { dv += A[l] * RK_B[l]; dq += A[l] * RKN.BB[l]; }
            dv += A[5] * RK_B[5];
            vs = v + h * dv; // y_new
            qs = q + h * v + dq * h2;
        }
        A[6] = row_acc(M, T, qs, vs);
        double ev = A[0] * RK_E[0], eq = A[0] * RKN.EE[0] + A[1] * RKN.EE[1];
#pragma unroll
        for (int l = 2; l < 6; ++l) { ev += A[l] * RK_E[l]; eq += A[l] * RKN.EE[l]; }
        ev += A[6] * RK_E[6];
        const double e_q = eq * h2 / (atol + fmax(fabs(q), fabs(qs)) * rtol);
        const double e_v = ev * h / (atol + fmax(fabs(v), fabs(vs)) * rtol);
        const double en = sqrt(group_sum(e_q * e_q + e_v * e_v)) * inv_sqrt14;
        if (en < 1) {
            double factor = (en == 0) ? 10.0 : fmin(10.0, 0.9 * pow_m5th(en));
            if (s.rejected) factor = fmin(1.0, factor);
            s.h_abs *= factor;
            s.t = t_new;
            s.q = qs;
            s.v = vs;
            s.a0 = A[6];
            s.in_step = false;
        } else {
            s.h_abs *= fmax(0.2, 0.9 * pow_m5th(en));
            s.rejected = true;
        }
    }
    return 1;
}

// the uninterrupted solve
template <typename RM>
__device__ __forceinline__ bool rk45_rows(const RM &M, double T, double &q_out, int &attempts) {
    RkState s;
    rk45_begin(M, T, s);
    const bool ok = rk45_advance(M, T, s, 0) > 0;
    q_out = s.q;  // on failure the last accepted q, as scipy's sol.y[:, -1] (exo_model.h rk45_solve)
    attempts = s.guard;
    return ok;
}

// carried state of a budgeted solve: lane field f of sub-lane sb (0..15),
// group field f of group g (t, h_abs, attempts, flags)
__device__ __forceinline__ size_t rk_lane(int sb, int f, int e, int N) { return (size_t)(sb * 4 + f) * N + e; }
__device__ __forceinline__ size_t rk_grp(int g, int f, int e, int N) { return (size_t)(64 + g * 4 + f) * N + e; }

__device__ __forceinline__ void rk_save(const Dev &S, int e, int sub, int grp, int r, const RkState &s, double T) {
    const int N = S.N;
    S.rk[rk_lane(sub, 0, e, N)] = s.q;
    S.rk[rk_lane(sub, 1, e, N)] = s.v;
    S.rk[rk_lane(sub, 2, e, N)] = s.a0;
    S.rk[rk_lane(sub, 3, e, N)] = T;
    if (r == 0) {
        S.rk[rk_grp(grp, 0, e, N)] = s.t;
        S.rk[rk_grp(grp, 1, e, N)] = s.h_abs;
        S.rk[rk_grp(grp, 2, e, N)] = (double)s.guard;
        S.rk[rk_grp(grp, 3, e, N)] = (double)((s.rejected ? 1 : 0) | (s.in_step ? 2 : 0));
    }
}

__device__ __forceinline__ void rk_load(const Dev &S, int e, int sub, int grp, RkState &s, double &T) {
    const int N = S.N;
    s.q = S.rk[rk_lane(sub, 0, e, N)];
    s.v = S.rk[rk_lane(sub, 1, e, N)];
    s.a0 = S.rk[rk_lane(sub, 2, e, N)];
    T = S.rk[rk_lane(sub, 3, e, N)];
    s.t = S.rk[rk_grp(grp, 0, e, N)];
    s.h_abs = S.rk[rk_grp(grp, 1, e, N)];
    s.guard = (int)S.rk[rk_grp(grp, 2, e, N)];
    const int fl = (int)S.rk[rk_grp(grp, 3, e, N)];
    s.rejected = fl & 1;
    s.in_step = (fl & 2) != 0;
}

// CoMs of the lane's two k-links (actuator j: K_LINK[2j], K_LINK[2j + 1])
// from the FK frames, given their rows v1, v2 (U.anc, loaded with the
// kernel-start batch).  The first anchors of actuators 0, 1 (links 9, 12) sit
// on the humerus, those of 2..6 on the base (U.kbase); the second anchors of
// actuators 0, 1 (links 5, 6) on the forearm, those of 2..6 on the humerus.
// Same operands and operations as the per-link form (a runtime index into the
// by-value kernel argument per link, U.xyz[link], compiled to a load from the
// kernarg segment behind a vmcnt(0) in each divergent branch): bit-identical.
__device__ __forceinline__ void anchors(int j, const double *v1, const double *v2, const double *R2,
                                        const double *p0, const double *R4, const double *p3, double *k1, double *k2) {
    double h1[3], f2[3], h2[3];
    xform(R2, p0, v1, h1);
    xform(R4, p3, v2, f2);
    xform(R2, p0, v2, h2);
    const bool arm = j < 2;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        k1[d] = arm ? h1[d] : v1[d];
        k2[d] = arm ? f2[d] : h2[d];
    }
}

// The solve of this lane's row with the selected RHS exchange (template PULL
// of the kernel): begin (a fresh solve) or continue the carried state `s`,
// at most `budget` attempts (0: to the end).
template <int PULL, int EPB>
__device__ __forceinline__ int solve_rows(const RowM &M0, int r, double T, RkState &s, bool begin, int budget) {
    if constexpr (PULL == 1) {
        const RowD M{M0, r >= 4};
        if (begin) rk45_begin(M, T, s);
        return rk45_advance(M, T, s, budget);
    } else if constexpr (PULL == 2) {
        __shared__ double2 s_qv[64 * EPB / 4];
        __shared__ double s_rr[64 * EPB / 4];
        const RowL M{M0, s_qv, s_rr, (int)threadIdx.x, (int)(threadIdx.x & ~63u)};
        if (begin) rk45_begin(M, T, s);
        return rk45_advance(M, T, s, budget);
    } else {
        if (begin) rk45_begin(M0, T, s);
        return rk45_advance(M0, T, s, budget);
    }
}

// The sparse RHS rows of this lane (row r of the env's I^-1, D, S).
__device__ __forceinline__ RowM load_rows(const Dev &S, int e, int r, int gbase) {
    const int N = S.N;
    RowM M0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        constexpr unsigned long long KDS[4] = {pack_col(RP_DSYM, 0), pack_col(RP_DSYM, 1), pack_col(RP_DSYM, 2),
                                               pack_col(RP_DSYM, 3)};
        constexpr unsigned long long KIS[4] = {pack_col(RP_ISYM, 0), pack_col(RP_ISYM, 1), pack_col(RP_ISYM, 2),
                                               pack_col(RP_ISYM, 3)};
        constexpr unsigned long long KDC[4] = {pack_col(RP_DCOL, 0), pack_col(RP_DCOL, 1), pack_col(RP_DCOL, 2),
                                               pack_col(RP_DCOL, 3)};
        constexpr unsigned long long KIC[4] = {pack_col(RP_ICOL, 0), pack_col(RP_ICOL, 1), pack_col(RP_ICOL, 2),
                                               pack_col(RP_ICOL, 3)};
        const int ds = tab_at(KDS[m], r), is = tab_at(KIS[m], r);
        // unconditional loads (field 0 for the pad entries), zeroed by a select
        const double dv = S.dnz[(size_t)(ds >= 0 ? ds : 0) * N + e];
        const double sv = S.snz[(size_t)(ds >= 0 ? ds : 0) * N + e];
        const double iv = S.iinv[(size_t)(is >= 0 ? is : 0) * N + e];
        M0.d[m] = ds >= 0 ? dv : 0.0;
        M0.s[m] = ds >= 0 ? sv : 0.0;
        M0.ii[m] = is >= 0 ? iv : 0.0;
        M0.dsrc[m] = gbase + tab_at(KDC[m], r);
        M0.isrc[m] = gbase + tab_at(KIC[m], r);
    }
    return M0;
}

// The actuated lane r's joint (:421-433): lane r holds q[r]; joint 0
// (shoulder z) <- q[2], 1 (y) <- q[0], 2 (x) <- q[1], 3 (elbow y) <- q[3],
// 4 <- q[4] (lanes 5..7: r, unused)
__device__ __forceinline__ int lane_joint(int r) { return (r == 0) ? 1 : (r == 1) ? 2 : (r == 2) ? 0 : r; }

// The operands of finish_solve that do not depend on the solve, loaded before
// it instead of after it (each was a memory latency on the slowest wave's
// tail): the imu sample of the lane's joint at counter c (issued right before
// the solve), and the joint's position before the motor step (with the
// kernel-start batch; only this lane writes it, after the solve).
struct Targets {
    double imu_v, q0;
    double lim[4];  // U.lim[r]: the joint's {lo, hi} and the boundary check's degree bounds
};
__device__ __forceinline__ void load_lims(const Urdf &U, int r, Targets &tg) {
#pragma unroll
    for (int k = 0; k < 4; ++k) tg.lim[k] = U.lim[r][k];
}
__device__ __forceinline__ double imu_at(const Dev &S, int motion, int joint, int c) {
    const int col = (joint == 0) ? 4 : (joint == 1) ? 3 : (joint == 2) ? 2 : (joint == 3) ? 0 : 1;
    return S.imu[((size_t)motion * 5 + col) * S.Lmax + c];
}

// After a solve of the step whose counter was c (:417-433): the amplitude
// into info (both groups), then -- actuated group -- the joint targets, the
// idealised motor step or the multibody targets, and the
// joint-range violation count.
__device__ __forceinline__ void finish_solve(const Dev &S, const Urdf &U, int e, int grp, int r, int ebase,
                                             const Targets &tg, double qr, float *info) {
    const int N = S.N;
    const double qdeg = qr * (180 / PI); // :417-418
    if (info && r < 7) info[(size_t)e * INFO + (grp == 0 ? 14 : 28) + r] = (float)qdeg;
    if (grp != 0) return;
    // ---- :421-433 joint targets and the idealised motor step
    const int joint = lane_joint(r);
    const double ang = tg.imu_v + (joint < 4 ? qdeg : 0.0);
    bool viol = false;
    if (r < 5) {
        if (S.mb_tgt) { // multibody mode: exo_multibody_kernel runs stepSimulation next
            S.mb_tgt[(size_t)joint * N + e] = ang * (PI / 180);
            if (r == 0) S.mb_flag[e] = 1;
        } else {
            const double q0 = tg.q0;
            const double nq = q0 + 0.1 * (ang * (PI / 180) - q0);
            S.phys_q[(size_t)joint * N + e] = fmin(fmax(nq, tg.lim[0]), tg.lim[1]);
        }
        if (joint < 4) viol = !(tg.lim[2] < ang && ang < tg.lim[3]); // check_movement_boundaries (:594-605)
    }
    const unsigned long long m = __ballot(viol);
    if (r == 0 && ((m >> ebase) & 0xFull)) S.viol[e] += 1;
}

// Budgeted step, an env whose solve(s) a previous launch left unfinished: no
// new step in this launch (its action is not consumed, the caller's mask
// leaves it out); its observation row is carried into this launch's output
// buffer (obs_cur -> obs: the trainer alternates two buffers); each pending
// group continues its solve, and a solve that completes finishes its step.
template <int PULL, int EPB>
__device__ void resume_env(const Dev &S, const Urdf &U, int e, int sub, int grp, int r, int gbase, int ebase,
                           int pend, float *obs, const float *obs_cur, float *info) {
    if (obs_cur) {
#pragma unroll
        for (int k = 0; k < OBS / 16; ++k) obs[(size_t)e * OBS + sub + 16 * k] = obs_cur[(size_t)e * OBS + sub + 16 * k];
    }
    const bool mine = (pend >> grp) & 1;
    int res = 1;
    RkState st;
    Targets tg{0.0, 0.0};
    if (mine) {
        const RowM M0 = load_rows(S, e, r, gbase);
        const int joint = lane_joint(r);
        tg.imu_v = imu_at(S, S.motion[e], joint, S.counts[e] - 1);
        tg.q0 = S.phys_q[(size_t)(joint < 5 ? joint : 4) * S.N + e];
        load_lims(U, r, tg);
        double T;
        rk_load(S, e, sub, grp, st, T);
        res = solve_rows<PULL, EPB>(M0, r, T, st, false, S.budget);
        if (res == 0) rk_save(S, e, sub, grp, r, st, T);
        if (res < 0) atomicOr(S.err, 1);
    }
    const unsigned long long m = __ballot(mine && res == 0 && r == 0);
    if (sub == 0) S.pend[e] = (uint8_t)(((m >> ebase) & 1) | (((m >> (ebase + 8)) & 1) << 1));
    if (!mine || res == 0) return;
#ifdef EXO_STAMPS
    if (g_exo_rksteps && r == 0) g_exo_rksteps[(size_t)grp * S.N + e] = st.guard;  // the solve's total attempts
#endif
    finish_solve(S, U, e, grp, r, ebase, tg, st.q, info);
}

// 16 envs (4 wavefronts) per workgroup: the state is SoA over envs, so one
// 128-byte line of a double field holds 16 consecutive envs -- a 4-env
// workgroup left each line to four workgroups on (round-robin) different XCDs
// and HBM fetched it up to four times (PMC: 3.1x the algorithmic bytes).
constexpr int RP_ENVS_PER_BLOCK = 16;

// PULL: the RHS neighbour exchange -- 0 LDS permutes, 1 DPP lane moves, 2 LDS slots (default)
// BUD: budgeted solves (S.budget > 0, S.pend / S.rk allocated; exo_set_step_budget)
template <int PULL, int EPB = RP_ENVS_PER_BLOCK, bool BUD = false>
__global__ __launch_bounds__(64 * EPB / 4) void exo_step_rp_kernel(
    Dev S, Urdf U, const float *__restrict__ act, float *__restrict__ obs, float *__restrict__ rew,
    uint8_t *__restrict__ done, float *__restrict__ info, const uint8_t *__restrict__ active,
    const float *__restrict__ obs_cur) {
    const int lane = threadIdx.x & 63;
    const int sub = lane & 15, grp = sub >> 3, r = sub & 7, gbase = lane & ~7, ebase = lane & ~15;
    const int e = blockIdx.x * EPB + (threadIdx.x >> 4);
    if (e >= S.N) return;
    const int N = S.N, c = S.counts[e], L = S.L[e];
    if constexpr (BUD) {
        const int pend = S.pend[e];  // uniform over the env's 16 lanes
        if (pend) {
            resume_env<PULL, EPB>(S, U, e, sub, grp, r, gbase, ebase, pend, obs, obs_cur, info);
            return;
        }
    }
    if ((active && !active[e]) || c >= L - 1) return; // uniform over the env's 16 lanes
    STAMP(0);

    const double maxS = S.maxSE[e], maxE = S.maxSE[(size_t)N + e];
    const float *a = act + (size_t)e * ACT;

    // ---- forward kinematics of the state left by the last stepSimulation (all lanes)
    // the five joint sincos are spread over the env's lanes (lane sub takes
    // joint sub % 5) and shared through wave-private LDS slots: one sincos
    // chain per lane instead of five in a row (ocml's sincos ends in a
    // divergent-branch check, so five calls did not overlap)
    __shared__ double2 s_fk[64 * EPB / 4];
    const int jt = lane_joint(r), jq = jt < 5 ? jt : 4;
    const double qk = S.phys_q[(size_t)(sub % 5) * N + e];
    const double qj = S.phys_q[(size_t)jq * N + e];  // this lane's joint before the motor step (finish_solve)
    double refo[6], refn[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) refo[j] = S.ref[(size_t)j * N + e];
    // ---- every other load of the step, issued now: one memory latency for the
    // whole step instead of one per phase (the loads go out in the order the
    // phases below consume them; nothing is stored before this point)
    const int j = r < 7 ? r : 6;  // this lane's actuator (lanes r == 7 duplicate actuator 6 and discard it)
    double sh1[3], sh2[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        sh1[d] = S.shift[(size_t)((2 * j) * 3 + d) * N + e];
        sh2[d] = S.shift[(size_t)((2 * j + 1) * 3 + d) * N + e];
    }
    double av1[3], av2[3];  // this lane's anchor rows (anchors())
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        av1[d] = U.anc[r][d];
        av2[d] = U.anc[r][3 + d];
    }
    const double pa_j = S.prev_a[(size_t)j * N + e];
    const double pa2_j = S.prev2_a[(size_t)j * N + e];
    float posv_old[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) posv_old[d] = S.posv[(size_t)(j * 3 + d) * N + e];
    const int motion = S.motion[e];
    Targets tg;
    tg.q0 = qj;
    load_lims(U, r, tg);
#ifdef EXO_STAMPS_MEMWAIT
    // diagnostic: when the kernel-start loads have all returned (serialises the prologue)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    STAMP(8);
#endif
    double R2[9], R4[9], p0[3], p3[3];
    {
        double sk, ck;
        sincos(qk, &sk, &ck);
        s_fk[threadIdx.x] = make_double2(sk, ck);
        __builtin_amdgcn_wave_barrier();
        double2 sc[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) sc[k] = s_fk[(threadIdx.x & ~15u) + k];  // lane k of the env: joint k
        double Rt[9], R0[9], R1[9], R3[9];
        p0[0] = U.xyz[0][0]; p0[1] = U.xyz[0][1]; p0[2] = U.xyz[0][2] + 0.1;
        mul_rz(U.Ro[0], sc[0].y, sc[0].x, R0);
        matmul3(R0, U.Ro[1], Rt); mul_rz(Rt, sc[1].y, sc[1].x, R1);
        matmul3(R1, U.Ro[2], Rt); mul_rz(Rt, sc[2].y, sc[2].x, R2);
        xform(R2, p0, U.xyz[3], p3);
        matmul3(R2, U.Ro[3], Rt); mul_rz(Rt, sc[3].y, sc[3].x, R3);
        matmul3(R3, U.Ro[4], Rt); mul_rz(Rt, sc[4].y, sc[4].x, R4);
        refn[0] = p0[0]; refn[1] = p0[1]; refn[2] = p0[2];
        xform(R3, p3, U.com3, &refn[3]);
    }
    // read-only operands of the reward, the observation and the solve's
    // torque, issued after the FK (the kernel-start batch above is what the FK
    // and the actuators wait for; these return under the actuator phase)
    const double tr_j = S.tremor[((size_t)c * 7 + j) * N + e];
    const int r4 = r & 3;  // tremor rows 0..3 of the observation at c - 1, c + 1
    const double tm1 = S.tremor[((size_t)(c > 0 ? c - 1 : 0) * 7 + r4) * N + e];
    const double tp1 = S.tremor[((size_t)(c + 1) * 7 + r4) * N + e];
    const double c_naxes = cfg(S, C_NAXES, e), c_maxrew = cfg(S, C_MAXREW, e);
    const double c_nrm = j < 2 ? cfg(S, C_MAXE0, e) : cfg(S, C_MAXS0, e);
    const int seq = S.seq[e];

    STAMP(1);
    // ---- actuator j = r (lanes r == 7 duplicate actuator 6 and discard it)
    double k1[3], k2[3], tx, ty, tz;
    float pv[3];
    {
        anchors(j, av1, av2, R2, p0, R4, p3, k1, k2);
        if (S.mb_q) { // multibody mode: the k-links sit at their prismatic joint positions
            const int kl1 = klink(2 * j), kl2 = klink(2 * j + 1);
            slide(U, kl1, R2, R4, S.mb_q[(size_t)kl1 * N + e], k1);
            slide(U, kl2, R2, R4, S.mb_q[(size_t)kl2 * N + e], k2);
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            k1[d] += sh1[d];
            k2[d] += sh2[d];
        }
        const double dx = (k2[0] + 5) - (k1[0] + 5), dy = (k2[1] + 5) - (k1[1] + 5), dz = (k2[2] + 5) - (k1[2] + 5);
        const double Fj = (((double)a[j] + 1) / 2) * (j < 2 ? maxE : maxS);
        const double fx = cos_atan2(dy, dx) * Fj, fy = cos_atan2(dx, dy) * Fj, fz = cos_atan2(dz, dx) * Fj;
        const int ro = (j < 2) ? 3 : 0; // elbow reference for actuators 1, 2
#pragma unroll
        for (int d = 0; d < 3; ++d) pv[d] = (float)(k2[d] - (ro ? refo[3 + d] : refo[d])); // stale ref (A.3)
        const double r0 = (ro ? refn[3] : refn[0]) - k2[0], r1 = (ro ? refn[4] : refn[1]) - k2[1],
                     r2 = (ro ? refn[5] : refn[2]) - k2[2];
        tx = fy * r2 - fz * r1;
        ty = fz * r0 - fx * r2;
        tz = fx * r1 - fy * r0;
    }
    STAMP(2);
    // the torque sums of :394-400 through wave-private LDS slots: every lane
    // stores its actuator's (tx, ty, tz); lane r < 3 reads component {1, 0,
    // 2}[r] of actuators 3, 4, 5, 7, 6 (lanes 2, 3, 4, 6, 5) and sums them in
    // that order, lane 3 takes |ty| of actuators 1 and 2 -- 7 reads where the
    // whole 7 x 3 table took 42 permutes (same sums: bit-identical)
    __shared__ double s_tq[3][64 * EPB / 4];
    s_tq[0][threadIdx.x] = tx;
    s_tq[1][threadIdx.x] = ty;
    s_tq[2][threadIdx.x] = tz;
    __builtin_amdgcn_wave_barrier();
    double at_r;
    {
        const unsigned eb = threadIdx.x & ~15u;  // the env's lane 0
        const double *col = s_tq[r == 1 ? 0 : (r == 2 ? 2 : 1)];
        const double t0 = col[eb], t1 = col[eb + 1], t2 = col[eb + 2], t3 = col[eb + 3], t4 = col[eb + 4],
                     t5 = col[eb + 5], t6 = col[eb + 6];
        at_r = r < 3 ? t2 + t3 + t4 + t6 + t5 : (r == 3 ? fabs(t0) - fabs(t1) : 0.0);
    }
    STAMP(6);
    // per-lane values of this lane's actuator j / joint row r (dynamic indices
    // into small register arrays would go to scratch)
    const double F_j = (((double)a[j] + 1) / 2) * (j < 2 ? maxE : maxS); // :256-266
    const double tr_r = (r < 7) ? tr_j : 0.0;
    const double Ta_r = tr_r + at_r;
    // every lane has read the carried state it needs; lanes of this env now
    // overwrite it (counts, ref, posv, prev actions, later the joints)
    // an env's 16 lanes sit in one wavefront, so only this wave's own loads
    // must have returned before its lanes overwrite the carried state: wait for
    // them (vmcnt 0; the "memory" clobber keeps the compiler from moving a
    // store above it) instead of a workgroup barrier, which also waited for the
    // other waves of the workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the ODE's matrix rows (12 loads, nothing in this kernel writes them),
    // issued only now: they return under the reward / observation / state
    // phase instead of queueing with the kernel-start batch the FK and the
    // actuators wait for
    const RowM M0 = load_rows(S, e, r, gbase);

    // reward terms (:341-366), term i on lane r = i of the actuated group (no
    // divergent per-term branches in one lane: every lane takes its two
    // divisions at once), summed over the 8-lane group by the butterfly; the
    // sums' order differs from the reference's i = 0..6 loop only by rounding
    double g_unw, g_st, g_nred, g_sa, g_sm;
    {
        const double eps = 1e-10;
        const bool live = r < 7, axis = r < 4, sel = axis && ((seq >> r) & 1);
        const double Tabs = fabs(Ta_r), tabs = fabs(tr_r);
        const double st_i = (Tabs - tabs) / tabs + 1;
        const double vv = (Tabs - tabs) / (tabs + eps) * 100;
        const double d = F_j - 2 * pa_j + pa2_j;
        g_unw = group_sum((axis && !sel) ? Tabs : 0.0);
        g_st = group_sum(sel ? st_i : 0.0);
        g_nred = group_sum((live && isfinite(vv) && vv < 0) ? 1.0 : 0.0);
        g_sa = group_sum(live ? F_j : 0.0);
        g_sm = group_sum(live ? d * d : 0.0);
    }

    // the four exponential reward terms (:341-366) on lanes 0..3 of the group
    // (one division chain and one exp per lane where lane 0 ran all four),
    // gathered into lane 0 by quad broadcasts; each term's operations as in
    // the one-lane form (r_sm's 0.05 * exp(.) commutes exactly)
    double r_k;
    {
        const double eps = 1e-10, Msum = maxE + maxS, naxes = c_naxes, sm = g_sm / 7;
        const double num = r == 0 ? g_unw : r == 1 ? -g_st + eps : r == 2 ? g_sa : sm;
        const double den = r == 0 ? Msum / 4 / naxes : r == 1 ? naxes : r == 2 ? Msum / 2 : Msum / 4;
        const double q = num / den;
        const double y = exp(r == 1 ? q : -q + eps);
        r_k = y * (r == 0 ? 0.5 : r == 1 ? 0.9 : 0.05);
    }
    const double r_tor = dpp_d<0x55>(r_k), r_ctl = dpp_d<0xAA>(r_k), r_sm = dpp_d<0xFF>(r_k);  // lanes 1, 2, 3 of the quad

    // ---- reward, done, observation, info, carried state (:341-366, :448-469, :487-570)
    if (grp == 0) {
        if (r == 0) {
            const double r_unw = r_k;
            const double r_axis = (int)g_nred * 0.5;
            rew[e] = (float)((r_axis + r_tor + r_sm + r_ctl + r_unw) / c_maxrew);
            done[e] = (uint8_t)(c + 1 >= L - 1);
            if (info) {
                float *io = info + (size_t)e * INFO;
                io[35] = (float)r_unw; io[36] = (float)r_tor; io[37] = (float)r_axis; io[38] = (float)r_ctl;
                io[39] = (float)r_sm;
            }
            S.counts[e] = c + 1;
        }
        STAMP(7);
        float *o = obs + (size_t)e * OBS;
        if (r < 7) {
            const double nrm = c_nrm;
            o[j] = (float)((c > 2 ? pa_j : 0.0) / nrm); // forces at c-1 (zero on an episode's first step)
            o[7 + j] = (float)(F_j / nrm);
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const size_t idx = (size_t)(j * 3 + d) * N + e;
                o[26 + j * 3 + d] = posv_old[d];
                o[47 + j * 3 + d] = pv[d];
                S.posv[idx] = pv[d];
            }
            if (info) {
                float *io = info + (size_t)e * INFO;
                io[j] = (float)at_r;
                io[7 + j] = (float)Ta_r;
                io[21 + j] = (float)tr_r;
            }
            S.prev2_a[(size_t)j * N + e] = pa_j;
            S.prev_a[(size_t)j * N + e] = F_j;
        } else { // lane 7: the reference link positions
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                o[68 + d] = (float)refo[d];
                o[74 + d] = (float)refn[d];
                S.ref[(size_t)d * N + e] = refn[d];
            }
        }
    } else if (r < 4) { // tremor rows 0..3 at c-1, c, c+1
        const double tn = (r < 3) ? 10.0 : 5.0;
        float *o = obs + (size_t)e * OBS;
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const double v = (b == 1) ? tr_r : (b == 0 ? tm1 : tp1);
            o[14 + b * 4 + r] = (float)(v / tn);
        }
    }

    // the imu sample for the joint targets, loaded now: its latency runs under
    // the solve (no vector-memory wait inside it); at kernel start its address
    // waited for `motion`, which stalled the in-order wave before the FK
    tg.imu_v = imu_at(S, motion, jt, c);  // every lane: in bounds, used by the actuated rows < 5
    STAMP(3);
    // ---- the two joint ODE solves (:409-414), one row per lane
    const double T = (r < 7) ? (grp == 0 ? Ta_r : tr_r) : 0.0;
    RkState st;
    const int res = solve_rows<PULL, EPB>(M0, r, T, st, true, BUD ? S.budget : 0);
    if constexpr (BUD) {
        // unfinished within the budget: the state is carried to the next launch
        if (res == 0) rk_save(S, e, sub, grp, r, st, T);
        const unsigned long long pm = __ballot(res == 0 && r == 0);
        if (sub == 0) S.pend[e] = (uint8_t)(((pm >> ebase) & 1) | (((pm >> (ebase + 8)) & 1) << 1));
        if (res == 0) return;
    }
    if (res < 0) atomicOr(S.err, 1);
#ifdef EXO_STAMPS
    if (g_exo_rksteps && r == 0) g_exo_rksteps[(size_t)grp * N + e] = st.guard;
#endif
    STAMP(4);
    // a failed solve (step below the spacing of t, or the device's 4,096-attempt
    // guard) continues from its last accepted q, as scipy's sol.y[:, -1]
    finish_solve(S, U, e, grp, r, ebase, tg, st.q, info);
    STAMP(5);
}

} // namespace

#ifdef EXO_STAMPS
extern "C" int exo_debug_set_stamps(unsigned long long *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_exo_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : -5;
}
extern "C" int exo_debug_set_rksteps(int32_t *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_exo_rksteps), &buf, sizeof(buf)) == hipSuccess ? 0 : -5;
}
#endif

namespace exo {
hipError_t launch_exo_step_rp(const Dev &S, const Urdf &U, const float *act, float *obs, float *rew, uint8_t *done,
                              float *info, const uint8_t *active, hipStream_t stream, bool shared,
                              const float *obs_cur) {
    // RHS neighbour exchange (EXO_RP_GATHER, all bit-identical): 2 = wave-private
    // LDS slots, 16-byte writes / reads (default: 26.8 vs 31.1 us at 4,096 envs,
    // profiles/r02f_raw/ab_pull.txt); 0 = LDS permutes (ds_bpermute, 4 32-bit
    // moves per (q, v) pull); 1 = DPP lane moves (slower still: two dword moves
    // per fp64 pull plus the DPP hazard waits -- 38.2 vs 34.9 us against 0);
    // r06: the slots for (q, v) and DPP moves for r (the second exchange of a
    // stage) tied the slots alone in the 256-thread shape (22.1-22.3 us) and
    // lost in the shared one (27.4 vs 26.9: two waves per SIMD share the
    // VALU), bit-identical -- not kept (profiles/r06_step/r06p)
    static const int pull = [] {
        const char *v = getenv("EXO_RP_GATHER");
        return v ? atoi(v) : 2;
    }();
    // shared: 32 envs per 512-thread workgroup (two waves per SIMD, a CU
    // filled by one workgroup): 4,096 envs take 128 CUs and leave the rest
    // whole for kernels running beside the step (the trainer's fused TD7
    // passes need a CU's full register file); 16 envs / 256 threads spread
    // over every CU (fastest alone)
    // budgeted solves (exo_set_step_budget): the LDS-slot exchange only
    if (S.budget > 0) {
        if (shared) {
            hipLaunchKernelGGL((exo_step_rp_kernel<2, 32, true>), dim3((S.N + 31) / 32), dim3(512), 0, stream, S, U,
                               act, obs, rew, done, info, active, obs_cur);
        } else {
            hipLaunchKernelGGL((exo_step_rp_kernel<2, RP_ENVS_PER_BLOCK, true>),
                               dim3((S.N + RP_ENVS_PER_BLOCK - 1) / RP_ENVS_PER_BLOCK),
                               dim3(64 * RP_ENVS_PER_BLOCK / 4), 0, stream, S, U, act, obs, rew, done, info, active,
                               obs_cur);
        }
        return hipGetLastError();
    }
    if (shared && pull != 1) {
        const dim3 grid((S.N + 31) / 32), block(512);
        if (pull == 2)
            hipLaunchKernelGGL((exo_step_rp_kernel<2, 32>), grid, block, 0, stream, S, U, act, obs, rew, done, info,
                               active, obs_cur);
        else
            hipLaunchKernelGGL((exo_step_rp_kernel<0, 32>), grid, block, 0, stream, S, U, act, obs, rew, done, info,
                               active, obs_cur);
        return hipGetLastError();
    }
    const dim3 grid((S.N + RP_ENVS_PER_BLOCK - 1) / RP_ENVS_PER_BLOCK), block(64 * RP_ENVS_PER_BLOCK / 4);
    if (pull == 1)
        hipLaunchKernelGGL(exo_step_rp_kernel<1>, grid, block, 0, stream, S, U, act, obs, rew, done, info, active,
                           obs_cur);
    else if (pull == 2)
        hipLaunchKernelGGL(exo_step_rp_kernel<2>, grid, block, 0, stream, S, U, act, obs, rew, done, info, active,
                           obs_cur);
    else
        hipLaunchKernelGGL(exo_step_rp_kernel<0>, grid, block, 0, stream, S, U, act, obs, rew, done, info, active,
                           obs_cur);
    return hipGetLastError();
}
} // namespace exo
