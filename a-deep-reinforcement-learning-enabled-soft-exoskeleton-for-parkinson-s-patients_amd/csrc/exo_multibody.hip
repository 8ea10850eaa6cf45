// exo_multibody.hip -- multibody ("fidelity") stepSimulation of the
// exoskeleton URDF (Environment/Exoskeleton_env.py:433)
// on gfx950.
//
// The default physics of exo_step is the idealised motor model of SURVEY.md
// A.2.  This kernel is the Bullet-equivalent alternative (exo_set_physics):
// Featherstone recursions over the 19-joint tree (5 revolute arm joints, 14
// prismatic actuator anchors), the joint motors and the violated joint limits
// as rows of a joint-space projected Gauss-Seidel (sequential impulse) solve,
// and semi-implicit Euler.  oracle/multibody.c states the model, its
// (unverified) Bullet constants, and is the checker.
//
// Layout: one env per 32-lane group (two envs per wavefront, 8 per
// workgroup), lane d owns joint d.  Per-link spatial quantities meet in LDS;
// the arm lanes do the inward (subtree) sums; the solve broadcasts each row's
// impulse with v_readlane (SGPRs, no LDS round trip) and every lane updates
// its own joint velocity with its row of M^-1.
//
// Same mathematics as the oracle, different factorisation (results agree to
// rounding, tests/test_multibody*.py):
//  * forward dynamics as qdd = -M^-1 h (Composite-Rigid-Body M, Newton-Euler
//    bias h with qdd = 0) instead of the Articulated-Body Algorithm: the solver
//    needs M^-1 anyway;
//  * M is an "arrow": each of the 9 k-links on the arm couples only with its
//    arm ancestors (b_k) and itself (D_k), so M^-1 follows from the 5x5 Schur
//    complement P = (M_arm - sum_k b_k b_k^T / D_k)^-1;
//  * the 5 k-links on the base are decoupled one-DOF systems.
#include <hip/hip_runtime.h>

#include "exo_model.h"

using namespace exo;

namespace {

constexpr int MB_G = 32;   // lanes per env
constexpr int MB_ENVS = 8; // envs per workgroup
constexpr int NC = 14;     // coupled joints: the arm (0..4) and its k-links (5..13)

struct EnvLds {
    double S[NJ][6];   // motion subspaces, world frame, about the world origin
    double qd[NJ];
    double in[NJ][10]; // rigid-body inertia {m, h = m c, Ibar about the origin: xx xy xz yy yz zz}
    double f[NJ][6];   // Newton-Euler link forces at qdd = 0
    double M[5][5];    // arm block of the joint-space inertia
    double b[NC][5];   // rows 5..13: S_j . I_k S_k of k-link k with its arm ancestors j
    double D[NJ];      // S_k . I_k S_k of the k-links
    double h[NJ];      // joint bias forces
};

__device__ __forceinline__ void cross3(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
// motion cross product v xm x
__device__ __forceinline__ void crm(const double *v, const double *x, double *o) {
    double t[3];
    cross3(v, x, o);
    cross3(v, x + 3, o + 3);
    cross3(v + 3, x, t);
    o[3] += t[0]; o[4] += t[1]; o[5] += t[2];
}
// force cross product v xf f
__device__ __forceinline__ void crf(const double *v, const double *f, double *o) {
    double t[3];
    cross3(v, f, o);
    cross3(v + 3, f + 3, t);
    o[0] += t[0]; o[1] += t[1]; o[2] += t[2];
    cross3(v, f + 3, o + 3);
}
// inertia {m, h, Ibar} times a motion vector [w; u]: [Ibar w + h x u; m u - h x w]
__device__ __forceinline__ void imul(const double *in, const double *x, double *o) {
    const double *Ib = in + 4;
    double t[3];
    cross3(in + 1, x + 3, t);
    o[0] = Ib[0] * x[0] + Ib[1] * x[1] + Ib[2] * x[2] + t[0];
    o[1] = Ib[1] * x[0] + Ib[3] * x[1] + Ib[4] * x[2] + t[1];
    o[2] = Ib[2] * x[0] + Ib[4] * x[1] + Ib[5] * x[2] + t[2];
    cross3(in + 1, x, t);
    o[3] = in[0] * x[3] - t[0];
    o[4] = in[0] * x[4] - t[1];
    o[5] = in[0] * x[5] - t[2];
}
__device__ __forceinline__ double dot6(const double *a, const double *b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
__device__ __forceinline__ double dot5(const double *a, const double *b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4];
}

// value of lane j of this lane's 32-lane group (j a compile-time constant):
// v_readlane into SGPRs for both groups of the wavefront, then a select
__device__ __forceinline__ double group_bcast(double x, int j, bool upper) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    const int l0 = __builtin_amdgcn_readlane(lo, j), h0 = __builtin_amdgcn_readlane(hi, j);
    const int l1 = __builtin_amdgcn_readlane(lo, 32 + j), h1 = __builtin_amdgcn_readlane(hi, 32 + j);
    return upper ? __hiloint2double(h1, l1) : __hiloint2double(h0, l0);
}

__global__ __launch_bounds__(MB_G *MB_ENVS) void exo_multibody_kernel(Dev S, Urdf U, MbModel P,
                                                                      const double *__restrict__ tgt,
                                                                      uint8_t *__restrict__ flag, int clear_flag) {
    __shared__ EnvLds lds[MB_ENVS];
    const int g = threadIdx.x / MB_G, d = threadIdx.x % MB_G;
    const bool upper = (threadIdx.x & 63) >= 32;
    const int N = S.N;
    const int e = blockIdx.x * MB_ENVS + g;
    const bool work = e < N && (!flag || flag[e]);
    const bool own = work && d < NJ;
    EnvLds &L = lds[g];
    // arm ancestors of joint d and the frame its joint hangs from
    const int npar = d < 5 ? d : (d <= 6 ? 5 : (d <= 13 ? 3 : 0));
    const int nwalk = d < 5 ? d + 1 : npar;

    double q = 0.0, qd = 0.0, qa[5];
    if (own) { q = S.mb_q[(size_t)d * N + e]; qd = S.mb_qd[(size_t)d * N + e]; }
#pragma unroll
    for (int j = 0; j < 5; ++j) qa[j] = work ? S.mb_q[(size_t)j * N + e] : 0.0;

    // ---- kinematics: walk the arm to joint d (arm lanes) or to its parent link
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, o[3] = {0.0, 0.0, 0.1}; // base at [0,0,0.1] (sim:18)
    double ax[3] = {0, 0, 1};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        if (i < nwalk) {
            double Rj[9], oi[3], s, c;
            matmul3(R, U.Ro[i], Rj);
            xform(R, o, U.xyz[i], oi);
            sincos(qa[i], &s, &c);
            mul_rz(Rj, c, s, R);
            ax[0] = Rj[2]; ax[1] = Rj[5]; ax[2] = Rj[8];
            o[0] = oi[0]; o[1] = oi[1]; o[2] = oi[2];
        }
    }
    double Sd[6], cm[3], Ic[9], m;
    if (d < 5) {
        Sd[0] = ax[0]; Sd[1] = ax[1]; Sd[2] = ax[2];
        cross3(o, ax, Sd + 3);
        xform(R, o, P.com[d < 5 ? d : 0], cm);
        double Rw[9];
        matmul3(R, P.Rin[d < 5 ? d : 0], Rw);
        const double *Id = P.Id[d < 5 ? d : 0];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b)
                Ic[a * 3 + b] = Rw[a * 3] * Id[0] * Rw[b * 3] + Rw[a * 3 + 1] * Id[1] * Rw[b * 3 + 1] +
                                Rw[a * 3 + 2] * Id[2] * Rw[b * 3 + 2];
        m = P.m[d < 5 ? d : 0];
    } else {
        const int k = (d < NJ ? d : 5) - 5;
        double jo[3], a3[3];
        xform(R, o, U.xyz[k + 5], jo);
        const double *z = U.kz[k];
#pragma unroll
        for (int a = 0; a < 3; ++a) a3[a] = R[a * 3] * z[0] + R[a * 3 + 1] * z[1] + R[a * 3 + 2] * z[2];
#pragma unroll
        for (int a = 0; a < 3; ++a) cm[a] = jo[a] + q * a3[a];
        Sd[0] = Sd[1] = Sd[2] = 0.0;
        Sd[3] = a3[0]; Sd[4] = a3[1]; Sd[5] = a3[2];
#pragma unroll
        for (int a = 0; a < 9; ++a) Ic[a] = (a % 4 == 0) ? 1.0 : 0.0;
        m = 1.0;
    }
    // {m, h, Ibar = Ic + m (|c|^2 E - c c^T)}
    double in[10];
    {
        const double cc = cm[0] * cm[0] + cm[1] * cm[1] + cm[2] * cm[2];
        in[0] = m; in[1] = m * cm[0]; in[2] = m * cm[1]; in[3] = m * cm[2];
        in[4] = Ic[0] + m * (cc - cm[0] * cm[0]);
        in[5] = Ic[1] - m * cm[0] * cm[1];
        in[6] = Ic[2] - m * cm[0] * cm[2];
        in[7] = Ic[4] + m * (cc - cm[1] * cm[1]);
        in[8] = Ic[5] - m * cm[1] * cm[2];
        in[9] = Ic[8] + m * (cc - cm[2] * cm[2]);
    }
    if (own) {
#pragma unroll
        for (int r = 0; r < 6; ++r) L.S[d][r] = Sd[r];
#pragma unroll
        for (int r = 0; r < 10; ++r) L.in[d][r] = in[r];
        L.qd[d] = qd;
    }
    __syncthreads();

    // ---- outward pass: velocity and bias acceleration (qdd = 0, gravity as an
    // upward base acceleration), Newton-Euler force of link d incl. Bullet's damping
    double v[6] = {0, 0, 0, 0, 0, 0}, acc[6] = {0, 0, 0, 0, 0, P.g};
    if (own) {
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const bool anc = a < npar, self = a == 5;
            if (anc || self) {
                double vJ[6], c6[6];
#pragma unroll
                for (int r = 0; r < 6; ++r) vJ[r] = anc ? L.S[a < 5 ? a : 0][r] * L.qd[a < 5 ? a : 0] : Sd[r] * qd;
#pragma unroll
                for (int r = 0; r < 6; ++r) v[r] += vJ[r];
                crm(v, vJ, c6);
#pragma unroll
                for (int r = 0; r < 6; ++r) acc[r] += c6[r];
            }
        }
    }
    double f[6];
    {
        double Ia[6], Iv[6], gy[6];
        imul(in, acc, Ia);
        imul(in, v, Iv);
        crf(v, Iv, gy);
        double t[3], vc[3];
        cross3(v, cm, t);
#pragma unroll
        for (int a = 0; a < 3; ++a) vc[a] = v[3 + a] + t[a];
        const double nv = sqrt(vc[0] * vc[0] + vc[1] * vc[1] + vc[2] * vc[2]);
        const double nw = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        double fl[3], ta[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            fl[a] = m * vc[a] * (P.lin_damp + P.lin_damp * nv);
            ta[a] = (Ic[a * 3] * v[0] + Ic[a * 3 + 1] * v[1] + Ic[a * 3 + 2] * v[2]) * (P.ang_damp + P.ang_damp * nw);
        }
        cross3(cm, fl, t);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            f[a] = Ia[a] + gy[a] + (ta[a] + t[a]);
            f[3 + a] = Ia[3 + a] + gy[3 + a] + fl[a];
        }
    }
    if (own) {
#pragma unroll
        for (int r = 0; r < 6; ++r) L.f[d][r] = f[r];
    }
    __syncthreads();

    // ---- inward pass: composite inertias of the arm subtrees (CRBA), bias forces
    if (own) {
        double F[6];
        if (d < 5) {
            double IC[10], fs[6];
#pragma unroll
            for (int r = 0; r < 10; ++r) IC[r] = in[r];
#pragma unroll
            for (int r = 0; r < 6; ++r) fs[r] = f[r];
            const int ub = d >= 3 ? 6 : 13; // subtree of joint d: d..6 (elbow) or d..13
            for (int k = d + 1; k <= ub; ++k) {
#pragma unroll
                for (int r = 0; r < 10; ++r) IC[r] += L.in[k][r];
#pragma unroll
                for (int r = 0; r < 6; ++r) fs[r] += L.f[k][r];
            }
            imul(IC, Sd, F);
            L.M[d][d] = dot6(Sd, F);
#pragma unroll
            for (int j = 0; j < 5; ++j)
                if (j < d) {
                    const double mj = dot6(L.S[j], F);
                    L.M[d][j] = mj;
                    L.M[j][d] = mj;
                }
            L.h[d] = dot6(Sd, fs);
        } else {
            imul(in, Sd, F);
            L.D[d] = dot6(Sd, F);
            L.h[d] = dot6(Sd, f);
            if (d < NC) {
#pragma unroll
                for (int j = 0; j < 5; ++j) L.b[d][j] = (j < npar) ? dot6(L.S[j], F) : 0.0;
            }
        }
    }
    __syncthreads();

    // ---- M^-1: Schur complement of the arrow, inverted per lane (5x5 SPD)
    double row[NC], diag = 1.0, vs = 0.0;
#pragma unroll
    for (int j = 0; j < NC; ++j) row[j] = 0.0;
    if (own) {
        double A[5][5], Pm[5][5];
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) A[i][j] = L.M[i][j];
        for (int k = 5; k < NC; ++k) {
            const double ik = 1.0 / L.D[k];
            double bk[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) bk[j] = L.b[k][j];
#pragma unroll
            for (int i = 0; i < 5; ++i)
#pragma unroll
                for (int j = 0; j < 5; ++j) A[i][j] -= bk[i] * bk[j] * ik;
        }
        // Gauss-Jordan without pivoting (symmetric positive definite)
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) Pm[i][j] = (i == j) ? 1.0 : 0.0;
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            const double ip = 1.0 / A[c][c];
#pragma unroll
            for (int j = 0; j < 5; ++j) { A[c][j] *= ip; Pm[c][j] *= ip; }
#pragma unroll
            for (int r = 0; r < 5; ++r)
                if (r != c) {
                    const double fr = A[r][c];
#pragma unroll
                    for (int j = 0; j < 5; ++j) { A[r][j] -= fr * A[c][j]; Pm[r][j] -= fr * Pm[c][j]; }
                }
        }
        // x = P g, g = e_d (arm) / b_d (arm k-link)
        double gv[5], x[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) gv[j] = d < 5 ? (j == d ? 1.0 : 0.0) : (d < NC ? L.b[d][j] : 0.0);
#pragma unroll
        for (int i = 0; i < 5; ++i) x[i] = dot5(Pm[i], gv);
        if (d < 5) {
#pragma unroll
            for (int j = 0; j < 5; ++j) row[j] = x[j];
#pragma unroll
            for (int k = 5; k < NC; ++k) row[k] = -dot5(L.b[k], x) / L.D[k];
            diag = dot5(gv, x);
        } else if (d < NC) {
            const double iD = 1.0 / L.D[d];
#pragma unroll
            for (int j = 0; j < 5; ++j) row[j] = -x[j] * iD;
#pragma unroll
            for (int k = 5; k < NC; ++k) row[k] = (k == d ? iD : 0.0) + dot5(L.b[k], x) * iD / L.D[k];
            diag = iD + dot5(gv, x) * iD / L.D[d];
        } else {
            diag = 1.0 / L.D[d];
        }
        // free motion qdd = -M^-1 h, predicted velocity (btMultiBody: v* = qd + dt qdd, clamped)
        double qdd = 0.0;
        if (d < NC) {
#pragma unroll
            for (int j = 0; j < NC; ++j) qdd -= row[j] * L.h[j];
        } else {
            qdd = -L.h[d] * diag;
        }
        vs = fmin(fmax(qd + DT * qdd, -P.max_vel), P.max_vel);
    }

    // ---- rows: violated limit (if any) and the joint motor of joint d
    const double lo = d < 5 ? U.lo[d < 5 ? d : 0] : -0.5, hi = d < 5 ? U.hi[d < 5 ? d : 0] : 0.5;
    const double pl = q - lo, pu = hi - q;
    const bool has_lim = own && (pl <= 0.0 || pu <= 0.0);
    const double sl = pl <= 0.0 ? 1.0 : -1.0;
    const double wl = -(pl <= 0.0 ? pl : pu) * P.erp / DT;
    const double kp = d < 5 ? P.kp : 0.0, target = (own && d < 5) ? tgt[(size_t)d * N + e] : 0.0;
    const double imp = d < 5 ? P.motor_imp : P.passive_imp;
    const double wm = kp * (target - q) / DT + vs + P.kd * (0.0 - vs);
    const double dinv = 1.0 / diag;
    double lam_l = 0.0, lam_m = 0.0;
    const bool any_lim = __ballot(has_lim) != 0ull; // wave uniform

    // ---- projected Gauss-Seidel sweeps (rows in Bullet's creation order).
    // The 5 base k-links' rows touch only their own velocity (their rows and
    // columns of M^-1 are zero elsewhere), so their sweeps run on their own
    // lanes first; the joint-coupled rows 0..13 then sweep with broadcasts.
    // Row j's impulse change is computed on every lane from its own row and
    // read from lane j (v_readlane); only lane j keeps its new impulse.
    const double sl_eff = has_lim ? sl : 0.0; // lanes without a violated limit broadcast 0
    if (own && d >= NC) {
        for (int it = 0; it < P.iters; ++it) {
            if (has_lim) {
                const double nl = fmin(fmax(lam_l + (wl - sl * vs) * dinv, 0.0), P.limit_imp);
                vs += diag * ((nl - lam_l) * sl);
                lam_l = nl;
            }
            const double nl = fmin(fmax(lam_m + (wm - vs) * dinv, -imp), imp);
            vs += diag * (nl - lam_m);
            lam_m = nl;
        }
    }
    for (int it = 0; it < P.iters; ++it) {
        if (any_lim) {
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const double nl = fmin(fmax(lam_l + (wl - sl * vs) * dinv, 0.0), P.limit_imp);
                const double dl = (nl - lam_l) * sl_eff;
                lam_l = d == j ? nl : lam_l;
                vs += row[j] * group_bcast(dl, j, upper);
            }
        }
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const double nl = fmin(fmax(lam_m + (wm - vs) * dinv, -imp), imp);
            const double dl = nl - lam_m;
            lam_m = d == j ? nl : lam_m;
            vs += row[j] * group_bcast(dl, j, upper);
        }
    }

    // ---- semi-implicit Euler
    if (own) {
        q += DT * vs;
        S.mb_q[(size_t)d * N + e] = q;
        S.mb_qd[(size_t)d * N + e] = vs;
        if (d < 5) S.phys_q[(size_t)d * N + e] = q;
    }
    if (work && d == 0 && clear_flag) flag[e] = 0;
}

} // namespace

namespace exo {
hipError_t launch_exo_multibody(const Dev &S, const Urdf &U, const MbModel &M, const double *tgt, uint8_t *flag,
                                int clear_flag, hipStream_t stream) {
    hipLaunchKernelGGL(exo_multibody_kernel, dim3((S.N + MB_ENVS - 1) / MB_ENVS), dim3(MB_G * MB_ENVS), 0, stream,
                       S, U, M, tgt, flag, clear_flag);
    return hipGetLastError();
}
} // namespace exo
