// exo_model.h -- constants and device math of the exoskeleton environment
// (gfx950).  Everything here is fp64: the reference computes in numpy float64
// and only casts the observation to float32 (Exoskeleton_env.py:568).
//
// Citations are path:line into the reference repository.
#pragma once
#ifdef EXO_HOST_ONLY // host-side unit tests compile this header with gcc (tests/native)
#define __host__
#define __device__
#define __forceinline__ inline
#else
#include <hip/hip_runtime.h>
#endif
#include "philox.h"
#include <math.h>
#include <stdint.h>

namespace exo {

constexpr int OBS = 80, ACT = 7, INFO = 40;
constexpr int MAX_L = 512;             // longest supported motion (reference: 347 samples)
constexpr int T_PER_LANE = MAX_L / 64; // reset kernel: tremor samples per lane
constexpr double DT = 1.0 / 40.0;      // Exoskeleton_env.py:59
constexpr double PI = 3.141592653589793;

// ---------------------------------------------------------------------------
// Anatomical matrices, Utilities/differential_eq_matrices.py:41-69.  Domain
// randomisation multiplies entries by (1 + noise) (domain_randomization_
// anatomical_matrices.py:24), so their zero pattern is invariant:
//   D, S: blocks {0,1,2,3} (with D/S[1][3] = D/S[2][3] = 0) and {4,5,6}
//   I   : blocks {0,3,6} and {1,2,4,5}
// The device keeps only the 21 structural non-zeros of D and S and the two
// diagonal blocks of I^-1 (9 + 16 values).
// ---------------------------------------------------------------------------
constexpr double I0[49] = {0.269, 0, 0, 0.076, 0, 0, -0.014, 0, 0.196, 0.083, 0, -0.002, 0.009, 0,
                           0, 0.083, 0.079, 0, 0, 0.011, 0, 0.076, 0, 0, 0.076, 0, 0, -0.012,
                           0, -0.002, 0, 0, 0.002, 0, 0, 0, 0.009, 0.011, 0, 0, 0.003, 0,
                           -0.014, 0, 0, -0.012, 0, 0, 0.003};
constexpr double D0[49] = {0.756, 0.184, 0.020, 0.187, 0, 0, 0, 0.184, 0.383, 0.267, 0, 0, 0, 0,
                           0.020, 0.267, 0.524, 0, 0, 0, 0, 0.187, 0, 0, 0.607, 0, 0, 0,
                           0, 0, 0, 0, 0.021, 0.001, 0.008, 0, 0, 0, 0, 0.001, 0.028, -0.003,
                           0, 0, 0, 0, 0.008, -0.003, 0.082};
constexpr double S0[49] = {10.80, 2.626, 0.279, 2.670, 0, 0, 0, 2.626, 5.468, 3.821, 0, 0, 0, 0,
                           0.279, 3.821, 7.486, 0, 0, 0, 0, 2.670, 0, 0, 8.670, 0, 0, 0,
                           0, 0, 0, 0, 0.756, 0.018, 0.291, 0, 0, 0, 0, 0.018, 0.992, -0.099,
                           0, 0, 0, 0, 0.291, -0.099, 2.920};
constexpr int NNZ = 21;
// (row, col) of the structural non-zeros of D and S, row-major
constexpr int NZ_R[NNZ] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6};
constexpr int NZ_C[NNZ] = {0, 1, 2, 3, 0, 1, 2, 0, 1, 2, 0, 3, 4, 5, 6, 4, 5, 6, 4, 5, 6};
// D and S are exactly symmetric after domain randomisation (the noise is
// symmetrised before it multiplies the symmetric matrix, :19-24), so only the
// 14 upper-triangle non-zeros are stored; NZ_U maps non-zero k to them.
constexpr int NSYM = 14;
constexpr int NZ_U[NNZ] = {0, 1, 2, 3, 1, 4, 5, 2, 5, 6, 3, 7, 8, 9, 10, 9, 11, 12, 10, 12, 13};
constexpr int SYM_R[NSYM] = {0, 0, 0, 0, 1, 1, 2, 3, 4, 4, 4, 5, 5, 6};
constexpr int SYM_C[NSYM] = {0, 1, 2, 3, 1, 2, 2, 3, 4, 5, 6, 5, 6, 6};
// I^-1 is stored as the upper triangles of its two diagonal blocks (6 + 10).
constexpr int B1[3] = {0, 3, 6};
constexpr int B2[4] = {1, 2, 4, 5};
constexpr int B1U[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
constexpr int B2U[4][4] = {{6, 7, 8, 9}, {7, 10, 11, 12}, {8, 11, 13, 14}, {9, 12, 14, 15}};
constexpr int NINV = 16;

// Butcher tableau of scipy RK45 (scipy/integrate/_ivp/rk.py class RK45)
constexpr double RK_A[6][5] = {
    {0, 0, 0, 0, 0},
    {1.0 / 5, 0, 0, 0, 0},
    {3.0 / 40, 9.0 / 40, 0, 0, 0},
    {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
    {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
    {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
constexpr double RK_B[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
constexpr double RK_E[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525, 1.0 / 40};

// ---------------------------------------------------------------------------
// URDF (Simulation/exo_v3.urdf).  Joint order == pybullet link index.
// Revolute joints 0..4: shoulder z, shoulder y, shoulder x, elbow y, elbow z.
// ---------------------------------------------------------------------------
constexpr int NJ = 19;
// link handles read by get_actuator_positions, in read order
// (Exoskeleton_sim_pybullet.py:48-61, :129-142): act11, act12, act21, ... act72
constexpr int K_LINK[14] = {9, 5, 12, 6, 15, 8, 17, 11, 14, 7, 18, 13, 16, 10};

struct Urdf {           // filled on the host (exo_create) and passed by value
    double Ro[5][9];    // origin rotation (rpy) of the 5 revolute joints
    double xyz[NJ][3];  // joint origin translations
    double kbase[5][3]; // world positions of the base-fixed k-links (joints 14..18)
    double com3[3];     // auxlink3 CoM in its frame (exo_v3.urdf:84)
    double lo[5], hi[5];// revolute limits (exo_v3.urdf:17,37,57,77,97)
    double kz[14][3];   // prismatic joints 5..18: axis (0 0 1) of the joint frame in the parent frame
    // row-parallel step (exo_step_rp.hip): lane r's actuator j = min(r, 6) anchor
    // rows, [0..2] U.xyz (links 9, 12) or U.kbase (the base-fixed links) of
    // K_LINK[2j], [3..5] U.xyz of K_LINK[2j + 1] -- read per lane with the
    // kernel-start loads instead of a runtime index per link
    double anc[8][6];
    // and its joint-target limits (finish_solve): lane r < 5 drives joint
    // (r == 0 ? 1 : r == 1 ? 2 : r == 2 ? 0 : r): {lo, hi} of the joint, then
    // check_movement_boundaries' degree bounds (joints 0..3; 0 for the rest)
    double lim[8][4];
};

// Multibody physics mode (csrc/exo_multibody.hip): <inertial> data of the arm
// links (exo_v3.urdf:23-27, 43-47, 63-67, 83-87, 103-107; the k-links have mass
// 1 and unit inertia) and the solver constants (include/exo_amd.h exo_mb_params).
struct MbModel {
    double m[5], com[5][3], Rin[5][9], Id[5][3];
    double g, kp, kd, motor_imp, passive_imp, limit_imp, erp, lin_damp, ang_damp, max_vel;
    int iters;
};

// ---------------------------------------------------------------------------
// Device state, structure of arrays, env index fastest.
// ---------------------------------------------------------------------------
enum CfgIdx { C_AMP0, C_AMP1, C_H1A, C_H1B, C_H2A, C_H2B, C_MAXS0, C_MAXE0, C_SHIFT, C_ACTR, C_MATF,
              C_MAXREW, C_NAXES, C_COUNT };

struct Dev {
    int N, n_motions, Lmax;
    const int32_t *motion, *L, *seq; // seq: 7-bit mask
    const double *cfg;               // [C_COUNT][N]
    const double *imu;               // [n_motions][5][Lmax] degrees
    double *tremor;                  // [Lmax][7][N]
    double *iinv;                    // [16][N] upper triangles of the I^-1 blocks
    double *dnz, *snz;               // [14][N] upper-triangle non-zeros of D, S
    double *shift;                   // [42][N]
    double *maxSE;                   // [2][N]
    uint32_t *episode;               // [N]
    int32_t *counts;                 // [N]
    double *phys_q;                  // [5][N]
    double *ref;                     // [6][N] cached reference link CoMs (shoulder xyz, elbow xyz)
    float *posv;                     // [21][N] position vectors of the previous read
    double *prev_a, *prev2_a;        // [7][N]
    int32_t *err;                    // [1] sticky error bits
    int32_t *viol;                   // [N] steps with a joint-range violation
    // multibody physics mode only (nullptr in the idealised mode):
    double *mb_q, *mb_qd;            // [19][N] joint positions / velocities (rows 0..4 mirror phys_q)
    double *mb_tgt;                  // [5][N] POSITION_CONTROL targets written by the step kernel (rad)
    uint8_t *mb_flag;                // [N] 1 = the step kernel stepped the env, the physics kernel follows
    // tremor model of the reset (exo_set_tremor_model): per-axis maxima and sign mode
    double tjmax[7];                 // joint_max_values (generate_parkinson_tremor.py:59)
    int32_t tsign;                   // EXO_TREMOR_SIGN_*: per sample (:70), one per axis, none
    // budgeted step (exo_set_step_budget; row-parallel kernels): at most `budget`
    // RK45 step attempts per solve and launch, an unfinished solve's state carried
    // to the next launch; an env with a pending solve starts no new step
    int32_t budget;                  // 0 = unlimited (pend / rk unused)
    uint8_t *pend;                   // [N] bit 0: the actuated solve pending, bit 1: the tremor-only solve
    double *rk;                      // [RK_FIELDS][N] carried solver state (exo_step_rp.hip rk_field)
};
constexpr int RK_FIELDS = 72;       // 16 lanes x (q, v, a0, T) + 2 groups x (t, h_abs, attempts, flags)

__host__ __device__ inline void matmul3(const double *A, const double *B, double *C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

// R * Rz(q): rotate the frame about its own z axis
__host__ __device__ inline void mul_rz(const double *R, double c, double s, double *O) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        O[i * 3 + 0] = R[i * 3] * c + R[i * 3 + 1] * s;
        O[i * 3 + 1] = -R[i * 3] * s + R[i * 3 + 1] * c;
        O[i * 3 + 2] = R[i * 3 + 2];
    }
}

__host__ __device__ inline void xform(const double *R, const double *p, const double *v, double *o) {
#pragma unroll
    for (int a = 0; a < 3; ++a) o[a] = p[a] + R[a * 3] * v[0] + R[a * 3 + 1] * v[1] + R[a * 3 + 2] * v[2];
}

// Multibody mode: a k-link (joint 5..18) slides qk along its joint axis,
// which is kz in the parent frame R (R4 for k12/k22, R2 for the humerus
// k-links, the world for the base k-links).
__host__ __device__ __forceinline__ void slide(const Urdf &U, int link, const double *R2, const double *R4, double qk,
                                               double *o) {
    const double *z = U.kz[link - 5];
    const double *R = (link == 5 || link == 6) ? R4 : R2;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double ax = link >= 14 ? z[a] : R[a * 3] * z[0] + R[a * 3 + 1] * z[1] + R[a * 3 + 2] * z[2];
        o[a] += qk * ax;
    }
}

// Forward kinematics of the link CoMs that getLinkState(...)[0] returns
// (Exoskeleton_sim_pybullet.py:129-142, 194-195, 348-349) for revolute
// positions q[5]; prismatic actuator anchors are held at 0
// unless qp (positions of joints 5..18, multibody mode) is given.
// act[k] = CoM of link K_LINK[k] (without the dummy shift); ref = links 0, 3.
__host__ __device__ inline void link_coms(const Urdf &U, const double *q, double act[14][3], double ref[6],
                                          const double *qp = nullptr) {
    double Rt[9], R0[9], R1[9], R2[9], R3[9], R4[9];
    double p0[3] = {U.xyz[0][0], U.xyz[0][1], U.xyz[0][2] + 0.1}; // base at [0,0,0.1] (sim:18)
    double s, c;
    sincos(q[0], &s, &c); mul_rz(U.Ro[0], c, s, R0);               // auxlink1
    matmul3(R0, U.Ro[1], Rt); sincos(q[1], &s, &c); mul_rz(Rt, c, s, R1); // auxlink2 (origin offset 0)
    matmul3(R1, U.Ro[2], Rt); sincos(q[2], &s, &c); mul_rz(Rt, c, s, R2); // humerus
    double p3[3];
    xform(R2, p0, U.xyz[3], p3);
    matmul3(R2, U.Ro[3], Rt); sincos(q[3], &s, &c); mul_rz(Rt, c, s, R3); // auxlink3
    matmul3(R3, U.Ro[4], Rt); sincos(q[4], &s, &c); mul_rz(Rt, c, s, R4); // alkar (origin offset 0)
    ref[0] = p0[0]; ref[1] = p0[1]; ref[2] = p0[2];
    xform(R3, p3, U.com3, &ref[3]);
#pragma unroll
    for (int k = 0; k < 14; ++k) {
        const int j = K_LINK[k];
        if (j == 5 || j == 6) xform(R4, p3, U.xyz[j], act[k]);             // k12, k22 on the forearm
        else if (j >= 14) { act[k][0] = U.kbase[j - 14][0]; act[k][1] = U.kbase[j - 14][1]; act[k][2] = U.kbase[j - 14][2]; }
        else xform(R2, p0, U.xyz[j], act[k]);                               // k11..k72 on the humerus
        if (qp) slide(U, j, R2, R4, qp[j - 5], act[k]);
    }
}

// cos(atan2(y, x)) without the transcendental pair: x / hypot(x, y), with the
// atan2 conventions for a zero radius (cos(+-0) = 1, cos(+-pi) = -1).
__host__ __device__ inline double cos_atan2(double y, double x) {
    double r = sqrt(x * x + y * y);
    return (r == 0.0) ? (signbit(x) ? -1.0 : 1.0) : x / r;
}

// ---------------------------------------------------------------------------
// Joint ODE I q'' + D q' + K q = T, y0 = 0, solved over [0, dt] with scipy's
// RK45 step control (Utilities/calculate_joint_angles.py:5-22).
// ---------------------------------------------------------------------------
struct OdeM {
    double ii[NINV];
    double dn[NSYM], sn[NSYM];
};

// acceleration part of dqdt (calculate_joint_angles.py:12): I^-1 (T - D v - K q)
__host__ __device__ __forceinline__ void ode_acc(const OdeM &M, const double *T, const double *q, const double *v, double *a) {
    double r[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        double dq = 0.0, kq = 0.0;
#pragma unroll
        for (int k = 0; k < NNZ; ++k)
            if (NZ_R[k] == i) { dq += M.dn[NZ_U[k]] * v[NZ_C[k]]; kq += M.sn[NZ_U[k]] * q[NZ_C[k]]; }
        r[i] = T[i] - dq - kq;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
        a[B1[i]] = M.ii[B1U[i][0]] * r[B1[0]] + M.ii[B1U[i][1]] * r[B1[1]] + M.ii[B1U[i][2]] * r[B1[2]];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        a[B2[i]] = M.ii[B2U[i][0]] * r[B2[0]] + M.ii[B2U[i][1]] * r[B2[1]] + M.ii[B2U[i][2]] * r[B2[2]] +
                   M.ii[B2U[i][3]] * r[B2[3]];
}

// Second-order form of the RK45 tableau.  With y = [q, v] and f = [v, a(q, v)]
// the velocity half of every stage derivative is the stage velocity itself,
// so a stage needs only the earlier ACCELERATIONS:
//   v_s = v + h sum_l A[s][l] a_l,   q_s = q + h C[s] v + h^2 sum_l AA[s][l] a_l,
// with AA = A.A.  y_new and the error estimate follow the same way (the 7th
// "stage" of the error estimate is y_new, whose coefficients are B).  This
// stores 7 x 7 accelerations instead of 7 x 14 derivatives; it is the same
// method and the same step-size control as scipy's RK45, rounded differently
// (differences ~1e-16 relative per operation, see tests).
struct RK2 {
    double C[6];
    double AA[6][5];
    double BB[6]; // sum_j B[j] A[j][l]
    double EE[7]; // sum_j E[j] A7[j][l], A7 = A with row 6 := B
    constexpr RK2() : C{}, AA{}, BB{}, EE{} {
        for (int s = 0; s < 6; ++s) {
            double cs = 0;
            for (int j = 0; j < 5; ++j) cs += RK_A[s][j];
            C[s] = cs;
            for (int l = 0; l < 5; ++l) {
                double acc = 0;
                for (int j = 0; j < 6; ++j) acc += RK_A[s][j < 5 ? j : 0] * (j < 5 ? RK_A[j][l] : 0.0);
                AA[s][l] = acc;
            }
        }
        for (int l = 0; l < 6; ++l) {
            double acc = 0;
            for (int j = 0; j < 6; ++j) acc += RK_B[j] * (l < 5 ? RK_A[j][l] : 0.0);
            BB[l] = acc;
        }
        for (int l = 0; l < 7; ++l) {
            double acc = 0;
            for (int j = 0; j < 7; ++j) {
                double ajl = 0;
                if (j < 6) ajl = (l < 5) ? RK_A[j][l] : 0.0;
                else ajl = (l < 6) ? RK_B[l] : 0.0;
                acc += RK_E[j] * ajl;
            }
            EE[l] = acc;
        }
    }
};
constexpr RK2 RKN{};

__host__ __device__ __forceinline__ double rms14(const double *x) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 14; ++i) s += x[i] * x[i];
    return sqrt(s) / 3.7416573867739413; // np.linalg.norm(x) / 14 ** 0.5 (scipy common.py norm)
}

// x^(-1/5) for the step-size controller (scipy rk.py `error_norm **
// error_exponent`, common.py select_initial_step): the library pow(double) is a
// ~100-instruction dependent chain (extended-precision log and exp), paid once
// per step attempt on the solve's critical path.  Here: a float seed from the
// hardware v_log_f32 / v_exp_f32 (relative error ~3e-7), then one
// second-order correction in fp64: with e = 1 - x*y^5,
// x^(-1/5) = y*(1 - e)^(-1/5) = y*(1 + e/5 + 3e^2/25 + O(e^3)); |e| < 2e-6,
// so the truncation is < 1e-18 (checked against long-double powers on 4e5
// arguments in [1e-30, 1e30]: within 1 ulp of x^-0.2, as numpy's pow is).
// Outside [1e-30, 1e30] (float range), for NaN and in host builds the library
// pow runs.
#ifndef EXO_FASTPOW
#define EXO_FASTPOW 1
#endif
__host__ __device__ __forceinline__ double pow_m5th(double x) {
#if EXO_FASTPOW && defined(__HIP_DEVICE_COMPILE__)
    if (!(x > 1e-30 && x < 1e30)) return pow(x, -0.2);
    const float l2 = __builtin_amdgcn_logf((float)x); // log2
    const float yf = __builtin_amdgcn_exp2f(-0.2f * l2);
    const double y = (double)yf, y2 = y * y, y5 = y2 * y2 * y;
    const double e = fma(-x, y5, 1.0);
    const double r = fma(y * e, fma(e, 0.12, 0.2), y);
    // the double -0.2 is -(1/5 + 1.11e-17): x^-0.2 = x^(-1/5) * (1 - 1.11e-17 ln x)
    // (up to 7 ulp at x = 1e30 without it); within 1 ulp of pow(x, -0.2) after it
    return fma(r, -1.1102230246251565e-17 * 0.6931471805599453 * (double)l2, r);
#else
    return pow(x, -0.2);
#endif
}

// Returns false if scipy would have failed (step size underflow) or the
// attempt guard tripped; q_out is then NaN.
__host__ __device__ inline bool rk45_solve(const OdeM &M, const double *T, double *q_out) {
    const double rtol = 1e-3, atol = 1e-6, tb = DT;
    double q[7], v[7], a0[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) { q[i] = 0.0; v[i] = 0.0; }
    ode_acc(M, T, q, v, a0);
    // select_initial_step (scipy common.py) with y0 = 0: d0 = 0 -> h0 = 1e-6,
    // f0 = [0, a0], y1 = h0 f0 = [0, h0 a0]
    double h_abs;
    {
        double tmp[14], y1v[7], a1[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) { tmp[i] = 0.0; tmp[7 + i] = a0[i] / atol; }
        const double d1 = rms14(tmp);
        const double h0 = 1e-6;
#pragma unroll
        for (int i = 0; i < 7; ++i) y1v[i] = h0 * a0[i];
        ode_acc(M, T, q, y1v, a1);
#pragma unroll
        for (int i = 0; i < 7; ++i) { tmp[i] = (y1v[i] - 0.0) / atol; tmp[7 + i] = (a1[i] - a0[i]) / atol; }
        const double d2 = rms14(tmp) / h0;
        // scipy's (0.01 / max(d1, d2)) ** (1 / (order + 1)) with the library pow:
        // once per solve, and 1 / pow_m5th would add a rounding (<= 3 ulp)
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
        h_abs = fmin(fmin(100 * h0, h1), tb);
    }
    double t = 0.0;
    int guard = 0;
    bool ok = true;
    while (t != tb && ok) {
        const double min_step = 10 * fabs(nextafter(t, INFINITY) - t);
        if (h_abs < min_step) h_abs = min_step;
        bool rejected = false, accepted = false;
        while (!accepted) {
            if (h_abs < min_step || ++guard > 4096) { ok = false; break; }
            double t_new = t + h_abs;
            if (t_new - tb > 0) t_new = tb;
            const double h = t_new - t, h2 = h * h;
            h_abs = fabs(h);
            double A[7][7], qs[7], vs[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) A[0][i] = a0[i];
#pragma unroll
            for (int st = 1; st < 6; ++st) {
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    double dv = 0.0, dq = 0.0;
#pragma unroll
                    for (int l = 0; l < st; ++l) { dv += A[l][i] * RK_A[st][l]; dq += A[l][i] * RKN.AA[st][l]; }
                    vs[i] = v[i] + dv * h;
                    qs[i] = q[i] + RKN.C[st] * h * v[i] + dq * h2;
                }
                ode_acc(M, T, qs, vs, A[st]);
            }
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                double dv = A[0][i] * RK_B[0], dq = A[0][i] * RKN.BB[0] + A[1][i] * RKN.BB[1];
#pragma unroll
                for (int l = 2; l < 5; ++l) { dv += A[l][i] * RK_B[l]; dq += A[l][i] * RKN.BB[l]; }
                dv += A[5][i] * RK_B[5]; // B[1] = 0; BB[5] = 0
                vs[i] = v[i] + h * dv; // y_new
                qs[i] = q[i] + h * v[i] + dq * h2;
            }
            ode_acc(M, T, qs, vs, A[6]);
            double e[14];
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                double ev = A[0][i] * RK_E[0], eq = A[0][i] * RKN.EE[0] + A[1][i] * RKN.EE[1];
#pragma unroll
                for (int l = 2; l < 6; ++l) { ev += A[l][i] * RK_E[l]; eq += A[l][i] * RKN.EE[l]; }
                ev += A[6][i] * RK_E[6]; // E[1] = 0; EE[6] = 0
                e[i] = eq * h2 / (atol + fmax(fabs(q[i]), fabs(qs[i])) * rtol);
                e[7 + i] = ev * h / (atol + fmax(fabs(v[i]), fabs(vs[i])) * rtol);
            }
            const double en = rms14(e);
            if (en < 1) {
                double factor = (en == 0) ? 10.0 : fmin(10.0, 0.9 * pow_m5th(en));
                if (rejected) factor = fmin(1.0, factor);
                h_abs *= factor;
                t = t_new;
#pragma unroll
                for (int i = 0; i < 7; ++i) { q[i] = qs[i]; v[i] = vs[i]; a0[i] = A[6][i]; }
                accepted = true;
            } else {
                h_abs *= fmax(0.2, 0.9 * pow_m5th(en));
                rejected = true;
            }
        }
    }
#pragma unroll
    // scipy's solve_ivp on failure (rk.py: step size below the spacing of t):
    // status -1 and sol.y up to the last accepted step, whose q the reference
    // takes (calculate_joint_angles.py:20); `ok` flags it (sticky error bit)
    for (int i = 0; i < 7; ++i) q_out[i] = q[i];
    return ok;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based draws for the reset path.
// ---------------------------------------------------------------------------

// Unit uniform number p of the draw stream of (env, episode): 53-bit, [0, 1).
__host__ __device__ inline double philox_u01(uint64_t seed, uint32_t env, uint32_t episode, uint32_t p) {
    uint32_t c[4] = {p >> 1, episode, env, 0x45584F31u};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t a = (p & 1) ? c[2] : c[0], b = (p & 1) ? c[3] : c[1];
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

#ifndef EXO_HOST_ONLY
// row-parallel step (csrc/exo_step_rp.hip): 16 lanes per env, for small env counts
hipError_t launch_exo_step_rp(const Dev &S, const Urdf &U, const float *act, float *obs, float *rew, uint8_t *done,
                              float *info, const uint8_t *active, hipStream_t stream, bool shared = false,
                              const float *obs_cur = nullptr);
// multibody stepSimulation (csrc/exo_multibody.hip) of the envs with flag[e] != 0
// (flag NULL = all); tgt [5][N]; clear_flag: zero the flags afterwards
struct MbModel;
hipError_t launch_exo_multibody(const Dev &S, const Urdf &U, const MbModel &M, const double *tgt, uint8_t *flag,
                                int clear_flag, hipStream_t stream);
#endif

// URDF numbers, Simulation/exo_v3.urdf (kept literally: 3.141593 is not pi)
constexpr double J_XYZ[NJ][3] = {
    {0.010000, -0.475000, 1.200000}, {0, 0, 0}, {0, 0, 0}, {0.480000, 0, 0}, {0, 0, -0.000000},
    {0.080234, -0.000000, -0.220137}, {-0.069766, -0.000000, -0.220137},
    {0.300000, 0.000000, 0.075000}, {0.200000, 0.000000, 0.075000}, {0.250000, 0.000000, 0.075000},
    {0.300000, 0.000000, -0.075000}, {0.200000, 0.000000, -0.075000}, {0.250000, 0.000000, -0.075000},
    {0.250000, -0.075000, 0.000000},
    {0.150000, -0.275000, 0.900000}, {0.150000, -0.275000, 1.100000}, {-0.150000, -0.275000, 0.900000},
    {-0.150000, -0.275000, 1.100000}, {0.010000, -0.475000, 1.290000}};
constexpr double J_RPY[5][3] = {{-3.141593, 3.141593, -3.141593}, {-1.570796, 3.141593, -3.141593},
                                {1.570796, 3.141593, 1.570796}, {1.570796, -1.570796, 0.000000},
                                {1.570796, 3.141593, -3.141593}};

// origin rpy of the prismatic joints 5..18 (exo_v3.urdf:120, 139, 158, ...)
constexpr double J_RPY_K[3][3] = {{3.141593, 3.089233, 3.141593},   // k12, k22 (on alkar)
                                  {-0.000000, 4.590216, -0.000000}, // k52 .. k62 (on the humerus)
                                  {-3.141593, 3.141593, -3.141593}};// k51 .. k61 (on the base)
inline int rpy_k_row(int joint) { return joint <= 6 ? 0 : (joint <= 13 ? 1 : 2); }

// <inertial> of the arm links 0..4 (exo_v3.urdf:23-27, 43-47, 63-67, 83-87, 103-107)
constexpr double L_MASS[5] = {0.20000000298023, 0.20000000298023, 2.0, 0.11219999939203, 1.1219999790192};
constexpr double L_COM[5][3] = {{0, 0, 0}, {0, 0, 0}, {0.230000, 0, 0}, {0, 0.500000, -0.000000},
                                {0.005234, 0, -0.245137}};
constexpr double L_IRPY[5][3] = {{-3.141593, 3.141593, -3.141593}, {1.570796, 3.141593, -3.141593},
                                 {-0.000000, -1.570796, 0.000000}, {1.570796, 3.141593, -3.141593},
                                 {-3.141593, 3.141593, -3.141593}};
constexpr double L_IDIAG[5][3] = {{0.00058960002794266, 0.00058960002794266, 0.0001124999968335},
                                  {0.00058960002794266, 0.00058960002794266, 0.0001124999968335},
                                  {0.05895833298564, 0.05895833298564, 0.011250000447035},
                                  {0.00039539280435958, 0.00039539280435958, 3.5410318407441e-05},
                                  {0.039536823770183, 0.039536823770183, 0.0035406111384836}};

// URDF rpy -> rotation Rz(yaw) Ry(pitch) Rx(roll)
inline void rpy_to_R(const double *r, double *R) {
    const double cr = cos(r[0]), sr = sin(r[0]), cp = cos(r[1]), sp = sin(r[1]), cy = cos(r[2]), sy = sin(r[2]);
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

// Host-side precomputation of the multibody model's constant part.
inline void build_mb_model(MbModel &M) {
    for (int i = 0; i < 5; ++i) {
        M.m[i] = L_MASS[i];
        rpy_to_R(L_IRPY[i], M.Rin[i]);
        for (int a = 0; a < 3; ++a) { M.com[i][a] = L_COM[i][a]; M.Id[i][a] = L_IDIAG[i][a]; }
    }
}

// Host-side precomputation of the constant part of the kinematic tree.
inline void build_urdf(Urdf &U) {
    for (int j = 0; j < 5; ++j) rpy_to_R(J_RPY[j], U.Ro[j]);
    for (int j = 5; j < NJ; ++j) {
        double R[9];
        rpy_to_R(J_RPY_K[rpy_k_row(j)], R);
        U.kz[j - 5][0] = R[2]; U.kz[j - 5][1] = R[5]; U.kz[j - 5][2] = R[8];
    }
    for (int j = 0; j < NJ; ++j)
        for (int a = 0; a < 3; ++a) U.xyz[j][a] = J_XYZ[j][a];
    for (int k = 0; k < 5; ++k)
        for (int a = 0; a < 3; ++a) U.kbase[k][a] = J_XYZ[14 + k][a] + (a == 2 ? 0.1 : 0.0);
    for (int r = 0; r < 8; ++r) {
        const int j = r < 7 ? r : 6, l1 = K_LINK[2 * j], l2 = K_LINK[2 * j + 1];
        for (int a = 0; a < 3; ++a) {
            U.anc[r][a] = l1 >= 14 ? U.kbase[l1 - 14][a] : U.xyz[l1][a];
            U.anc[r][3 + a] = U.xyz[l2][a];
        }
    }
    U.com3[0] = 0.0; U.com3[1] = 0.5; U.com3[2] = -0.0;
    const double lo[5] = {-1.3962633609772, -0.69813168048859, -2.6441738605499, -0.034906584769487, -1.5184364318848};
    const double hi[5] = {1.3962633609772, 2.8187066316605, 0.78539800643921, 2.6179938726127, 1.3962633609772};
    for (int j = 0; j < 5; ++j) { U.lo[j] = lo[j]; U.hi[j] = hi[j]; }
    const double blo[4] = {-80, -40, -151.5, -10}, bhi[4] = {80, 160.5, 33.5, 150}; // Exoskeleton_env.py:594-605
    for (int r = 0; r < 8; ++r) {
        const int jt = (r == 0) ? 1 : (r == 1) ? 2 : (r == 2) ? 0 : r;
        U.lim[r][0] = jt < 5 ? U.lo[jt] : 0.0;
        U.lim[r][1] = jt < 5 ? U.hi[jt] : 0.0;
        U.lim[r][2] = jt < 4 ? blo[jt] : 0.0;
        U.lim[r][3] = jt < 4 ? bhi[jt] : 0.0;
    }
}

} // namespace exo
