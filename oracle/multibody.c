/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see exo_oracle.c).
 *
 * Multibody ("fidelity") physics of the exoskeleton URDF for the stepSimulation
 * call of Environment/Exoskeleton_env.py:433: a plain-C, fp64, dense,
 * deliberately generic restatement that checks the HIP kernel
 * (csrc/exo_multibody.hip), which uses a structured (arrow) factorisation
 * instead.  SURVEY.md 8(f) row 2.
 *
 * Model (Bullet's btMultiBody pipeline; the constants are
 * Bullet knowledge and UNVERIFIED -- pybullet 3.2.5 is not installed, so this
 * mode is "parity unpinned" against Bullet; it is pinned against the
 * idealised model it must reduce to when the solver converges, and against
 * its own invariants):
 *   1. forward dynamics with the Articulated-Body Algorithm (Featherstone,
 *      world-frame spatial algebra), gravity -9.81 z (Exoskeleton_env.py:116),
 *      Bullet's link damping (linear/angular, k1 = k2) and the gyroscopic term;
 *      v* = qd + dt qdd, |v*| <= max coordinate velocity;
 *   2. a joint-space sequential-impulse (projected Gauss-Seidel) solve over
 *      the rows {violated joint limits (creation order: joints 0..18), joint
 *      motors 0..18}:
 *        motor row j : J = e_j, target kp (q*_j - q_j)/dt + v*_j + kd (0 - v*_j),
 *                      |impulse| <= maxImpulse.  Revolute joints 0..4 carry the
 *                      POSITION_CONTROL targets of sim:109-117 (kp 0.1, kd 1,
 *                      force 1e5 -> 1e5 dt); prismatic joints the default
 *                      velocity motors (kp 0, kd 1, maxImpulse 1);
 *        limit row   : created when q_j has crossed a URDF limit
 *                      (exo_v3.urdf:17,37,57,77,97; +-0.5 for the prismatic
 *                      joints), J = +-e_j, target -erp * pen / dt, impulse in
 *                      [0, limit impulse];
 *      every row uses the inverse joint-space inertia M^-1 (Bullet:
 *      calcAccelerationDeltasMultiDof), `iters` sweeps;
 *   3. semi-implicit Euler: q += dt v, qd = v.
 * The mass matrix is built with the Composite-Rigid-Body Algorithm and
 * inverted densely; the Recursive Newton-Euler Algorithm is provided so the
 * tests can check M qdd_ABA + h_RNEA = tau.
 *
 * Citations are path:line into the reference repository.
 */
#include <math.h>
#include <string.h>

#include "multibody.h"

#define NL 19

/* Simulation/exo_v3.urdf, joints in file order == pybullet link index */
static const int PAR[NL] = {-1, 0, 1, 2, 3, 4, 4, 2, 2, 2, 2, 2, 2, 2, -1, -1, -1, -1, -1};
static const int REV[NL] = {1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static const double XYZ[NL][3] = {
    {0.010000, -0.475000, 1.200000}, {0, 0, 0}, {0, 0, 0}, {0.480000, 0, 0}, {0, 0, -0.000000},
    {0.080234, -0.000000, -0.220137}, {-0.069766, -0.000000, -0.220137},
    {0.300000, 0.000000, 0.075000}, {0.200000, 0.000000, 0.075000}, {0.250000, 0.000000, 0.075000},
    {0.300000, 0.000000, -0.075000}, {0.200000, 0.000000, -0.075000}, {0.250000, 0.000000, -0.075000},
    {0.250000, -0.075000, 0.000000},
    {0.150000, -0.275000, 0.900000}, {0.150000, -0.275000, 1.100000}, {-0.150000, -0.275000, 0.900000},
    {-0.150000, -0.275000, 1.100000}, {0.010000, -0.475000, 1.290000}};
static const double RPY[NL][3] = {
    {-3.141593, 3.141593, -3.141593}, {-1.570796, 3.141593, -3.141593}, {1.570796, 3.141593, 1.570796},
    {1.570796, -1.570796, 0.000000}, {1.570796, 3.141593, -3.141593},
    {3.141593, 3.089233, 3.141593}, {3.141593, 3.089233, 3.141593},
    {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000},
    {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000},
    {-0.000000, 4.590216, -0.000000},
    {-3.141593, 3.141593, -3.141593}, {-3.141593, 3.141593, -3.141593}, {-3.141593, 3.141593, -3.141593},
    {-3.141593, 3.141593, -3.141593}, {-3.141593, 3.141593, -3.141593}};
/* <inertial> blocks: exo_v3.urdf:23-27, 43-47, 63-67, 83-87, 103-107; the k-links
 * (:129-132 ...) have mass 1, unit inertia and no inertial origin */
static const double MASS5[5] = {0.20000000298023, 0.20000000298023, 2.0, 0.11219999939203, 1.1219999790192};
static const double COM5[5][3] = {{0, 0, 0}, {0, 0, 0}, {0.230000, 0, 0}, {0, 0.500000, -0.000000},
                                  {0.005234, 0, -0.245137}};
static const double IRPY5[5][3] = {{-3.141593, 3.141593, -3.141593}, {1.570796, 3.141593, -3.141593},
                                   {-0.000000, -1.570796, 0.000000}, {1.570796, 3.141593, -3.141593},
                                   {-3.141593, 3.141593, -3.141593}};
static const double IDIAG5[5][3] = {{0.00058960002794266, 0.00058960002794266, 0.0001124999968335},
                                    {0.00058960002794266, 0.00058960002794266, 0.0001124999968335},
                                    {0.05895833298564, 0.05895833298564, 0.011250000447035},
                                    {0.00039539280435958, 0.00039539280435958, 3.5410318407441e-05},
                                    {0.039536823770183, 0.039536823770183, 0.0035406111384836}};
static const double LO5[5] = {-1.3962633609772, -0.69813168048859, -2.6441738605499, -0.034906584769487,
                              -1.5184364318848};
static const double HI5[5] = {1.3962633609772, 2.8187066316605, 0.78539800643921, 2.6179938726127,
                              1.3962633609772};

void oracle_mb_default_params(mb_params *p) {
    p->dt = 1.0 / 40.0;            /* Exoskeleton_env.py:59, setTimeStep :117 */
    p->gravity = 9.81;             /* :116 */
    p->kp = 0.1;                   /* pybullet setJointMotorControlArray default positionGain */
    p->kd = 1.0;                   /* ... default velocityGain */
    p->motor_impulse = 1e5 / 40.0; /* default force 1e5 x dt */
    p->passive_impulse = 1.0;      /* createJointMotors: velocity motors, maxMotorImpulse 1 */
    p->limit_impulse = 100.0;      /* btMultiBodyConstraint default max applied impulse */
    p->erp = 0.2;                  /* btContactSolverInfo default m_erp */
    p->lin_damp = 0.04;            /* btMultiBody default linear damping */
    p->ang_damp = 0.04;            /* btMultiBody default angular damping */
    p->max_vel = 100.0;            /* btMultiBody default max coordinate velocity */
    p->iters = 50;                 /* pybullet default numSolverIterations */
}

static void rpy_mat(const double *rpy, double R[9]) {
    double cr = cos(rpy[0]), sr = sin(rpy[0]), cp = cos(rpy[1]), sp = sin(rpy[1]), cy = cos(rpy[2]),
           sy = sin(rpy[2]);
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

static void mm3(const double *A, const double *B, double *C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

static void cross(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

typedef struct {
    double R[NL][9], P[NL][3]; /* link frame (joint frame moved by q) */
    double S[NL][6];           /* motion subspace, world frame, about the world origin */
    double I[NL][36];          /* spatial inertia, world frame, about the world origin */
    double com[NL][3];
    double m[NL], Ic[NL][9];
} mb_kin;

/* Spatial inertia about the origin of a body with mass m, CoM c and rotational
 * inertia Ic about the CoM (angular rows first): [[Ic - m cx cx, m cx], [-m cx, m E]]. */
static void rb_inertia(double m, const double *c, const double *Ic, double *I6) {
    const double X[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
    double XX[9];
    mm3(X, X, XX);
    memset(I6, 0, 36 * sizeof(double));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            I6[i * 6 + j] = Ic[i * 3 + j] - m * XX[i * 3 + j];
            I6[i * 6 + 3 + j] = m * X[i * 3 + j];
            I6[(3 + i) * 6 + j] = -m * X[i * 3 + j];
        }
    for (int i = 0; i < 3; ++i) I6[(3 + i) * 6 + 3 + i] = m;
}

static void kinematics(const double *q, mb_kin *k) {
    for (int i = 0; i < NL; ++i) {
        double Rp[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, pp[3] = {0, 0, 0.1}; /* basePosition [0,0,0.1] (sim:18) */
        if (PAR[i] >= 0) { memcpy(Rp, k->R[PAR[i]], sizeof Rp); memcpy(pp, k->P[PAR[i]], sizeof pp); }
        double Ro[9], Rj[9];
        rpy_mat(RPY[i], Ro);
        mm3(Rp, Ro, Rj);
        double o[3], ax[3] = {Rj[2], Rj[5], Rj[8]}; /* joint axis (0 0 1) in the joint frame */
        for (int a = 0; a < 3; ++a)
            o[a] = pp[a] + Rp[a * 3] * XYZ[i][0] + Rp[a * 3 + 1] * XYZ[i][1] + Rp[a * 3 + 2] * XYZ[i][2];
        if (REV[i]) {
            const double c = cos(q[i]), s = sin(q[i]);
            const double Rz[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
            mm3(Rj, Rz, k->R[i]);
            memcpy(k->P[i], o, sizeof o);
            k->S[i][0] = ax[0]; k->S[i][1] = ax[1]; k->S[i][2] = ax[2];
            cross(o, ax, &k->S[i][3]);
        } else {
            memcpy(k->R[i], Rj, sizeof Rj);
            for (int a = 0; a < 3; ++a) k->P[i][a] = o[a] + q[i] * ax[a];
            k->S[i][0] = k->S[i][1] = k->S[i][2] = 0;
            k->S[i][3] = ax[0]; k->S[i][4] = ax[1]; k->S[i][5] = ax[2];
        }
        double Rin[9], d[3];
        if (i < 5) {
            double Ri[9];
            rpy_mat(IRPY5[i], Ri);
            mm3(k->R[i], Ri, Rin);
            for (int a = 0; a < 3; ++a)
                k->com[i][a] = k->P[i][a] + k->R[i][a * 3] * COM5[i][0] + k->R[i][a * 3 + 1] * COM5[i][1] +
                               k->R[i][a * 3 + 2] * COM5[i][2];
            k->m[i] = MASS5[i];
            memcpy(d, IDIAG5[i], sizeof d);
        } else {
            memcpy(Rin, k->R[i], sizeof Rin);
            memcpy(k->com[i], k->P[i], sizeof k->com[i]);
            k->m[i] = 1.0;
            d[0] = d[1] = d[2] = 1.0;
        }
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b)
                k->Ic[i][a * 3 + b] = Rin[a * 3] * d[0] * Rin[b * 3] + Rin[a * 3 + 1] * d[1] * Rin[b * 3 + 1] +
                                      Rin[a * 3 + 2] * d[2] * Rin[b * 3 + 2];
        rb_inertia(k->m[i], k->com[i], k->Ic[i], k->I[i]);
    }
}

static void mv6(const double *M, const double *v, double *o) {
    for (int i = 0; i < 6; ++i) {
        double s = 0;
        for (int j = 0; j < 6; ++j) s += M[i * 6 + j] * v[j];
        o[i] = s;
    }
}
static double dot6(const double *a, const double *b) {
    double s = 0;
    for (int i = 0; i < 6; ++i) s += a[i] * b[i];
    return s;
}
/* motion cross product v xm u */
static void crm(const double *v, const double *u, double *o) {
    double t[3];
    cross(v, u, o);
    cross(v, u + 3, o + 3);
    cross(v + 3, u, t);
    for (int a = 0; a < 3; ++a) o[3 + a] += t[a];
}
/* force cross product v xf f */
static void crf(const double *v, const double *f, double *o) {
    double t[3];
    cross(v, f, o);
    cross(v + 3, f + 3, t);
    for (int a = 0; a < 3; ++a) o[a] += t[a];
    cross(v, f + 3, o + 3);
}

/* Bullet's link damping (btMultiBody::computeAccelerationsArticulatedBodyAlgorithmMultiDof,
 * k1 = k2 = damping): resisting force m vc (k + k|vc|) at the CoM and torque
 * Ic w (k + k|w|), as a spatial force about the origin. */
static void damping(const mb_kin *k, int i, const double *v, const mb_params *p, double *f) {
    double vc[3], t[3];
    cross(v, k->com[i], t);
    for (int a = 0; a < 3; ++a) vc[a] = v[3 + a] + t[a];
    const double nv = sqrt(vc[0] * vc[0] + vc[1] * vc[1] + vc[2] * vc[2]);
    const double nw = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    double fl[3], ta[3];
    for (int a = 0; a < 3; ++a) {
        fl[a] = k->m[i] * vc[a] * (p->lin_damp + p->lin_damp * nv);
        ta[a] = (k->Ic[i][a * 3] * v[0] + k->Ic[i][a * 3 + 1] * v[1] + k->Ic[i][a * 3 + 2] * v[2]) *
                (p->ang_damp + p->ang_damp * nw);
    }
    cross(k->com[i], fl, t);
    for (int a = 0; a < 3; ++a) { f[a] = ta[a] + t[a]; f[3 + a] = fl[a]; }
}

/* Articulated-Body Algorithm: qdd for joint forces tau (fixed base; gravity as
 * an upward base acceleration). */
void oracle_mb_aba(const double *q, const double *qd, const double *tau, const mb_params *p, double *qdd) {
    mb_kin k;
    kinematics(q, &k);
    double v[NL][6], c[NL][6], pA[NL][6], IA[NL][36], U[NL][6], D[NL], u[NL], a[NL][6];
    for (int i = 0; i < NL; ++i) {
        double vJ[6], Iv[6], f[6];
        for (int r = 0; r < 6; ++r) vJ[r] = k.S[i][r] * qd[i];
        for (int r = 0; r < 6; ++r) v[i][r] = (PAR[i] >= 0 ? v[PAR[i]][r] : 0.0) + vJ[r];
        crm(v[i], vJ, c[i]);
        memcpy(IA[i], k.I[i], sizeof IA[i]);
        mv6(k.I[i], v[i], Iv);
        crf(v[i], Iv, pA[i]);
        damping(&k, i, v[i], p, f);
        for (int r = 0; r < 6; ++r) pA[i][r] += f[r];
    }
    for (int i = NL - 1; i >= 0; --i) {
        mv6(IA[i], k.S[i], U[i]);
        D[i] = dot6(k.S[i], U[i]);
        u[i] = (tau ? tau[i] : 0.0) - dot6(k.S[i], pA[i]);
        const int pi = PAR[i];
        if (pi < 0) continue;
        double Ia[36], pa[6], Iac[6];
        for (int r = 0; r < 6; ++r)
            for (int s = 0; s < 6; ++s) Ia[r * 6 + s] = IA[i][r * 6 + s] - U[i][r] * U[i][s] / D[i];
        mv6(Ia, c[i], Iac);
        for (int r = 0; r < 6; ++r) pa[r] = pA[i][r] + Iac[r] + U[i][r] * u[i] / D[i];
        for (int r = 0; r < 36; ++r) IA[pi][r] += Ia[r];
        for (int r = 0; r < 6; ++r) pA[pi][r] += pa[r];
    }
    const double a0[6] = {0, 0, 0, 0, 0, p->gravity};
    for (int i = 0; i < NL; ++i) {
        const double *ap = PAR[i] >= 0 ? a[PAR[i]] : a0;
        for (int r = 0; r < 6; ++r) a[i][r] = ap[r] + c[i][r];
        qdd[i] = (u[i] - dot6(U[i], a[i])) / D[i];
        for (int r = 0; r < 6; ++r) a[i][r] += k.S[i][r] * qdd[i];
    }
}

/* Recursive Newton-Euler: joint forces for (q, qd, qdd), same gravity / damping. */
void oracle_mb_rnea(const double *q, const double *qd, const double *qdd, const mb_params *p, double *tau) {
    mb_kin k;
    kinematics(q, &k);
    double v[NL][6], a[NL][6], f[NL][6];
    const double a0[6] = {0, 0, 0, 0, 0, p->gravity};
    for (int i = 0; i < NL; ++i) {
        double vJ[6], c[6], Iv[6], Ia[6], g[6], d[6];
        for (int r = 0; r < 6; ++r) vJ[r] = k.S[i][r] * qd[i];
        for (int r = 0; r < 6; ++r) v[i][r] = (PAR[i] >= 0 ? v[PAR[i]][r] : 0.0) + vJ[r];
        crm(v[i], vJ, c);
        const double *ap = PAR[i] >= 0 ? a[PAR[i]] : a0;
        for (int r = 0; r < 6; ++r) a[i][r] = ap[r] + k.S[i][r] * qdd[i] + c[r];
        mv6(k.I[i], a[i], Ia);
        mv6(k.I[i], v[i], Iv);
        crf(v[i], Iv, g);
        damping(&k, i, v[i], p, d);
        for (int r = 0; r < 6; ++r) f[i][r] = Ia[r] + g[r] + d[r];
    }
    for (int i = NL - 1; i >= 0; --i) {
        tau[i] = dot6(k.S[i], f[i]);
        if (PAR[i] >= 0)
            for (int r = 0; r < 6; ++r) f[PAR[i]][r] += f[i][r];
    }
}

/* Composite-Rigid-Body Algorithm: joint-space inertia M (19 x 19, row-major). */
void oracle_mb_mass(const double *q, double *M) {
    mb_kin k;
    kinematics(q, &k);
    double IC[NL][36];
    memcpy(IC, k.I, sizeof IC);
    for (int i = NL - 1; i >= 0; --i)
        if (PAR[i] >= 0)
            for (int r = 0; r < 36; ++r) IC[PAR[i]][r] += IC[i][r];
    memset(M, 0, NL * NL * sizeof(double));
    for (int i = 0; i < NL; ++i) {
        double F[6];
        mv6(IC[i], k.S[i], F);
        M[i * NL + i] = dot6(k.S[i], F);
        for (int j = PAR[i]; j >= 0; j = PAR[j]) M[i * NL + j] = M[j * NL + i] = dot6(k.S[j], F);
    }
}

/* World CoMs of the 19 links for all 19 joint positions (19 x 3). */
void oracle_mb_link_coms(const double *q, double *com) {
    mb_kin k;
    kinematics(q, &k);
    for (int i = 0; i < NL; ++i)
        for (int a = 0; a < 3; ++a) com[i * 3 + a] = k.com[i][a];
}

/* Gauss-Jordan inverse with partial pivoting (n <= NL). */
static int inverse(const double *A, double *Ai, int n) {
    double W[NL][2 * NL];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 2 * n; ++j) W[i][j] = j < n ? A[i * n + j] : (j - n == i ? 1.0 : 0.0);
    for (int c = 0; c < n; ++c) {
        int piv = c;
        for (int r = c + 1; r < n; ++r)
            if (fabs(W[r][c]) > fabs(W[piv][c])) piv = r;
        if (W[piv][c] == 0.0) return -1;
        if (piv != c)
            for (int j = 0; j < 2 * n; ++j) { double t = W[c][j]; W[c][j] = W[piv][j]; W[piv][j] = t; }
        const double d = W[c][c];
        for (int j = 0; j < 2 * n; ++j) W[c][j] /= d;
        for (int r = 0; r < n; ++r)
            if (r != c) {
                const double f = W[r][c];
                if (f != 0.0)
                    for (int j = 0; j < 2 * n; ++j) W[r][j] -= f * W[c][j];
            }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) Ai[i * n + j] = W[i][n + j];
    return 0;
}

/* One stepSimulation of the multibody model.  q, qd (19) are updated in place;
 * tgt5 = the revolute POSITION_CONTROL targets (rad).  stats (optional, 4):
 * [number of limit rows, max |motor residual| of the revolute rows after the
 * sweeps (rad/s), sum |impulse| of the prismatic motors, sum |impulse| of the
 * revolute motors]. */
int oracle_mb_step(double *q, double *qd, const double *tgt5, const mb_params *p, double *stats) {
    const double dt = p->dt;
    double qdd[NL], v[NL], M[NL * NL], Mi[NL * NL];
    oracle_mb_aba(q, qd, NULL, p, qdd);
    for (int j = 0; j < NL; ++j) {
        v[j] = qd[j] + dt * qdd[j];
        if (v[j] > p->max_vel) v[j] = p->max_vel;
        if (v[j] < -p->max_vel) v[j] = -p->max_vel;
    }
    oracle_mb_mass(q, M);
    if (inverse(M, Mi, NL)) return -1;
    /* rows: violated limits (lower, upper per joint), then the 19 motors */
    int dof[3 * NL], nrow = 0, nlim = 0;
    double sgn[3 * NL], w[3 * NL], lo[3 * NL], hi[3 * NL], lam[3 * NL];
    for (int j = 0; j < NL; ++j) {
        const double l = REV[j] ? LO5[j] : -0.5, h = REV[j] ? HI5[j] : 0.5;
        const double pen[2] = {q[j] - l, h - q[j]};
        for (int side = 0; side < 2; ++side) {
            if (pen[side] > 0) continue;
            dof[nrow] = j; sgn[nrow] = side ? -1.0 : 1.0;
            w[nrow] = -pen[side] * p->erp / dt;
            lo[nrow] = 0.0; hi[nrow] = p->limit_impulse;
            ++nrow; ++nlim;
        }
    }
    for (int j = 0; j < NL; ++j) {
        const double kp = REV[j] ? p->kp : 0.0, target = REV[j] ? tgt5[j] : 0.0;
        const double imp = REV[j] ? p->motor_impulse : p->passive_impulse;
        dof[nrow] = j; sgn[nrow] = 1.0;
        w[nrow] = kp * (target - q[j]) / dt + v[j] + p->kd * (0.0 - v[j]);
        lo[nrow] = -imp; hi[nrow] = imp;
        ++nrow;
    }
    for (int r = 0; r < nrow; ++r) lam[r] = 0.0;
    for (int it = 0; it < p->iters; ++it)
        for (int r = 0; r < nrow; ++r) {
            const int j = dof[r];
            double dl = (w[r] - sgn[r] * v[j]) / Mi[j * NL + j];
            double nl = lam[r] + dl;
            if (nl < lo[r]) nl = lo[r];
            if (nl > hi[r]) nl = hi[r];
            dl = nl - lam[r];
            lam[r] = nl;
            for (int d = 0; d < NL; ++d) v[d] += Mi[d * NL + j] * sgn[r] * dl;
        }
    if (stats) {
        double res = 0.0, pimp = 0.0, rimp = 0.0;
        for (int r = nlim; r < nrow; ++r) {
            const int j = dof[r];
            if (REV[j]) {
                const double e = fabs(w[r] - v[j]);
                if (e > res) res = e;
                rimp += fabs(lam[r]);
            } else {
                pimp += fabs(lam[r]);
            }
        }
        stats[0] = nlim; stats[1] = res; stats[2] = pimp; stats[3] = rimp;
    }
    for (int j = 0; j < NL; ++j) { q[j] += dt * v[j]; qd[j] = v[j]; }
    return 0;
}
