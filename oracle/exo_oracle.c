/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, fp64, single-threaded restatement of the reference's environment
 * hot path (TomasDelaney/...Parkinson-s-Patients).  It is the CHECKER for the
 * HIP kernels in ../a-deep-...-patients_amd/csrc and the "port" CPU baseline in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product never links or calls it.
 *
 * Parity pinning: every function below is checked against golden vectors
 * produced by the reference itself (tests/golden/make_golden.py imports the
 * reference from /root/reference with pybullet/gym stubbed out):
 *   - tests/golden/ode_cases.npz  pins solve_diff_eq (scipy RK45)
 *   - tests/golden/env_m*.npz     pins reset()/step() end to end.
 * The Bullet dynamics (stepSimulation) are NOT pinned (pybullet 3.2.5 is not
 * installed anywhere here): both the golden stub and this file implement the
 * idealised position-motor model of SURVEY.md A.2, with URDF forward
 * kinematics taken from Simulation/exo_v3.urdf.
 *
 * Citations are path:line into the reference repository.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "multibody.h"

#define DT (1.0 / 40.0) /* Environment/Exoskeleton_env.py:59 */

/* ------------------------------------------------------------------------ */
/* scipy RK45 (Dormand-Prince 5(4)), as used by solve_ivp defaults.          */
/* Utilities/calculate_joint_angles.py:5-22 calls                             */
/*   solve_ivp(dqdt, [0, dt], zeros(14))  -> rtol 1e-3, atol 1e-6.            */
/* Step control follows scipy/integrate/_ivp/rk.py (RungeKutta._step_impl)    */
/* and common.py (select_initial_step, norm).                                 */
/* ------------------------------------------------------------------------ */
/* RK_C is not needed: dqdt does not depend on t. */
static const double RK_A[6][5] = {
    {0, 0, 0, 0, 0},
    {1.0 / 5, 0, 0, 0, 0},
    {3.0 / 40, 9.0 / 40, 0, 0, 0},
    {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
    {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
    {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
static const double RK_B[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
static const double RK_E[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200, -22.0 / 525, 1.0 / 40};

typedef struct {
    double lu[49];
    int piv[7];
    const double *D, *K, *T;
    int nfev;
} ode_sys;

/* LU with partial pivoting (the algorithm np.linalg.solve -> LAPACK dgesv uses). */
static void lu_factor(const double *A, double *lu, int *piv) {
    memcpy(lu, A, 49 * sizeof(double));
    for (int k = 0; k < 7; ++k) {
        int p = k;
        double best = fabs(lu[k * 7 + k]);
        for (int i = k + 1; i < 7; ++i)
            if (fabs(lu[i * 7 + k]) > best) { best = fabs(lu[i * 7 + k]); p = i; }
        piv[k] = p;
        if (p != k)
            for (int j = 0; j < 7; ++j) { double t = lu[k * 7 + j]; lu[k * 7 + j] = lu[p * 7 + j]; lu[p * 7 + j] = t; }
        double r = 1.0 / lu[k * 7 + k];
        for (int i = k + 1; i < 7; ++i) {
            double l = lu[i * 7 + k] * r;
            lu[i * 7 + k] = l;
            for (int j = k + 1; j < 7; ++j) lu[i * 7 + j] -= l * lu[k * 7 + j];
        }
    }
}

static void lu_solve(const double *lu, const int *piv, double *b) {
    for (int k = 0; k < 7; ++k)
        if (piv[k] != k) { double t = b[k]; b[k] = b[piv[k]]; b[piv[k]] = t; }
    for (int i = 1; i < 7; ++i)
        for (int j = 0; j < i; ++j) b[i] -= lu[i * 7 + j] * b[j];
    for (int i = 6; i >= 0; --i) {
        for (int j = i + 1; j < 7; ++j) b[i] -= lu[i * 7 + j] * b[j];
        b[i] /= lu[i * 7 + i];
    }
}

/* dqdt of calculate_joint_angles.py:7-15 */
static void rhs(ode_sys *s, const double *y, double *f) {
    double r[7];
    for (int i = 0; i < 7; ++i) {
        double dq = 0.0, kq = 0.0;
        for (int j = 0; j < 7; ++j) { dq += s->D[i * 7 + j] * y[7 + j]; kq += s->K[i * 7 + j] * y[j]; }
        r[i] = s->T[i] - dq - kq;
    }
    lu_solve(s->lu, s->piv, r);
    for (int i = 0; i < 7; ++i) { f[i] = y[7 + i]; f[7 + i] = r[i]; }
    s->nfev++;
}

static double rms14(const double *x) {
    double s = 0.0;
    for (int i = 0; i < 14; ++i) s += x[i] * x[i];
    return sqrt(s) / sqrt(14.0);
}

/* Returns q(dt) (7) for y0 = 0; *nfev receives the number of RHS evaluations. */
int oracle_solve_diff_eq(const double *I, const double *D, const double *K, const double *T, double *q_out,
                         int *nfev) {
    const double rtol = 1e-3, atol = 1e-6, t_bound = DT;
    ode_sys s;
    s.D = D; s.K = K; s.T = T; s.nfev = 0;
    lu_factor(I, s.lu, s.piv);
    double y[14] = {0}, f[14];
    rhs(&s, y, f);
    /* select_initial_step (common.py:68-134), y0 = 0 */
    double h_abs;
    {
        double sc[14], tmp[14];
        for (int i = 0; i < 14; ++i) { sc[i] = atol + fabs(y[i]) * rtol; tmp[i] = y[i] / sc[i]; }
        double d0 = rms14(tmp);
        for (int i = 0; i < 14; ++i) tmp[i] = f[i] / sc[i];
        double d1 = rms14(tmp);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        if (h0 > t_bound) h0 = t_bound;
        double y1[14], f1[14];
        for (int i = 0; i < 14; ++i) y1[i] = y[i] + h0 * f[i];
        rhs(&s, y1, f1);
        for (int i = 0; i < 14; ++i) tmp[i] = (f1[i] - f[i]) / sc[i];
        double d2 = rms14(tmp) / h0;
        double h1;
        if (d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
        else h1 = pow(0.01 / fmax(d1, d2), 1.0 / 5.0);
        h_abs = fmin(fmin(100 * h0, h1), t_bound);
    }
    double t = 0.0;
    const double err_exp = -1.0 / 5.0;
    while (t != t_bound) { /* base.py:189, rk.py _step_impl */
        double min_step = 10 * fabs(nextafter(t, INFINITY) - t);
        if (h_abs < min_step) h_abs = min_step;
        int rejected = 0;
        for (;;) {
            if (h_abs < min_step) { /* scipy: status -1, sol.y up to the last accepted step */
                for (int i = 0; i < 7; ++i) q_out[i] = y[i];
                if (nfev) *nfev = s.nfev;
                return 1;
            }
            double h = h_abs, t_new = t + h;
            if (t_new - t_bound > 0) t_new = t_bound;
            h = t_new - t;
            h_abs = fabs(h);
            double Kst[7][14], ynew[14], fnew[14], ys[14];
            memcpy(Kst[0], f, sizeof f);
            for (int st = 1; st < 6; ++st) {
                for (int i = 0; i < 14; ++i) {
                    double dy = 0.0;
                    for (int j = 0; j < st; ++j) dy += Kst[j][i] * RK_A[st][j];
                    ys[i] = y[i] + dy * h;
                }
                rhs(&s, ys, Kst[st]);
            }
            for (int i = 0; i < 14; ++i) {
                double acc = 0.0;
                for (int j = 0; j < 6; ++j) acc += Kst[j][i] * RK_B[j];
                ynew[i] = y[i] + h * acc;
            }
            rhs(&s, ynew, fnew);
            memcpy(Kst[6], fnew, sizeof fnew);
            double e[14];
            for (int i = 0; i < 14; ++i) {
                double acc = 0.0;
                for (int j = 0; j < 7; ++j) acc += Kst[j][i] * RK_E[j];
                double sc = atol + fmax(fabs(y[i]), fabs(ynew[i])) * rtol;
                e[i] = acc * h / sc;
            }
            double en = rms14(e);
            if (en < 1) {
                double factor = (en == 0) ? 10.0 : fmin(10.0, 0.9 * pow(en, err_exp));
                if (rejected) factor = fmin(1.0, factor);
                h_abs *= factor;
                t = t_new;
                memcpy(y, ynew, sizeof y);
                memcpy(f, fnew, sizeof f);
                break;
            }
            h_abs *= fmax(0.2, 0.9 * pow(en, err_exp));
            rejected = 1;
        }
    }
    for (int i = 0; i < 7; ++i) q_out[i] = y[i];
    if (nfev) *nfev = s.nfev;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* URDF forward kinematics: Simulation/exo_v3.urdf (joints in file order ==   */
/* pybullet link index; Environment/Exoskeleton_sim_pybullet.py:21-63).       */
/* ------------------------------------------------------------------------ */
#define NJ 19
static const int J_PARENT[NJ] = {-1, 0, 1, 2, 3, 4, 4, 2, 2, 2, 2, 2, 2, 2, -1, -1, -1, -1, -1};
static const int J_REVOLUTE[NJ] = {1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static const double J_XYZ[NJ][3] = {
    {0.010000, -0.475000, 1.200000}, {0, 0, 0}, {0, 0, 0}, {0.480000, 0, 0}, {0, 0, -0.000000},
    {0.080234, -0.000000, -0.220137}, {-0.069766, -0.000000, -0.220137},
    {0.300000, 0.000000, 0.075000}, {0.200000, 0.000000, 0.075000}, {0.250000, 0.000000, 0.075000},
    {0.300000, 0.000000, -0.075000}, {0.200000, 0.000000, -0.075000}, {0.250000, 0.000000, -0.075000},
    {0.250000, -0.075000, 0.000000},
    {0.150000, -0.275000, 0.900000}, {0.150000, -0.275000, 1.100000}, {-0.150000, -0.275000, 0.900000},
    {-0.150000, -0.275000, 1.100000}, {0.010000, -0.475000, 1.290000}};
static const double J_RPY[NJ][3] = {
    {-3.141593, 3.141593, -3.141593}, {-1.570796, 3.141593, -3.141593}, {1.570796, 3.141593, 1.570796},
    {1.570796, -1.570796, 0.000000}, {1.570796, 3.141593, -3.141593},
    {3.141593, 3.089233, 3.141593}, {3.141593, 3.089233, 3.141593},
    {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000},
    {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000}, {-0.000000, 4.590216, -0.000000},
    {-0.000000, 4.590216, -0.000000},
    {-3.141593, 3.141593, -3.141593}, {-3.141593, 3.141593, -3.141593}, {-3.141593, 3.141593, -3.141593},
    {-3.141593, 3.141593, -3.141593}, {-3.141593, 3.141593, -3.141593}};
/* child-link inertial origins (CoM in link frame): exo_v3.urdf:24,44,64,84,104; k-links 0 */
static const double J_COM[NJ][3] = {{0, 0, 0}, {0, 0, 0}, {0.230000, 0, 0}, {0, 0.500000, -0.000000},
                                    {0.005234, 0, -0.245137}};
static const double J_LO[5] = {-1.3962633609772, -0.69813168048859, -2.6441738605499, -0.034906584769487,
                               -1.5184364318848};
static const double J_HI[5] = {1.3962633609772, 2.8187066316605, 0.78539800643921, 2.6179938726127,
                               1.3962633609772};

static void rpy_mat(const double *rpy, double R[9]) {
    double cr = cos(rpy[0]), sr = sin(rpy[0]), cp = cos(rpy[1]), sp = sin(rpy[1]), cy = cos(rpy[2]),
           sy = sin(rpy[2]);
    /* Rz(y) Ry(p) Rx(r) */
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
}

static void matmul3(const double *A, const double *B, double *C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

/* World CoM of all 19 links for revolute positions q[5] (prismatic held at 0). */
void oracle_link_coms(const double *q5, double *com /* 19x3 */) {
    double R[NJ][9], P[NJ][3];
    for (int i = 0; i < NJ; ++i) {
        double Rp[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, pp[3] = {0, 0, 0.1};
        if (J_PARENT[i] >= 0) { memcpy(Rp, R[J_PARENT[i]], sizeof Rp); memcpy(pp, P[J_PARENT[i]], sizeof pp); }
        double Ro[9], Rj[9];
        rpy_mat(J_RPY[i], Ro);
        matmul3(Rp, Ro, Rj);
        for (int a = 0; a < 3; ++a)
            P[i][a] = pp[a] + Rp[a * 3] * J_XYZ[i][0] + Rp[a * 3 + 1] * J_XYZ[i][1] + Rp[a * 3 + 2] * J_XYZ[i][2];
        if (J_REVOLUTE[i]) {
            double c = cos(q5[i]), s = sin(q5[i]);
            double Rz[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
            matmul3(Rj, Rz, R[i]);
        } else {
            memcpy(R[i], Rj, sizeof Rj);
        }
        const double *cm = (i < 5) ? J_COM[i] : (const double[3]){0, 0, 0};
        for (int a = 0; a < 3; ++a)
            com[i * 3 + a] = P[i][a] + R[i][a * 3] * cm[0] + R[i][a * 3 + 1] * cm[1] + R[i][a * 3 + 2] * cm[2];
    }
}

/* ------------------------------------------------------------------------ */
/* Environment state: Environment/Exoskeleton_env.py:38-175                   */
/* ------------------------------------------------------------------------ */
static const double I0[49] = {0.269, 0, 0, 0.076, 0, 0, -0.014, 0, 0.196, 0.083, 0, -0.002, 0.009, 0,
                              0, 0.083, 0.079, 0, 0, 0.011, 0, 0.076, 0, 0, 0.076, 0, 0, -0.012,
                              0, -0.002, 0, 0, 0.002, 0, 0, 0, 0.009, 0.011, 0, 0, 0.003, 0,
                              -0.014, 0, 0, -0.012, 0, 0, 0.003}; /* differential_eq_matrices.py:41-49 */
static const double D0[49] = {0.756, 0.184, 0.020, 0.187, 0, 0, 0, 0.184, 0.383, 0.267, 0, 0, 0, 0,
                              0.020, 0.267, 0.524, 0, 0, 0, 0, 0.187, 0, 0, 0.607, 0, 0, 0,
                              0, 0, 0, 0, 0.021, 0.001, 0.008, 0, 0, 0, 0, 0.001, 0.028, -0.003,
                              0, 0, 0, 0, 0.008, -0.003, 0.082}; /* :52-58 */
static const double S0[49] = {10.80, 2.626, 0.279, 2.670, 0, 0, 0, 2.626, 5.468, 3.821, 0, 0, 0, 0,
                              0.279, 3.821, 7.486, 0, 0, 0, 0, 2.670, 0, 0, 8.670, 0, 0, 0,
                              0, 0, 0, 0, 0.756, 0.018, 0.291, 0, 0, 0, 0, 0.018, 0.992, -0.099,
                              0, 0, 0, 0, 0.291, -0.099, 2.920}; /* :61-67 */

/* link handles Exoskeleton_sim_pybullet.py:48-63, read order :129-142 */
static const int K_LINK[14] = {9, 5, 12, 6, 15, 8, 17, 11, 14, 7, 18, 13, 16, 10};

typedef struct {
    /* constructor arguments */
    int L;
    const double *imu; /* [5][L] deg: elbow_y, elbow_z, shoulder_x, shoulder_y, shoulder_z */
    int seq[7];
    double amp[2], h1[2], h2[2], maxS0, maxE0, shift_r, act_r, mat_f;
    /* per episode */
    double *tremor; /* [7][L] */
    double I[49], D[49], S[49], shift[42], maxS, maxE, mag;
    double *forces; /* [7][L]  ep_state_values actuator forces */
    int counts;
    /* carried state */
    double phys_q[5];
    double ref_cached[6];   /* act_shoulder/elbow_reference_positions (sim:80-81,194-195,348-349) */
    double ref_cur[6], ref_prev[6];
    double pos_vect[21], prev_pos_vect[21];
    double prev_action[7], second_prev_action[7];
    double com[NJ * 3];     /* link CoMs cached at the last stepSimulation */
    double max_reward;
    int n_axes;
    /* stepSimulation model: 0 idealised motors, 1 multibody (multibody.c) */
    int physics;
    mb_params mb;
    double mb_q[NJ], mb_qd[NJ], mb_stats[4];
} oracle_env;

oracle_env *oracle_env_create(int L, const double *imu, const int *seq, const double *amp, const double *h1,
                              const double *h2, double maxS0, double maxE0, double shift_r, double act_r,
                              double mat_f) {
    oracle_env *e = (oracle_env *)calloc(1, sizeof(oracle_env));
    e->L = L; e->imu = imu;
    for (int i = 0; i < 7; ++i) { e->seq[i] = seq[i]; e->n_axes += seq[i]; }
    e->amp[0] = amp[0]; e->amp[1] = amp[1]; e->h1[0] = h1[0]; e->h1[1] = h1[1]; e->h2[0] = h2[0]; e->h2[1] = h2[1];
    e->maxS0 = maxS0; e->maxE0 = maxE0; e->shift_r = shift_r; e->act_r = act_r; e->mat_f = mat_f;
    e->tremor = (double *)calloc((size_t)7 * L, sizeof(double));
    e->forces = (double *)calloc((size_t)7 * L, sizeof(double));
    /* :167-169 */
    e->max_reward = e->n_axes * 0.5 + 0.9 + 0.05 + 0.05 + 0.5;
    double z[5] = {0};
    oracle_link_coms(z, e->com); /* loadURDF at q = 0 (sim:18) */
    oracle_mb_default_params(&e->mb);
    return e;
}

void oracle_env_destroy(oracle_env *e) {
    if (!e) return;
    free(e->tremor); free(e->forces); free(e);
}

int oracle_draws_per_episode(int L) { return 208 + 8 * L; }

/* add_symmetric_noise: Utilities/domain_randomization_anatomical_matrices.py:4-27 */
static void sym_noise(const double *M, double f, const double *u, double *out) {
    double n[49];
    for (int i = 0; i < 49; ++i) n[i] = -f + (f - (-f)) * u[i];
    for (int i = 0; i < 7; ++i)
        for (int j = 0; j < 7; ++j) {
            double s = (n[i * 7 + j] + n[j * 7 + i]) / 2;
            out[i * 7 + j] = M[i * 7 + j] + s * M[i * 7 + j];
        }
}

static void read_actuators(oracle_env *e, double act[14][3]) {
    /* get_actuator_positions: sim:119-158 */
    for (int k = 0; k < 14; ++k)
        for (int a = 0; a < 3; ++a) act[k][a] = e->com[K_LINK[k] * 3 + a] + e->shift[k * 3 + a];
}

static void pos_vect(oracle_env *e, double act[14][3], double *out) {
    /* get_actuator_pos_vect (effective def) sim:300-336: act_j2 - cached ref */
    for (int j = 0; j < 7; ++j) {
        const double *ref = (j < 2) ? &e->ref_cached[3] : &e->ref_cached[0];
        for (int a = 0; a < 3; ++a) out[j * 3 + a] = act[2 * j + 1][a] - ref[a];
    }
}

static void read_refs(oracle_env *e, double *out6) {
    /* return_reference_dummy_pos sim:338-351 (links 0 and 3) */
    for (int a = 0; a < 3; ++a) { out6[a] = e->com[0 * 3 + a]; out6[3 + a] = e->com[3 * 3 + a]; }
    memcpy(e->ref_cached, out6, 6 * sizeof(double));
}

static void pack_obs(oracle_env *e, float *obs) {
    /* update_state_vector: Exoskeleton_env.py:487-570 */
    int c = e->counts, k = 0;
    const double nrm[7] = {e->maxE0, e->maxE0, e->maxS0, e->maxS0, e->maxS0, e->maxS0, e->maxS0};
    for (int back = 2; back >= 1; --back)
        for (int j = 0; j < 7; ++j) obs[k++] = (float)(e->forces[j * e->L + c - back] / nrm[j]);
    const double tn[4] = {10, 10, 10, 5};
    for (int back = 2; back >= 0; --back)
        for (int j = 0; j < 4; ++j) obs[k++] = (float)(e->tremor[j * e->L + c - back] / tn[j]);
    for (int i = 0; i < 21; ++i) obs[k++] = (float)e->prev_pos_vect[i];
    for (int i = 0; i < 21; ++i) obs[k++] = (float)e->pos_vect[i];
    for (int i = 0; i < 6; ++i) obs[k++] = (float)e->ref_prev[i];
    for (int i = 0; i < 6; ++i) obs[k++] = (float)e->ref_cur[i];
}

/* initialize_movement: Exoskeleton_env.py:193-254 with the draw order of SURVEY.md 3.2.
 * draws: 208 + 8L unit uniforms in [0,1). */
void oracle_env_reset(oracle_env *e, const double *u, float *obs) {
    const int L = e->L;
    int p = 0;
    memset(e->forces, 0, sizeof(double) * 7 * L);
    /* :198-199 */
    double range = e->amp[1] - e->amp[0];
    e->mag = e->amp[0] + (u[p++] * range);
    /* generate_parkinson_tremor.py:5-21 */
    double f1 = e->h1[0] + (e->h1[1] - e->h1[0]) * u[p++];
    double f2 = e->h2[0] + (e->h2[1] - e->h2[0]) * u[p++];
    const double *noise_u = &u[p];
    p += L;
    double stop = L * DT, step = stop / (L - 1); /* np.linspace(0, L*dt, L) */
    double w1 = 2 * M_PI * f1, w2 = 2 * M_PI * f2;
    double *wave1 = (double *)malloc(sizeof(double) * L), *wave2 = (double *)malloc(sizeof(double) * L),
           *acc = (double *)malloc(sizeof(double) * L);
    for (int t = 0; t < L; ++t) {
        double tt = (t == L - 1) ? stop : t * step;
        wave1[t] = sin(w1 * tt);
        wave2[t] = sin(w2 * tt);
    }
    /* generate_joint_torques_train :31-73 */
    const double jmax0[7] = {2.5, 5, 10, 5, 5, 0.5, 0.5};
    for (int i = 0; i < 7; ++i) {
        double a1 = pow(10.0, (-5.0 + (0.0 - (-5.0)) * u[p++]) / 20);
        double a2 = pow(10.0, (-20.0 + (-10.0 - (-20.0)) * u[p++]) / 20);
        double mn = INFINITY, mx = -INFINITY;
        for (int t = 0; t < L; ++t) {
            acc[t] = (a1 * wave1[t] + a2 * wave2[t] + noise_u[t] * 0.001) * e->seq[i];
            if (acc[t] < mn) mn = acc[t];
            if (acc[t] > mx) mx = acc[t];
        }
        double jm = jmax0[i] * e->mag;
        for (int t = 0; t < L; ++t) {
            double v = (-1 + 2 * (acc[t] - mn) / (mx - mn)) * jm;
            if (!isfinite(v)) v = 0.0;
            double sgn = (u[p + t] < 0.5) ? -1.0 : 1.0;
            e->tremor[i * L + t] = v * sgn;
        }
        p += L;
    }
    free(wave1); free(wave2); free(acc);
    /* :208-210 */
    sym_noise(I0, e->mat_f, &u[p], e->I); p += 49;
    sym_noise(D0, e->mat_f, &u[p], e->D); p += 49;
    sym_noise(S0, e->mat_f, &u[p], e->S); p += 49;
    /* create_dummy_shift sim:98-107 */
    for (int i = 0; i < 42; ++i) e->shift[i] = -e->shift_r + (e->shift_r - (-e->shift_r)) * u[p++];
    /* :216-217 */
    double lo = 1 - e->act_r, hi = 1 + e->act_r;
    e->maxS = e->maxS0 * (lo + (hi - lo) * u[p++]);
    e->maxE = e->maxE0 * (lo + (hi - lo) * u[p++]);
    e->counts = 2;
    /* :229-250; set_joint_position has no effect before stepSimulation */
    double act[14][3];
    read_actuators(e, act);
    pos_vect(e, act, e->prev_pos_vect);
    read_refs(e, e->ref_prev);
    pos_vect(e, act, e->pos_vect);
    read_refs(e, e->ref_cur);
    pack_obs(e, obs);
}

static void cross3(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

/* step: Exoskeleton_env.py:368-471.  info[40] = actuator_torques, torque_val, ampl_val,
 * tremor_torque_val, tremor_ampl_val, reward_unwanted, _torque, _axis, _control, _smoothness. */
int oracle_env_step(oracle_env *e, const double *a, float *obs, double *reward, int *done, double *info,
                    double *targets_out) {
    const int L = e->L, c = e->counts;
    if (c >= L - 1) return -1;
    double F[7];
    for (int j = 0; j < 2; ++j) F[j] = ((a[j] + 1) / 2) * e->maxE; /* transform_action :256-266 */
    for (int j = 2; j < 7; ++j) F[j] = ((a[j] + 1) / 2) * e->maxS;
    for (int j = 0; j < 7; ++j) e->forces[j * L + c] = F[j];
    double act[14][3];
    read_actuators(e, act);
    memcpy(e->ref_prev, e->ref_cur, sizeof e->ref_prev);
    /* get_force_components sim:207-298 */
    double Fc[7][3];
    const double sv = 5;
    for (int j = 0; j < 7; ++j) {
        const double *k1 = act[2 * j], *k2 = act[2 * j + 1];
        double dx = (k2[0] + sv) - (k1[0] + sv), dy = (k2[1] + sv) - (k1[1] + sv), dz = (k2[2] + sv) - (k1[2] + sv);
        Fc[j][0] = cos(atan2(dy, dx)) * F[j];
        Fc[j][1] = cos(atan2(dx, dy)) * F[j];
        Fc[j][2] = cos(atan2(dz, dx)) * F[j];
    }
    memcpy(e->prev_pos_vect, e->pos_vect, sizeof e->pos_vect);
    pos_vect(e, act, e->pos_vect);
    read_refs(e, e->ref_cur);
    /* get_torques :177-187 with get_radius_vectors sim:192-205 */
    double tau[7][3];
    for (int j = 0; j < 7; ++j) {
        const double *ref = (j < 2) ? &e->ref_cached[3] : &e->ref_cached[0];
        double r[3] = {ref[0] - act[2 * j + 1][0], ref[1] - act[2 * j + 1][1], ref[2] - act[2 * j + 1][2]};
        cross3(Fc[j], r, tau[j]);
    }
    /* :394-400 (actuators 3,4,5,7,6 in that order) */
    double at[7] = {tau[2][1] + tau[3][1] + tau[4][1] + tau[6][1] + tau[5][1],
                    tau[2][0] + tau[3][0] + tau[4][0] + tau[6][0] + tau[5][0],
                    tau[2][2] + tau[3][2] + tau[4][2] + tau[6][2] + tau[5][2],
                    fabs(tau[0][1]) - fabs(tau[1][1]), 0, 0, 0};
    double tr[7], T[7];
    for (int j = 0; j < 7; ++j) { tr[j] = e->tremor[j * L + c]; T[j] = tr[j] + at[j]; }
    double qa[7], qt[7];
    /* a failed solve (> 0) continues from its last accepted q, as solve_ivp */
    if (oracle_solve_diff_eq(e->I, e->D, e->S, T, qa, NULL) < 0) return -2;
    if (oracle_solve_diff_eq(e->I, e->D, e->S, tr, qt, NULL) < 0) return -2;
    const double r2d = 180 / M_PI, d2r = M_PI / 180;
    for (int j = 0; j < 7; ++j) { qa[j] *= r2d; qt[j] *= r2d; }
    /* :421-431; imu columns: 0 elbow_y, 1 elbow_z, 2 shoulder_x, 3 shoulder_y, 4 shoulder_z */
    double sz = e->imu[4 * L + c] + qa[2], sy = e->imu[3 * L + c] + qa[0], sx = e->imu[2 * L + c] + qa[1],
           ey = e->imu[0 * L + c] + qa[3];
    double tgt[5] = {sz * d2r, sy * d2r, sx * d2r, ey * d2r, e->imu[1 * L + c] * d2r};
    if (targets_out) memcpy(targets_out, tgt, sizeof tgt);
    if (e->physics == 1) {
        /* stepSimulation: multibody dynamics + joint-space impulse solve (multibody.c) */
        if (oracle_mb_step(e->mb_q, e->mb_qd, tgt, &e->mb, e->mb_stats)) return -3;
        for (int j = 0; j < 5; ++j) e->phys_q[j] = e->mb_q[j];
        oracle_mb_link_coms(e->mb_q, e->com);
    } else {
        /* stepSimulation: idealised position motors, limits clamp */
        for (int j = 0; j < 5; ++j) {
            double q = e->phys_q[j] + 0.1 * (tgt[j] - e->phys_q[j]);
            e->phys_q[j] = fmin(fmax(q, J_LO[j]), J_HI[j]);
        }
        oracle_link_coms(e->phys_q, e->com);
    }
    /* get_reward :341-366 */
    const double eps = 1e-10;
    double M = e->maxE + e->maxS;
    double unwanted = 0.0;
    for (int j = 0; j < 4; ++j) if (e->seq[j] == 0) unwanted += fabs(T[j]);
    double r_unw = exp(-(unwanted / (M / 4 / e->n_axes)) + eps) * 0.5;
    double st = 0.0;
    for (int j = 0; j < 4; ++j) if (e->seq[j] == 1) st += (fabs(T[j]) - fabs(tr[j])) / fabs(tr[j]) + 1;
    double r_tor = exp((-st + eps) / e->n_axes) * 0.9;
    int nred = 0;
    for (int j = 0; j < 7; ++j) {
        double v = (fabs(T[j]) - fabs(tr[j])) / (fabs(tr[j]) + eps) * 100;
        if (!isfinite(v)) v = 0.0;
        if (v < 0) nred++;
    }
    double r_axis = nred * 0.5;
    double sa = 0.0;
    for (int j = 0; j < 7; ++j) sa += F[j];
    double r_ctl = exp(-(sa / (M / 2)) + eps) * 0.05;
    double sm = 0.0;
    for (int j = 0; j < 7; ++j) { double d = F[j] - 2 * e->prev_action[j] + e->second_prev_action[j]; sm += d * d; }
    sm /= 7;
    double r_sm = 0.05 * exp(-(sm / (M / 4)) + eps);
    *reward = (r_axis + r_tor + r_sm + r_ctl + r_unw) / e->max_reward;
    e->counts = c + 1;
    pack_obs(e, obs);
    memcpy(e->second_prev_action, e->prev_action, sizeof F);
    memcpy(e->prev_action, F, sizeof F);
    *done = e->counts >= L - 1;
    if (info) {
        for (int j = 0; j < 7; ++j) {
            info[j] = at[j]; info[7 + j] = T[j]; info[14 + j] = qa[j]; info[21 + j] = tr[j]; info[28 + j] = qt[j];
        }
        info[35] = r_unw; info[36] = r_tor; info[37] = r_axis; info[38] = r_ctl; info[39] = r_sm;
    }
    return 0;
}

/* accessors for tests */
const double *oracle_env_tremor(const oracle_env *e) { return e->tremor; }
void oracle_env_episode(const oracle_env *e, double *I, double *D, double *S, double *shift, double *maxSE) {
    memcpy(I, e->I, sizeof e->I); memcpy(D, e->D, sizeof e->D); memcpy(S, e->S, sizeof e->S);
    memcpy(shift, e->shift, sizeof e->shift);
    maxSE[0] = e->maxS; maxSE[1] = e->maxE;
}
void oracle_env_phys(const oracle_env *e, double *q5) { memcpy(q5, e->phys_q, sizeof e->phys_q); }
int oracle_env_counts(const oracle_env *e) { return e->counts; }
/* multibody mode: select it (with optional parameters) and read / write the 19-joint state */
void oracle_env_set_physics(oracle_env *e, int mode, const mb_params *p) {
    e->physics = mode;
    if (p) e->mb = *p;
}
void oracle_env_mb_state(const oracle_env *e, double *q19, double *qd19, double *stats4) {
    if (q19) memcpy(q19, e->mb_q, sizeof e->mb_q);
    if (qd19) memcpy(qd19, e->mb_qd, sizeof e->mb_qd);
    if (stats4) memcpy(stats4, e->mb_stats, sizeof e->mb_stats);
}
void oracle_env_set_mb_state(oracle_env *e, const double *q19, const double *qd19) {
    memcpy(e->mb_q, q19, sizeof e->mb_q);
    memcpy(e->mb_qd, qd19, sizeof e->mb_qd);
    for (int j = 0; j < 5; ++j) e->phys_q[j] = q19[j];
    oracle_mb_link_coms(e->mb_q, e->com);
}

/* ------------------------------------------------------------------------ */
/* CPU baseline driver: n_envs envs stepped sequentially on one core with     */
/* random actions; draws from a splitmix64 stream.  Returns env-steps done.   */
/* ------------------------------------------------------------------------ */
static uint64_t sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01(uint64_t *s) { return (sm64(s) >> 11) * (1.0 / 9007199254740992.0); }

long oracle_bench(int n_envs, const double *imu_all /* [8][5][Lmax] */, const int *lens, int Lmax, long max_steps,
                  uint64_t seed) {
    const int seq[7] = {0, 1, 0, 1, 0, 0, 0};
    const double amp[2] = {0.95, 1.05}, h1[2] = {4, 6}, h2[2] = {8, 10};
    oracle_env **envs = (oracle_env **)calloc(n_envs, sizeof(void *));
    double **imus = (double **)calloc(n_envs, sizeof(void *));
    uint64_t s = seed;
    float obs[80];
    double *draws = (double *)malloc(sizeof(double) * (208 + 8 * Lmax));
    for (int i = 0; i < n_envs; ++i) {
        int m = i % 8, L = lens[m];
        imus[i] = (double *)malloc(sizeof(double) * 5 * L);
        for (int c = 0; c < 5; ++c) memcpy(imus[i] + c * L, imu_all + ((size_t)m * 5 + c) * Lmax, sizeof(double) * L);
        envs[i] = oracle_env_create(L, imus[i], seq, amp, h1, h2, 40, 20, 0.02, 0.03, 0.1);
    }
    long steps = 0;
    while (steps < max_steps) {
        for (int i = 0; i < n_envs; ++i) {
            for (int k = 0; k < 208 + 8 * envs[i]->L; ++k) draws[k] = u01(&s);
            oracle_env_reset(envs[i], draws, obs);
        }
        int active = n_envs;
        while (active > 0 && steps < max_steps) {
            active = 0;
            for (int i = 0; i < n_envs; ++i) {
                if (envs[i]->counts >= envs[i]->L - 1) continue;
                double a[7], r;
                int d;
                for (int j = 0; j < 7; ++j) a[j] = 2 * u01(&s) - 1;
                oracle_env_step(envs[i], a, obs, &r, &d, NULL, NULL);
                steps++;
                if (!d) active++;
            }
        }
    }
    for (int i = 0; i < n_envs; ++i) { oracle_env_destroy(envs[i]); free(imus[i]); }
    free(envs); free(imus); free(draws);
    return steps;
}
