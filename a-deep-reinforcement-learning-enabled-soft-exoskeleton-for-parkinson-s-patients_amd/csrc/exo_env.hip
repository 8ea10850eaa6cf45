// exo_env.hip -- vectorised exoskeleton environment for MI355X (gfx950).
//
// Kernels
//   exo_reset_kernel : 16 envs per 256-thread workgroup, 16 threads per env.
//                      They sweep the tremor samples (generate_parkinson_
//                      tremor.py:31-73; coalesced table stores), the domain-
//                      randomised matrices (Exoskeleton_env.py:208-210) and the
//                      dummy shift (Exoskeleton_sim_pybullet.py:98-107); one
//                      thread per env inverts the two diagonal blocks of I and
//                      packs the reset observation (Exoskeleton_env.py:220-254).
//                      exo_reset_list_kernel: the same with one wavefront per
//                      listed env (async episodes' short lists).
//   exo_step_kernel  : two lanes per env.  Both lanes run the kinematics and
//                      torque model (Exoskeleton_env.py:369-406); lane 0 solves
//                      the actuated joint ODE, lane 1 the tremor-only ODE
//                      (:409-414), then lane 0 finishes the step (targets,
//                      motor update, reward, observation; :417-471).
//   exo_multibody_kernel (csrc/exo_multibody.hip): the multibody stepSimulation
//                      that follows the step kernel in EXO_PHYS_MULTIBODY mode.
//
// C ABI: include/exo_amd.h.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "exo_amd.h"
#include "exo_model.h"

using namespace exo;

namespace {

__device__ __forceinline__ double cfg(const Dev &S, int k, int e) { return S.cfg[(size_t)k * S.N + e]; }

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

struct Draws {
    const double *buf; // injected stream or nullptr (Philox)
    uint64_t seed;
    uint32_t env, episode;
    __device__ __forceinline__ double operator()(int p) const {
        return buf ? buf[p] : philox_u01(seed, env, episode, (uint32_t)p);
    }
};

// Invert a small dense matrix (Gauss-Jordan, partial pivoting), fp64.  Every
// index is a compile-time one (the pivot row swap is a select per row): with
// `a[p * n + j]` for the runtime pivot p the arrays lived in scratch memory,
// 46 scratch accesses on the reset's serial tail (r06).  Same operations in
// the same order: bit-identical.
template <int n>
__device__ __forceinline__ void invert(double *a /* n*n, destroyed */, double *inv) {
#pragma unroll
    for (int i = 0; i < n * n; ++i) inv[i] = (i % (n + 1) == 0) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = fabs(a[k * n + k]);
#pragma unroll
        for (int i = k + 1; i < n; ++i) {
            const double v = fabs(a[i * n + k]);
            if (v > best) { best = v; p = i; }
        }
#pragma unroll
        for (int i = k + 1; i < n; ++i) {
            const bool sw = p == i;
#pragma unroll
            for (int j = 0; j < n; ++j) {
                const double t = a[k * n + j], u = inv[k * n + j];
                a[k * n + j] = sw ? a[i * n + j] : t;
                a[i * n + j] = sw ? t : a[i * n + j];
                inv[k * n + j] = sw ? inv[i * n + j] : u;
                inv[i * n + j] = sw ? u : inv[i * n + j];
            }
        }
        const double r = 1.0 / a[k * n + k];
#pragma unroll
        for (int j = 0; j < n; ++j) { a[k * n + j] *= r; inv[k * n + j] *= r; }
#pragma unroll
        for (int i = 0; i < n; ++i) {
            if (i == k) continue;
            const double m = a[i * n + k];
#pragma unroll
            for (int j = 0; j < n; ++j) { a[i * n + j] -= m * a[k * n + j]; inv[i * n + j] -= m * inv[k * n + j]; }
        }
    }
}

// ---------------------------------------------------------------------------
// reset: initialize_movement (Exoskeleton_env.py:193-254).  The draw stream
// follows the reference's np.random call order:
//   0 magnitude, 1 f1, 2 f2, 3..3+L-1 white noise,
//   per axis i: base_i = 3+L+i(L+2): a1, a2, L signs,
//   17+8L: I noise (49), D noise (49), S noise (49), 164+8L: shift (42),
//   206+8L: shoulder force scale, elbow force scale.
// ---------------------------------------------------------------------------
// The resets of EPW envs by one workgroup of EPW x TS threads: thread
// (el = tid % EPW, tl = tid / EPW) works for env slot el and sweeps its tremor
// samples t = tl, tl + TS, ...  With EPW = 16 the 16 threads of a (sample,
// axis) store 16 consecutive envs' values -- one whole 128-byte line of the
// [Lmax][7][N] tremor table per store instruction -- where one wavefront per
// env stored each value to a line of its own (r05: 275 us per 4,096-env reset,
// the line-scattered stores).  The arithmetic of every value is the one-env
// sequence of the reference (numpy order, no contraction), so the tables are
// bit-identical to the per-env kernel's.  e < 0: an idle slot (it joins the
// barriers, stores nothing).  draws: the slot's injected stream or nullptr
// (Philox).
template <int EPW, int TS>
__device__ void reset_group(const Dev &S, const Urdf &U, int e, const double *draws, uint64_t seed, float *obs) {
    // numpy evaluates every expression of the reset without fused multiply-add;
    // keep the rounding identical (bit-exact D, S, shift and force scales).
#pragma clang fp contract(off)
    constexpr int NT = EPW * TS, NW = NT / 64;
    static_assert(NT % 64 == 0 && 64 % EPW == 0, "whole wavefronts, a slot's threads spread over lanes");
    const int el = threadIdx.x % EPW, tl = threadIdx.x / EPW, w = threadIdx.x / 64;
    const bool on = e >= 0;
    const int ee = on ? e : 0;
    if (on && tl == 0 && S.pend) S.pend[e] = 0;  // a solve still carried by a budgeted step is dropped
    const int N = S.N, L = on ? S.L[ee] : 0, seq = S.seq[ee];
    const uint32_t ep = S.episode[ee];
    const Draws D{draws, seed, (uint32_t)ee, ep};

    __shared__ double sA[EPW][14], sMn[NW][EPW][7], sMx[NW][EPW][7];
    __shared__ double sI[EPW][49], sD[EPW][49], sS[EPW][49], sShift[EPW][42], sTrem[EPW][3][4], sInv[EPW][NINV];

    // ---- tremor (generate_parkinson_tremor.py:5-28, :31-73) -------------
    const double amp0 = cfg(S, C_AMP0, ee), amp1 = cfg(S, C_AMP1, ee);
    const double h1a = cfg(S, C_H1A, ee), h1b = cfg(S, C_H1B, ee), h2a = cfg(S, C_H2A, ee), h2b = cfg(S, C_H2B, ee);
    double mag = 0, f1 = 0, f2 = 0;
    if (on) {
        mag = amp0 + (D(0) * (amp1 - amp0)); // :198-199
        f1 = h1a + (h1b - h1a) * D(1);
        f2 = h2a + (h2b - h2a) * D(2);
    }
    const double stop = L * DT, step = stop / (L - 1); // np.linspace(0, L*dt, L)
    const double w1 = 2 * PI * f1, w2 = 2 * PI * f2;
    // the 14 amplitudes, one pow per thread of the slot
    for (int j = tl; j < 14; j += TS) {
        const int i = j % 7, b = 3 + L + i * (L + 2);
        sA[el][j] = !on ? 0.0
                    : j < 7 ? pow(10.0, (-5.0 + (0.0 - (-5.0)) * D(b)) / 20)
                            : pow(10.0, (-20.0 + (-10.0 - (-20.0)) * D(b + 1)) / 20);
    }
    __syncthreads();
    double a1[7], a2[7], mn[7], mx[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        a1[i] = sA[el][i];
        a2[i] = sA[el][7 + i];
        mn[i] = INFINITY;
        mx[i] = -INFINITY;
    }
    for (int t = tl; t < L; t += TS) {
        const double tt = (t == L - 1) ? stop : t * step;
        const double wv1 = sin(w1 * tt), wv2 = sin(w2 * tt), nz = D(3 + t) * 0.001;
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const double acc = (a1[i] * wv1 + a2[i] * wv2 + nz) * (double)((seq >> i) & 1);
            mn[i] = fmin(mn[i], acc);
            mx[i] = fmax(mx[i], acc);
        }
    }
    // min / max over the slot's threads: lanes EPW apart in a wavefront, then
    // the wavefronts through LDS (fmin / fmax are exact: any order)
#pragma unroll
    for (int i = 0; i < 7; ++i) {
#pragma unroll
        for (int o = EPW; o < 64; o <<= 1) {
            mn[i] = fmin(mn[i], __shfl_xor(mn[i], o, 64));
            mx[i] = fmax(mx[i], __shfl_xor(mx[i], o, 64));
        }
    }
    if (NW > 1) {
        if ((threadIdx.x & 63) < EPW) {
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                sMn[w][el][i] = mn[i];
                sMx[w][el][i] = mx[i];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            mn[i] = sMn[0][el][i];
            mx[i] = sMx[0][el][i];
#pragma unroll
            for (int v = 1; v < NW; ++v) {
                mn[i] = fmin(mn[i], sMn[v][el][i]);
                mx[i] = fmax(mx[i], sMx[v][el][i]);
            }
        }
    }
    // joint_max_values (:59): the shipped table unless exo_set_tremor_model chose another
    for (int t = tl; t < L; t += TS) {
        const double tt = (t == L - 1) ? stop : t * step;
        const double wv1 = sin(w1 * tt), wv2 = sin(w2 * tt), nz = D(3 + t) * 0.001;
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const double acc = (a1[i] * wv1 + a2[i] * wv2 + nz) * (double)((seq >> i) & 1);
            double v = (-1 + 2 * (acc - mn[i]) / (mx[i] - mn[i])) * (S.tjmax[i] * mag);
            if (!isfinite(v)) v = 0.0; // np.nan_to_num (:67)
            // np.random.choice([-1, 1], L) per sample (:70); the diagnostic
            // models use the axis's first sign draw for every sample, or none
            const int ts = S.tsign == EXO_TREMOR_SIGN_PER_AXIS ? 0 : t;
            const double sgn = (S.tsign != EXO_TREMOR_SIGN_NONE && D(3 + L + i * (L + 2) + 2 + ts) < 0.5) ? -1.0
                                                                                                            : 1.0;
            v *= sgn;
            S.tremor[((size_t)t * 7 + i) * N + e] = v;
            if (t < 3 && i < 4) sTrem[el][t][i] = v;
        }
    }

    // ---- domain-randomised matrices (domain_randomization_...py:4-27) ----
    const double mf = cfg(S, C_MATF, ee);
    const int pI = 17 + 8 * L;
    if (on) {
        for (int j = tl; j < 49; j += TS) {
            const int r = j / 7, c = j % 7, tr = c * 7 + r;
            double n0, n1, s;
            n0 = -mf + (mf - (-mf)) * D(pI + j); n1 = -mf + (mf - (-mf)) * D(pI + tr);
            s = (n0 + n1) / 2; sI[el][j] = I0[j] + s * I0[j];
            n0 = -mf + (mf - (-mf)) * D(pI + 49 + j); n1 = -mf + (mf - (-mf)) * D(pI + 49 + tr);
            s = (n0 + n1) / 2; sD[el][j] = D0[j] + s * D0[j];
            n0 = -mf + (mf - (-mf)) * D(pI + 98 + j); n1 = -mf + (mf - (-mf)) * D(pI + 98 + tr);
            s = (n0 + n1) / 2; sS[el][j] = S0[j] + s * S0[j];
        }
        const double sr = cfg(S, C_SHIFT, ee);
        for (int j = tl; j < 42; j += TS) {
            const double v = -sr + (sr - (-sr)) * D(pI + 147 + j);
            sShift[el][j] = v;
            S.shift[(size_t)j * N + e] = v;
        }
    }
    __syncthreads();
    if (on) {
        for (int k = tl; k < NSYM; k += TS) { // the upper-triangle non-zeros of D and S
            int r = 0, c = 0;
#pragma unroll
            for (int q = 0; q < NSYM; ++q)
                if (q == k) { r = SYM_R[q]; c = SYM_C[q]; }
            S.dnz[(size_t)k * N + e] = sD[el][r * 7 + c];
            S.snz[(size_t)k * N + e] = sS[el][r * 7 + c];
        }
        if (tl == 0) {
            double a3[9], i3[9], a4[16], i4[16];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) a3[i * 3 + j] = sI[el][B1[i] * 7 + B1[j]];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) a4[i * 4 + j] = sI[el][B2[i] * 7 + B2[j]];
            invert<3>(a3, i3);
            invert<4>(a4, i4);
            for (int i = 0; i < 3; ++i)
                for (int j = i; j < 3; ++j) sInv[el][B1U[i][j]] = i3[i * 3 + j];
            for (int i = 0; i < 4; ++i)
                for (int j = i; j < 4; ++j) sInv[el][B2U[i][j]] = i4[i * 4 + j];
        }
    }
    __syncthreads();
    if (!on) return;
    for (int k = tl; k < NINV; k += TS) S.iinv[(size_t)k * N + e] = sInv[el][k];
    if (tl != 0) return;
    // ---- actuator force scale (:216-217) --------------------------------
    const double ar = cfg(S, C_ACTR, e), lo = 1 - ar, hi = 1 + ar;
    const double maxS = cfg(S, C_MAXS0, e) * (lo + (hi - lo) * D(pI + 189));
    const double maxE = cfg(S, C_MAXE0, e) * (lo + (hi - lo) * D(pI + 190));
    S.maxSE[e] = maxS;
    S.maxSE[(size_t)N + e] = maxE;
    S.counts[e] = 2;
    S.episode[e] = ep + 1;

    // ---- reset observation (:229-254).  No stepSimulation in between, so
    // both reads see the same physics state; prev_position_vectors uses the
    // reference positions cached by the previous read.
    double q[5], act[14][3], ref[6], refc[6];
#pragma unroll
    for (int j = 0; j < 5; ++j) q[j] = S.phys_q[(size_t)j * N + e];
#pragma unroll
    for (int j = 0; j < 6; ++j) refc[j] = S.ref[(size_t)j * N + e];
    link_coms(U, q, act, ref);
    float *o = obs ? obs + (size_t)e * OBS : nullptr;
    float ob[OBS];
#pragma unroll
    for (int i = 0; i < 14; ++i) ob[i] = 0.0f; // ep_state_values forces are zero at c-2, c-1
    const double tn[4] = {10, 10, 10, 5};
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) ob[14 + t * 4 + i] = (float)(sTrem[el][t][i] / tn[i]);
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double p = act[2 * j + 1][a] + sShift[el][(2 * j + 1) * 3 + a];
            const double rc = (j < 2) ? refc[3 + a] : refc[a];
            const double rn = (j < 2) ? ref[3 + a] : ref[a];
            ob[26 + j * 3 + a] = (float)(p - rc);
            const float pv = (float)(p - rn);
            ob[47 + j * 3 + a] = pv;
            S.posv[(size_t)(j * 3 + a) * N + e] = pv;
        }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        ob[68 + j] = (float)ref[j];
        ob[74 + j] = (float)ref[j];
        S.ref[(size_t)j * N + e] = ref[j];
    }
    if (o) {
#pragma unroll
        for (int i = 0; i < OBS; i += 4) *reinterpret_cast<float4 *>(o + i) = make_float4(ob[i], ob[i + 1], ob[i + 2], ob[i + 3]);
    }
}

// bulk resets (exo_reset, exo_reset_from_draws; Exoskeleton_env.py:473-478 ->
// initialize_movement, :193-254): 16 envs per 256-thread workgroup -- every
// env (slot = env index; mask: those set), or the n listed envs with their
// injected draw streams
constexpr int RESET_EPW = 16, RESET_TS = 32;
__global__ __launch_bounds__(RESET_EPW *RESET_TS) void exo_reset_kernel(Dev S, Urdf U, const uint8_t *mask,
                                                                        const int32_t *ids, int n,
                                                                        const double *draws, int draw_stride,
                                                                        uint64_t seed, float *obs) {
    const int slot = blockIdx.x * RESET_EPW + (int)threadIdx.x % RESET_EPW;
    int e = -1;
    if (ids) {
        if (slot < n) e = ids[slot];
    } else if (slot < S.N && !(mask && !mask[slot])) {
        e = slot;
    }
    reset_group<RESET_EPW, RESET_TS>(S, U, e, draws && slot < n ? draws + (size_t)slot * draw_stride : nullptr,
                                     seed, obs);
}

// the envs listed in ids[0 .. *n_ids) (exo_episode_advance's compacted list,
// a dozen envs per iteration at 4,096 envs): one wavefront per env as the
// latency of a short list wants, a small fixed grid, each wavefront taking
// every gridDim.x-th listed env
__global__ __launch_bounds__(64) void exo_reset_list_kernel(Dev S, Urdf U, const int32_t *ids,
                                                            const int32_t *n_ids, uint64_t seed, float *obs) {
    const int n = *n_ids;
    for (int k = blockIdx.x; k < n; k += gridDim.x) reset_group<1, 64>(S, U, ids[k], nullptr, seed, obs);
}

// ---------------------------------------------------------------------------
// step (Exoskeleton_env.py:368-471).  Thread pair per env.  Everything the
// step returns except the joint-angle part of `info` depends only on the
// physics state read at the start of the step (the observation never sees the
// ODE result), so role 0 finishes observation, reward, done and the carried
// state BEFORE the solves; only the joint targets / motor update (role 0) and
// the two `ampl` info blocks need the ODE.  That keeps the epilogue out of the
// register budget of the RK45 loop.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void exo_step_kernel(Dev S, Urdf U, const float *__restrict__ act,
                                                       float *__restrict__ obs, float *__restrict__ rew,
                                                       uint8_t *__restrict__ done, float *__restrict__ info,
                                                       const uint8_t *__restrict__ active) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int e = gid >> 1, role = gid & 1;
    if (e >= S.N) return;
    const int N = S.N, c = S.counts[e], L = S.L[e];
    if ((active && !active[e]) || c >= L - 1) return; // both lanes of the pair agree

    double T[7];
    {
        const double maxS = S.maxSE[e], maxE = S.maxSE[(size_t)N + e];
        // transform_action (:256-266)
        double F[7];
        const float *a = act + (size_t)e * ACT;
#pragma unroll
        for (int j = 0; j < 7; ++j) F[j] = (((double)a[j] + 1) / 2) * (j < 2 ? maxE : maxS);
        // link reads of the state left by the last stepSimulation
        double q[5], ak[14][3], refn[6], refo[6];
#pragma unroll
        for (int j = 0; j < 5; ++j) q[j] = S.phys_q[(size_t)j * N + e];
#pragma unroll
        for (int j = 0; j < 6; ++j) refo[j] = S.ref[(size_t)j * N + e];
        if (S.mb_q) { // multibody mode: the k-links sit at their prismatic joint positions
            double qp[14];
#pragma unroll
            for (int j = 0; j < 14; ++j) qp[j] = S.mb_q[(size_t)(5 + j) * N + e];
            link_coms(U, q, ak, refn, qp);
        } else {
            link_coms(U, q, ak, refn);
        }
#pragma unroll
        for (int k = 0; k < 14; ++k)
#pragma unroll
            for (int a3 = 0; a3 < 3; ++a3) ak[k][a3] += S.shift[(size_t)(k * 3 + a3) * N + e];

        // get_force_components (sim:207-298) and get_torques (:177-187)
        double tau[7][3];
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const double *k1 = ak[2 * j], *k2 = ak[2 * j + 1];
            const double dx = (k2[0] + 5) - (k1[0] + 5), dy = (k2[1] + 5) - (k1[1] + 5), dz = (k2[2] + 5) - (k1[2] + 5);
            const double fx = cos_atan2(dy, dx) * F[j], fy = cos_atan2(dx, dy) * F[j], fz = cos_atan2(dz, dx) * F[j];
            const double *rn = (j < 2) ? &refn[3] : &refn[0];
            const double r0 = rn[0] - k2[0], r1 = rn[1] - k2[1], r2 = rn[2] - k2[2];
            tau[j][0] = fy * r2 - fz * r1; // np.cross(F, r)
            tau[j][1] = fz * r0 - fx * r2;
            tau[j][2] = fx * r1 - fy * r0;
        }
        // :394-400, summed in the reference's actuator order 3, 4, 5, 7, 6
        double at[4];
        at[0] = tau[2][1] + tau[3][1] + tau[4][1] + tau[6][1] + tau[5][1];
        at[1] = tau[2][0] + tau[3][0] + tau[4][0] + tau[6][0] + tau[5][0];
        at[2] = tau[2][2] + tau[3][2] + tau[4][2] + tau[6][2] + tau[5][2];
        at[3] = fabs(tau[0][1]) - fabs(tau[1][1]);

        double tr[7], Ta[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            tr[j] = S.tremor[((size_t)c * 7 + j) * N + e];
            Ta[j] = tr[j] + (j < 4 ? at[j] : 0.0); // :406
            T[j] = role == 0 ? Ta[j] : tr[j];
        }

        if (role == 0) {
            // get_reward (:268-366)
            const int seq = S.seq[e];
            const double eps = 1e-10, Msum = maxE + maxS, naxes = cfg(S, C_NAXES, e);
            double pa[7], pa2[7];
#pragma unroll
            for (int j = 0; j < 7; ++j) { pa[j] = S.prev_a[(size_t)j * N + e]; pa2[j] = S.prev2_a[(size_t)j * N + e]; }
            double unw = 0.0, st = 0.0;
            int nred = 0;
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                const double Tabs = fabs(Ta[j]), tabs = fabs(tr[j]);
                if (j < 4) {
                    if ((seq >> j) & 1) st += (Tabs - tabs) / tabs + 1;
                    else unw += Tabs;
                }
                const double v = (Tabs - tabs) / (tabs + eps) * 100;
                if (isfinite(v) && v < 0) nred++; // nan_to_num then "< 0"
            }
            const double r_unw = exp(-(unw / (Msum / 4 / naxes)) + eps) * 0.5;
            const double r_tor = exp((-st + eps) / naxes) * 0.9;
            const double r_axis = nred * 0.5;
            double sa = 0.0, sm = 0.0;
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                sa += F[j];
                const double d = F[j] - 2 * pa[j] + pa2[j];
                sm += d * d;
            }
            sm /= 7;
            const double r_ctl = exp(-(sa / (Msum / 2)) + eps) * 0.05;
            const double r_sm = 0.05 * exp(-(sm / (Msum / 4)) + eps);
            rew[e] = (float)((r_axis + r_tor + r_sm + r_ctl + r_unw) / cfg(S, C_MAXREW, e));
            done[e] = (uint8_t)(c + 1 >= L - 1); // :457-458

            // update_state_vector (:487-570) with counts = c + 1
            float ob[OBS];
            const double maxS0 = cfg(S, C_MAXS0, e), maxE0 = cfg(S, C_MAXE0, e);
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                const double nrm = j < 2 ? maxE0 : maxS0;
                ob[j] = (float)((c > 2 ? pa[j] : 0.0) / nrm); // ep_state_values[c-1] is 0 on the first step
                ob[7 + j] = (float)(F[j] / nrm);
            }
            const double tn[4] = {10, 10, 10, 5};
#pragma unroll
            for (int b = 0; b < 3; ++b)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const double v = (b == 1) ? tr[i] : S.tremor[((size_t)(c - 1 + b) * 7 + i) * N + e];
                    ob[14 + b * 4 + i] = (float)(v / tn[i]);
                }
#pragma unroll
            for (int j = 0; j < 7; ++j)
#pragma unroll
                for (int a3 = 0; a3 < 3; ++a3) {
                    const int i = j * 3 + a3;
                    // get_actuator_pos_vect uses the reference positions cached by the previous read (sim:300-336)
                    const float p = (float)(ak[2 * j + 1][a3] - (j < 2 ? refo[3 + a3] : refo[a3]));
                    ob[26 + i] = S.posv[(size_t)i * N + e];
                    ob[47 + i] = p;
                    S.posv[(size_t)i * N + e] = p;
                }
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                ob[68 + j] = (float)refo[j];
                ob[74 + j] = (float)refn[j];
                S.ref[(size_t)j * N + e] = refn[j];
            }
            float *o = obs + (size_t)e * OBS;
#pragma unroll
            for (int i = 0; i < OBS; i += 4) *reinterpret_cast<float4 *>(o + i) = make_float4(ob[i], ob[i + 1], ob[i + 2], ob[i + 3]);
            if (info) {
                float *io = info + (size_t)e * INFO;
#pragma unroll
                for (int j = 0; j < 7; ++j) {
                    io[j] = (float)(j < 4 ? at[j] : 0.0);
                    io[7 + j] = (float)Ta[j];
                    io[21 + j] = (float)tr[j];
                }
                io[35] = (float)r_unw; io[36] = (float)r_tor; io[37] = (float)r_axis; io[38] = (float)r_ctl;
                io[39] = (float)r_sm;
            }
            S.counts[e] = c + 1;
#pragma unroll
            for (int j = 0; j < 7; ++j) { S.prev2_a[(size_t)j * N + e] = pa[j]; S.prev_a[(size_t)j * N + e] = F[j]; }
        }
    }

    // ---- the two joint ODE solves (:409-414) ------------------------------
    OdeM M;
#pragma unroll
    for (int k = 0; k < NINV; ++k) M.ii[k] = S.iinv[(size_t)k * N + e];
#pragma unroll
    for (int k = 0; k < NSYM; ++k) { M.dn[k] = S.dnz[(size_t)k * N + e]; M.sn[k] = S.snz[(size_t)k * N + e]; }
    double qs[7];
    if (!rk45_solve(M, T, qs)) atomicOr(S.err, 1);
    const double r2d = 180 / PI, d2r = PI / 180;
#pragma unroll
    for (int j = 0; j < 7; ++j) qs[j] *= r2d; // :417-418
    if (info) {
        float *io = info + (size_t)e * INFO + (role == 0 ? 14 : 28); // ampl_val / tremor_ampl_val
#pragma unroll
        for (int j = 0; j < 7; ++j) io[j] = (float)qs[j];
    }
    if (role != 0) return;
    // :421-433 joint targets, then the motors move (idealised Bullet)
    const double *imu = S.imu + (size_t)S.motion[e] * 5 * S.Lmax;
    const double ang[4] = {imu[4 * S.Lmax + c] + qs[2], imu[3 * S.Lmax + c] + qs[0], imu[2 * S.Lmax + c] + qs[1],
                           imu[0 * S.Lmax + c] + qs[3]}; // shoulder z, y, x, elbow y (deg)
    const double tgt[5] = {ang[0] * d2r, ang[1] * d2r, ang[2] * d2r, ang[3] * d2r, imu[1 * S.Lmax + c] * d2r};
    // check_movement_boundaries (:594-605) prints; the build counts the steps with a violation
    if (!(-80 < ang[0] && ang[0] < 80) || !(-40 < ang[1] && ang[1] < 160.5) || !(-151.5 < ang[2] && ang[2] < 33.5) ||
        !(-10 < ang[3] && ang[3] < 150))
        S.viol[e] += 1;
    if (S.mb_tgt) { // multibody mode: exo_multibody_kernel runs stepSimulation next
#pragma unroll
        for (int j = 0; j < 5; ++j) S.mb_tgt[(size_t)j * N + e] = tgt[j];
        S.mb_flag[e] = 1;
        return;
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const double q0 = S.phys_q[(size_t)j * N + e];
        const double nq = q0 + 0.1 * (tgt[j] - q0);
        S.phys_q[(size_t)j * N + e] = fmin(fmax(nq, U.lo[j]), U.hi[j]);
    }
}

} // namespace

// ===========================================================================
// C ABI
// ===========================================================================

// ---------------------------------------------------------------- metrics
// Tremor-suppression statistics of the training script
// (Simulation/Exoskeleton_agent_train.py:149-200) for every env the last step
// advanced, from its info row, on the device.  Per env: the per-axis torque
// and amplitude reductions (percent, nan_to_num), the end-effector amplitude
// change from Denavit-Hartenberg FK of the IMU angles with the suppressed and
// the unsuppressed tremor amplitudes added (Utilities/
// calculate_arm_end_effector_points.py:18-50), and the script's counters.
__device__ void dh_end_effector(const double th[7], double L1, double L2, double out[3]) {
    // A_i(alpha, a = 0, d, theta): alpha = (pi/2, pi/2, -pi/2, pi/2, pi/2, pi/2, pi/2), d = (0, 0, L1, 0, L2, 0, 0)
    const double alpha[7] = {PI / 2, PI / 2, -PI / 2, PI / 2, PI / 2, PI / 2, PI / 2};
    const double d[7] = {0, 0, L1, 0, L2, 0, 0};
    double T[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0}; // rows 0..2 of the running 4x4 product
    for (int k = 0; k < 7; ++k) {
        const double ct = cos(th[k]), st = sin(th[k]), ca = cos(alpha[k]), sa = sin(alpha[k]);
        const double A[12] = {ct, -st * ca, st * sa, 0.0, st, ct * ca, -ct * sa, 0.0, 0.0, sa, ca, d[k]};
        double R[12];
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 4; ++j) {
                double v = T[i * 4 + 0] * A[0 * 4 + j] + T[i * 4 + 1] * A[1 * 4 + j] + T[i * 4 + 2] * A[2 * 4 + j];
                if (j == 3) v += T[i * 4 + 3];
                R[i * 4 + j] = v;
            }
        }
        for (int i = 0; i < 12; ++i) T[i] = R[i];
    }
    out[0] = T[3];
    out[1] = T[7];
    out[2] = T[11];
}

__device__ __forceinline__ double pct_change(double v, double ref) { // nan_to_num((|v|-|ref|)/|ref|*100, 0, 0, 0)
    const double x = (fabs(v) - fabs(ref)) / fabs(ref) * 100.0;
    return isfinite(x) ? x : 0.0;
}

// 8 lanes per env (r04; one thread per env before: 27 us per 4,096-env launch,
// 16 workgroups, three serial DH chains of 7 fp64 sincos each per thread).
// Lane j < 7 owns joint j: its two percent changes and the sines and cosines
// of its angle in the three DH chains; lanes 0, 1, 2 then each multiply one
// chain (the same expressions in the same order as dh_end_effector, the sines
// and cosines fetched by shuffles) and lane 0 finishes the env.  Bit-identical
// to the per-thread form.
constexpr int TM_LANES = 8;
__device__ __forceinline__ double shfl8(double v, int src) { return __shfl(v, src, TM_LANES); }

__global__ __launch_bounds__(256) void tremor_metrics_kernel(Dev S, const float *__restrict__ info,
                                                             const uint8_t *__restrict__ stepped, double L1, double L2,
                                                             int disregard, float *__restrict__ metrics,
                                                             float *__restrict__ counters) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int e = g / TM_LANES, j = g % TM_LANES;
    if (e >= S.N) return;  // uniform over the env's 8 lanes
    float *m = metrics + (size_t)e * 16;
    if (stepped && !stepped[e]) {  // a done env's row of the step is zeros (:201-203); counters untouched
        if (j < 4) reinterpret_cast<float4 *>(m)[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    const float *in = info + (size_t)e * INFO;
    const int jj = j < 7 ? j : 6;  // lane 7 mirrors joint 6 (its values unused)
    double tr = pct_change(in[7 + jj], in[21 + jj]);   // torque_val vs tremor_torque_val
    double ta = pct_change(in[14 + jj], in[28 + jj]);  // ampl_val vs tremor_ampl_val
    // return_original_joint_angles at the post-step count: x, y, z, elbow y, elbow z, 0, 0 (degrees)
    const int cnt = S.counts[e];
    const double *imu = S.imu + (size_t)S.motion[e] * 5 * S.Lmax;
    const int colj = jj == 0 ? 2 : jj == 1 ? 3 : jj == 2 ? 4 : jj == 3 ? 0 : 1;
    const double o = jj < 5 ? imu[colj * S.Lmax + cnt] * (PI / 180) : 0.0;
    const double th0 = o, th1 = (double)in[14 + jj] * (PI / 180) + o, th2 = (double)in[28 + jj] * (PI / 180) + o;
    const double c0 = cos(th0), s0 = sin(th0), c1 = cos(th1), s1 = sin(th1), c2 = cos(th2), s2 = sin(th2);
    // lanes 0 / 1 / 2: the chain of q0 / q1 / q2 (dh_end_effector)
    const int base = threadIdx.x & ~(TM_LANES - 1);
    const double alpha[7] = {PI / 2, PI / 2, -PI / 2, PI / 2, PI / 2, PI / 2, PI / 2};
    const double d[7] = {0, 0, L1, 0, L2, 0, 0};
    double T[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const double ck0 = shfl8(c0, k), sk0 = shfl8(s0, k), ck1 = shfl8(c1, k), sk1 = shfl8(s1, k);
        const double ck2 = shfl8(c2, k), sk2 = shfl8(s2, k);
        const double ct = j == 0 ? ck0 : j == 1 ? ck1 : ck2, st = j == 0 ? sk0 : j == 1 ? sk1 : sk2;
        const double ca = cos(alpha[k]), sa = sin(alpha[k]);
        const double A[12] = {ct, -st * ca, st * sa, 0.0, st, ct * ca, -ct * sa, 0.0, 0.0, sa, ca, d[k]};
        double R[12];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                double v = T[i * 4 + 0] * A[0 * 4 + c] + T[i * 4 + 1] * A[1 * 4 + c] + T[i * 4 + 2] * A[2 * 4 + c];
                if (c == 3) v += T[i * 4 + 3];
                R[i * 4 + c] = v;
            }
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) T[i] = R[i];
    }
    (void)base;
    const double px = T[3], py = T[7], pz = T[11];
    const double p0x = shfl8(px, 0), p0y = shfl8(py, 0), p0z = shfl8(pz, 0);
    const double p1x = shfl8(px, 1), p1y = shfl8(py, 1), p1z = shfl8(pz, 1);
    const double p2x = shfl8(px, 2), p2y = shfl8(py, 2), p2z = shfl8(pz, 2);
    // counters (before the disregard clamp, :172-184): torque reductions of axes 0..3
    int neg = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) neg += shfl8(tr, k) < 0 ? 1 : 0;
    if (disregard) { // :186-191
        if (tr > 0) tr = 0;
        if (ta > 0) ta = 0;
    }
    int nzc = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) nzc += shfl8(tr, k) != 0.0 ? 1 : 0;
    if (j < 7) {
        m[j] = (float)tr;
        m[7 + j] = (float)ta;
    }
    if (j != 0) return;
    const double ds = sqrt((p1x - p0x) * (p1x - p0x) + (p1y - p0y) * (p1y - p0y) + (p1z - p0z) * (p1z - p0z));
    const double du = sqrt((p2x - p0x) * (p2x - p0x) + (p2y - p0y) * (p2y - p0y) + (p2z - p0z) * (p2z - p0z));
    double total = (ds - du) / du * 100.0;
    float *cn = counters + (size_t)e * 6;
    cn[0] += 4 - neg;
    cn[1] += neg;
    if (neg > 0) cn[2] += 1;
    if (total < 0) {
        cn[4] += 1;
        cn[5] = (float)total;
    } else {
        cn[3] += 1;
    }
    if (disregard && total > 0) total = 0;
    m[14] = (float)total;
    m[15] = nzc ? 1.f : 0.f;
}

// Evaluation-script statistics (Simulation/Evaluate_control_performance.py:
// 192-260), which differ from the training script's in four places: the
// reductions divide by |ref + 1e-10| (:197, :201), the SFE/SAA amplitudes are
// swapped before the DH FK (:208-209), the torque counters look at the env's
// tremor axes only with <= 0 (:233-241: every axis suppressed / any axis
// suppressed), and the episode's total-amplitude mean runs over the negative
// values (:262, :414).  counters [N][5] accumulate: all-axes-suppressed steps,
// any-axis-suppressed steps, total < 0 steps, total >= 0 steps, sum of the
// negative totals.
__global__ void eval_metrics_kernel(Dev S, const float *__restrict__ info, const uint8_t *__restrict__ stepped,
                                    double L1, double L2, float *__restrict__ counters) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= S.N || (stepped && !stepped[e])) return;
    const float *in = info + (size_t)e * INFO;
    const int seq = S.seq[e];
    bool all_sup = true, any_sup = false;
    for (int j = 0; j < 7; ++j) {
        if (!((seq >> j) & 1)) continue;
        const double ref = in[21 + j];
        double tr = (fabs((double)in[7 + j]) - fabs(ref)) / fabs(ref + 1e-10) * 100.0;
        if (!isfinite(tr)) tr = 0.0;
        all_sup &= tr <= 0.0;
        any_sup |= tr <= 0.0;
    }
    const int cnt = S.counts[e];
    const double *imu = S.imu + (size_t)S.motion[e] * 5 * S.Lmax;
    const int col[5] = {2, 3, 4, 0, 1};
    double q0[7], q1[7], q2[7];
    for (int j = 0; j < 7; ++j) {
        const int js = j == 0 ? 1 : (j == 1 ? 0 : j);  // amplitudes with axes 0 / 1 swapped
        const double o = j < 5 ? imu[col[j] * S.Lmax + cnt] * (PI / 180) : 0.0;
        q0[j] = o;
        q1[j] = (double)in[14 + js] * (PI / 180) + o;
        q2[j] = (double)in[28 + js] * (PI / 180) + o;
    }
    double p0[3], p1[3], p2[3];
    dh_end_effector(q0, L1, L2, p0);
    dh_end_effector(q1, L1, L2, p1);
    dh_end_effector(q2, L1, L2, p2);
    const double ds = sqrt((p1[0] - p0[0]) * (p1[0] - p0[0]) + (p1[1] - p0[1]) * (p1[1] - p0[1]) +
                           (p1[2] - p0[2]) * (p1[2] - p0[2]));
    const double du = sqrt((p2[0] - p0[0]) * (p2[0] - p0[0]) + (p2[1] - p0[1]) * (p2[1] - p0[1]) +
                           (p2[2] - p0[2]) * (p2[2] - p0[2]));
    const double total = (ds - du) / du * 100.0;
    float *cn = counters + (size_t)e * 5;
    if (all_sup) cn[0] += 1;
    if (any_sup) cn[1] += 1;
    if (total < 0) {
        cn[2] += 1;
        cn[4] += (float)total;
    } else {
        cn[3] += 1;
    }
}

// The synchronous-episode trainer's active mask (Simulation/Exoskeleton_agent_
// train.py:123-125: an env steps while its motion lasts): the step counter k
// (device int64) advances by one, saturating at rows - 1, and row k of the
// [rows][n] table is copied to active -- one single-workgroup launch inside
// the captured iteration, safe however many times a graph is replayed.  With
// score != nullptr the step's episode scores are accumulated first from the
// mask being replaced (:144, score += reward where the env stepped: float32
// reward into the float64 score, the value torch's where + add_ produce).
__global__ __launch_bounds__(1024) void active_advance_kernel(const uint8_t *__restrict__ table, int rows, int n,
                                                              long long *k, uint8_t *__restrict__ active,
                                                              int32_t *count, const float *__restrict__ rew,
                                                              double *__restrict__ score) {
    __shared__ int wsum[16];
    const long long k0 = *k;
    const long long kk = k0 + 1 < rows ? k0 + 1 : rows - 1;
    int c = 0;
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
        const uint8_t v = table[(size_t)kk * n + e];
        if (score) score[e] += active[e] ? (double)rew[e] : 0.0;
        active[e] = v;
        c += v != 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        *k = kk;
        if (count) {
            int t = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += wsum[w];
            *count = t;
        }
    }
}

struct exo_ctx {
    int device = 0;
    int N = 0, n_motions = 0, Lmax = 0;
    uint64_t seed = 0;
    Dev S{};
    Urdf U{};
    std::vector<int32_t> L_host, motion_host;
    std::vector<double> imu_host;
    std::vector<void *> allocs;
    float *obs_scratch = nullptr;
    int step_variant = EXO_STEP_AUTO;
    int physics = EXO_PHYS_IDEAL;
    MbModel mb{};
    double *mb_q = nullptr, *mb_qd = nullptr, *mb_tgt = nullptr;
    uint8_t *mb_flag = nullptr;
    unsigned long long *step_clock = nullptr; // exo_set_step_clock
    std::string err;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
        else prev = -1;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int fail(exo_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

int check(exo_ctx *c, hipError_t e, const char *what) {
    if (e == hipSuccess) return EXO_OK;
    return fail(c, EXO_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
T *dalloc(exo_ctx *c, size_t n) {
    void *p = nullptr;
    if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) return nullptr;
    (void)hipMemset(p, 0, n * sizeof(T));
    c->allocs.push_back(p);
    return static_cast<T *>(p);
}

} // namespace

namespace {
template <class T>
int read1(exo_ctx *c, const T *base, size_t idx, T *out) {
    return check(c, hipMemcpy(out, base + idx, sizeof(T), hipMemcpyDeviceToHost), "read-back");
}
template <class T>
int write1(exo_ctx *c, T *base, size_t idx, T v) {
    return check(c, hipMemcpy(base + idx, &v, sizeof(T), hipMemcpyHostToDevice), "write");
}
} // namespace

extern "C" {

int exo_create(const exo_env_config *cfgs, int32_t n_envs, const double *motion_angles, const int32_t *motion_lengths,
               int32_t n_motions, int32_t max_len, uint64_t seed, int32_t device, exo_ctx **out) {
    if (!out || !cfgs || !motion_angles || !motion_lengths || n_envs <= 0 || n_motions <= 0 || max_len <= 2 ||
        max_len > MAX_L)
        return EXO_EINVAL;
    *out = nullptr;
    for (int m = 0; m < n_motions; ++m)
        if (motion_lengths[m] < 4 || motion_lengths[m] > max_len) return EXO_EINVAL;
    std::vector<double> cfg((size_t)C_COUNT * n_envs);
    std::vector<int32_t> seq(n_envs), L(n_envs), mot(n_envs);
    for (int e = 0; e < n_envs; ++e) {
        const exo_env_config &c = cfgs[e];
        if (c.motion < 0 || c.motion >= n_motions) return EXO_EINVAL;
        int bits = 0, n = 0;
        for (int i = 0; i < 7; ++i) {
            if (c.tremor_sequence[i] != 0 && c.tremor_sequence[i] != 1) return EXO_EINVAL;
            bits |= c.tremor_sequence[i] << i;
            n += c.tremor_sequence[i];
        }
        if (n == 0) return EXO_EINVAL; // reward divides by the tremor axis count (:320, :337)
        seq[e] = bits;
        mot[e] = c.motion;
        L[e] = motion_lengths[c.motion];
        const double v[C_COUNT] = {c.tremor_amplitude_range[0], c.tremor_amplitude_range[1],
                                   c.first_harmonics_interval[0], c.first_harmonics_interval[1],
                                   c.second_harmonics_interval[0], c.second_harmonics_interval[1],
                                   c.max_force_shoulder, c.max_force_elbow, c.dr_actuator_end_pos_shift,
                                   c.dr_actuator_range, c.matrix_noise_fraction,
                                   n * 0.5 + 0.9 + 0.05 + 0.05 + 0.5, (double)n}; // max_reward :167-169
        for (int k = 0; k < C_COUNT; ++k) cfg[(size_t)k * n_envs + e] = v[k];
    }
    exo_ctx *c = new exo_ctx();
    c->device = device;
    c->N = n_envs;
    c->n_motions = n_motions;
    c->Lmax = max_len;
    c->seed = seed;
    c->L_host = L;
    c->motion_host = mot;
    c->imu_host.assign(motion_angles, motion_angles + (size_t)n_motions * 5 * max_len);
    build_urdf(c->U);
    DeviceGuard g(device);
    const size_t N = n_envs;
    Dev &S = c->S;
    S.N = n_envs; S.n_motions = n_motions; S.Lmax = max_len;
    int32_t *motion_d = dalloc<int32_t>(c, N), *L_d = dalloc<int32_t>(c, N), *seq_d = dalloc<int32_t>(c, N);
    double *cfg_d = dalloc<double>(c, cfg.size()), *imu_d = dalloc<double>(c, c->imu_host.size());
    S.tremor = dalloc<double>(c, (size_t)max_len * 7 * N);
    S.iinv = dalloc<double>(c, NINV * N);
    S.dnz = dalloc<double>(c, NSYM * N);
    S.snz = dalloc<double>(c, NSYM * N);
    S.shift = dalloc<double>(c, 42 * N);
    S.maxSE = dalloc<double>(c, 2 * N);
    S.episode = dalloc<uint32_t>(c, N);
    S.counts = dalloc<int32_t>(c, N);
    S.phys_q = dalloc<double>(c, 5 * N);
    S.ref = dalloc<double>(c, 6 * N);
    S.posv = dalloc<float>(c, 21 * N);
    S.prev_a = dalloc<double>(c, 7 * N);
    S.prev2_a = dalloc<double>(c, 7 * N);
    S.err = dalloc<int32_t>(c, 1);
    S.viol = dalloc<int32_t>(c, N);
    c->obs_scratch = dalloc<float>(c, N * OBS);
    for (void *p : c->allocs)
        if (!p) { exo_destroy(c); return EXO_ENOMEM; }
    if (!motion_d || !L_d || !seq_d || !cfg_d || !imu_d || !S.tremor || !S.iinv ||
        !S.dnz || !S.snz || !S.shift || !S.maxSE || !S.episode || !S.counts || !S.phys_q || !S.ref || !S.posv ||
        !S.prev_a || !S.prev2_a || !S.err || !S.viol || !c->obs_scratch) {
        exo_destroy(c);
        return EXO_ENOMEM;
    }
    S.motion = motion_d; S.L = L_d; S.seq = seq_d; S.cfg = cfg_d; S.imu = imu_d;
    exo_set_tremor_model(c, nullptr, EXO_TREMOR_SIGN_PER_SAMPLE); // the shipped tremor (generate_parkinson_tremor.py:59, :70)
    hipError_t e = hipMemcpy(motion_d, mot.data(), N * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(L_d, L.data(), N * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(seq_d, seq.data(), N * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(cfg_d, cfg.data(), cfg.size() * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(imu_d, c->imu_host.data(), c->imu_host.size() * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) { exo_destroy(c); return EXO_EDEVICE; }
    // the constructor runs initialize_movement() once (Exoskeleton_env.py:172)
    int rc = exo_reset(c, nullptr, c->obs_scratch, nullptr);
    if (rc == EXO_OK) rc = check(c, hipDeviceSynchronize(), "exo_create");
    if (rc != EXO_OK) { exo_destroy(c); return rc; }
    *out = c;
    return EXO_OK;
}

int exo_reset(exo_ctx *c, const uint8_t *mask_dev, float *obs_dev, void *stream) {
    if (!c) return EXO_EINVAL;
    DeviceGuard g(c->device);
    hipLaunchKernelGGL(exo_reset_kernel, dim3((c->N + RESET_EPW - 1) / RESET_EPW), dim3(RESET_EPW * RESET_TS), 0,
                       (hipStream_t)stream, c->S, c->U, mask_dev, (const int32_t *)nullptr, 0,
                       (const double *)nullptr, 0, c->seed, obs_dev);
    return check(c, hipGetLastError(), "exo_reset");
}

int exo_reset_from_draws(exo_ctx *c, const int32_t *env_ids_host, int32_t n, const double *draws_host, float *obs_dev,
                         void *stream) {
    if (!c || !env_ids_host || !draws_host || n <= 0) return EXO_EINVAL;
    for (int k = 0; k < n; ++k)
        if (env_ids_host[k] < 0 || env_ids_host[k] >= c->N) return fail(c, EXO_EINVAL, "env id out of range");
    DeviceGuard g(c->device);
    const int stride = EXO_DRAWS_PER_EPISODE(c->Lmax);
    int32_t *ids = nullptr;
    double *dr = nullptr;
    if (hipMalloc(&ids, n * 4) != hipSuccess || hipMalloc(&dr, (size_t)n * stride * 8) != hipSuccess) {
        (void)hipFree(ids);
        return fail(c, EXO_ENOMEM, "exo_reset_from_draws: out of memory");
    }
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemcpyAsync(ids, env_ids_host, n * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dr, draws_host, (size_t)n * stride * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(exo_reset_kernel, dim3((n + RESET_EPW - 1) / RESET_EPW), dim3(RESET_EPW * RESET_TS), 0,
                           s, c->S, c->U, (const uint8_t *)nullptr, ids, n, dr, stride, c->seed, obs_dev);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(ids);
    (void)hipFree(dr);
    return check(c, e, "exo_reset_from_draws");
}

// The step clock (exo_set_step_clock): one-lane kernels on the step's stream
// either side of the step launch read the 100 MHz wall clock; the second adds
// the interval to clk[1] and counts it in clk[2].  Stream order makes them
// bracket the step kernel inside a captured graph as well as eagerly.
namespace {
__global__ void step_clock_kernel(unsigned long long *clk, int end) {
    const unsigned long long t = wall_clock64();
    if (!end) {
        clk[0] = t;
    } else {
        clk[1] += t - clk[0];
        clk[2] += 1;
    }
}
} // namespace

int exo_step(exo_ctx *c, const float *act_dev, float *obs_dev, float *rew_dev, uint8_t *done_dev, float *info_dev,
             const uint8_t *active_dev, void *stream) {
    return exo_step_carry(c, act_dev, obs_dev, rew_dev, done_dev, info_dev, active_dev, nullptr, stream);
}

namespace {
bool rows_variant(const exo_ctx *c) {
    return c->step_variant == EXO_STEP_ROWS_SHARED || c->step_variant == EXO_STEP_ROWS ||
           (c->step_variant == EXO_STEP_AUTO && c->N <= 16384);
}

__global__ __launch_bounds__(1024) void budget_advance_kernel(const int32_t *counts, const int32_t *L,
                                                              const uint8_t *pend, int n, uint8_t *active,
                                                              int32_t *count, int32_t *remaining,
                                                              long long *steps_total) {
    __shared__ int wsum[2][16];
    int a = 0, rem = 0;
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
        const bool run = counts[e] < L[e] - 1, p = pend[e] != 0;
        active[e] = run && !p;
        a += run && !p;
        rem += run || p;
    }
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        rem += __shfl_xor(rem, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        wsum[0][threadIdx.x >> 6] = a;
        wsum[1][threadIdx.x >> 6] = rem;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int ta = 0, tr = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            ta += wsum[0][w];
            tr += wsum[1][w];
        }
        if (steps_total) *steps_total += *count;  // the envs the last launch stepped
        *count = ta;
        *remaining = tr;
    }
}

// Auto-reset episodes (VecTrainer episodes="async"): an env whose episode is
// over (its done step was taken: counts >= L - 1) is reset (mask for
// exo_reset_kernel) once that step's solve is complete -- the final step's
// motor update sets joint state the reset keeps, so a budgeted final solve
// still pending finishes in later launches first -- and steps again in the
// next launch; every env without a pending solve steps.  count = the envs of
// the next launch, steps_total += the envs the last launch stepped.
__global__ __launch_bounds__(1024) void episode_advance_kernel(const int32_t *counts, const int32_t *L,
                                                               const uint8_t *pend, int n, uint8_t *active,
                                                               int32_t *count, int32_t *reset_ids,
                                                               long long *steps_total) {
    __shared__ int wsum[16];
    __shared__ int nres;
    if (threadIdx.x == 0) nres = 0;
    __syncthreads();
    int a = 0;
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
        const bool fin = counts[e] >= L[e] - 1, p = pend && pend[e] != 0;
        if (fin && !p) reset_ids[atomicAdd(&nres, 1)] = e;  // list order is immaterial: resets are per env
        const bool run = !p;
        active[e] = run;
        a += run;
    }
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        int ta = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) ta += wsum[w];
        if (steps_total) *steps_total += *count;
        *count = ta;
        reset_ids[n] = nres;
    }
}
} // namespace

int exo_set_step_budget(exo_ctx *c, int32_t budget) {
    if (!c || budget < 0) return EXO_EINVAL;
    DeviceGuard g(c->device);
    if (budget > 0 && (!rows_variant(c) || c->physics != EXO_PHYS_IDEAL))
        return fail(c, EXO_EINVAL, "exo_set_step_budget: row-parallel step kernels and idealised physics only");
    int rc = check(c, hipDeviceSynchronize(), "exo_set_step_budget");
    if (rc) return rc;
    if (budget == 0) {
        if (c->S.pend) {
            std::vector<uint8_t> p(c->N);
            rc = check(c, hipMemcpy(p.data(), c->S.pend, c->N, hipMemcpyDeviceToHost), "exo_set_step_budget");
            if (rc) return rc;
            for (uint8_t v : p)
                if (v) return fail(c, EXO_EINVAL, "exo_set_step_budget: a solve is still pending");
        }
        c->S.budget = 0;
        return EXO_OK;
    }
    if (!c->S.pend) {
        c->S.pend = dalloc<uint8_t>(c, c->N);
        c->S.rk = dalloc<double>(c, (size_t)RK_FIELDS * c->N);
        if (!c->S.pend || !c->S.rk) return fail(c, EXO_ENOMEM, "exo_set_step_budget: out of memory");
    }
    c->S.budget = budget;
    return EXO_OK;
}

int exo_budget_advance(exo_ctx *c, uint8_t *active_dev, int32_t *count_dev, int32_t *remaining_dev,
                       int64_t *steps_total_dev, void *stream) {
    if (!c || !active_dev || !count_dev || !remaining_dev) return EXO_EINVAL;
    if (!c->S.pend) return fail(c, EXO_EINVAL, "exo_budget_advance: no step budget set");
    DeviceGuard g(c->device);
    hipLaunchKernelGGL(budget_advance_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, c->S.counts, c->S.L,
                       c->S.pend, c->N, active_dev, count_dev, remaining_dev, (long long *)steps_total_dev);
    return check(c, hipGetLastError(), "exo_budget_advance");
}

int exo_episode_advance(exo_ctx *c, uint8_t *active_dev, int32_t *count_dev, int32_t *reset_ws_dev,
                        int64_t *steps_total_dev, float *obs_dev, void *stream) {
    if (!c || !active_dev || !count_dev || !reset_ws_dev || !obs_dev) return EXO_EINVAL;
    DeviceGuard g(c->device);
    const hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(episode_advance_kernel, dim3(1), dim3(1024), 0, s, c->S.counts, c->S.L, c->S.pend, c->N,
                       active_dev, count_dev, reset_ws_dev, (long long *)steps_total_dev);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {  // a few envs end per launch (N / episode length): 64 wavefronts cover them
        hipLaunchKernelGGL(exo_reset_list_kernel, dim3(std::min(c->N, 64)), dim3(64), 0, s, c->S, c->U, reset_ws_dev,
                           reset_ws_dev + c->N, c->seed, obs_dev);
        e = hipGetLastError();
    }
    return check(c, e, "exo_episode_advance");
}

int exo_step_carry(exo_ctx *c, const float *act_dev, float *obs_dev, float *rew_dev, uint8_t *done_dev,
                   float *info_dev, const uint8_t *active_dev, const float *obs_cur_dev, void *stream) {
    if (!c || !act_dev || !obs_dev || !rew_dev || !done_dev) return EXO_EINVAL;
    DeviceGuard g(c->device);
    const bool shared = c->step_variant == EXO_STEP_ROWS_SHARED;
    const bool rows = rows_variant(c);
    if (c->S.budget > 0 && (!rows || c->physics != EXO_PHYS_IDEAL))
        return fail(c, EXO_EINVAL, "exo_step: the step budget needs the row-parallel kernel and idealised physics");
    hipError_t e = hipSuccess;
    if (c->step_clock) {
        hipLaunchKernelGGL(step_clock_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, c->step_clock, 0);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
    } else if (rows) {
        e = launch_exo_step_rp(c->S, c->U, act_dev, obs_dev, rew_dev, done_dev, info_dev, active_dev,
                               (hipStream_t)stream, shared, obs_cur_dev);
    } else {
        const int threads = 256, lanes = 2 * c->N;
        hipLaunchKernelGGL(exo_step_kernel, dim3((lanes + threads - 1) / threads), dim3(threads), 0,
                           (hipStream_t)stream, c->S, c->U, act_dev, obs_dev, rew_dev, done_dev, info_dev, active_dev);
        e = hipGetLastError();
    }
    if (e == hipSuccess && c->physics == EXO_PHYS_MULTIBODY) // stepSimulation (:433) of the envs just stepped
        e = launch_exo_multibody(c->S, c->U, c->mb, c->S.mb_tgt, c->S.mb_flag, 1, (hipStream_t)stream);
    if (e == hipSuccess && c->step_clock) {
        hipLaunchKernelGGL(step_clock_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, c->step_clock, 1);
        e = hipGetLastError();
    }
    return check(c, e, "exo_step");
}

void exo_multibody_default_params(exo_mb_params *p) {
    if (!p) return;
    p->gravity = 9.81;               // Exoskeleton_env.py:116
    p->kp = 0.1;                     // setJointMotorControlArray defaults (sim:115-117)
    p->kd = 1.0;
    p->motor_impulse = 1e5 * DT;     // default force 1e5, x timestep
    p->passive_impulse = 1.0;        // pybullet's default joint velocity motors
    p->limit_impulse = 100.0;        // btMultiBodyConstraint default
    p->erp = 0.2;                    // btContactSolverInfo default
    p->lin_damp = 0.04;              // btMultiBody defaults
    p->ang_damp = 0.04;
    p->max_vel = 100.0;
    p->iters = 50;                   // pybullet default numSolverIterations
}

int exo_set_physics(exo_ctx *c, int32_t mode, const exo_mb_params *params) {
    if (!c || (mode != EXO_PHYS_IDEAL && mode != EXO_PHYS_MULTIBODY)) return EXO_EINVAL;
    if (mode == EXO_PHYS_MULTIBODY && c->S.budget > 0)
        return fail(c, EXO_EINVAL, "exo_set_physics: the step budget needs idealised physics");
    exo_mb_params p;
    exo_multibody_default_params(&p);
    if (params) p = *params;
    if (p.iters < 0 || p.iters > 100000 || !(p.motor_impulse >= 0) || !(p.passive_impulse >= 0) ||
        !(p.limit_impulse >= 0) || !(p.max_vel > 0))
        return fail(c, EXO_EINVAL, "exo_set_physics: invalid multibody parameters");
    DeviceGuard g(c->device);
    const size_t N = c->N;
    int rc = check(c, hipDeviceSynchronize(), "exo_set_physics");
    if (rc) return rc;
    if (mode == EXO_PHYS_IDEAL) {
        c->physics = mode;
        c->S.mb_q = c->S.mb_qd = c->S.mb_tgt = nullptr;
        c->S.mb_flag = nullptr;
        return EXO_OK;
    }
    if (!c->mb_q) {
        c->mb_q = dalloc<double>(c, NJ * N);
        c->mb_qd = dalloc<double>(c, NJ * N);
        c->mb_tgt = dalloc<double>(c, 5 * N);
        c->mb_flag = dalloc<uint8_t>(c, N);
        if (!c->mb_q || !c->mb_qd || !c->mb_tgt || !c->mb_flag) return fail(c, EXO_ENOMEM, "exo_set_physics: out of memory");
    }
    if (c->physics != EXO_PHYS_MULTIBODY) {
        // continue from the current arm pose at rest, k-links at their load position 0
        hipError_t e = hipMemset(c->mb_q, 0, NJ * N * sizeof(double));
        if (e == hipSuccess) e = hipMemset(c->mb_qd, 0, NJ * N * sizeof(double));
        if (e == hipSuccess) e = hipMemset(c->mb_flag, 0, N);
        if (e == hipSuccess) e = hipMemcpy(c->mb_q, c->S.phys_q, 5 * N * sizeof(double), hipMemcpyDeviceToDevice);
        if ((rc = check(c, e, "exo_set_physics"))) return rc;
    }
    build_mb_model(c->mb);
    c->mb.g = p.gravity; c->mb.kp = p.kp; c->mb.kd = p.kd; c->mb.motor_imp = p.motor_impulse;
    c->mb.passive_imp = p.passive_impulse; c->mb.limit_imp = p.limit_impulse; c->mb.erp = p.erp;
    c->mb.lin_damp = p.lin_damp; c->mb.ang_damp = p.ang_damp; c->mb.max_vel = p.max_vel; c->mb.iters = p.iters;
    c->S.mb_q = c->mb_q; c->S.mb_qd = c->mb_qd; c->S.mb_tgt = c->mb_tgt; c->S.mb_flag = c->mb_flag;
    c->physics = mode;
    return EXO_OK;
}

int exo_multibody_advance(exo_ctx *c, const double *targets_dev, const uint8_t *mask_dev, void *stream) {
    if (!c || !targets_dev) return EXO_EINVAL;
    if (c->physics != EXO_PHYS_MULTIBODY) return fail(c, EXO_EINVAL, "exo_multibody_advance: physics is not multibody");
    DeviceGuard g(c->device);
    return check(c, launch_exo_multibody(c->S, c->U, c->mb, targets_dev, const_cast<uint8_t *>(mask_dev), 0,
                                         (hipStream_t)stream), "exo_multibody_advance");
}

int exo_get_multibody_state_host(exo_ctx *c, int32_t env, double *q19, double *qd19) {
    if (!c || env < 0 || env >= c->N || !q19 || !qd19) return EXO_EINVAL;
    if (c->physics != EXO_PHYS_MULTIBODY) return fail(c, EXO_EINVAL, "physics is not multibody");
    DeviceGuard g(c->device);
    int rc = check(c, hipDeviceSynchronize(), "sync");
    for (int j = 0; j < NJ && !rc; ++j) rc = read1(c, (const double *)c->mb_q, (size_t)j * c->N + env, &q19[j]);
    for (int j = 0; j < NJ && !rc; ++j) rc = read1(c, (const double *)c->mb_qd, (size_t)j * c->N + env, &qd19[j]);
    return rc;
}

int exo_set_multibody_state_host(exo_ctx *c, int32_t env, const double *q19, const double *qd19) {
    if (!c || env < 0 || env >= c->N || !q19 || !qd19) return EXO_EINVAL;
    if (c->physics != EXO_PHYS_MULTIBODY) return fail(c, EXO_EINVAL, "physics is not multibody");
    DeviceGuard g(c->device);
    int rc = check(c, hipDeviceSynchronize(), "sync");
    for (int j = 0; j < NJ && !rc; ++j) rc = write1(c, c->mb_q, (size_t)j * c->N + env, q19[j]);
    for (int j = 0; j < NJ && !rc; ++j) rc = write1(c, c->mb_qd, (size_t)j * c->N + env, qd19[j]);
    for (int j = 0; j < 5 && !rc; ++j) rc = write1(c, c->S.phys_q, (size_t)j * c->N + env, q19[j]);
    return rc;
}

int32_t exo_num_envs(const exo_ctx *c) { return c ? c->N : 0; }

int exo_episode_length(const exo_ctx *c, int32_t env, int32_t *L_out) {
    if (!c || env < 0 || env >= c->N || !L_out) return EXO_EINVAL;
    *L_out = c->L_host[env];
    return EXO_OK;
}

int exo_tremor_host(exo_ctx *c, int32_t env, double *out) {
    if (!c || env < 0 || env >= c->N || !out) return EXO_EINVAL;
    DeviceGuard g(c->device);
    const int L = c->L_host[env];
    int rc = check(c, hipDeviceSynchronize(), "sync");
    // strided gather: [t][axis][env]
    std::vector<double> col((size_t)L * 7);
    for (int t = 0; t < L && rc == EXO_OK; ++t)
        for (int i = 0; i < 7 && rc == EXO_OK; ++i) rc = read1(c, (const double *)c->S.tremor, ((size_t)t * 7 + i) * c->N + env, &col[(size_t)i * L + t]);
    if (rc == EXO_OK) std::memcpy(out, col.data(), col.size() * 8);
    return rc;
}

int exo_original_joint_angles_host(exo_ctx *c, int32_t env, double *out7) {
    // return_original_joint_angles (:580-592): x, y, z, elbow y, elbow z, 0, 0 at counts
    if (!c || env < 0 || env >= c->N || !out7) return EXO_EINVAL;
    DeviceGuard g(c->device);
    int32_t cnt = 0;
    int rc = read1(c, (const int32_t *)c->S.counts, env, &cnt);
    if (rc) return rc;
    const double *imu = c->imu_host.data() + (size_t)c->motion_host[env] * 5 * c->Lmax;
    const int col[5] = {2, 3, 4, 0, 1};
    for (int k = 0; k < 5; ++k) out7[k] = imu[col[k] * c->Lmax + cnt];
    out7[5] = out7[6] = 0.0;
    return EXO_OK;
}

int exo_episode_host(exo_ctx *c, int32_t env, double *D49, double *S49, double *Iinv49, double *shift42, double *maxSE2) {
    if (!c || env < 0 || env >= c->N) return EXO_EINVAL;
    DeviceGuard g(c->device);
    int rc = check(c, hipDeviceSynchronize(), "sync");
    const size_t N = c->N;
    double dn[NSYM], sn[NSYM], ii[NINV];
    for (int k = 0; k < NSYM && !rc; ++k) rc = read1(c, (const double *)c->S.dnz, k * N + env, &dn[k]);
    for (int k = 0; k < NSYM && !rc; ++k) rc = read1(c, (const double *)c->S.snz, k * N + env, &sn[k]);
    for (int k = 0; k < NINV && !rc; ++k) rc = read1(c, (const double *)c->S.iinv, k * N + env, &ii[k]);
    if (rc) return rc;
    if (D49 || S49) {
        for (int k = 0; k < 49; ++k) { if (D49) D49[k] = 0; if (S49) S49[k] = 0; }
        for (int k = 0; k < NNZ; ++k) {
            if (D49) D49[NZ_R[k] * 7 + NZ_C[k]] = dn[NZ_U[k]];
            if (S49) S49[NZ_R[k] * 7 + NZ_C[k]] = sn[NZ_U[k]];
        }
    }
    if (Iinv49) {
        for (int k = 0; k < 49; ++k) Iinv49[k] = 0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Iinv49[B1[i] * 7 + B1[j]] = ii[B1U[i][j]];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) Iinv49[B2[i] * 7 + B2[j]] = ii[B2U[i][j]];
    }
    for (int k = 0; k < 42 && shift42 && !rc; ++k) rc = read1(c, (const double *)c->S.shift, k * N + env, &shift42[k]);
    for (int k = 0; k < 2 && maxSE2 && !rc; ++k) rc = read1(c, (const double *)c->S.maxSE, k * N + env, &maxSE2[k]);
    return rc;
}

int exo_get_state_host(exo_ctx *c, int32_t env, double *out) {
    if (!c || env < 0 || env >= c->N || !out) return EXO_EINVAL;
    DeviceGuard g(c->device);
    int rc = check(c, hipDeviceSynchronize(), "sync");
    const size_t N = c->N;
    int32_t cnt = 0;
    uint32_t ep = 0;
    if (!rc) rc = read1(c, (const int32_t *)c->S.counts, env, &cnt);
    if (!rc) rc = read1(c, (const uint32_t *)c->S.episode, env, &ep);
    out[0] = cnt;
    for (int j = 0; j < 5 && !rc; ++j) rc = read1(c, (const double *)c->S.phys_q, j * N + env, &out[1 + j]);
    for (int j = 0; j < 6 && !rc; ++j) rc = read1(c, (const double *)c->S.ref, j * N + env, &out[6 + j]);
    for (int j = 0; j < 21 && !rc; ++j) {
        float v = 0;
        rc = read1(c, (const float *)c->S.posv, j * N + env, &v);
        out[12 + j] = v;
    }
    for (int j = 0; j < 7 && !rc; ++j) rc = read1(c, (const double *)c->S.prev_a, j * N + env, &out[33 + j]);
    for (int j = 0; j < 7 && !rc; ++j) rc = read1(c, (const double *)c->S.prev2_a, j * N + env, &out[40 + j]);
    for (int j = 0; j < 2 && !rc; ++j) rc = read1(c, (const double *)c->S.maxSE, j * N + env, &out[47 + j]);
    int32_t viol = 0;
    if (!rc) rc = read1(c, (const int32_t *)c->S.viol, env, &viol);
    out[49] = ep;
    out[50] = c->L_host[env];
    out[51] = c->motion_host[env];
    out[52] = viol;
    return rc;
}

int exo_set_state_host(exo_ctx *c, int32_t env, const double *in) {
    if (!c || env < 0 || env >= c->N || !in) return EXO_EINVAL;
    DeviceGuard g(c->device);
    int rc = check(c, hipDeviceSynchronize(), "sync");
    const size_t N = c->N;
    if (!rc) rc = write1(c, c->S.counts, env, (int32_t)in[0]);
    if (!rc) rc = write1(c, c->S.episode, env, (uint32_t)in[49]);
    if (!rc) rc = write1(c, c->S.viol, env, (int32_t)in[52]);
    for (int j = 0; j < 5 && !rc; ++j) rc = write1(c, c->S.phys_q, j * N + env, in[1 + j]);
    for (int j = 0; j < 6 && !rc; ++j) rc = write1(c, c->S.ref, j * N + env, in[6 + j]);
    for (int j = 0; j < 21 && !rc; ++j) rc = write1(c, c->S.posv, j * N + env, (float)in[12 + j]);
    for (int j = 0; j < 7 && !rc; ++j) rc = write1(c, c->S.prev_a, j * N + env, in[33 + j]);
    for (int j = 0; j < 7 && !rc; ++j) rc = write1(c, c->S.prev2_a, j * N + env, in[40 + j]);
    for (int j = 0; j < 2 && !rc; ++j) rc = write1(c, c->S.maxSE, j * N + env, in[47 + j]);
    return rc;
}

int exo_set_step_variant(exo_ctx *c, int32_t variant) {
    if (c && c->S.budget > 0 && variant == EXO_STEP_LANES)
        return fail(c, EXO_EINVAL, "exo_set_step_variant: the step budget needs a row-parallel kernel");
    if (!c || variant < EXO_STEP_AUTO || variant > EXO_STEP_ROWS_SHARED) return EXO_EINVAL;
    c->step_variant = variant;
    return EXO_OK;
}

int exo_set_step_clock(exo_ctx *c, unsigned long long *clock_dev, double *ticks_per_ms) {
    if (!c) return EXO_EINVAL;
    c->step_clock = clock_dev;
    if (ticks_per_ms) {
        int khz = 0;
        hipError_t e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device);
        if (e != hipSuccess || khz <= 0) return check(c, e != hipSuccess ? e : hipErrorInvalidValue, "exo_set_step_clock");
        *ticks_per_ms = (double)khz;
    }
    return EXO_OK;
}

int exo_set_tremor_model(exo_ctx *c, const double *jmax7, int32_t sign_mode) {
    if (!c || sign_mode < EXO_TREMOR_SIGN_PER_SAMPLE || sign_mode > EXO_TREMOR_SIGN_NONE) return EXO_EINVAL;
    static const double shipped[7] = {2.5, 5, 10, 5, 5, 0.5, 0.5}; // generate_parkinson_tremor.py:59
    for (int i = 0; i < 7; ++i) {
        const double v = jmax7 ? jmax7[i] : shipped[i];
        if (!(v >= 0) || !(v < 1e6)) return fail(c, EXO_EINVAL, "exo_set_tremor_model: invalid joint maximum");
        c->S.tjmax[i] = v;
    }
    c->S.tsign = sign_mode;
    return EXO_OK;
}

int exo_set_seed(exo_ctx *c, uint64_t seed) {
    if (!c) return EXO_EINVAL;
    c->seed = seed;
    return EXO_OK;
}

int exo_tremor_metrics(exo_ctx *c, const float *info_dev, const uint8_t *stepped_dev, double humerus_length,
                       double forearm_length, double hand_length, int32_t disregard, float *metrics_dev,
                       float *counters_dev, void *stream) {
    (void)hand_length; // the reference's DH table ends at the wrist (a = d = 0 for joints 6, 7)
    if (!c || !info_dev || !metrics_dev || !counters_dev) return EXO_EINVAL;
    DeviceGuard g(c->device);
    hipLaunchKernelGGL(tremor_metrics_kernel, dim3(((size_t)c->N * TM_LANES + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, c->S,
                       info_dev, stepped_dev, humerus_length, forearm_length, disregard, metrics_dev, counters_dev);
    return check(c, hipGetLastError(), "exo_tremor_metrics");
}

int exo_active_advance(const uint8_t *table_dev, int32_t rows, int32_t n, int64_t *k_dev, uint8_t *active_dev,
                       int32_t *count_dev, void *stream) {
    if (!table_dev || !k_dev || !active_dev || rows <= 0 || n <= 0) return EXO_EINVAL;
    hipLaunchKernelGGL(active_advance_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, table_dev, rows, n,
                       (long long *)k_dev, active_dev, count_dev, (const float *)nullptr, (double *)nullptr);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int exo_active_advance_score(const uint8_t *table_dev, int32_t rows, int32_t n, int64_t *k_dev, uint8_t *active_dev,
                             int32_t *count_dev, const float *reward_dev, double *score_dev, void *stream) {
    if (!table_dev || !k_dev || !active_dev || !reward_dev || !score_dev || rows <= 0 || n <= 0) return EXO_EINVAL;
    hipLaunchKernelGGL(active_advance_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, table_dev, rows, n,
                       (long long *)k_dev, active_dev, count_dev, reward_dev, score_dev);
    return hipGetLastError() == hipSuccess ? EXO_OK : EXO_EDEVICE;
}

int exo_eval_metrics(exo_ctx *c, const float *info_dev, const uint8_t *stepped_dev, double humerus_length,
                     double forearm_length, float *counters_dev, void *stream) {
    if (!c || !info_dev || !counters_dev) return EXO_EINVAL;
    DeviceGuard g(c->device);
    hipLaunchKernelGGL(eval_metrics_kernel, dim3((c->N + 255) / 256), dim3(256), 0, (hipStream_t)stream, c->S,
                       info_dev, stepped_dev, humerus_length, forearm_length, counters_dev);
    return check(c, hipGetLastError(), "exo_eval_metrics");
}

const char *exo_last_error(const exo_ctx *c) { return c ? c->err.c_str() : "null context"; }

void exo_destroy(exo_ctx *c) {
    if (!c) return;
    {
        DeviceGuard g(c->device);
        (void)hipDeviceSynchronize();
        for (void *p : c->allocs)
            if (p) (void)hipFree(p);
    }
    delete c;
}

} // extern "C"
