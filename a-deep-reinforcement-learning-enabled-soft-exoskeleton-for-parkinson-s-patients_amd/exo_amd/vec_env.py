"""VecExoskeletonEnv: N exoskeleton envs stepped by one HIP kernel launch.

Host-side mirror of ``ExoskeletonEnv_train`` (Environment/Exoskeleton_env.py:34)
for many envs at once.  All tensors live on the GPU; step/reset are
stream-ordered launches on torch's current stream (no host sync).
"""
import ctypes

import numpy as np
import torch

from . import _native as nat
from . import motions as motion_data

OBS_DIM, ACT_DIM, INFO_DIM = 80, 7, 40
STATE_DOUBLES = 53

# Defaults of Simulation/Exoskeleton_agent_train.py:28-44.  The reference env
# has no default for tremor_amplitude_range (Exoskeleton_env.py:41); [0.95,
# 1.05] is what both evaluation scripts pass.
DEFAULTS = dict(tremor_sequence=(0, 1, 0, 1, 0, 0, 0), tremor_amplitude_range=(0.95, 1.05),
                first_harmonics_interval=(4.0, 6.0), second_harmonics_interval=(8.0, 10.0),
                max_force_shoulder=40.0, max_force_elbow=20.0, dr_actuator_end_pos_shift=0.02,
                dr_actuator_range=0.03, matrix_noise_fraction=0.1)

INFO_SLICES = {"actuator_torques": slice(0, 7), "torque_val": slice(7, 14), "ampl_val": slice(14, 21),
               "tremor_torque_val": slice(21, 28), "tremor_ampl_val": slice(28, 35), "reward_unwanted": 35,
               "reward_torque": 36, "reward_axis": 37, "reward_control": 38, "reward_smoothness": 39}


def draws_per_episode(L):
    """np.random draws one reset consumes."""
    return 208 + 8 * int(L)


def _per_env(value, n, shape):
    a = np.asarray(value, dtype=np.float64)
    if a.shape == shape:
        return np.broadcast_to(a, (n,) + shape)
    if a.shape == (n,) + shape:
        return a
    raise ValueError(f"expected shape {shape} or {(n,) + shape}, got {a.shape}")


class VecExoskeletonEnv:
    """N independent envs; env i follows motion ``motions[i]`` (default i mod 8).

    Every constructor argument of ExoskeletonEnv_train may be given per env
    (leading dimension N) for domain-randomisation sweeps.
    """

    observation_dim, action_dim = OBS_DIM, ACT_DIM

    PHYSICS = {"ideal": 0, "multibody": 1}

    def __init__(self, n_envs, motions=None, seed=0, device=None, physics="ideal", multibody_params=None, **kwargs):
        self.device = nat.require_gpu(device)
        self.n = int(n_envs)
        unknown = set(kwargs) - set(DEFAULTS)
        if unknown:
            raise TypeError(f"unknown env arguments {sorted(unknown)}")
        p = dict(DEFAULTS, **kwargs)
        angles, lengths = motion_data.load()
        n_mot = lengths.size
        mot = np.arange(self.n) % n_mot if motions is None else np.asarray(motions, dtype=np.int64)
        if mot.shape != (self.n,) or mot.min() < 0 or mot.max() >= n_mot:
            raise ValueError("motions must hold one motion index in [0, 8) per env")
        seq = _per_env(p["tremor_sequence"], self.n, (7,))
        amp = _per_env(p["tremor_amplitude_range"], self.n, (2,))
        h1 = _per_env(p["first_harmonics_interval"], self.n, (2,))
        h2 = _per_env(p["second_harmonics_interval"], self.n, (2,))
        scal = {k: _per_env(p[k], self.n, ()) for k in ("max_force_shoulder", "max_force_elbow",
                                                       "dr_actuator_end_pos_shift", "dr_actuator_range",
                                                       "matrix_noise_fraction")}
        cfgs = (nat.ExoEnvConfig * self.n)()
        for i in range(self.n):
            c = cfgs[i]
            c.motion = int(mot[i])
            for j in range(7):
                c.tremor_sequence[j] = int(seq[i, j])
            for j in range(2):
                c.tremor_amplitude_range[j] = amp[i, j]
                c.first_harmonics_interval[j] = h1[i, j]
                c.second_harmonics_interval[j] = h2[i, j]
            for k, v in scal.items():
                setattr(c, k, float(v[i]))
        self.motions = mot
        self.tremor_sequence = np.asarray(seq, dtype=np.int64)
        self.max_force = (scal["max_force_shoulder"].copy(), scal["max_force_elbow"].copy())
        self.lengths_host = lengths[mot].astype(np.int64)
        self._ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = nat.lib().exo_create(cfgs, self.n, angles.ctypes.data_as(nat.P(ctypes.c_double)),
                                      lengths.ctypes.data_as(nat.P(ctypes.c_int32)), n_mot, angles.shape[2],
                                      ctypes.c_uint64(int(seed) & (2 ** 64 - 1)), self.device.index,
                                      ctypes.byref(self._ctx))
        nat.check(rc, "exo_create")
        self.max_len = int(angles.shape[2])
        self.lengths = torch.as_tensor(self.lengths_host, device=self.device)
        n_axes = self.tremor_sequence.sum(1)
        self.max_reward = n_axes * 0.5 + 0.9 + 0.05 + 0.05 + 0.5  # Exoskeleton_env.py:167-169
        self.physics = "ideal"
        if physics != "ideal" or multibody_params is not None:
            self.set_physics(physics, multibody_params)

    # ------------------------------------------------------------------ core
    def _stream(self):
        return nat.stream_ptr(self.device)

    def reset(self, mask=None, obs_out=None):
        """initialize_movement for envs with mask[i] (bool/uint8 [N] on device; None = all).
        Returns the observation tensor [N, 80] (rows of masked-out envs are left untouched
        when obs_out is given, uninitialised otherwise)."""
        obs = obs_out if obs_out is not None else torch.empty((self.n, OBS_DIM), dtype=torch.float32,
                                                               device=self.device)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            assert m.numel() == self.n
        self._check_out(obs, (self.n, OBS_DIM), torch.float32)
        nat.check(nat.lib().exo_reset(self._ctx, nat.ptr(m), nat.ptr(obs), self._stream()), "exo_reset", self._ctx)
        return obs

    def step(self, actions, active=None, out=None, with_info=True, obs_cur=None):
        """One step for every env (Exoskeleton_env.py:368-471).

        actions: float32 [N, 7] device tensor in [-1, 1].  active: optional
        bool/uint8 [N]; inactive envs and envs already done are skipped and
        their rows in the outputs are left untouched.  With a step budget
        (set_step_budget) an env with a pending solve continues it instead of
        stepping and, given obs_cur (the current observations), copies its row
        into the output buffer.  Returns
        (obs [N,80] f32, reward [N] f32, done [N] bool, info [N,40] f32 or None)."""
        a = actions
        if a.dtype != torch.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        assert a.shape == (self.n, ACT_DIM), a.shape
        if out is None:
            out = self.new_outputs(with_info)
        obs, rew, done, info = out
        act = None
        if active is not None:
            if active.dtype == torch.bool and active.device == self.device and active.is_contiguous():
                act = active.view(torch.uint8)  # same bytes, no conversion kernel
            else:
                act = active.to(device=self.device, dtype=torch.uint8).contiguous()
        rc = nat.lib().exo_step_carry(self._ctx, nat.ptr(a), nat.ptr(obs), nat.ptr(rew), nat.ptr(done),
                                      nat.ptr(info) if with_info else None, nat.ptr(act), nat.ptr(obs_cur),
                                      self._stream())
        nat.check(rc, "exo_step", self._ctx)
        return obs, rew, done.view(torch.bool), info

    step_budget = 0

    def set_step_budget(self, budget):
        """At most `budget` RK45 step attempts per ODE solve and launch (0 = no
        limit; include/exo_amd.h exo_set_step_budget): a stiff env's solve
        continues over several launches, its trajectory unchanged, instead of
        holding every launch for its whole solve."""
        nat.check(nat.lib().exo_set_step_budget(self._ctx, int(budget)), "exo_set_step_budget", self._ctx)
        self.step_budget = int(budget)

    def budget_advance(self, active, count, remaining, steps_total=None):
        """Budget mode's mask for the next launch (exo_budget_advance): active
        (bool [N]) = envs that will start a step, count (int32 [1]) their
        number, remaining (int32 [1]) the envs not finished, steps_total (int64
        [1]) += the envs the last launch stepped."""
        nat.check(nat.lib().exo_budget_advance(self._ctx, nat.ptr(active), nat.ptr(count), nat.ptr(remaining),
                                               nat.ptr(steps_total), self._stream()), "exo_budget_advance",
                  self._ctx)

    def episode_advance(self, active, count, obs_out, steps_total=None):
        """Auto-reset (exo_episode_advance): envs whose episode is over are
        reset in place, their observations written into obs_out (the buffer
        the last step wrote); active (bool [N]) = the envs of the next launch
        (all but those with a pending budgeted solve), count (int32 [1]) their
        number, steps_total (int64 [1]) += the envs the last launch stepped."""
        if getattr(self, "_reset_ws", None) is None:
            self._reset_ws = torch.zeros((self.n + 1,), dtype=torch.int32, device=self.device)
        self._check_out(obs_out, (self.n, OBS_DIM), torch.float32)
        nat.check(nat.lib().exo_episode_advance(self._ctx, nat.ptr(active), nat.ptr(count), nat.ptr(self._reset_ws),
                                                nat.ptr(steps_total), nat.ptr(obs_out), self._stream()),
                  "exo_episode_advance", self._ctx)

    def new_outputs(self, with_info=True):
        d = self.device
        return (torch.empty((self.n, OBS_DIM), dtype=torch.float32, device=d),
                torch.empty((self.n,), dtype=torch.float32, device=d),
                torch.zeros((self.n,), dtype=torch.uint8, device=d),
                torch.empty((self.n, INFO_DIM), dtype=torch.float32, device=d) if with_info else None)

    @staticmethod
    def _check_out(t, shape, dtype):
        if tuple(t.shape) != shape or t.dtype != dtype or not t.is_contiguous():
            raise ValueError(f"output buffer must be contiguous {dtype} {shape}")

    METRIC_SLICES = {"tremor_reduction": slice(0, 7), "tremor_reduction_ampl": slice(7, 14),
                     "tremor_reduction_ampl_total": 14, "any_reduction": 15}
    COUNTER_NAMES = ("tremor_when_reduction_nonneg", "tremor_when_reduction_neg", "tremor_reduction_in_episode",
                     "tremor_when_ampl_reduction_nonneg", "tremor_when_ampl_reduction_neg",
                     "tremor_ampl_total_reduction_ep")

    def tremor_metrics(self, info, stepped=None, counters=None, humerus_length=0.4, forearm_length=0.4,
                       hand_length=0.05, disregard=True, out=None):
        """The training script's per-step tremor-suppression statistics
        (Simulation/Exoskeleton_agent_train.py:149-200) for the envs the last
        step advanced, on the device.  info: that step's [N, 40] output;
        stepped: bool/uint8 [N] (the `active` mask passed to step(), before the
        step's done flags); counters [N, 6] float32 accumulate (COUNTER_NAMES).
        Returns (metrics [N, 16] per METRIC_SLICES, counters)."""
        if counters is None:
            counters = torch.zeros((self.n, 6), dtype=torch.float32, device=self.device)
        m = out if out is not None else torch.zeros((self.n, 16), dtype=torch.float32, device=self.device)
        st = None
        if stepped is not None:
            st = (stepped.view(torch.uint8) if stepped.dtype == torch.bool else stepped.to(torch.uint8)).contiguous()
        nat.check(nat.lib().exo_tremor_metrics(self._ctx, nat.ptr(info.contiguous()), nat.ptr(st),
                                               float(humerus_length), float(forearm_length), float(hand_length),
                                               int(bool(disregard)), nat.ptr(m), nat.ptr(counters), self._stream()),
                  "exo_tremor_metrics", self._ctx)
        return m, counters

    EVAL_COUNTER_NAMES = ("all_axes_suppressed", "any_axis_suppressed", "ampl_total_neg", "ampl_total_nonneg",
                          "ampl_total_neg_sum")

    def eval_metrics(self, info, stepped=None, counters=None, humerus_length=0.4, forearm_length=0.4):
        """The evaluation script's per-step statistics
        (Simulation/Evaluate_control_performance.py:192-260) for the envs the last
        step advanced, accumulated on the device into counters [N, 5] float32
        (EVAL_COUNTER_NAMES); see include/exo_amd.h exo_eval_metrics."""
        if counters is None:
            counters = torch.zeros((self.n, 5), dtype=torch.float32, device=self.device)
        st = None
        if stepped is not None:
            st = (stepped.view(torch.uint8) if stepped.dtype == torch.bool else stepped.to(torch.uint8)).contiguous()
        nat.check(nat.lib().exo_eval_metrics(self._ctx, nat.ptr(info.contiguous()), nat.ptr(st), float(humerus_length),
                                             float(forearm_length), nat.ptr(counters), self._stream()),
                  "exo_eval_metrics", self._ctx)
        return counters

    STEP_VARIANTS = {"auto": 0, "lanes": 1, "rows": 2, "rows_shared": 3}
    step_variant = "auto"

    def set_step_variant(self, name):
        """exo_step kernel: 'lanes' (one lane per ODE solve), 'rows' (16 lanes per
        env), 'auto' (rows for N <= 16384), 'rows_shared' (rows, 32 envs per
        512-thread workgroup: half the CUs at 4,096 envs, for a GPU shared with
        concurrent kernels -- the graph-replayed trainer picks it)."""
        nat.check(nat.lib().exo_set_step_variant(self._ctx, self.STEP_VARIANTS[name]), "exo_set_step_variant",
                  self._ctx)
        self.step_variant = name

    TREMOR_SIGN = {"per_sample": 0, "per_axis": 1, "none": 2}

    def set_tremor_model(self, jmax=None, sign="per_sample"):
        """Tremor of later resets (diagnostic, include/exo_amd.h
        exo_set_tremor_model): jmax = joint_max_values [7] before the
        magnitude (None: the shipped generate_parkinson_tremor.py:59 table);
        sign = 'per_sample' (the shipped :70), 'per_axis' or 'none'."""
        j = None if jmax is None else np.ascontiguousarray(jmax, dtype=np.float64)
        if j is not None and j.shape != (7,):
            raise ValueError("jmax must hold 7 values")
        nat.check(nat.lib().exo_set_tremor_model(self._ctx, None if j is None else j.ctypes.data_as(nat.P(ctypes.c_double)),
                                                 self.TREMOR_SIGN[sign]), "exo_set_tremor_model", self._ctx)

    def set_step_clock(self, on=True):
        """Step clock (include/exo_amd.h exo_set_step_clock): every later step
        launch -- eager or inside a captured graph -- is bracketed by device
        wall-clock reads on its stream.  Returns the clock tensor (int64 [3]:
        last start, summed ticks, steps); read it with step_clock_ms()."""
        if not on:
            nat.check(nat.lib().exo_set_step_clock(self._ctx, None, None), "exo_set_step_clock", self._ctx)
            return None
        self._clock = torch.zeros(3, dtype=torch.int64, device=self.device)
        rate = ctypes.c_double(0.0)
        nat.check(nat.lib().exo_set_step_clock(self._ctx, nat.ptr(self._clock), ctypes.byref(rate)),
                  "exo_set_step_clock", self._ctx)
        self._clock_rate = rate.value  # ticks per ms
        return self._clock

    def step_clock_ms(self):
        """(mean ms per bracketed step launch, steps) of the step clock; synchronises."""
        _, ticks, n = (int(x) for x in self._clock.cpu())
        return (ticks / self._clock_rate / n if n else float("nan")), n

    # ----------------------------------------------------- physics model
    @staticmethod
    def multibody_params(**overrides):
        """Default exo_mb_params (Bullet's defaults, include/exo_amd.h) with overrides."""
        p = nat.ExoMbParams()
        nat.lib().exo_multibody_default_params(ctypes.byref(p))
        for k, val in overrides.items():
            if not hasattr(p, k):
                raise TypeError(f"unknown multibody parameter {k!r}")
            setattr(p, k, val)
        return p

    def set_physics(self, physics, params=None):
        """stepSimulation model (Exoskeleton_env.py:433): 'ideal' -- the idealised
        position motors of SURVEY.md A.2 (default) -- or 'multibody' -- Featherstone
        dynamics of the 19-joint URDF tree with a joint-space impulse solve of the
        motors and joint limits (csrc/exo_multibody.hip).  params: a
        multibody_params() struct or a dict of overrides."""
        if physics not in self.PHYSICS:
            raise ValueError(f"physics must be one of {sorted(self.PHYSICS)}")
        if isinstance(params, dict):
            params = self.multibody_params(**params)
        nat.check(nat.lib().exo_set_physics(self._ctx, self.PHYSICS[physics],
                                            ctypes.byref(params) if params is not None else None),
                  "exo_set_physics", self._ctx)
        self.physics = physics

    def multibody_advance(self, targets, mask=None):
        """One multibody stepSimulation alone: targets float64 [5, N] device (rad)."""
        t = targets.to(device=self.device, dtype=torch.float64).contiguous()
        assert t.shape == (5, self.n), t.shape
        m = None if mask is None else mask.to(device=self.device, dtype=torch.uint8).contiguous()
        nat.check(nat.lib().exo_multibody_advance(self._ctx, nat.ptr(t), nat.ptr(m), self._stream()),
                  "exo_multibody_advance", self._ctx)

    def multibody_state(self, env):
        """(q[19], qd[19]) of one env's URDF joints (pybullet link order)."""
        q, qd = np.zeros(19), np.zeros(19)
        dp = lambda a: a.ctypes.data_as(nat.P(ctypes.c_double))  # noqa: E731
        nat.check(nat.lib().exo_get_multibody_state_host(self._ctx, env, dp(q), dp(qd)),
                  "exo_get_multibody_state_host", self._ctx)
        return q, qd

    def set_multibody_state(self, env, q, qd):
        q = np.ascontiguousarray(q, dtype=np.float64)
        qd = np.ascontiguousarray(qd, dtype=np.float64)
        assert q.shape == (19,) and qd.shape == (19,)
        dp = lambda a: a.ctypes.data_as(nat.P(ctypes.c_double))  # noqa: E731
        nat.check(nat.lib().exo_set_multibody_state_host(self._ctx, env, dp(q), dp(qd)),
                  "exo_set_multibody_state_host", self._ctx)

    # ------------------------------------------------------- parity / debug
    def reset_from_draws(self, env_ids, draws, obs_out=None):
        """Reset envs from explicit unit-uniform draw streams (the reference's
        np.random call order).  draws: list/array of 1-D float64 streams."""
        ids = np.ascontiguousarray(env_ids, dtype=np.int32)
        stride = draws_per_episode(self.max_len)
        buf = np.zeros((ids.size, stride))
        for k, d in enumerate(draws):
            d = np.asarray(d, dtype=np.float64)
            need = draws_per_episode(self.lengths_host[ids[k]])
            if d.size != need:
                raise ValueError(f"env {ids[k]} needs {need} draws, got {d.size}")
            buf[k, :need] = d
        obs = obs_out if obs_out is not None else torch.empty((self.n, OBS_DIM), dtype=torch.float32,
                                                               device=self.device)
        rc = nat.lib().exo_reset_from_draws(self._ctx, ids.ctypes.data_as(nat.P(ctypes.c_int32)), ids.size,
                                            buf.ctypes.data_as(nat.P(ctypes.c_double)), nat.ptr(obs),
                                            self._stream())
        nat.check(rc, "exo_reset_from_draws", self._ctx)
        return obs

    def tremor(self, env):
        L = int(self.lengths_host[env])
        out = np.zeros((7, L))
        nat.check(nat.lib().exo_tremor_host(self._ctx, env, out.ctypes.data_as(nat.P(ctypes.c_double))),
                  "exo_tremor_host", self._ctx)
        return out

    def episode(self, env):
        """(D, S, I^-1, dummy shift [14,3], (max_output_shoulder, max_output_elbow))"""
        D, S, Ii, sh, m = np.zeros(49), np.zeros(49), np.zeros(49), np.zeros(42), np.zeros(2)
        dp = lambda a: a.ctypes.data_as(nat.P(ctypes.c_double))  # noqa: E731
        nat.check(nat.lib().exo_episode_host(self._ctx, env, dp(D), dp(S), dp(Ii), dp(sh), dp(m)),
                  "exo_episode_host", self._ctx)
        return D.reshape(7, 7), S.reshape(7, 7), Ii.reshape(7, 7), sh.reshape(14, 3), m

    def get_state(self, env):
        out = np.zeros(STATE_DOUBLES)
        nat.check(nat.lib().exo_get_state_host(self._ctx, env, out.ctypes.data_as(nat.P(ctypes.c_double))),
                  "exo_get_state_host", self._ctx)
        return out

    def set_state(self, env, state):
        st = np.ascontiguousarray(state, dtype=np.float64)
        assert st.size == STATE_DOUBLES
        nat.check(nat.lib().exo_set_state_host(self._ctx, env, st.ctypes.data_as(nat.P(ctypes.c_double))),
                  "exo_set_state_host", self._ctx)

    def original_joint_angles(self, env):
        out = np.zeros(7)
        nat.check(nat.lib().exo_original_joint_angles_host(self._ctx, env,
                                                           out.ctypes.data_as(nat.P(ctypes.c_double))),
                  "exo_original_joint_angles_host", self._ctx)
        return out

    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            nat.lib().exo_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def unpack_info(info_row):
        """info dict of one env from a [40] info row (Exoskeleton_env.py:464-469)."""
        r = np.asarray(info_row, dtype=np.float64)
        return {k: (r[s].copy() if isinstance(s, slice) else float(r[s])) for k, s in INFO_SLICES.items()}
