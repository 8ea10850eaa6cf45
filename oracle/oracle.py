"""ORACLE -- test infrastructure only (see exo_oracle.c header).

ctypes wrapper around oracle/_build/libexo_oracle.so.  Importable only from
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libexo_oracle.so")
_lib = None

_d = ctypes.POINTER(ctypes.c_double)
_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)


class MBParams(ctypes.Structure):
    """mb_params of multibody.h (Bullet-equivalent step constants)."""
    _fields_ = [(n, ctypes.c_double) for n in ("dt", "gravity", "kp", "kd", "motor_impulse", "passive_impulse",
                                               "limit_impulse", "erp", "lin_damp", "ang_damp", "max_vel")] + \
               [("iters", ctypes.c_int)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_solve_diff_eq.argtypes = [_d, _d, _d, _d, _d, _i]
        L.oracle_link_coms.argtypes = [_d, _d]
        L.oracle_env_create.restype = ctypes.c_void_p
        L.oracle_env_create.argtypes = [ctypes.c_int, _d, _i, _d, _d, _d] + [ctypes.c_double] * 5
        L.oracle_env_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_env_reset.argtypes = [ctypes.c_void_p, _d, _f]
        L.oracle_env_step.argtypes = [ctypes.c_void_p, _d, _f, _d, _i, _d, _d]
        L.oracle_env_tremor.restype = _d
        L.oracle_env_tremor.argtypes = [ctypes.c_void_p]
        L.oracle_env_episode.argtypes = [ctypes.c_void_p, _d, _d, _d, _d, _d]
        L.oracle_env_phys.argtypes = [ctypes.c_void_p, _d]
        L.oracle_env_counts.argtypes = [ctypes.c_void_p]
        L.oracle_env_set_physics.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(MBParams)]
        L.oracle_env_mb_state.argtypes = [ctypes.c_void_p, _d, _d, _d]
        L.oracle_env_set_mb_state.argtypes = [ctypes.c_void_p, _d, _d]
        L.oracle_mb_default_params.argtypes = [ctypes.POINTER(MBParams)]
        L.oracle_mb_aba.argtypes = [_d, _d, _d, ctypes.POINTER(MBParams), _d]
        L.oracle_mb_rnea.argtypes = [_d, _d, _d, ctypes.POINTER(MBParams), _d]
        L.oracle_mb_mass.argtypes = [_d, _d]
        L.oracle_mb_link_coms.argtypes = [_d, _d]
        L.oracle_mb_step.argtypes = [_d, _d, _d, ctypes.POINTER(MBParams), _d]
        L.oracle_bench.restype = ctypes.c_long
        L.oracle_bench.argtypes = [ctypes.c_int, _d, _i, ctypes.c_int, ctypes.c_long, ctypes.c_uint64]
        _lib = L
    return _lib


def _p(a, t=_d):
    return a.ctypes.data_as(t)


def solve_diff_eq(I, D, K, T):
    q = np.zeros(7)
    n = ctypes.c_int(0)
    args = [np.ascontiguousarray(x, dtype=np.float64) for x in (I, D, K, T)]
    rc = lib().oracle_solve_diff_eq(*[_p(a) for a in args], _p(q), ctypes.byref(n))
    if rc < 0:
        raise RuntimeError("RK45 solve failed")
    # rc 1: scipy's "required step size is less than spacing between numbers" --
    # solve_ivp returns status -1 with sol.y up to the last accepted step, whose
    # q the reference uses (calculate_joint_angles.py:20): q is that
    return q, n.value


def link_coms(q5):
    q5 = np.ascontiguousarray(q5, dtype=np.float64)
    out = np.zeros((19, 3))
    lib().oracle_link_coms(_p(q5), _p(out))
    return out


# ---------------------------------------------------------------- multibody
def mb_params(**overrides):
    p = MBParams()
    lib().oracle_mb_default_params(ctypes.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def _vec(x, n=19):
    a = np.ascontiguousarray(x, dtype=np.float64)
    assert a.shape == (n,), a.shape
    return a


def mb_aba(q, qd, tau=None, params=None):
    """Articulated-Body Algorithm: joint accelerations (19)."""
    p = params or mb_params()
    out = np.zeros(19)
    t = None if tau is None else _p(_vec(tau))
    lib().oracle_mb_aba(_p(_vec(q)), _p(_vec(qd)), t, ctypes.byref(p), _p(out))
    return out


def mb_rnea(q, qd, qdd, params=None):
    """Recursive Newton-Euler: joint forces (19)."""
    p = params or mb_params()
    out = np.zeros(19)
    lib().oracle_mb_rnea(_p(_vec(q)), _p(_vec(qd)), _p(_vec(qdd)), ctypes.byref(p), _p(out))
    return out


def mb_mass(q):
    """Composite-Rigid-Body Algorithm: joint-space inertia (19 x 19)."""
    out = np.zeros((19, 19))
    lib().oracle_mb_mass(_p(_vec(q)), _p(out))
    return out


def mb_link_coms(q):
    out = np.zeros((19, 3))
    lib().oracle_mb_link_coms(_p(_vec(q)), _p(out))
    return out


def mb_step(q, qd, targets, params=None):
    """One multibody stepSimulation: returns (q', qd', stats[4])."""
    p = params or mb_params()
    q, qd = _vec(q).copy(), _vec(qd).copy()
    st = np.zeros(4)
    rc = lib().oracle_mb_step(_p(q), _p(qd), _p(_vec(targets, 5)), ctypes.byref(p), _p(st))
    if rc:
        raise RuntimeError("singular joint-space inertia")
    return q, qd, st


class OracleEnv:
    """One reference env (fp64), driven by explicit draw streams."""

    def __init__(self, imu, seq, amp, h1, h2, maxS0, maxE0, shift_r, act_r, mat_f):
        self.imu = np.ascontiguousarray(imu, dtype=np.float64)  # [5, L]
        self.L = self.imu.shape[1]
        self._seq = np.ascontiguousarray(seq, dtype=np.int32)
        self._amp, self._h1, self._h2 = (np.ascontiguousarray(x, dtype=np.float64) for x in (amp, h1, h2))
        self.h = lib().oracle_env_create(self.L, _p(self.imu), _p(self._seq, _i), _p(self._amp), _p(self._h1),
                                         _p(self._h2), maxS0, maxE0, shift_r, act_r, mat_f)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_env_destroy(self.h)
            self.h = None

    def reset(self, draws):
        draws = np.ascontiguousarray(draws, dtype=np.float64)
        assert draws.size == 208 + 8 * self.L
        obs = np.zeros(80, dtype=np.float32)
        lib().oracle_env_reset(self.h, _p(draws), _p(obs, _f))
        return obs

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.float64)
        obs = np.zeros(80, dtype=np.float32)
        r = ctypes.c_double(0)
        d = ctypes.c_int(0)
        info = np.zeros(40)
        tgt = np.zeros(5)
        rc = lib().oracle_env_step(self.h, _p(a), _p(obs, _f), ctypes.byref(r), ctypes.byref(d), _p(info), _p(tgt))
        if rc != 0:
            raise IndexError("step past the end of the reference motion")
        return obs, r.value, bool(d.value), info, tgt

    def tremor(self):
        p = lib().oracle_env_tremor(self.h)
        return np.ctypeslib.as_array(p, shape=(7 * self.L,)).reshape(7, self.L).copy()

    def episode(self):
        I, D, S, sh, m = np.zeros(49), np.zeros(49), np.zeros(49), np.zeros(42), np.zeros(2)
        lib().oracle_env_episode(self.h, _p(I), _p(D), _p(S), _p(sh), _p(m))
        return I.reshape(7, 7), D.reshape(7, 7), S.reshape(7, 7), sh.reshape(14, 3), m

    def phys_q(self):
        q = np.zeros(5)
        lib().oracle_env_phys(self.h, _p(q))
        return q

    def set_physics(self, mode, params=None):
        """mode 'ideal'  or 'multibody' (multibody.c)."""
        m = {"ideal": 0, "multibody": 1}[mode]
        lib().oracle_env_set_physics(self.h, m, ctypes.byref(params) if params is not None else None)

    def mb_state(self):
        q, qd, st = np.zeros(19), np.zeros(19), np.zeros(4)
        lib().oracle_env_mb_state(self.h, _p(q), _p(qd), _p(st))
        return q, qd, st

    def set_mb_state(self, q, qd):
        lib().oracle_env_set_mb_state(self.h, _p(_vec(q)), _p(_vec(qd)))

    @property
    def counts(self):
        return lib().oracle_env_counts(self.h)


def bench(n_envs, angles, lengths, max_steps, seed=0):
    """Single-core CPU baseline: returns env-steps executed."""
    angles = np.ascontiguousarray(angles, dtype=np.float64)
    lengths = np.ascontiguousarray(lengths, dtype=np.int32)
    return lib().oracle_bench(n_envs, _p(angles), _p(lengths, _i), angles.shape[2], max_steps, seed)
