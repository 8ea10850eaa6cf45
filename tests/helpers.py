"""Shared helpers for the parity tests (test infrastructure)."""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
MODEL_HOST_SO = os.path.join(REPO, "tests", "native", "_build", "libmodel_host.so")

NZ_R = [0, 0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6]
NZ_C = [0, 1, 2, 3, 0, 1, 2, 0, 1, 2, 0, 3, 4, 5, 6, 4, 5, 6, 4, 5, 6]
SYM_R = [0, 0, 0, 0, 1, 1, 2, 3, 4, 4, 4, 5, 5, 6]
SYM_C = [0, 1, 2, 3, 1, 2, 2, 3, 4, 5, 6, 5, 6, 6]
B1, B2 = [0, 3, 6], [1, 2, 4, 5]


def golden_env(m):
    return np.load(os.path.join(GOLDEN, f"env_m{m}.npz"), allow_pickle=False)


def env_kwargs(d):
    return dict(tremor_sequence=d["tremor_seq"], tremor_amplitude_range=d["amp_range"],
                first_harmonics_interval=d["harm1"], second_harmonics_interval=d["harm2"],
                max_force_shoulder=float(d["max_force"][0]), max_force_elbow=float(d["max_force"][1]),
                dr_actuator_end_pos_shift=float(d["dr"][0]), dr_actuator_range=float(d["dr"][1]),
                matrix_noise_fraction=float(d["dr"][2]))


def episode_steps(d, ep):
    idx = np.nonzero(d["step_ep"] == ep)[0]
    return idx


def model_host():
    """gcc build of csrc/exo_model.h (the device math) for host-side tests."""
    src = os.path.join(REPO, "tests", "native", "model_host.cpp")
    hdr = os.path.join(PKG, "csrc", "exo_model.h")
    if not os.path.exists(MODEL_HOST_SO) or os.path.getmtime(MODEL_HOST_SO) < max(os.path.getmtime(src),
                                                                                   os.path.getmtime(hdr)):
        os.makedirs(os.path.dirname(MODEL_HOST_SO), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-D_GNU_SOURCE", "-DEXO_HOST_ONLY",
                        "-ffp-contract=off", "-I", os.path.join(PKG, "csrc"), "-o", MODEL_HOST_SO, src], check=True)
    L = ctypes.CDLL(MODEL_HOST_SO)
    d = ctypes.POINTER(ctypes.c_double)
    L.mh_rk45.argtypes = [d] * 5
    L.mh_link_coms.argtypes = [d] * 3
    L.mh_cos_atan2.restype = ctypes.c_double
    L.mh_cos_atan2.argtypes = [ctypes.c_double] * 2
    L.mh_philox_u01.restype = ctypes.c_double
    L.mh_philox_u01.argtypes = [ctypes.c_ulonglong, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]
    return L


def pack_ode(I, D, S):
    """Device layout of the episode matrices: I^-1 block upper triangles (16), D/S sym non-zeros (14)."""
    Ii = np.linalg.inv(I)
    b1 = Ii[np.ix_(B1, B1)]
    b2 = Ii[np.ix_(B2, B2)]
    ii = np.concatenate([b1[np.triu_indices(3)], b2[np.triu_indices(4)]])
    dn = np.array([D[r, c] for r, c in zip(SYM_R, SYM_C)])
    sn = np.array([S[r, c] for r, c in zip(SYM_R, SYM_C)])
    return ii, dn, sn


def philox_draws(L, seed, env, episode, lib=None):
    lib = lib or model_host()
    n = 208 + 8 * int(L)
    return np.array([lib.mh_philox_u01(seed, env, episode, p) for p in range(n)])


# ----------------------------------------------------------------------------
# td7_full.npz: the TD7 update at the bench's own shape (configs[1]: zs/enc 300,
# critic/actor 320, 8 strata x 128 rows).  The batches are regenerated from a
# seeded PCG64 stream (their float64 sums are stored in the fixture and
# checked), so the fixture holds only the reference's outputs.
TD7_FULL_HP = dict(zs_dim=300, enc_hdim=300, critic_hdim=320, actor_hdim=320, batch_size=128)
TD7_FULL_ENVS = 8
TD7_FULL_STEPS = 3
# td7_wide.npz: configs[4]'s wide TD7 (every MLP 1,024 wide, zs 1,024), same batches
TD7_WIDE_HP = dict(zs_dim=1024, enc_hdim=1024, critic_hdim=1024, actor_hdim=1024, batch_size=128)
TD7_WIDE_STEPS = 2
TD7_GOLDENS = {"td7_full": (TD7_FULL_HP, TD7_FULL_STEPS), "td7_wide": (TD7_WIDE_HP, TD7_WIDE_STEPS)}
TD7_FULL_LEARNING_STEPS = 500000
TD7_FULL_SAMPLES = 512
# running Q-target clamp bounds injected before the first step (:243; 0/0 until
# the first target refresh otherwise, which would hide the clamp)
TD7_FULL_QBOUNDS = (-1.5, 2.0)


def td7_full_batch(step):
    """(state, action, next_state, reward, not_done, noise) of golden step `step` (float32 numpy)."""
    B = TD7_FULL_ENVS * TD7_FULL_HP["batch_size"]
    rng = np.random.Generator(np.random.PCG64(9000 + step))
    s = rng.normal(0, 1, (B, 80)).astype(np.float32)
    a = rng.uniform(-1, 1, (B, 7)).astype(np.float32)
    s2 = (s + 0.1 * rng.normal(0, 1, (B, 80))).astype(np.float32)
    r = rng.uniform(-2, 3, (B, 1)).astype(np.float32)
    nd = (rng.uniform(0, 1, (B, 1)) > 0.02).astype(np.float32)
    nz = rng.normal(0, 1, (B, 7)).astype(np.float32)
    return s, a, s2, r, nd, nz


def td7_full_sample_index(name, numel):
    """Fixed flat indices at which a parameter / gradient tensor is sampled."""
    if numel <= TD7_FULL_SAMPLES:
        return np.arange(numel, dtype=np.int64)
    seed = sum(ord(c) * (i + 1) for i, c in enumerate(name))
    return np.sort(np.random.Generator(np.random.PCG64(seed)).choice(numel, TD7_FULL_SAMPLES, replace=False))


# ----------------------------------------------------------------------------
# select_action_full.npz (make_golden.py --only select_action_full): select_action
# at the bench's widths: (name, Hyperparameters overrides, torch seed).
# The Pink agent's defaults (zs / enc 300, critic 320, actor 300, the shipped
# checkpoints' shapes) and TD7_multi_agent.py's actor width 320 (the bench).
SELECT_FULL = [("pink300", {}, 41), ("actor320", {"actor_hdim": 320}, 42)]
SELECT_FULL_ROWS = 256
SELECT_FULL_PERTURB = 0.02


def select_full_states():
    """SELECT_FULL_ROWS real observations: every 7th step of the motion-0..7
    golden traces (env_m*.npz step_obs, the reference env's own outputs)."""
    obs = np.concatenate([np.load(os.path.join(GOLDEN, f"env_m{m}.npz"))["step_obs"] for m in range(8)])
    return obs[::7][:SELECT_FULL_ROWS].astype(np.float32)


def select_full_perturb(module, seed):
    """Move the live nets off the checkpoint copies: p += PERTURB * N(0, 1)
    from PCG64(seed + k) for the k-th parameter (named_parameters order);
    tests/test_select_full_gpu.py applies the same to the build's nets."""
    import torch
    with torch.no_grad():
        for k, (_, p) in enumerate(module.named_parameters()):
            z = np.random.Generator(np.random.PCG64(seed + k)).normal(0, 1, tuple(p.shape)).astype(np.float32)
            p.add_(SELECT_FULL_PERTURB * torch.from_numpy(z))
