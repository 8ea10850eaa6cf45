"""GPU parity of the HIP environment kernels (exo_reset_kernel / exo_step_kernel)
against the reference's golden traces and the CPU oracle.

Tolerances: the kernels compute in fp64 like the reference; they differ from it
only by rounding (I^-1 multiply instead of LU, cos(atan2(y,x)) = x/hypot(x,y),
FMA contraction, RK45 stages in second-order storage form).  Observations are
float32 in the reference (Exoskeleton_env.py:568) and must match to 1 ulp-level
(atol 2e-6 relative to magnitude); rewards (fp32 output of an fp64 value) to
2e-6 relative; info (fp32 output) to 1e-5 relative / 1e-6 absolute; joint
positions (fp64 state) to 1e-9 rad; done indices exactly; tremor tables to
1e-13 relative (device sin/pow and FMA contraction round differently from
numpy by a few ulp; the D/S matrices, dummy shift and force scales are
bit-exact).
"""
import numpy as np
import pytest
import torch

import oracle as O
from helpers import env_kwargs, episode_steps, golden_env, model_host, philox_draws

pytestmark = pytest.mark.gpu


def _close_obs(a, b):
    np.testing.assert_allclose(a, b, rtol=2e-6, atol=2e-6)


VARIANTS = ["rows", "lanes", "rows_shared"]


def _batched_golden_env(variant="auto"):
    from exo_amd import VecExoskeletonEnv
    gold = [golden_env(m) for m in range(8)]
    kw = {}
    per = [env_kwargs(d) for d in gold]
    for k in per[0]:
        kw[k] = np.stack([np.asarray(p[k], dtype=np.float64) for p in per])
    env = VecExoskeletonEnv(8, motions=list(range(8)), seed=5, **kw)
    env.set_step_variant(variant)
    # exo_create already ran the constructor's initialize_movement on Philox
    # draws; the goldens' episode 0 IS that constructor call, whose link-read
    # cache is still all zeros (Exoskeleton_sim_pybullet.py:80-81).  Restore
    # the freshly-loaded state so reset_from_draws(ep0) replays it.
    for m in range(8):
        st = env.get_state(m)
        st[6:12] = 0.0
        st[49] = 0
        env.set_state(m, st)
    return env, gold


def test_reset_matches_reference_draws():
    env, gold = _batched_golden_env()
    for ep in (0, 1):
        obs = env.reset_from_draws(list(range(8)), [d[f"ep{ep}_draws"] for d in gold]).cpu().numpy()
        for m, d in enumerate(gold):
            _close_obs(obs[m], d[f"ep{ep}_obs"])
            if ep == 1:
                np.testing.assert_allclose(env.tremor(m), d["ep1_tremor"], rtol=1e-13, atol=1e-14)
                Dm, S, Iinv, sh, mm = env.episode(m)
                np.testing.assert_array_equal(Dm, d["ep1_D"])
                np.testing.assert_array_equal(S, d["ep1_S"])
                np.testing.assert_allclose(Iinv, np.linalg.inv(d["ep1_I"]), rtol=1e-12, atol=1e-9)
                np.testing.assert_array_equal(sh, d["ep1_shift"])
                assert mm[0] == d["ep1_maxS"] and mm[1] == d["ep1_maxE"]
                st = env.get_state(m)
                assert st[0] == 2 and st[50] == d["L"] and st[51] == m


@pytest.mark.parametrize("variant", VARIANTS)
def test_steps_match_reference_traces_with_active_mask(variant):
    """All 8 motions in one batch; envs whose golden episode is shorter wait
    (inactive) like the training script's per-env `done` skip."""
    env, gold = _batched_golden_env(variant)
    env.reset_from_draws(list(range(8)), [d["ep0_draws"] for d in gold])
    out = env.new_outputs(True)
    for ep in (1, 2):
        env.reset_from_draws(list(range(8)), [d[f"ep{ep}_draws"] for d in gold])
        idx = [episode_steps(d, ep) for d in gold]
        nmax = max(i.size for i in idx)
        for k in range(nmax):
            act = np.zeros((8, 7), dtype=np.float32)
            active = np.zeros(8, dtype=bool)
            for m in range(8):
                if k < idx[m].size:
                    act[m] = gold[m]["step_action"][idx[m][k]]
                    active[m] = True
            obs, rew, done, info = env.step(torch.as_tensor(act, device=env.device),
                                            active=torch.as_tensor(active, device=env.device), out=out)
            obs, rew, done, info = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy(), info.cpu().numpy()
            for m in np.nonzero(active)[0]:
                d, j = gold[m], idx[m][k]
                _close_obs(obs[m], d["step_obs"][j])
                np.testing.assert_allclose(rew[m], d["step_reward"][j], rtol=2e-6, atol=1e-7)
                assert bool(done[m]) == bool(d["step_done"][j]), (ep, k, m)
                np.testing.assert_allclose(info[m], d["step_info"][j], rtol=1e-5, atol=1e-6)
                st = env.get_state(int(m)) if k % 37 == 0 or k == idx[m].size - 1 else None
                if st is not None:
                    np.testing.assert_allclose(st[1:6], d["step_q_after"][j], rtol=0, atol=1e-9)
                    assert st[0] == d["step_counts"][j]
        if ep == 1:
            for m in range(8):
                assert gold[m]["step_done"][idx[m][-1]]
                assert idx[m].size == int(gold[m]["L"]) - 3


@pytest.mark.parametrize("variant", VARIANTS)
def test_done_envs_are_skipped(variant):
    from exo_amd import VecExoskeletonEnv
    env = VecExoskeletonEnv(8, seed=3)
    env.set_step_variant(variant)
    env.reset()
    out = env.new_outputs(True)
    a = torch.zeros((8, 7), device=env.device)
    L = env.lengths_host
    for k in range(int(L.max()) + 5):
        env.step(a, out=out)
    st = np.array([env.get_state(m)[0] for m in range(8)])
    np.testing.assert_array_equal(st, L - 1)


@pytest.mark.parametrize("variant", VARIANTS)
def test_philox_path_matches_oracle_at_scale(variant):
    """4096 envs on Philox draws; a sample of envs is replayed on the oracle
    with the same draw streams and random actions."""
    from exo_amd import VecExoskeletonEnv, motions
    N, seed = 4096, 99
    env = VecExoskeletonEnv(N, seed=seed)  # episode 0 drawn by the constructor
    env.set_step_variant(variant)
    obs0 = env.reset().cpu().numpy()       # episode 1
    angles, lengths = motions.load()
    lib = model_host()
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (12, N, 7)).astype(np.float32)
    outs = []
    o = env.new_outputs(True)
    for k in range(12):
        ob, r, dn, inf = env.step(torch.as_tensor(acts[k], device=env.device), out=o)
        outs.append((ob.cpu().numpy().copy(), r.cpu().numpy().copy(), inf.cpu().numpy().copy()))
    for e in [0, 1, 7, 8, 1023, 2047, 3001, 4095]:
        m = e % 8
        L = int(lengths[m])
        cfg = env_kwargs_default()
        oe = O.OracleEnv(angles[m][:, :L], cfg["seq"], cfg["amp"], cfg["h1"], cfg["h2"], 40.0, 20.0, 0.02, 0.03, 0.1)
        oe.reset(philox_draws(L, seed, e, 0, lib))
        ob = oe.reset(philox_draws(L, seed, e, 1, lib))
        _close_obs(obs0[e], ob)
        for k in range(12):
            ob, r, dn, info, _ = oe.step(acts[k][e].astype(np.float64))
            _close_obs(outs[k][0][e], ob)
            np.testing.assert_allclose(outs[k][1][e], r, rtol=2e-6, atol=1e-7)
            np.testing.assert_allclose(outs[k][2][e], info, rtol=1e-5, atol=1e-6)


def env_kwargs_default():
    return dict(seq=np.array([0, 1, 0, 1, 0, 0, 0], dtype=np.int32), amp=np.array([0.95, 1.05]),
                h1=np.array([4.0, 6.0]), h2=np.array([8.0, 10.0]))


def test_state_roundtrip_and_reset_mask():
    from exo_amd import VecExoskeletonEnv
    env = VecExoskeletonEnv(16, seed=11)
    env.reset()
    a = torch.full((16, 7), 0.3, device=env.device)
    for _ in range(5):
        env.step(a)
    st = env.get_state(3)
    env.set_state(3, st)
    np.testing.assert_array_equal(env.get_state(3), st)
    mask = torch.zeros(16, dtype=torch.bool, device=env.device)
    mask[3] = True
    env.reset(mask=mask)
    assert env.get_state(3)[0] == 2 and env.get_state(4)[0] == 7
    assert env.get_state(3)[49] == st[49] + 1  # episode counter advanced only for env 3


def test_drop_in_single_env_api():
    import Environment.Exoskeleton_env as E
    np.random.seed(0)
    env = E.ExoskeletonEnv_train(reference_motion_file_num="2", tremor_sequence=np.array([0, 1, 0, 1, 0, 0, 0]),
                                 tremor_amplitude_range=np.array([0.95, 1.05]),
                                 first_harmonics_interval=np.array([4, 6]),
                                 second_harmonics_interval=np.array([8, 10]), max_force_shoulder=40,
                                 max_force_elbow=20)
    assert env.observation_space.shape == (80,) and env.action_space.shape == (7,)
    obs, score = env.reset()
    assert obs.shape == (80,) and obs.dtype == np.float32 and score == 2
    n = 0
    done = False
    while not done:
        obs, r, done, trunc, info = env.step(np.random.uniform(-1, 1, 7))
        n += 1
        assert isinstance(r, float) and trunc is False
        assert set(info) == {"actuator_torques", "torque_val", "ampl_val", "tremor_torque_val", "tremor_ampl_val",
                             "reward_unwanted", "reward_torque", "reward_axis", "reward_control",
                             "reward_smoothness"}
    assert n == env.return_max_length() - 3
    with pytest.raises(IndexError):
        env.step(np.zeros(7))
    seq, mx = env.return_generated_tremor_data()
    assert mx.shape == (7,) and mx[1] > 0 and mx[0] == 0
    assert len(env.return_original_joint_angles()) == 7
    env.close()


def test_kernel_variants_agree():
    """Row-parallel and one-lane-per-solve kernels on identical states (N not a
    multiple of 4 to exercise the partial last block)."""
    from exo_amd import VecExoskeletonEnv
    envs = []
    for v in VARIANTS:
        e = VecExoskeletonEnv(1030, seed=21)
        e.set_step_variant(v)
        e.reset()
        envs.append(e)
    rng = np.random.default_rng(4)
    for k in range(40):
        a = torch.as_tensor(rng.uniform(-1, 1, (1030, 7)).astype(np.float32), device=envs[0].device)
        outs = [[t.cpu().numpy() for t in (o[0], o[1], o[3])] for o in (e.step(a) for e in envs)]
        o0 = outs[0]
        for o1 in outs[1:]:
            np.testing.assert_allclose(o0[0], o1[0], rtol=1e-6, atol=1e-7)
            np.testing.assert_allclose(o0[1], o1[1], rtol=1e-6, atol=1e-8)
            np.testing.assert_allclose(o0[2], o1[2], rtol=1e-5, atol=1e-7)
    for i in (0, 513, 1029):
        for e in envs[1:]:
            np.testing.assert_allclose(envs[0].get_state(i), e.get_state(i), rtol=1e-9, atol=1e-12)
    # the two row-parallel launch shapes run the same code per env: bit-identical
    for i in (0, 513, 1029):
        np.testing.assert_array_equal(envs[0].get_state(i), envs[2].get_state(i))


@pytest.mark.parametrize("variant", VARIANTS)
def test_domain_randomisation_sweep_matches_oracle(variant):
    """BASELINE configs[3]: 16,384 envs with per-env DR draws
    (matrix_noise_fraction ~ U(0.05, 0.25), dr_actuator_range ~ U(0, 0.1),
    dr_actuator_end_pos_shift ~ U(0, 0.04), tremor magnitude range [0.1, 1.0]
    -- Exoskeleton_env.py:70's range); a sample of envs replayed on the oracle
    with each env's own parameters and draw streams."""
    from exo_amd import VecExoskeletonEnv, motions
    N, seed = 16384, 2024
    rng = np.random.default_rng(3)
    mat_f = rng.uniform(0.05, 0.25, N)
    act_r = rng.uniform(0.0, 0.1, N)
    shift_r = rng.uniform(0.0, 0.04, N)
    env = VecExoskeletonEnv(N, seed=seed, matrix_noise_fraction=mat_f, dr_actuator_range=act_r,
                            dr_actuator_end_pos_shift=shift_r, tremor_amplitude_range=(0.1, 1.0))
    env.set_step_variant(variant)
    obs0 = env.reset().cpu().numpy()
    angles, lengths = motions.load()
    lib = model_host()
    acts = rng.uniform(-1, 1, (6, N, 7)).astype(np.float32)
    outs = []
    o = env.new_outputs(True)
    for k in range(6):
        ob, r, dn, inf = env.step(torch.as_tensor(acts[k], device=env.device), out=o)
        outs.append((ob.cpu().numpy().copy(), r.cpu().numpy().copy(), inf.cpu().numpy().copy()))
    cfg = env_kwargs_default()
    for e in [0, 5, 4097, 9999, 16383]:
        m = e % 8
        L = int(lengths[m])
        oe = O.OracleEnv(angles[m][:, :L], cfg["seq"], np.array([0.1, 1.0]), cfg["h1"], cfg["h2"], 40.0, 20.0,
                         shift_r[e], act_r[e], mat_f[e])
        oe.reset(philox_draws(L, seed, e, 0, lib))
        ob = oe.reset(philox_draws(L, seed, e, 1, lib))
        _close_obs(obs0[e], ob)
        _, D, S, sh, mx = oe.episode()
        Dg, Sg, _, shg, mxg = env.episode(e)   # per-env DR draws: bit-exact
        np.testing.assert_array_equal(Dg, D)
        np.testing.assert_array_equal(Sg, S)
        np.testing.assert_array_equal(shg, sh)
        np.testing.assert_array_equal(mxg, mx)
        for k in range(6):
            ob, r, dn, info, _ = oe.step(acts[k][e].astype(np.float64))
            _close_obs(outs[k][0][e], ob)
            np.testing.assert_allclose(outs[k][1][e], r, rtol=2e-6, atol=1e-7)
            np.testing.assert_allclose(outs[k][2][e], info, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("model", [("shipped", None, "per_sample"), ("docstring_axis", [10, 5, 2.5, 5, 5, .5, .5], "per_axis"),
                                   ("docstring_none", [10, 5, 2.5, 5, 5, .5, .5], "none")])
def test_tremor_model_knob(model):
    """exo_set_tremor_model (the diagnostic tremor models of tools/eval_hypotheses.py):
    the reset's tremor table against a numpy restatement of
    generate_parkinson_tremor.py:5-73 fed the same draws, with the given
    joint maxima and sign mode; the draw stream is the same in every mode."""
    from exo_amd import VecExoskeletonEnv, draws_per_episode
    name, jmax, sign = model
    n = 8
    seq = np.array([1, 1, 1, 1, 0, 1, 0])
    env = VecExoskeletonEnv(n, seed=3, tremor_sequence=seq, tremor_amplitude_range=(0.9, 1.1))
    env.set_tremor_model(jmax, sign)
    J = np.array(jmax if jmax is not None else [2.5, 5, 10, 5, 5, 0.5, 0.5])
    rng = np.random.default_rng(11)
    draws = [rng.random(draws_per_episode(int(L))) for L in env.lengths_host]
    env.reset_from_draws(np.arange(n), draws)
    for e in range(n):
        L, u = int(env.lengths_host[e]), draws[e]
        mag = 0.9 + u[0] * 0.2
        f1, f2 = 4 + 2 * u[1], 8 + 2 * u[2]
        t = np.linspace(0, L / 40, L)
        w1, w2, noise = np.sin(2 * np.pi * f1 * t), np.sin(2 * np.pi * f2 * t), u[3:3 + L] * 0.001
        want = np.zeros((7, L))
        for i in range(7):
            b = 3 + L + i * (L + 2)
            a1, a2 = 10 ** ((-5 + 5 * u[b]) / 20), 10 ** ((-20 + 10 * u[b + 1]) / 20)
            acc = (a1 * w1 + a2 * w2 + noise) * seq[i]
            with np.errstate(invalid="ignore"):
                v = np.nan_to_num((-1 + 2 * (acc - acc.min()) / (acc.max() - acc.min())) * J[i] * mag)
            s = {"per_sample": np.where(u[b + 2:b + 2 + L] < 0.5, -1.0, 1.0),
                 "per_axis": np.where(u[b + 2] < 0.5, -1.0, 1.0), "none": 1.0}[sign]
            want[i] = v * s
        np.testing.assert_allclose(env.tremor(e), want, rtol=0, atol=1e-12 * J.max(), err_msg=f"{name} env {e}")
    if sign != "per_sample":  # no per-sample flips: every axis reaches its maximum jmax * magnitude
        for e in range(n):
            mx = env.tremor(e).max(axis=1)
            mag = 0.9 + draws[e][0] * 0.2
            np.testing.assert_allclose(mx[seq == 1], (J * mag)[seq == 1], rtol=1e-12)


def test_step_clock_brackets_every_step_launch():
    """exo_set_step_clock (bench.py's in-window env-step time for configs[3] /
    [4]): counts every step launch, eager and graph-replayed, measures a
    positive time no longer than the HIP-event time around the same launches,
    leaves the step's outputs unchanged, and stops counting when turned off."""
    from exo_amd import VecExoskeletonEnv
    n = 64
    outs = []
    for clocked in (False, True):
        env = VecExoskeletonEnv(n, seed=5)
        env.reset()
        clk = env.set_step_clock() if clocked else None
        g = torch.Generator(device="cuda").manual_seed(9)
        obs = []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            act = torch.rand((n, 7), device="cuda", generator=g) * 2 - 1
            obs.append(env.step(act)[0].clone())
        e1.record()
        torch.cuda.synchronize()
        outs.append(torch.stack(obs))
        if clocked:
            ms, cnt = env.step_clock_ms()
            assert cnt == 5 and 0 < ms <= e0.elapsed_time(e1) / 5 * 1.05
            # captured: the clock kernels replay with the step
            act = torch.zeros((n, 7), device="cuda")
            o = env.new_outputs(True)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                from exo_amd.graphs import new_graph
                graph = new_graph()
                with torch.cuda.graph(graph, stream=s):
                    env.step(act, out=o)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            base = int(clk[2])
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize()
            assert int(clk[2]) == base + 3
            env.set_step_clock(False)
            env.step(act)
            torch.cuda.synchronize()
            assert int(clk[2]) == base + 3
    torch.testing.assert_close(outs[0], outs[1], rtol=0, atol=0)
