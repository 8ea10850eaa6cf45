"""Tremor-suppression statistics (Simulation/Exoskeleton_agent_train.py:149-200,
Utilities/calculate_arm_end_effector_points.py:18-50): the numpy oracle
against the reference's golden vectors (CPU), and the device kernel
(exo_tremor_metrics) against the oracle on a live env (GPU)."""
import numpy as np
import pytest
import torch

from helpers import GOLDEN


def test_oracle_dh_fk_matches_reference():
    import metrics as M
    g = np.load(f"{GOLDEN}/dh_fk.npz")
    for th, ln, pos in zip(g["theta"], g["lengths"], g["position"]):
        np.testing.assert_allclose(M.end_effector(th, *ln), pos, rtol=1e-13, atol=1e-15)


def test_oracle_step_metrics_match_reference():
    import metrics as M
    g = np.load(f"{GOLDEN}/metrics_cases.npz")
    for k in range(g["torque_val"].shape[0]):
        tr, ta, tot, cnt, _ = M.step_metrics(g["torque_val"][k], g["tremor_torque_val"][k], g["ampl_val"][k],
                                             g["tremor_ampl_val"][k], g["original_deg"][k])
        np.testing.assert_allclose(tr, g["tremor_reduction"][k], rtol=1e-13, atol=1e-12)
        np.testing.assert_allclose(ta, g["tremor_reduction_ampl"][k], rtol=1e-13, atol=1e-12)
        np.testing.assert_allclose(tot, g["ampl_total"][k], rtol=1e-12, atol=1e-12)
        np.testing.assert_array_equal(cnt, g["counter_deltas"][k])


@pytest.mark.gpu
def test_device_metrics_match_oracle_on_live_env():
    import metrics as M
    from exo_amd import VecExoskeletonEnv
    from exo_amd.vec_env import INFO_SLICES
    n = 64
    env = VecExoskeletonEnv(n, seed=11)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    counters = torch.zeros((n, 6), device="cuda")
    ref_counters = np.zeros((n, 6))
    for step in range(6):
        act = torch.rand((n, 7), device="cuda", generator=g) * 2 - 1
        active = torch.ones(n, dtype=torch.bool, device="cuda")
        active[step::7] = False
        obs, rew, done, info = env.step(act, active=active)
        m, counters = env.tremor_metrics(info, stepped=active, counters=counters)
        mh, ih = m.cpu().numpy(), info.cpu().numpy().astype(np.float64)
        for e in range(n):
            if not bool(active[e]):
                assert not mh[e].any()  # a done env's row of the step is zeros (:201-203)
                continue
            orig = env.original_joint_angles(e)
            tr, ta, tot, cnt, last = M.step_metrics(ih[e, INFO_SLICES["torque_val"]], ih[e, INFO_SLICES["tremor_torque_val"]],
                                                    ih[e, INFO_SLICES["ampl_val"]], ih[e, INFO_SLICES["tremor_ampl_val"]],
                                                    orig)
            np.testing.assert_allclose(mh[e, 0:7], tr, rtol=2e-5, atol=2e-4)
            np.testing.assert_allclose(mh[e, 7:14], ta, rtol=2e-5, atol=2e-4)
            np.testing.assert_allclose(mh[e, 14], tot, rtol=1e-4, atol=1e-4)
            ref_counters[e, :5] += cnt
            if last is not None:
                ref_counters[e, 5] = last
    c = counters.cpu().numpy()
    np.testing.assert_array_equal(c[:, :5], ref_counters[:, :5])
    np.testing.assert_allclose(c[:, 5], ref_counters[:, 5], rtol=1e-4, atol=1e-4)


def test_oracle_eval_counters_swap_and_selection():
    """Evaluate_control_performance.py:192-247 restated: the SFE/SAA swap only
    changes the FK total, the torque counters only look at the tremor axes."""
    import metrics as M
    orig = np.array([10.0, -20.0, 30.0, 40.0, 5.0, 0.0, 0.0])
    torque = np.array([1.0, -3.0, 0.5, 2.0, 0.0, 0.0, 0.0])
    tremor = np.array([2.0, 1.0, 0.0, 4.0, 0.0, 0.0, 0.0])
    ampl, tampl = np.array([1.0, 2.0, 0.5, 0.3, 0, 0, 0]), np.array([2.0, 1.0, 0.4, 0.6, 0, 0, 0])
    c = M.eval_step_counters(torque, tremor, ampl, tampl, orig, [1, 1, 0, 1, 0, 0, 0])
    # axis 0: (1-2)/2 < 0; axis 1: (3-1)/1 > 0; axis 3: (2-4)/4 < 0 -> not all, any
    assert c[0] == 0.0 and c[1] == 1.0
    c2 = M.eval_step_counters(torque, tremor, ampl, tampl, orig, [1, 0, 0, 1, 0, 0, 0])
    assert c2[0] == 1.0 and c2[1] == 1.0
    # the swap: same as the training-script total on pre-swapped amplitudes
    sw = [1, 0, 2, 3, 4, 5, 6]
    _, _, tot, _, _ = M.step_metrics(torque, tremor, ampl[sw], tampl[sw], orig, disregard=False)
    assert c[2] == float(tot < 0) and c[3] == float(not tot < 0)
    np.testing.assert_allclose(c[4], tot if tot < 0 else 0.0, rtol=1e-12)


@pytest.mark.gpu
def test_device_eval_counters_match_oracle_on_live_env():
    import metrics as M
    from exo_amd import VecExoskeletonEnv
    from exo_amd.vec_env import INFO_SLICES
    n = 64
    seqs = np.zeros((n, 7), dtype=np.int64)
    for e in range(n):
        seqs[e, :4] = [(e + 1) >> k & 1 for k in range(4)]
    seqs[seqs[:, :4].sum(1) == 0, 3] = 1
    env = VecExoskeletonEnv(n, seed=5, tremor_sequence=seqs)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    counters = torch.zeros((n, 5), device="cuda")
    ref = np.zeros((n, 5))
    for step in range(6):
        act = torch.rand((n, 7), device="cuda", generator=g) * 2 - 1
        active = torch.ones(n, dtype=torch.bool, device="cuda")
        active[step::5] = False
        obs, rew, done, info = env.step(act, active=active)
        counters = env.eval_metrics(info, stepped=active, counters=counters)
        ih = info.cpu().numpy().astype(np.float64)
        for e in range(n):
            if bool(active[e]):
                ref[e] += M.eval_step_counters(ih[e, INFO_SLICES["torque_val"]], ih[e, INFO_SLICES["tremor_torque_val"]],
                                               ih[e, INFO_SLICES["ampl_val"]], ih[e, INFO_SLICES["tremor_ampl_val"]],
                                               env.original_joint_angles(e), seqs[e])
    c = counters.cpu().numpy()
    np.testing.assert_array_equal(c[:, :4], ref[:, :4])
    np.testing.assert_allclose(c[:, 4], ref[:, 4], rtol=1e-4, atol=1e-3)
