"""The CPU oracle (oracle/exo_oracle.c) against the reference's golden vectors."""
import numpy as np
import pytest

import oracle as O
from helpers import episode_steps, golden_env, GOLDEN
from exo_amd import motions


def test_ode_matches_scipy_rk45():
    o = np.load(f"{GOLDEN}/ode_cases.npz")
    for i in range(len(o["T"])):
        q, nfev = O.solve_diff_eq(o["I"][i], o["D"][i], o["S"][i], o["T"][i])
        ref = o["q"][i]
        scale = max(np.abs(ref).max(), 1e-300)
        assert np.abs(q - ref).max() <= 1e-10 * scale, i
        assert nfev >= 8


def test_zero_torque_gives_zero():
    o = np.load(f"{GOLDEN}/ode_cases.npz")
    q, _ = O.solve_diff_eq(o["I"][0], o["D"][0], o["S"][0], np.zeros(7))
    assert np.all(q == 0)


def test_urdf_zero_config_coms():
    import json
    j = json.load(open(f"{GOLDEN}/urdf_links.json"))
    np.testing.assert_allclose(O.link_coms(np.zeros(5)), np.array(j["zero_config_coms"]), atol=1e-12)


@pytest.mark.parametrize("m", range(8))
def test_env_episodes_match_reference(m):
    d = golden_env(m)
    L = int(d["L"])
    angles, lengths = motions.load()
    assert lengths[m] == L
    e = O.OracleEnv(angles[m][:, :L], d["tremor_seq"], d["amp_range"], d["harm1"], d["harm2"], d["max_force"][0],
                    d["max_force"][1], d["dr"][0], d["dr"][1], d["dr"][2])
    np.testing.assert_array_equal(e.reset(d["ep0_draws"]), d["ep0_obs"])
    for ep in (1, 2):
        np.testing.assert_array_equal(e.reset(d[f"ep{ep}_draws"]), d[f"ep{ep}_obs"])
        np.testing.assert_array_equal(e.tremor(), d[f"ep{ep}_tremor"])
        I, D, S, sh, mm = e.episode()
        np.testing.assert_array_equal(I, d[f"ep{ep}_I"])
        np.testing.assert_array_equal(D, d[f"ep{ep}_D"])
        np.testing.assert_array_equal(S, d[f"ep{ep}_S"])
        np.testing.assert_array_equal(sh, d[f"ep{ep}_shift"])
        assert mm[0] == d[f"ep{ep}_maxS"] and mm[1] == d[f"ep{ep}_maxE"]
        for k in episode_steps(d, ep):
            obs, r, done, info, tgt = e.step(d["step_action"][k])
            np.testing.assert_array_equal(obs, d["step_obs"][k])
            assert abs(r - d["step_reward"][k]) <= 1e-12
            assert done == bool(d["step_done"][k])
            np.testing.assert_allclose(info, d["step_info"][k], rtol=1e-9, atol=1e-10)
            np.testing.assert_allclose(tgt, d["step_targets"][k], rtol=0, atol=1e-12)
            np.testing.assert_allclose(e.phys_q(), d["step_q_after"][k], rtol=0, atol=1e-12)
    # the full first episode ends exactly at L - 3 steps (done index is bit-exact)
    n1 = episode_steps(d, 1).size
    assert n1 == L - 3 and d["step_done"][episode_steps(d, 1)[-1]]
    with pytest.raises(IndexError):
        for _ in range(L):
            e.step(np.zeros(7))
