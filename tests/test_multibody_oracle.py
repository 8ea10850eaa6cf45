"""The multibody stepSimulation oracle (oracle/multibody.c).

Bullet itself is absent (pybullet 3.2.5 is not installed), so this mode is
"parity unpinned" against the reference's physics engine.  What is pinned:
  * Featherstone's three recursions agree with each other: the Articulated-Body
    Algorithm's accelerations reproduce the applied joint forces through the
    Recursive Newton-Euler Algorithm and through M qdd + h with the
    Composite-Rigid-Body mass matrix (1e-12 relative);
  * the mass matrix is symmetric positive definite with the URDF tree's
    sparsity (k-links couple only with their ancestors);
  * the model reduces to the idealised motor model of SURVEY.md A.2 (which the
    reference goldens pin, tests/test_oracle.py) whenever the impulse solve
    converges: the first step from rest, and every step of the golden episodes
    of motions 4..7, agree with the idealised model to 1e-12 rad;
  * violated joint limits push back, free k-links fall under gravity.
"""
import numpy as np
import pytest

import oracle as O
from helpers import episode_steps, golden_env
from exo_amd import motions

PARENT = [-1, 0, 1, 2, 3, 4, 4, 2, 2, 2, 2, 2, 2, 2, -1, -1, -1, -1, -1]


def _ancestors(i):
    out = set()
    while PARENT[i] >= 0:
        i = PARENT[i]
        out.add(i)
    return out


def _random_state(rng, spread=1.0):
    q = rng.uniform(-spread, spread, 19)
    q[5:] *= 0.2
    return q, rng.uniform(-2, 2, 19)


def test_aba_rnea_crba_agree():
    rng = np.random.default_rng(0)
    for _ in range(20):
        q, qd = _random_state(rng)
        tau = rng.uniform(-5, 5, 19)
        qdd = O.mb_aba(q, qd, tau)
        np.testing.assert_allclose(O.mb_rnea(q, qd, qdd), tau, rtol=0, atol=1e-12 * 10)
        M = O.mb_mass(q)
        h = O.mb_rnea(q, qd, np.zeros(19))
        np.testing.assert_allclose(M @ qdd + h, tau, rtol=0, atol=1e-12 * 10)


def test_mass_matrix_structure():
    rng = np.random.default_rng(1)
    for _ in range(10):
        q, _ = _random_state(rng)
        M = O.mb_mass(q)
        assert np.array_equal(M, M.T)
        assert np.linalg.eigvalsh(M).min() > 0
        for i in range(19):
            for j in range(19):
                related = i == j or j in _ancestors(i) or i in _ancestors(j)
                if not related:
                    assert M[i, j] == 0.0, (i, j)
        # the k-links have unit mass along their axes
        np.testing.assert_allclose(np.diag(M)[5:], 1.0, rtol=1e-12)


def test_free_k_links_fall_along_their_axes():
    # at rest, without solver rows, a base k-link (vertical axis up to the
    # 3.141593-vs-pi tilt of its rpy) accelerates at -g
    qdd = O.mb_aba(np.zeros(19), np.zeros(19))
    np.testing.assert_allclose(qdd[14:], -9.81, rtol=1e-10)


def test_first_step_from_rest_is_the_idealised_motor_step():
    tgt = np.array([0.2, 0.3, -0.4, 0.5, 0.1])
    q, qd, st = O.mb_step(np.zeros(19), np.zeros(19), tgt)
    np.testing.assert_allclose(q[:5], 0.1 * tgt, rtol=0, atol=1e-14)
    np.testing.assert_allclose(q[5:], 0.0, atol=1e-15)
    assert st[0] == 0 and st[1] < 1e-12


def test_violated_limit_pushes_back():
    # a base k-link 0.1 m beyond its +0.5 m limit: the limit row (target -erp
    # pen / dt = -0.8 m/s) outlasts its velocity motor (impulse <= 1 N s)
    q = np.zeros(19)
    q[14] = 0.6
    q1, qd1, st = O.mb_step(q, np.zeros(19), np.zeros(5))
    assert st[0] == 1
    np.testing.assert_allclose(qd1[14], -0.2 * 0.1 / (1 / 40), rtol=1e-9)
    # rows are swept limits first, motors second (Bullet's creation order): an
    # unsaturated revolute motor overrides its joint's limit row ...
    q = np.zeros(19)
    q[3] = 2.7  # elbow y beyond its upper limit 2.6179938726127 (exo_v3.urdf:77)
    tgt = np.array([0.0, 0.0, 0.0, 3.0, 0.0])
    q1, qd1, st = O.mb_step(q, np.zeros(19), tgt)
    np.testing.assert_allclose(qd1[3], 0.1 * (3.0 - 2.7) * 40, rtol=1e-9)
    # ... a saturated one does not
    q1, qd1, st = O.mb_step(q, np.zeros(19), tgt, O.mb_params(motor_impulse=1e-4))
    assert qd1[3] < 0.0 and q1[3] < q[3]


@pytest.mark.parametrize("m", [4, 5, 6, 7])
def test_converged_golden_episodes_equal_the_idealised_model(m):
    d = golden_env(m)
    L = int(d["L"])
    angles, _ = motions.load()
    envs = []
    for mode in ("ideal", "multibody"):
        e = O.OracleEnv(angles[m][:, :L], d["tremor_seq"], d["amp_range"], d["harm1"], d["harm2"], d["max_force"][0],
                        d["max_force"][1], d["dr"][0], d["dr"][1], d["dr"][2])
        e.set_physics(mode)
        e.reset(d["ep0_draws"])
        envs.append(e)
    for e in envs:
        e.reset(d["ep1_draws"])
    for k in episode_steps(d, 1):
        o1 = envs[0].step(d["step_action"][k])
        o2 = envs[1].step(d["step_action"][k])
        np.testing.assert_allclose(envs[1].phys_q(), envs[0].phys_q(), rtol=0, atol=1e-12)
        np.testing.assert_allclose(o2[0], o1[0], rtol=1e-6, atol=1e-7)
        q, qd, st = envs[1].mb_state()
        assert st[1] < 1e-9 and np.abs(q[5:]).max() < 1e-12
