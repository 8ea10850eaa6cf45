"""Host (gcc) build of the device math in csrc/exo_model.h vs the oracle and the
reference's RK45 goldens.  Validates the algorithms the HIP kernels run (RK45 in
second-order storage form, URDF FK, cos(atan2) identity, Philox draws) without
a GPU."""
import ctypes
import math

import numpy as np

import oracle as O
from helpers import GOLDEN, model_host, pack_ode

D = ctypes.POINTER(ctypes.c_double)


def _rk45(L, I, Dm, S, T):
    ii, dn, sn = pack_ode(I, Dm, S)
    T = np.ascontiguousarray(T, dtype=np.float64)
    q = np.zeros(7)
    rc = L.mh_rk45(ii.ctypes.data_as(D), dn.ctypes.data_as(D), sn.ctypes.data_as(D), T.ctypes.data_as(D),
                   q.ctypes.data_as(D))
    assert rc == 0
    return q


def test_rk45_second_order_form_matches_scipy():
    L = model_host()
    o = np.load(f"{GOLDEN}/ode_cases.npz")
    for i in range(len(o["T"])):
        q = _rk45(L, o["I"][i], o["D"][i], o["S"][i], o["T"][i])
        ref = o["q"][i]
        assert np.abs(q - ref).max() <= 1e-10 * max(np.abs(ref).max(), 1e-300), i


def test_matrices_keep_the_block_structure():
    o = np.load(f"{GOLDEN}/ode_cases.npz")
    for i in range(len(o["T"])):
        I, Dm, S = o["I"][i], o["D"][i], o["S"][i]
        assert np.all(I[np.ix_([0, 3, 6], [1, 2, 4, 5])] == 0)
        assert np.all(Dm[:4, 4:] == 0) and np.all(S[:4, 4:] == 0)
        assert Dm[1, 3] == 0 and Dm[2, 3] == 0 and S[1, 3] == 0 and S[2, 3] == 0
        np.testing.assert_array_equal(Dm, Dm.T)
        np.testing.assert_array_equal(S, S.T)


def test_fk_matches_oracle():
    L = model_host()
    rng = np.random.default_rng(0)
    K = [9, 5, 12, 6, 15, 8, 17, 11, 14, 7, 18, 13, 16, 10]
    for _ in range(50):
        q5 = rng.uniform(-1.5, 1.5, 5)
        act, ref = np.zeros(42), np.zeros(6)
        L.mh_link_coms(q5.ctypes.data_as(D), act.ctypes.data_as(D), ref.ctypes.data_as(D))
        com = O.link_coms(q5)
        np.testing.assert_allclose(act.reshape(14, 3), com[K], atol=1e-14)
        np.testing.assert_allclose(ref, np.concatenate([com[0], com[3]]), atol=1e-14)


def test_cos_atan2_identity():
    L = model_host()
    rng = np.random.default_rng(1)
    cases = [(0.0, 0.0), (0.0, -0.0), (-0.0, 0.0), (-0.0, -0.0), (1e-3, 0.0), (0.0, -2.0), (5.0, 1e-300)]
    cases += [tuple(x) for x in rng.normal(0, 1, (2000, 2))]
    for y, x in cases:
        ref = math.cos(math.atan2(y, x))
        assert abs(L.mh_cos_atan2(y, x) - ref) <= 4e-16, (y, x)


def test_philox_draws_are_uniform_and_distinct():
    L = model_host()
    u = np.array([L.mh_philox_u01(123, e, ep, p) for e in range(4) for ep in range(3) for p in range(2000)])
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01 and abs(u.var() - 1 / 12) < 0.005
    assert np.unique(u).size == u.size
    hist, _ = np.histogram(u, bins=20, range=(0, 1))
    chi2 = ((hist - u.size / 20) ** 2 / (u.size / 20)).sum()
    assert chi2 < 60  # 19 dof, p ~ 1e-6
