"""The row-parallel step kernel's three RHS neighbour-exchange forms (csrc/exo_step_rp.hip,
EXO_RP_GATHER: 2 = wave-private LDS slots (default), 0 = ds_bpermute permutes, 1 = DPP
lane moves) evaluate the same terms in the same order, so they must agree BIT FOR BIT on
every output and on the carried state, in both row-parallel launch shapes.

The exchange form is read once per process (a static in the launcher), so each form runs
in its own child process; this parent never touches the GPU.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd")

WORKER = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from exo_amd import VecExoskeletonEnv
out = {}
n = 1030  # not a multiple of the workgroup's env count: partial last block
for variant in ("rows", "rows_shared"):
    env = VecExoskeletonEnv(n, seed=33)
    env.set_step_variant(variant)
    env.reset()
    rng = np.random.default_rng(9)
    obs, rew, info = [], [], []
    for k in range(24):
        a = torch.as_tensor(rng.uniform(-1, 1, (n, 7)).astype(np.float32), device=env.device)
        o, r, d, i = env.step(a)
        obs.append(o.cpu().numpy()); rew.append(r.cpu().numpy()); info.append(i.cpu().numpy())
    out[variant + "_obs"] = np.stack(obs)
    out[variant + "_rew"] = np.stack(rew)
    out[variant + "_info"] = np.stack(info)
    out[variant + "_state"] = np.stack([env.get_state(e) for e in range(0, n, 7)])
    env.close()
np.savez(sys.argv[2], **out)
"""


def _run(form, path):
    env = dict(os.environ, EXO_RP_GATHER=str(form))
    subprocess.run([sys.executable, "-c", WORKER, PKG, path], check=True, env=env, timeout=300)
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


def test_rhs_exchange_forms_are_bit_identical(tmp_path):
    res = {f: _run(f, str(tmp_path / f"form{f}.npz")) for f in (2, 0, 1)}
    for k, v in res[2].items():
        assert np.isfinite(v).all(), k
        for f in (0, 1):
            np.testing.assert_array_equal(v, res[f][k], err_msg=f"EXO_RP_GATHER={f} vs 2: {k}")
