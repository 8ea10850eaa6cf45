"""BASELINE.json configurations run end to end on the MI355X (the bench's own
loop: VecTrainer, HIP-graph replays), with a sample of envs replayed on the
oracle (oracle/exo_oracle.c) from the same Philox draw streams and the
actions the policy actually took.

* configs[4]: 65,536 envs, wide TD7 (every MLP and zs 1,024), fp16 MFMA
  operands -- the update itself is pinned by tests/test_td7_full.py against
  the reference's wide golden; here the whole iteration runs at scale.
"""
import numpy as np
import pytest
import torch

import oracle as O
from helpers import model_host, philox_draws

pytestmark = pytest.mark.gpu

SEQ = np.array([0, 1, 0, 1, 0, 0, 0], dtype=np.int32)


def _close_obs(a, b):
    np.testing.assert_allclose(a, b, rtol=2e-6, atol=2e-6)


def _run_and_check(N, hp, precision, seed, sample, iters=5):
    from exo_amd import VecExoskeletonEnv, motions
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent
    torch.manual_seed(seed)
    env = VecExoskeletonEnv(N, seed=seed)
    agent = Agent(80, 7, 1, env_num=8, hp=hp, precision=precision, n_envs=N, graph_safe=True)
    tr = VecTrainer(env, agent)
    idx = torch.as_tensor(sample, device=env.device)
    obs = [tr.obs.index_select(0, idx).cpu().numpy()]
    acts = []
    before = torch.cat([p.detach().reshape(-1) for p in agent.learner.critic.parameters()]).clone()
    for _ in range(iters):
        assert tr.step() == N   # every motion runs >= 229 steps: all envs active
        acts.append(tr.last_actions.index_select(0, idx).cpu().numpy())
        obs.append(tr.obs.index_select(0, idx).cpu().numpy())
    torch.cuda.synchronize()
    assert len(tr.graphs) == 2 and agent.learner.training_steps == iters
    after = torch.cat([p.detach().reshape(-1) for p in agent.learner.critic.parameters()])
    assert torch.isfinite(after).all() and not torch.equal(before, after)
    for m in (agent.learner.actor, agent.learner.encoder):
        assert all(torch.isfinite(p).all() for p in m.parameters())
    angles, lengths = motions.load()
    lib = model_host()
    for j, e in enumerate(sample):
        m = e % 8
        L = int(lengths[m])
        oe = O.OracleEnv(angles[m][:, :L], SEQ, [0.95, 1.05], [4, 6], [8, 10], 40.0, 20.0, 0.02, 0.03, 0.1)
        oe.reset(philox_draws(L, seed, e, 0, lib))
        _close_obs(obs[0][j], oe.reset(philox_draws(L, seed, e, 1, lib)))
        for k in range(iters):
            assert np.all(np.abs(acts[k][j]) <= 1.0)
            ob, r, done, _, _ = oe.step(acts[k][j].astype(np.float64))
            _close_obs(obs[k + 1][j], ob)
            assert not done


def test_configs4_wide_iteration_65536_envs():
    from exo_amd.td7 import Hyperparameters
    hp = Hyperparameters(zs_dim=1024, enc_hdim=1024, critic_hdim=1024, actor_hdim=1024)
    _run_and_check(65536, hp, "fp16", 4242, [0, 1, 9, 4095, 32767, 40001, 65535])


def test_configs1_iteration_4096_envs():
    from exo_amd.td7 import Hyperparameters
    _run_and_check(4096, Hyperparameters(), "bf16", 77, [0, 3, 8, 2049, 4095])
