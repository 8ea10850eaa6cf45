"""T4: Agent.maybe_train_and_checkpoint / train_and_reset
(Agent/TD7_multi_agent.py:296-325) against the reference's decisions over 40
recorded episodes (tests/golden/checkpoint_policy.npz, train() stubbed to its
step counter): early policy-evaluation stop, checkpoint refresh of the actor
and the fixed encoder, the steps_before_checkpointing switch with
reset_weight and max_eps_when_checkpointing.  Exact: the logic is host-side
scalar bookkeeping."""
import numpy as np
import pytest
import torch

from helpers import GOLDEN
from exo_amd.td7 import Agent, GradSync, Hyperparameters, TD7Learner


def _hp(g):
    steps, max_eps, w = g["hp"]
    return Hyperparameters(zs_dim=8, enc_hdim=8, critic_hdim=8, actor_hdim=8, batch_size=4,
                           steps_before_checkpointing=int(steps), max_eps_when_checkpointing=int(max_eps),
                           reset_weight=float(w))


def _replay(ag, g):
    L = ag.learner

    def stub_train():
        L.training_steps += 1
    ag.train = stub_train
    for j, (n, r) in enumerate(zip(g["ep_len"], g["ret"])):
        with torch.no_grad():
            L.actor.l3.bias[0] = float(j)
            L.fixed_encoder.zs1.bias[0] = float(j)
        ag.maybe_train_and_checkpoint(int(n), float(r))
        got = [ag.eps_since_update, ag.timesteps_since_update, ag.max_eps_before_update, ag.min_return,
               ag.best_min_return, L.training_steps, float(L.checkpoint_actor.l3.bias[0].detach()),
               float(L.checkpoint_encoder.zs1.bias[0].detach())]
        np.testing.assert_array_equal(np.array(got, dtype=np.float64), g["trace"][j], err_msg=f"episode {j}")


def test_checkpoint_policy_matches_reference_cpu():
    g = np.load(f"{GOLDEN}/checkpoint_policy.npz", allow_pickle=False)
    ag = Agent.__new__(Agent)  # the host logic without the GPU replay buffer
    ag.hp = _hp(g)
    ag.sync = GradSync(None)
    ag.learner = TD7Learner(80, 7, ag.hp, learning_steps=1000, device="cpu", fused_adam=False)
    ag._init_checkpointing()
    _replay(ag, g)


@pytest.mark.gpu
def test_checkpoint_policy_matches_reference_gpu_agent():
    g = np.load(f"{GOLDEN}/checkpoint_policy.npz", allow_pickle=False)
    ag = Agent(80, 7, 1, learning_steps=1000, hp=_hp(g), env_num=2, device="cuda", buffer_size=64)
    _replay(ag, g)
