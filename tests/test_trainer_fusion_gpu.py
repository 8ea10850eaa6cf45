"""The graph-replayed trainer on the fused TD7 path (bf16, the bench's widths):
its scheduling options change where work runs, never what it computes.

* the optimiser steps inside the weight-gradient launches (td7f_wgrad_adam),
  as separate fused step+repack launches (td7f_adam_pack) and as the
  unfused td7_adam_step_multi + td7f_pack pair train to the same weights bit
  for bit (each launch is pinned to the next by tests/test_adam_pack_gpu.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(seed=0, n_envs=512):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(seed)
    hp = Hyperparameters(target_update_rate=7)
    env = VecExoskeletonEnv(n_envs, seed=seed)
    agent = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=1 << 14, precision="bf16", graph_safe=True)
    assert agent.learner.fused is not None
    return VecTrainer(env, agent, use_graphs=True), agent


def _params(agent):
    L = agent.learner
    return [p.detach().clone() for m in (L.actor, L.critic, L.encoder, L.actor_target, L.critic_target)
            for p in m.parameters()]


def _assert_same(a, b):
    assert len(a) == len(b)
    for k, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), f"parameter {k} differs"


@pytest.mark.parametrize("mode", ["adam_pack", "unfused"])
def test_optimiser_placement_does_not_change_training(mode, monkeypatch):
    import exo_amd.rollout as rollout
    import exo_amd.td7 as td7
    t1, a1 = _make(seed=6)
    for _ in range(10):
        t1.step()
    torch.cuda.synchronize()
    ref = _params(a1)
    monkeypatch.setattr(td7, "WGRAD_ADAM", False)
    if mode == "unfused":
        monkeypatch.setattr(td7, "ADAM_PACK", False)
        monkeypatch.setattr(rollout, "ENC_STEP_BRANCH", False)
    t2, a2 = _make(seed=6)
    for _ in range(10):
        t2.step()
    torch.cuda.synchronize()
    _assert_same(_params(a2), ref)


def test_fused_priority_update_and_next_sample_does_not_change_training(monkeypatch):
    """LAP.update_priority + the next iteration's sample as one launch
    (lap_update_sample_rng, r04) against the two launches: the same weights
    and replay trees after 12 graph-replayed iterations (a target refresh
    included)."""
    from exo_amd.replay import LAP
    outs = []
    for fused in (False, True):
        monkeypatch.setattr(LAP, "fuse_update_sample", fused)
        t, a = _make(seed=4)
        for _ in range(12):
            t.step()
        torch.cuda.synchronize()
        outs.append((_params(a), a.replay_buffer._tree.clone()))
    _assert_same(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_priority_update_after_the_critic_pass_does_not_change_training(monkeypatch):
    """LAP.update_priority_and_sample_td forked right after the critic pass
    (priorities from its |td|, r04) against the update after the weight-
    gradient launch (td7f_wgrad's priorities): the same weights, replay trees
    and batches bit for bit."""
    import exo_amd.rollout as rollout
    monkeypatch.setattr(rollout.VecTrainer, "us_after_critic", False)
    t1, a1 = _make(seed=9)
    for _ in range(10):
        t1.step()
    torch.cuda.synchronize()
    ref, tree_ref = _params(a1), a1.replay_buffer._tree.clone()
    monkeypatch.setattr(rollout.VecTrainer, "us_after_critic", True)
    t2, a2 = _make(seed=9)
    for _ in range(10):
        t2.step()
    torch.cuda.synchronize()
    _assert_same(_params(a2), ref)
    assert torch.equal(a2.replay_buffer._tree, tree_ref)
