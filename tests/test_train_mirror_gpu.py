"""configs[0] ("single exoskeleton env, TD7 agent 1k steps, seed 0"): the
training driver that mirrors Simulation/Exoskeleton_agent_train.py
(<pkg>/Simulation/Exoskeleton_agent_train.py, the four SURVEY §0 fixes marked
FIX 1-4) run through the drop-in ExoskeletonEnv_train, Agent,
LAP.add(tremor_num=i), maybe_train_and_checkpoint and save, then a load round
trip of the 8 checkpoint files.  The warm-up is lowered to 300 steps so the
policy (select_action on 1-D states) drives the later episodes."""
import os
import sys

import numpy as np
import pytest
import torch

from helpers import PKG

pytestmark = pytest.mark.gpu


def test_training_mirror_configs0(tmp_path):
    sys.path.insert(0, os.path.join(PKG, "Simulation"))
    import Exoskeleton_agent_train as drv
    args = drv.parse_args(["--seed", "0", "--n_steps", "1000", "--warmup", "300", "--num_reference_motions", "1",
                           "--save_dir", str(tmp_path), "--buffer_size", "20000", "--quiet"])
    out = drv.train(args)
    agent = out["agent"]
    L = agent.learner
    # motion 0: L = 232 -> 229 steps per episode; 1,000 steps -> 5 rounds
    assert out["steps"] == 5 * 229 and out["rounds"] == 5
    # every round trains round(mean(ep_len)) = 230 steps (:208, :315-325)
    assert L.training_steps == 5 * 230
    assert agent.replay_buffer.size == 5 * 229
    assert out["scores"].shape == (5, 1) and np.isfinite(out["scores"]).all()
    for m in (L.actor, L.critic, L.encoder):
        assert all(torch.isfinite(p).all() for p in m.parameters())
    # the policy drove rounds 3-5 with exploration: the noise scale decreased once per call
    assert L.exploration_noise < agent.hp.exploration_noise
    # the 8 checkpoint files (:330-345) load back into a fresh agent
    for suf in agent.SUFFIXES:
        assert os.path.exists(out["save_prefix"] + suf), suf
    from exo_amd.td7 import Agent
    ag2 = Agent(80, 7, 1, env_num=1, buffer_size=64)
    ag2.load(out["save_prefix"])
    for name in ("actor", "critic", "encoder", "checkpoint_actor", "checkpoint_encoder"):
        for p, q in zip(getattr(L, name).parameters(), getattr(ag2.learner, name).parameters()):
            torch.testing.assert_close(p, q, rtol=0, atol=0)
    torch.testing.assert_close(ag2.learner.critic_optimizer.m, L.critic_optimizer.m, rtol=0, atol=0)
    # the loaded agent acts like the saved one
    s = np.random.default_rng(0).normal(size=(4, 80)).astype(np.float32)
    np.testing.assert_allclose(ag2.select_action(s, use_checkpoint=True, use_exploration=False),
                               agent.select_action(s, use_checkpoint=True, use_exploration=False), atol=0, rtol=0)
    assert os.path.exists(os.path.join(str(tmp_path), "algo_score.npz"))
