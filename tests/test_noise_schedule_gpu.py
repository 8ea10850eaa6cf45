"""The exploration-noise schedule on the device: the reference
decrements exploration_noise once per select_action call on a Python float64
(Agent/TD7_multi_agent.py:207, called once per running env by
Simulation/Exoskeleton_agent_train.py:128).  The build keeps sigma as a float32
device scalar and subtracts dec * (running envs) once per vectorised step.
Nothing in the reference pins which rounding is right (parity unpinned); this
pins the drift over a long horizon against the float64 recurrence, and the
data-parallel rule (every rank's envs count: the decrement scales with the
world size)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fused", [True, False])
def test_sigma_tracks_the_float64_recurrence(fused, monkeypatch):
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(0)
    if not fused:
        monkeypatch.setenv("EXO_TD7_FUSED", "0")
    N, steps = 4096, 1000
    ag = Agent(80, 7, 1, learning_steps=6_000_000, env_num=8, hp=Hyperparameters(), precision="bf16", n_envs=N,
               buffer_size=1024)
    assert (ag.learner.fused is not None) == fused
    obs = torch.randn(N, 80, device="cuda")
    count = torch.tensor([N], dtype=torch.int32, device="cuda")
    dec = ag.learner.action_noise_decrease
    want = float(ag.hp.exploration_noise)
    for k in range(steps):
        n = N - (k % 7) * 100  # envs finishing at different steps
        count.fill_(n)
        ag.select_action_batch(obs, dec_count=count)
        for _ in range(n):  # the script: one float64 subtraction per select_action call
            want -= dec
    got = float(ag.learner.exploration_noise_t)
    # float32 storage: at most half an ulp per update (ulp(0.1) = 7.45e-9)
    assert abs(got - want) <= steps * 3.8e-9, (got, want)
    assert abs(got - want) / abs(want) < 1e-4


def test_data_parallel_decrement_counts_every_rank():
    """GradSync.world scales the per-step decrement: a replica decrements by
    every rank's running envs (ranks step identical env layouts)."""
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(0)
    ag = Agent(80, 7, 1, learning_steps=100_000, env_num=8, hp=Hyperparameters(), precision="bf16", n_envs=64,
               buffer_size=1024)
    ag.sync.world = 4  # as a 4-rank process group reports it
    obs = torch.randn(64, 80, device="cuda")
    count = torch.tensor([64], dtype=torch.int32, device="cuda")
    s0 = float(ag.learner.exploration_noise_t)
    ag.select_action_batch(obs, dec_count=count)
    assert np.isclose(s0 - float(ag.learner.exploration_noise_t), 4 * 64 * ag.learner.action_noise_decrease,
                      rtol=1e-4)
