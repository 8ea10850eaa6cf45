"""select_action ahead (VecTrainer.select_ahead, r04): in an iteration that does
not update the actor, the next step's actions are computed at the end of the
rollout branch; the next iteration starts with its env step.  The same
launches on the same inputs in the same order (the exploration-noise stream
and its scale included), so trajectories and weights are bit-identical to
selecting at the start of each iteration -- for both policy-update parities,
policy_freq 3, async and synchronous episodes (across a round reset, where
nothing is selected ahead), the fused and the per-layer TD7 paths."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(ahead, monkeypatch, fused, policy_freq=2, episodes="sync", iters=12, near_round_end=False):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    monkeypatch.setattr(VecTrainer, "select_ahead", ahead)
    torch.manual_seed(5)
    if fused:
        hp = Hyperparameters(batch_size=32, policy_freq=policy_freq, target_update_rate=7)
        kw = dict(precision="bf16")
    else:
        hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16,
                             policy_freq=policy_freq, target_update_rate=7)
        kw = {}
    env = VecExoskeletonEnv(64, seed=5)
    ag = Agent(80, 7, 1, hp=hp, env_num=8, n_envs=64, buffer_size=8192, graph_safe=True, **kw)
    tr = VecTrainer(env, ag, episodes=episodes)
    out = []
    for i in range(iters):
        if near_round_end and i == 4:
            tr.k = tr.round_len - 3  # the next steps cross the round's end (both arms alike)
        tr.step()
        out.append((tr.last_actions.clone(), tr.obs.clone()))
    torch.cuda.synchronize()
    w = [p.detach().clone() for m in (ag.learner.actor, ag.learner.critic, ag.learner.encoder) for p in m.parameters()]
    return tr, out, w, float(ag.learner.exploration_noise_t)


@pytest.mark.parametrize("fused,policy_freq,episodes,near_end", [
    (True, 2, "async", False), (True, 2, "sync", True), (False, 3, "sync", False), (False, 2, "async", False)])
def test_select_ahead_is_bit_identical(monkeypatch, fused, policy_freq, episodes, near_end):
    t0, o0, w0, s0 = _run(False, monkeypatch, fused, policy_freq, episodes, near_round_end=near_end)
    t1, o1, w1, s1 = _run(True, monkeypatch, fused, policy_freq, episodes, near_round_end=near_end)
    for i, ((a0, b0), (a1, b1)) in enumerate(zip(o0, o1)):
        torch.testing.assert_close(a1, a0, rtol=0, atol=0, msg=f"actions, iteration {i}")
        torch.testing.assert_close(b1, b0, rtol=0, atol=0, msg=f"observations, iteration {i}")
    for x, y in zip(w0, w1):
        torch.testing.assert_close(y, x, rtol=0, atol=0)
    assert s0 == s1
    assert any(k[4] for k in t1.graphs) and any(k[5] for k in t1.graphs)
    assert not any(k[4] or k[5] for k in t0.graphs)
