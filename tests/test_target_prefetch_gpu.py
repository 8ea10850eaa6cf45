"""Cross-iteration prefetch of the critic's inputs (VecTrainer.prefetch_targets,
TD7Learner.prefetch_targets): the fixed embeddings and the target heads of the
next batch computed at the end of the current iteration.  The same launches on
the same inputs in the same order (the target-noise stream included), so the
trained weights are bit-identical to computing them inside the next
iteration -- through target refreshes (where the trainer does not prefetch),
both policy-update parities, graph capture and replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(prefetch, iters, monkeypatch, episodes="sync"):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    monkeypatch.setattr(VecTrainer, "prefetch_targets", prefetch)
    torch.manual_seed(11)
    hp = Hyperparameters(batch_size=32, target_update_rate=5)  # the fused widths (300 / 320)
    env = VecExoskeletonEnv(64, seed=11)
    ag = Agent(80, 7, 1, hp=hp, env_num=8, precision="bf16", n_envs=64, buffer_size=8192, graph_safe=True)
    assert ag.learner.fused is not None
    tr = VecTrainer(env, ag, episodes=episodes)
    for _ in range(iters):
        tr.step()
    torch.cuda.synchronize()
    w = {n: [p.detach().clone() for p in getattr(ag.learner, n).parameters()] for n in ("actor", "critic", "encoder")}
    return tr, w


@pytest.mark.parametrize("episodes", ["sync", "async"])
def test_prefetched_targets_are_bit_identical(monkeypatch, episodes):
    iters = 17  # target refreshes after steps 5, 10, 15; 3 eager warm-up iterations
    tr_off, w_off = _run(False, iters, monkeypatch, episodes)
    tr_on, w_on = _run(True, iters, monkeypatch, episodes)
    for n in w_off:
        for a, b in zip(w_off[n], w_on[n]):
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    # steady state reads and writes a slot; the iteration before a refresh
    # does not prefetch, the one after it computes its own inputs
    keys = set(tr_on.graphs)
    assert any(k[2] and k[3] for k in keys)
    assert any(k[2] and not k[3] for k in keys)
    assert any(not k[2] and k[3] for k in keys)
    assert all(not k[2] and not k[3] for k in tr_off.graphs)


def test_agent_train_drops_prefetched_inputs(monkeypatch):
    """An Agent.train() between trainer iterations samples its own batch: the
    prefetched slot no longer matches the trainer's next batch and is dropped
    (the next iteration computes its inputs itself)."""
    tr, _ = _run(True, 6, monkeypatch)
    L = tr.agent.learner
    assert L.prefetch_ready(tr._cur)
    tr.agent.train()
    assert not L.prefetch_ready(0) and not L.prefetch_ready(1)
    tr.step()
    torch.cuda.synchronize()
    assert all(torch.isfinite(p).all() for p in L.critic.parameters())
