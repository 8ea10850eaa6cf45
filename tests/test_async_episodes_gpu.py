"""Auto-reset (asynchronous) episodes: exo_episode_advance resets every env
whose episode is over in place and lets every other env step again (except a
budgeted solve that is pending).  Parity: each env's sequence of transitions
equals the one the same env produces when the host resets it with the
reference's reset (exo_reset with a mask) at the end of each of its episodes
(Exoskeleton_env.py:473-478 after the done step, :448/:457) -- bit for bit,
with and without a step budget."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _host_driven(N, seed, acts_of, M):
    """Reference run: every env steps every launch; when an env has taken its
    episode's L - 3 steps the host resets it (masked exo_reset into the
    observation buffer the step wrote).  Returns rewards [M, N] and
    observations [M, N, 80] of each env's first M transitions."""
    from exo_amd import VecExoskeletonEnv
    env = VecExoskeletonEnv(N, seed=seed)
    dev = env.device
    steps_per_ep = env.lengths_host - 3
    obs = env.reset()
    outs = [env.new_outputs(True), env.new_outputs(True)]
    rew_rec = np.zeros((M, N), np.float32)
    obs_rec = np.zeros((M, N, 80), np.float32)
    j = np.zeros(N, np.int64)      # transitions taken so far
    in_ep = np.zeros(N, np.int64)  # steps into the current episode
    par = 0
    for t in range(M):
        ob, r, d, _ = env.step(acts_of(t, j), out=outs[par])
        rew_rec[t] = r.cpu().numpy()
        obs_rec[t] = ob.cpu().numpy()
        done_h = d.cpu().numpy().astype(bool)
        in_ep += 1
        fin = in_ep >= steps_per_ep
        np.testing.assert_array_equal(done_h, fin)  # the done index of the reference
        if fin.any():
            env.reset(mask=torch.as_tensor(fin, device=dev), obs_out=ob)
            in_ep[fin] = 0
        j += 1
        par ^= 1
    return rew_rec, obs_rec


@pytest.mark.parametrize("budget", [0, 3])
def test_episode_advance_equals_host_driven_resets(budget):
    from exo_amd import VecExoskeletonEnv
    N, seed = 1030, 41
    env = VecExoskeletonEnv(N, seed=seed)
    M = int(env.lengths_host.min()) - 3 + 12  # motion 0's envs cross an episode end and reset
    rng = np.random.default_rng(5)
    A = rng.uniform(-1, 1, (M, N, 7)).astype(np.float32)

    def acts_of(t, j):  # env e's j-th transition takes A[j[e], e]
        return torch.as_tensor(A[np.minimum(j, M - 1), np.arange(N)], device="cuda")

    want_r, want_o = _host_driven(N, seed, lambda t, j: acts_of(t, j), M)
    if budget:
        env.set_step_budget(budget)
    dev = env.device
    obs = env.reset()
    outs = [env.new_outputs(True), env.new_outputs(True)]
    active = torch.ones(N, dtype=torch.bool, device=dev)
    count = torch.full((1,), N, dtype=torch.int32, device=dev)
    total = torch.zeros((1,), dtype=torch.int64, device=dev)
    j = np.zeros(N, np.int64)
    got_r = np.zeros((M, N), np.float32)
    got_o = np.zeros((M, N, 80), np.float32)
    par, launches, stepped_sum = 0, 0, 0
    while (j < M).any():
        act_h = active.cpu().numpy().astype(bool) & (j < M)
        assert int(count) == int(active.sum())
        ob, r, _, _ = env.step(acts_of(0, j), active=torch.as_tensor(act_h, device=dev), out=outs[par],
                               obs_cur=obs if budget else None)
        stepped_sum += int(act_h.sum())
        idx = np.flatnonzero(act_h)
        rh, oh = r.cpu().numpy(), ob.cpu().numpy()
        got_r[j[idx], idx] = rh[idx]
        got_o[j[idx], idx] = oh[idx]
        j[idx] += 1
        count.fill_(int(act_h.sum()))  # the launch's envs (the masked tail of the test included)
        env.episode_advance(active, count, ob, total)
        obs, par = ob, par ^ 1
        launches += 1
        assert launches < M * (4096 // max(budget, 1) + 2), "does not converge"
    np.testing.assert_array_equal(got_r, want_r)
    np.testing.assert_array_equal(got_o, want_o)
    assert int(total) == stepped_sum
    if budget:
        assert launches > M  # solves were carried


def _trainer(episodes, seed, budget=0):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(seed)
    hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16,
                         target_update_rate=50)
    env = VecExoskeletonEnv(64, seed=seed)
    if budget:
        env.set_step_budget(budget)
    agent = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=8192, graph_safe=True)
    return VecTrainer(env, agent, episodes=episodes), env, agent


@pytest.mark.parametrize("budget", [0, 4])
def test_async_trainer_in_graphs(budget):
    """Graph-replayed trainer with async episodes.  Until the first episode
    ends (motion 0: 229 steps) it is the synchronous trainer bit for bit (same
    seeds: weights, observations, env states); past it (240 iterations)
    motion 0's envs have been reset inside the captured iterations and run
    their next episode while the others continue theirs -- no host round, no
    idle envs."""
    first_end = 229
    res = {}
    for eps in ("sync", "async"):
        tr, env, ag = _trainer(eps, 3, budget)
        for _ in range(first_end - 1):
            n = tr.step()
            assert n == (0 if budget else 64)
        torch.cuda.synchronize()
        res[eps] = ([p.detach().clone() for p in ag.learner.actor.parameters()], tr.obs.clone(),
                    [env.get_state(e) for e in (0, 1, 63)])
        if eps == "async":
            for _ in range(240 - (first_end - 1)):
                assert tr.step() == (0 if budget else 64)
            torch.cuda.synchronize()
            assert tr.resets == 0
            total = tr.env_steps_total()
            if budget:
                assert 0 < total < 64 * 240
            else:
                assert total == 64 * 240
                counts = np.array([env.get_state(e)[0] for e in range(64)])
                m0 = np.arange(64) % 8 == 0
                np.testing.assert_array_equal(counts[m0], 2 + 240 - first_end)  # reset, 11 steps into episode 2
                np.testing.assert_array_equal(counts[~m0], 2 + 240)
            assert torch.isfinite(tr.obs).all()
    (pa, oa, sa), (pb, ob, sb) = res["sync"], res["async"]
    for x, y in zip(pa, pb):
        torch.testing.assert_close(x, y, rtol=0, atol=0)
    torch.testing.assert_close(oa, ob, rtol=0, atol=0)
    for x, y in zip(sa, sb):
        np.testing.assert_array_equal(x, y)


def test_async_refuses_pink():
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16)
    env = VecExoskeletonEnv(16, seed=1)
    agent = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=1024)
    with pytest.raises(ValueError):
        VecTrainer(env, agent, exploration="pink", episodes="async")
