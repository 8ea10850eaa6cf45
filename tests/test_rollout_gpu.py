"""The HIP-graph-replayed training iteration (exo_amd.rollout.VecTrainer)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(use_graphs, seed=0, policy_freq=2):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(seed)
    hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16, target_update_rate=5,
                         policy_freq=policy_freq)
    env = VecExoskeletonEnv(64, seed=seed)
    agent = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=4096, graph_safe=use_graphs)
    return VecTrainer(env, agent, use_graphs=use_graphs), env, agent


def test_graph_replay_matches_eager_bookkeeping():
    te, env_e, ag_e = _make(False)
    tg, env_g, ag_g = _make(True)
    for _ in range(12):
        assert te.step() == tg.step()
    torch.cuda.synchronize()
    # policy_freq 2: parity and observation buffer alternate in lockstep (further keys:
    # the target-prefetch variants around the target refreshes, target_update_rate 5)
    assert len({k[:2] for k in tg.graphs}) == 2
    np.testing.assert_array_equal(ag_e.replay_buffer.size_s.cpu().numpy(), ag_g.replay_buffer.size_s.cpu().numpy())
    np.testing.assert_array_equal(ag_e.replay_buffer.ptr_s.cpu().numpy(), ag_g.replay_buffer.ptr_s.cpu().numpy())
    assert ag_g.learner.training_steps == 12
    c_e = [env_e.get_state(i)[0] for i in range(64)]
    c_g = [env_g.get_state(i)[0] for i in range(64)]
    assert c_e == c_g
    for p in ag_g.learner.critic.parameters():
        assert torch.isfinite(p).all()
    # the graphs really train: the running Q bound moved and the targets were refreshed at step 10
    assert float(ag_g.learner.max) > -1e8
    assert float(ag_g.learner.max_target) == float(ag_g.learner.max) or ag_g.learner.training_steps % 5 != 0


def test_graph_replay_is_deterministic_for_identical_seeds():
    t1, _, a1 = _make(True, seed=3)
    for _ in range(9):
        t1.step()
    snap = [p.detach().clone() for p in a1.learner.actor.parameters()]
    t2, _, a2 = _make(True, seed=3)
    for _ in range(9):
        t2.step()
    torch.cuda.synchronize()
    for p, q in zip(snap, a2.learner.actor.parameters()):
        torch.testing.assert_close(p, q, rtol=0, atol=0)


@pytest.mark.parametrize("layout", ["single", "split"])
def test_graph_replay_matches_eager_numerics(layout):
    """Same seeds -> the graph-replayed iterations (both parities, several
    replays each) train the nets to the same weights as eager execution.
    'split' is the data-parallel 3-graph layout (pack/unpack around the
    gradient all-reduce), exercised here at world size 1."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import graph_vs_eager
    assert graph_vs_eager.run(layout, iters=10) <= 1e-5


def test_graph_replay_matches_eager_with_policy_freq_3():
    """policy_freq 3: the policy-update parity no longer flips with the
    observation buffer, so graphs are keyed by (parity, buffer) -- 4 captures
    -- and every replay reads the observation buffer of its own iteration
    (keyed by parity alone a replay read a stale buffer)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import graph_vs_eager
    assert graph_vs_eager.run("single", iters=12, policy_freq=3) <= 1e-5
    tg, _, _ = _make(True, policy_freq=3)
    for _ in range(12):
        tg.step()
    assert sorted({k[:2] for k in tg.graphs}) == [(False, 0), (False, 1), (True, 0), (True, 1)]


def test_pink_exploration_trainer_runs_in_graphs():
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(0)
    hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16)
    env = VecExoskeletonEnv(64, seed=2)
    agent = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=4096, graph_safe=True)
    tr = VecTrainer(env, agent, exploration="pink")
    for _ in range(8):
        tr.step()
    torch.cuda.synchronize()
    assert len(tr.graphs) == 2 and int(tr.k_dev) == 8  # one increment per rollout
    assert torch.isfinite(tr.last_actions).all() and float(tr.last_actions.abs().max()) <= 1.0


def test_active_advance_saturates_and_copies_rows():
    """exo_active_advance: the device step counter advances by one per call and
    saturates at the last row, whose copy lands in the active mask (graph
    replays past a round's end stay in bounds)."""
    from exo_amd import _native as nat
    table = (torch.arange(4 * 70, device="cuda").view(4, 70) % 3 == 0).contiguous()
    k = torch.zeros(1, dtype=torch.int64, device="cuda")
    act = torch.zeros(70, dtype=torch.bool, device="cuda")
    cnt = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    for want in (1, 2, 3, 3, 3):
        nat.check(nat.lib().exo_active_advance(nat.ptr(table), 4, 70, nat.ptr(k), nat.ptr(act),
                                               nat.ptr(cnt) if want != 2 else None,
                                               nat.stream_ptr(torch.device("cuda", 0))), "exo_active_advance")
        torch.cuda.synchronize()
        assert int(k) == want
        assert torch.equal(act, table[want])
        if want != 2:  # the active count of the copied row (NULL: left alone)
            assert int(cnt) == int(table[want].sum())


@pytest.mark.parametrize("episodes", ["sync", "async"])
def test_pair_graphs_are_bit_identical(monkeypatch, episodes):
    """EXO_PAIR_GRAPHS (two iterations per graph replay, r04): the same
    launches in the same order -- weights, observations and replay rows bit
    for bit against one graph per iteration, through target refreshes
    (target_update_rate 5: single graphs around them)."""
    from exo_amd.rollout import VecTrainer
    res = []
    for pair in (False, True):
        monkeypatch.setattr(VecTrainer, "pair_graphs", pair)
        monkeypatch.setenv("EXO_EPISODES", episodes)
        tr, env, ag = _make(True, seed=4)
        tr.plan(17)  # pairs only inside an announced run
        obs = []
        for _ in range(17):
            tr.step()
            obs.append(tr.obs.clone())
        torch.cuda.synchronize()
        res.append((tr, obs, [p.detach().clone() for m in (ag.learner.actor, ag.learner.critic) for p in m.parameters()],
                    ag.replay_buffer.state.clone()))
    (t0, o0, w0, r0), (t1, o1, w1, r1) = res
    for i, (a, b) in enumerate(zip(o0, o1)):
        torch.testing.assert_close(b, a, rtol=0, atol=0, msg=f"iteration {i}")
    for a, b in zip(w0, w1):
        torch.testing.assert_close(b, a, rtol=0, atol=0)
    torch.testing.assert_close(r1, r0, rtol=0, atol=0)
    assert any(k[0] == "pair" for k in t1.graphs) and not any(k[0] == "pair" for k in t0.graphs)


@pytest.mark.parametrize("episodes,split", [("sync", "0"), ("async", "0"), ("sync", "1"), ("async", "1")])
def test_overlapped_pairs_are_bit_identical(monkeypatch, episodes, split):
    """EXO_OVERLAP_PAIRS (r05): an actor iteration and the critic-only one after
    it in one graph, the second's target chain / fixed / encoder passes beside
    the first's actor passes (its rollout and critic step wait for them).  The
    same launches on the same inputs: weights, observations, replay rows and
    sum trees bit for bit against one graph per iteration, through target
    refreshes (target_update_rate 5: unpaired graphs around them).  Fused
    bf16 passes (the overlap needs the fused update), 256-wide nets.  split
    "1" (r06): the second iteration's select_action in two launches, its zs
    half from the iteration's start (EXO_SPLIT_SELECT)."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    monkeypatch.setattr(VecTrainer, "split_select", split)
    res = []
    for overlap in (False, True):
        monkeypatch.setattr(VecTrainer, "overlap_pairs", overlap)
        monkeypatch.setenv("EXO_EPISODES", episodes)
        torch.manual_seed(6)
        hp = Hyperparameters(zs_dim=256, enc_hdim=256, critic_hdim=256, actor_hdim=256, batch_size=32,
                             target_update_rate=5)
        env = VecExoskeletonEnv(256, seed=6)
        ag = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=4096, graph_safe=True, precision="bf16")
        assert ag.learner.fused_train
        tr = VecTrainer(env, ag)
        tr.plan(20)  # pairs only inside an announced run (20: the last pair ends at it)
        obs = []
        for _ in range(20):
            tr.step()
            obs.append(tr.obs.clone())
        torch.cuda.synchronize()
        L = ag.learner
        res.append((tr, obs, [p.detach().clone() for m in (L.actor, L.critic, L.encoder) for p in m.parameters()],
                    ag.replay_buffer.state.clone(), ag.replay_buffer._tree.clone()))
    (t0, o0, w0, r0, s0), (t1, o1, w1, r1, s1) = res
    for i, (a, b) in enumerate(zip(o0, o1)):
        torch.testing.assert_close(b, a, rtol=0, atol=0, msg=f"iteration {i}")
    for a, b in zip(w0, w1):
        torch.testing.assert_close(b, a, rtol=0, atol=0)
    torch.testing.assert_close(r1, r0, rtol=0, atol=0)
    torch.testing.assert_close(s1, s0, rtol=0, atol=0)
    assert any(k[-1] == "overlap" for k in t1.graphs) and not any(k[0] == "pair" for k in t0.graphs)


def test_pairs_never_run_past_the_announced_steps(monkeypatch):
    """Without plan() every step() is exactly one iteration's GPU work (no
    pair graph); with plan(n) a pair starts only where two announced calls
    remain, so after n calls exactly n iterations have run: the same weights
    as n unpaired iterations (n odd and even)."""
    from exo_amd.rollout import VecTrainer
    monkeypatch.setattr(VecTrainer, "pair_graphs", True)
    for n in (12, 13):
        res = []
        for planned in (False, True):
            tr, env, ag = _make(True, seed=8)
            if planned:
                tr.plan(n)
            for _ in range(n):
                tr.step()
            torch.cuda.synchronize()
            assert any(k[0] == "pair" for k in tr.graphs) == planned
            assert ag.learner.training_steps == n
            res.append([p.detach().clone() for p in ag.learner.critic.parameters()])
        for a, b in zip(*res):
            torch.testing.assert_close(b, a, rtol=0, atol=0)


@pytest.mark.parametrize("episodes", ["sync", "async"])
def test_prepare_records_the_window_graphs_without_running_them(monkeypatch, episodes):
    """VecTrainer.prepare (r06): after the eager warm-up,
    plan(n) + prepare() records the graphs the next n steps replay -- the two
    single-iteration graphs and the overlapped pair -- without running them, so
    those n steps capture nothing and the run is bit-identical to the same
    steps without prepare (weights, observations, replay rows, sum trees)."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    monkeypatch.setenv("EXO_EPISODES", episodes)
    res = []
    for prep in (False, True):
        torch.manual_seed(6)
        hp = Hyperparameters(zs_dim=256, enc_hdim=256, critic_hdim=256, actor_hdim=256, batch_size=32)
        env = VecExoskeletonEnv(256, seed=6)
        ag = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=4096, graph_safe=True, precision="bf16")
        tr = VecTrainer(env, ag)
        tr.plan(3)
        for _ in range(3):  # the eager warm-up iterations only
            tr.step()
        tr.plan(12)
        if prep:
            assert not tr.graphs
            made = tr.prepare()
            assert made == 3 and len(tr.graphs) == 3 and any(k[-1] == "overlap" for k in tr.graphs)
            assert ag.learner.training_steps == 3 and tr.iters == 3
            keys = set(tr.graphs)
            assert tr.prepare() == 0
        obs = []
        for _ in range(12):
            tr.step()
            obs.append(tr.obs.clone())
        torch.cuda.synchronize()
        if prep:
            assert set(tr.graphs) == keys
        L = ag.learner
        res.append((obs, [p.detach().clone() for m in (L.actor, L.critic, L.encoder) for p in m.parameters()],
                    ag.replay_buffer.state.clone(), ag.replay_buffer._tree.clone()))
    (o0, w0, r0, s0), (o1, w1, r1, s1) = res
    for i, (a, b) in enumerate(zip(o0, o1)):
        torch.testing.assert_close(b, a, rtol=0, atol=0, msg=f"iteration {i}")
    for a, b in zip(w0, w1):
        torch.testing.assert_close(b, a, rtol=0, atol=0)
    torch.testing.assert_close(r1, r0, rtol=0, atol=0)
    torch.testing.assert_close(s1, s0, rtol=0, atol=0)
