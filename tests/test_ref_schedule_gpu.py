"""The reference training schedule in the vectorised trainer:
exo_amd.rollout.RefScheduleTrainer against the drop-in training-script mirror
(<pkg>/Simulation/Exoskeleton_agent_train.py, the reference's
Simulation/Exoskeleton_agent_train.py:110-211 with FIX 1-4).

Both runs: 8 envs (one per motion), seed 0, the same injected reset draws per
(round, env), the script's own action choice (np.random.uniform during the
warm-up, then the drop-in's per-env select_action with Gaussian exploration,
drawn from np.random in the script's order -- injected into the trainer
through its action_source hook).  Everything else is each side's own code:
the mirror steps 8 one-env objects, adds transitions one by one with
LAP.add(tremor_num=i) and calls Agent.train() eagerly inside
maybe_train_and_checkpoint; the trainer steps all envs in one launch, inserts
with lap_store_batch_ref (the shared pointer on the device) and replays its
training steps from HIP graphs.  The per-round decision trace
(training_steps, eps_since_update, min/best_min_return, checkpoint refreshes)
and the final weights -- live and checkpoint nets, optimiser moments -- must
agree bit for bit."""
import os
import sys

import numpy as np
import pytest
import torch

from helpers import PKG

pytestmark = pytest.mark.gpu

E = 8
BUF = 4096


def _draws(rnd, motion, L):
    from exo_amd.vec_env import draws_per_episode
    return np.random.default_rng(7919 * rnd + motion).random(draws_per_episode(L))


def _record(agent, trace):
    """Wrap agent.maybe_train_and_checkpoint to append its state after each round."""
    orig = agent.maybe_train_and_checkpoint

    def wrapped(ep_timesteps, ep_return, train=None):
        refreshed = agent.checkpoint_refreshes
        orig(ep_timesteps, ep_return, train=train)
        L = agent.learner
        trace.append((ep_timesteps, ep_return, L.training_steps, agent.eps_since_update, agent.min_return,
                      agent.best_min_return, agent.max_eps_before_update,
                      agent.checkpoint_refreshes - refreshed))
    agent.maybe_train_and_checkpoint = wrapped


def _run_mirror(tmp_path, rounds, warmup, precision, monkeypatch):
    sys.path.insert(0, os.path.join(PKG, "Simulation"))
    import Exoskeleton_agent_train as drv
    from exo_amd import td7

    class InjectedEnv(drv.ExoskeletonEnv_train):
        def __init__(self, *a, **kw):
            super().__init__(*a, seed=1234, **kw)  # explicit seed: no np.random draw at construction
            self._round = 0

        def reset(self):
            obs = self._vec.reset_from_draws([0], [_draws(self._round, int(self.file_num), self.max_count)])
            self._round += 1
            self._done = False
            self.state = obs[0].cpu().numpy()
            return self.state, self.counts

    trace = []
    orig_init = td7.Agent.__init__

    def init(self, *a, **kw):
        orig_init(self, *a, **kw)
        _record(self, trace)
    monkeypatch.setattr(drv, "ExoskeletonEnv_train", InjectedEnv)
    monkeypatch.setattr(td7.Agent, "__init__", init)
    args = drv.parse_args(["--seed", "0", "--n_steps", "1000000", "--warmup", str(warmup), "--save_dir",
                           str(tmp_path), "--buffer_size", str(BUF), "--max_rounds", str(rounds), "--quiet",
                           "--precision", precision])
    out = drv.train(args)
    monkeypatch.undo()
    _run_mirror.round_stats = out["round_stats"]
    return out["agent"], trace, out["steps"]


def _run_trainer(rounds, warmup, precision):
    import random
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent

    torch.manual_seed(0)
    np.random.seed(0)
    random.seed(0)
    env = VecExoskeletonEnv(E, seed=1234)
    agent = Agent(80, 7, 1, learning_steps=1000000, env_num=E, buffer_size=BUF, precision=precision)
    trace = []
    _record(agent, trace)
    rs = np.random.mtrand._rand  # the script's global np.random stream (seeded above)

    def actions(tr, random_phase):
        """The script's choice per running env, in env order (:125-131)."""
        act = np.zeros((E, 7))
        obs = tr.obs.cpu().numpy() if not random_phase else None
        for i in np.flatnonzero(tr.active_host[tr.k]):
            if random_phase:
                act[i] = np.clip(rs.uniform(-1, 1, 7), -1, 1)
            else:
                act[i] = agent.select_action(obs[i].astype(np.float64), use_checkpoint=False, use_exploration=True)
        return act

    def resets(rnd, obs_out):
        Ls = env.lengths_host
        env.reset_from_draws(np.arange(E), [_draws(rnd, m, int(Ls[m])) for m in range(E)], obs_out=obs_out)

    tr = RefScheduleTrainer(env, agent, warmup=warmup, action_source=actions, reset_source=resets, stats=True)
    for _ in range(rounds):
        tr.run_round()
    torch.cuda.synchronize()
    return agent, trace, tr


@pytest.mark.parametrize("precision,rounds", [("fp32", 4), ("bf16", 3)])
def test_ref_schedule_matches_training_mirror(tmp_path, monkeypatch, precision, rounds):
    warmup = 3257  # rounds 1-2 random (steps_count 2,257 <= warmup < 4,514: :210-211), then the policy
    ag_m, tr_m, steps_m = _run_mirror(tmp_path, rounds, warmup, precision, monkeypatch)
    ag_v, tr_v, trainer = _run_trainer(rounds, warmup, precision)
    assert steps_m == trainer.steps_count == rounds * 2257
    assert [t[0] for t in tr_m] == [283] * rounds  # round(mean(ep_len)) of the 8 motions
    # the decision trace, bit for bit
    assert len(tr_m) == len(tr_v) == rounds
    for r, (a, b) in enumerate(zip(tr_m, tr_v)):
        assert a == b, f"round {r + 1}: mirror {a} vs trainer {b}"
    assert sum(t[7] for t in tr_v) >= 1  # at least one checkpoint refresh happened
    # the replay: same shared pointer state, same stored transitions and priorities
    rb_m, rb_v = ag_m.replay_buffer, ag_v.replay_buffer
    assert (rb_m.ptr, rb_m.count, rb_m.size) == rb_v.ref_pointer()
    n = rb_m.size + 1
    for name in ("state", "action", "next_state", "reward", "not_done"):
        torch.testing.assert_close(getattr(rb_v, name)[:, :n], getattr(rb_m, name)[:, :n], rtol=0, atol=0)
    torch.testing.assert_close(rb_v._tree, rb_m._tree, rtol=0, atol=0)
    # the nets after the bursts: live, target, checkpoint, optimiser moments
    Lm, Lv = ag_m.learner, ag_v.learner
    for name in ("actor", "critic", "encoder", "actor_target", "critic_target", "fixed_encoder",
                 "fixed_encoder_target", "checkpoint_actor", "checkpoint_encoder"):
        for p, q in zip(getattr(Lm, name).parameters(), getattr(Lv, name).parameters()):
            torch.testing.assert_close(q, p, rtol=0, atol=0, msg=name)
    for opt in ("actor_optimizer", "critic_optimizer", "encoder_optimizer"):
        torch.testing.assert_close(getattr(Lv, opt).m, getattr(Lm, opt).m, rtol=0, atol=0)
        torch.testing.assert_close(getattr(Lv, opt).v, getattr(Lm, opt).v, rtol=0, atol=0)
    assert float(Lv.exploration_noise_t) == float(Lm.exploration_noise_t) < ag_m.hp.exploration_noise
    assert len([k for k in trainer.graphs if k[0] == "train"]) == 2  # bursts replayed from graphs
    # the script's per-round tremor statistics (:149-205, :213-317) on the
    # device (exo_tremor_metrics, fp32 per step) against the mirror's numpy
    _check_round_stats(_run_mirror.round_stats, trainer.round_stats, rounds)


def _check_round_stats(want, got, rounds):
    assert len(want) == len(got) == rounds
    for r, (a, b) in enumerate(zip(want, got)):
        assert set(a) == set(b)
        for k in a:
            np.testing.assert_allclose(b[k], a[k], rtol=1e-4, atol=2e-4, err_msg=f"round {r + 1}: {k}")


def test_ref_schedule_device_path():
    """Without hooks: device uniform warm-up actions, then the batched fused
    select_action (bf16) whose exploration noise drops once per RUNNING env;
    graph-replayed rollouts and bursts; the schedule's bookkeeping."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent
    torch.manual_seed(0)
    N = 64
    env = VecExoskeletonEnv(N, seed=5)
    agent = Agent(80, 7, 1, learning_steps=100000, env_num=E, buffer_size=2 * BUF, precision="bf16", n_envs=N)
    tr = RefScheduleTrainer(env, agent, warmup=1)
    A = int((env.lengths_host - 3).sum())
    n1, b1 = tr.run_round()  # random actions (allow_train is set after this round)
    assert (n1, b1) == (A, 283) and tr.allow_train and tr.trace[0]["random_actions"]
    s0 = float(agent.learner.exploration_noise_t)
    n2, b2 = tr.run_round()  # the policy
    torch.cuda.synchronize()
    assert (n2, b2) == (A, 283) and not tr.trace[1]["random_actions"]
    # one decrement per select_action call of the script = per running env-step (:125-128, :207)
    want = s0 - A * agent.learner.action_noise_decrease
    # (344 f32 decrements of at most half an ulp each; decrementing by all N envs would be 4e-3 lower)
    assert abs(float(agent.learner.exploration_noise_t) - want) < 5e-6
    assert agent.learner.training_steps == 2 * 283 and tr.steps_count == 2 * A
    assert tr.trace[0]["checkpoint_refreshed"]  # the first round always checkpoints (best_min_return = -1e8)
    # the shared pointer advanced once per E adds
    ptr, count, size = agent.replay_buffer.ref_pointer()
    assert count == 2 * A and ptr == size == -(-2 * A // E)
    assert int(agent.replay_buffer.size_s.min()) == int(agent.replay_buffer.size_s.max()) == size
    assert ("roll", True, 0, False) in tr.graphs and ("roll", False, 0, False) in tr.graphs
    assert ("train", True) in tr.graphs and ("train", False) in tr.graphs
    for m in (agent.learner.actor, agent.learner.critic, agent.learner.encoder):
        assert all(torch.isfinite(p).all() for p in m.parameters())
    # the checkpoint policy acts (a refresh copied the actor of its round)
    a = agent.select_action(np.zeros((3, 80), np.float32), use_checkpoint=True, use_exploration=False)
    assert np.isfinite(a).all() and a.shape == (3, 7)


def test_round_graph_rollout_matches_per_step_rollout():
    """RefScheduleTrainer's round graph (the round's rollout steps as one graph,
    each step's replay insert on a branch beside the next step's select_action)
    against per-step graph replays: after every round (with its training
    burst) the replay storage and sum trees, the episode scores, the env state and every network weight are bit-identical (six
    rounds: three random ones -- per step, then the random round graph
    captured and replayed, whose uniform actions of step k+1 must not reach
    step k's insert still running on its branch -- then three policy rounds
    the same way)."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    outs = []
    N = 32
    A = N // E * 2257  # active env-steps per round
    for rg in (False, True, "serial"):
        torch.manual_seed(3)
        env = VecExoskeletonEnv(N, seed=9)
        hp = Hyperparameters(batch_size=32)  # the bench's widths: the fused select in the round graph
        agent = Agent(80, 7, 1, hp=hp, learning_steps=100000, env_num=E, buffer_size=2 * BUF, precision="bf16",
                      n_envs=N, graph_safe=True)
        tr = RefScheduleTrainer(env, agent, warmup=2 * A + 1, round_graph=rg)
        scores = []
        for _ in range(6):  # 3 random, 3 policy: per step, then the round graph captured and replayed
            tr.run_round()
            scores.append(tr.score.clone())
        torch.cuda.synchronize()
        rb = agent.replay_buffer
        # (_u: the host-RNG sampling scratch, unused and uninitialised with the
        # device RNG; _ref_ws / _ref_add_ws: the per-step and the planned
        # inserts' scratch -- the branch-overlapped round graph (rg True) keeps
        # the per-step inserts, the others plan the round, r05)
        st = {k: v.detach().clone() for k, v in rb.__dict__.items()
              if isinstance(v, torch.Tensor) and k not in ("_u", "_ref_ws", "_ref_add_ws")}
        w = [p.detach().clone() for m in (agent.learner.actor, agent.learner.critic, agent.learner.encoder)
             for p in m.parameters()]
        obs = tr.obs.clone()
        outs.append((st, w, scores, obs, [t["training_steps"] for t in tr.trace]))
        assert [t["random_actions"] for t in tr.trace] == [True] * 3 + [False] * 3
        assert tr._use_plan() == (rg is not True)
        if rg:
            assert {k[:2] for k in tr._round_graphs} == {("round", True), ("round", False)}
    a = outs[0]
    for b in outs[1:]:  # the branch-overlapped and the serial ("serial": inserts in line) round graphs
        assert a[4] == b[4]
        for k in a[0]:
            torch.testing.assert_close(a[0][k], b[0][k], rtol=0, atol=0, msg=f"replay {k}")
        for x, y in zip(a[1], b[1]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)
        for x, y in zip(a[2], b[2]):
            torch.testing.assert_close(x, y, rtol=0, atol=0)
        torch.testing.assert_close(a[3], b[3], rtol=0, atol=0)


def test_fused_score_matches_torch_where_add():
    """The episode scores accumulated inside the mask-advance launch
    (exo_active_advance_score) are bit-identical to torch's
    score.add_(rew.where(active, 0.0)) (Exoskeleton_agent_train.py:144), over
    a random and a policy round with envs finishing at different steps."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    outs = []
    for fused in (False, True):
        torch.manual_seed(5)
        N = 24
        env = VecExoskeletonEnv(N, seed=4)
        agent = Agent(80, 7, 1, hp=Hyperparameters(batch_size=32), learning_steps=100000, env_num=E,
                      buffer_size=2 * BUF, precision="bf16", n_envs=N, graph_safe=True)
        tr = RefScheduleTrainer(env, agent, warmup=1)
        tr.fused_score = fused
        scores = []
        for _ in range(3):
            tr.run_round()
            scores.append(tr.score.clone())
        torch.cuda.synchronize()
        outs.append((scores, [t["ep_return"] for t in tr.trace]))
    for x, y in zip(outs[0][0], outs[1][0]):
        torch.testing.assert_close(x, y, rtol=0, atol=0)
    assert outs[0][1] == outs[1][1]


def test_burst_prefetch_is_bit_identical(monkeypatch):
    """RefScheduleTrainer.burst_prefetch (r04): each burst step samples the
    next step's batch at its end (update + sample in one launch) -- the same
    launches in the same order as sampling at the start of every step: the
    nets, trees, replay and decision trace bit for bit."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent
    out = []
    for on, pairs in (("0", False), ("1", False), ("1", True)):
        monkeypatch.setenv("EXO_BURST_PREFETCH", on)
        # r05: with prefetch, an actor step and the critic-only step after it
        # run as one overlapped graph inside a burst (RefScheduleTrainer._run_train_pair)
        monkeypatch.setattr(RefScheduleTrainer, "overlap_pairs", pairs)
        torch.manual_seed(0)
        env = VecExoskeletonEnv(64, seed=5)
        agent = Agent(80, 7, 1, learning_steps=100000, env_num=E, buffer_size=2 * BUF, precision="bf16", n_envs=64)
        tr = RefScheduleTrainer(env, agent, warmup=1)
        for _ in range(3):
            tr.run_round()
        torch.cuda.synchronize()
        L = agent.learner
        out.append(([p.detach().clone() for m in (L.actor, L.critic, L.encoder) for p in m.parameters()],
                    agent.replay_buffer._tree.clone(), [dict(t) for t in tr.trace], tr))
    (w0, t0, d0, tr0), (w1, t1, d1, tr1), (w2, t2, d2, tr2) = out
    for w, t, d in ((w1, t1, d1), (w2, t2, d2)):
        for a, b in zip(w0, w):
            torch.testing.assert_close(b, a, rtol=0, atol=0)
        torch.testing.assert_close(t, t0, rtol=0, atol=0)
        assert d0 == d
    assert any(len(k) == 5 for k in tr1.graphs if k[0] == "train")
    assert not any(len(k) == 5 for k in tr0.graphs if k[0] == "train")
    assert any(k[0] == "tpair" for k in tr2.graphs) and not any(k[0] == "tpair" for k in tr1.graphs)


def test_per_round_save_reloads_to_the_trainers_weights(tmp_path):
    """RefScheduleTrainer(save_prefix=...): agent.save(prefix) after every
    round (Exoskeleton_agent_train.py:290, TD7_multi_agent.py:330-345); the 8
    files of the last round, loaded into a fresh Agent (weights_only), hold the
    trainer's live nets, optimiser moments and checkpoint nets."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent
    torch.manual_seed(0)
    N = 64
    env = VecExoskeletonEnv(N, seed=5)
    agent = Agent(80, 7, 1, learning_steps=100000, env_num=E, buffer_size=2 * BUF, precision="bf16", n_envs=N)
    prefix = str(tmp_path / "test_agent")
    tr = RefScheduleTrainer(env, agent, warmup=1, save_prefix=prefix)
    for _ in range(2):
        tr.run_round()
    torch.cuda.synchronize()
    assert tr.saves == 2 and tr.save_seconds > 0
    assert all(os.path.exists(prefix + s) for s in Agent.SUFFIXES)
    fresh = Agent(80, 7, 1, learning_steps=100000, env_num=E, buffer_size=2 * BUF, precision="bf16", n_envs=N)
    fresh.load(prefix)
    La, Lb = agent.learner, fresh.learner
    for name in ("actor", "critic", "encoder", "checkpoint_actor", "checkpoint_encoder"):
        for p, q in zip(getattr(La, name).parameters(), getattr(Lb, name).parameters()):
            torch.testing.assert_close(q, p, rtol=0, atol=0, msg=name)
    for opt in ("actor_optimizer", "critic_optimizer", "encoder_optimizer"):
        torch.testing.assert_close(getattr(Lb, opt).m, getattr(La, opt).m, rtol=0, atol=0)
        torch.testing.assert_close(getattr(Lb, opt).v, getattr(La, opt).v, rtol=0, atol=0)
        assert float(getattr(Lb, opt)._step) == float(getattr(La, opt)._step) == La.training_steps // (
            2 if opt == "actor_optimizer" else 1)
