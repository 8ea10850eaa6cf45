"""Vectorised TD7 training loop on one GPU, replayed from HIP graphs.

One iteration = the reference training script's per-step work for every env
(Simulation/Exoskeleton_agent_train.py:123-147: select_action, env.step,
replay_buffer.add) plus one Agent.train() step (:208 / TD7_multi_agent.py:211).
Episodes are synchronous like the script (:110-123): all envs reset together
and done envs stay idle until the longest motion ends.

Everything inside an iteration is device work with no host synchronisation,
so it is captured once into HIP graphs and replayed:
  * world == 1: one graph per policy-update parity (actor updated or not);
  * world  > 1: the gradient all-reduces (RCCL) run eagerly between graphs
    (pre: rollout + encoder/critic grads, mid: optimiser steps + priorities +
    actor grads, post: actor step).
Host-side bookkeeping left outside the graphs: the env reset at the end of a
round, the target-network refresh every 250 steps (:284-293).
"""
import numpy as np
import torch

from . import _native as nat


class VecTrainer:
    def __init__(self, env, agent, strata=None, use_graphs=True, warmup_eager=3):
        self.env, self.agent = env, agent
        self.device = env.device
        self.n = env.n
        Ls = env.lengths_host
        self.round_len = int(Ls.max()) - 3
        self.active_table = torch.as_tensor(np.stack([Ls - 3 > k for k in range(self.round_len)]),
                                            device=self.device)
        self.active_counts = self.active_table.sum(1).cpu().numpy()
        self.strata = (torch.as_tensor(env.motions % agent.env_num, dtype=torch.int32, device=self.device)
                       if strata is None else strata)
        self.obs = env.reset()
        self.out = env.new_outputs(True)
        self.active = self.active_table[0].clone()
        self.k = 0
        self.use_graphs = use_graphs
        self.warmup_eager = warmup_eager
        self.iters = 0
        self.graphs = {}
        self.dp = agent.sync.active
        self.last_actions = None

    # ----------------------------------------------------------- pieces
    def _rollout(self):
        ag = self.agent
        act = ag.select_action_batch(self.obs)
        nobs, rew, done, info = self.env.step(act, active=self.active, out=self.out)
        ag.replay_buffer.add_batch(self.obs, act, nobs, rew, done, self.strata, self.active)
        self.obs.copy_(nobs)
        self.last_actions = act

    def _pre(self):
        self._rollout()
        ag = self.agent
        self._batch = ag.replay_buffer.sample()
        self._prio = ag.learner.phase_grads(*self._batch)

    def _mid(self, update_actor):
        ag = self.agent
        ag.learner.phase_steps()
        ag.replay_buffer.update_priority(self._prio)
        if update_actor:
            ag.learner.phase_actor_grads(self._batch[0], self._batch[1])

    def _post(self, update_actor):
        if update_actor:
            self.agent.learner.phase_actor_step()

    def _eager(self, update_actor):
        L = self.agent.learner
        self._pre()
        L.sync.allreduce_grads(L.grad_params())
        self._mid(update_actor)
        if update_actor:
            L.sync.allreduce_grads(L.grad_params(actor=True))
        self._post(update_actor)

    def _capture(self, update_actor):
        """Capture this parity's iteration; the capture itself performs one real iteration."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        pool = None  # one private pool per parity: the two parities replay in alternation
        parts = []
        with torch.cuda.stream(s):
            if not self.dp:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, stream=s):
                    self._pre()
                    self._mid(update_actor)
                    self._post(update_actor)
                parts = [g]
            else:
                L = self.agent.learner
                g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1, pool=pool, stream=s):
                    self._pre()
                pool = g1.pool()
                L.sync.allreduce_grads(L.grad_params())
                with torch.cuda.graph(g2, pool=pool, stream=s):
                    self._mid(update_actor)
                if update_actor:
                    L.sync.allreduce_grads(L.grad_params(actor=True))
                with torch.cuda.graph(g3, pool=pool, stream=s):
                    self._post(update_actor)
                parts = [g1, g2, g3]
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graphs[update_actor] = parts
        # capture records but does not execute: run the iteration now
        self._replay(update_actor)

    def _replay(self, update_actor):
        parts = self.graphs[update_actor]
        if not self.dp:
            parts[0].replay()
            return
        L = self.agent.learner
        parts[0].replay()
        L.sync.allreduce_grads(L.grad_params())
        parts[1].replay()
        if update_actor:
            L.sync.allreduce_grads(L.grad_params(actor=True))
        parts[2].replay()

    # ------------------------------------------------------------- step
    def step(self):
        """One training iteration; returns the number of active env-steps."""
        ag = self.agent
        L = ag.learner
        if self.k == self.round_len:
            self.env.reset(obs_out=self.obs)
            self.k = 0
        self.active.copy_(self.active_table[self.k])
        L.training_steps += 1
        update_actor = L.training_steps % ag.hp.policy_freq == 0
        if not self.use_graphs or self.iters < self.warmup_eager:
            self._eager(update_actor)
        elif update_actor not in self.graphs:
            self._capture(update_actor)
        else:
            self._replay(update_actor)
        if L.maybe_update_targets():
            ag.replay_buffer.reset_max_priority()
        n_active = int(self.active_counts[self.k])
        self.k += 1
        self.iters += 1
        return n_active
