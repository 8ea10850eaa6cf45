"""Vectorised TD7 training loop on one GPU, replayed from HIP graphs.

One iteration = the reference training script's per-step work for every env
(Simulation/Exoskeleton_agent_train.py:123-147: select_action, env.step,
replay_buffer.add) plus one Agent.train() step (:208 / TD7_multi_agent.py:211).
Episodes are synchronous like the script (:110-123): all envs reset together
and done envs stay idle until the longest motion ends.

Everything inside an iteration is device work with no host synchronisation,
so it is captured once into HIP graphs and replayed:
  * world == 1: one graph per policy-update parity (actor updated or not);
  * world  > 1: the collectives (RCCL) run eagerly between graphs: the
    encoder/critic gradient bucket after `pre` (rollout + grads), a MAX of
    max_priority after `mid` (optimiser steps + priorities + actor grads),
    the actor bucket before `post` (actor step).
Host-side bookkeeping left outside the graphs: the env reset at the end of a
round, the target-network refresh every 250 steps (:284-293).
"""
import os

import numpy as np
import torch

from . import _native as nat
from .td7 import ENC_STEP_BRANCH


def graph_reductions_ok(device, rows=1024, cols=300, replays=3):
    """Replay a captured multi-block column reduction a few times and compare
    with eager sums; raise if the HIP runtime replays it wrongly (see
    exo_amd/__init__.py: DEBUG_CLR_GRAPH_PACKET_CAPTURE must be 0 before the
    first GPU call of the process).  ~1 ms, once per trainer."""
    gen = torch.Generator(device=device).manual_seed(0)
    x = torch.randn(rows, cols, device=device, generator=gen)
    s = torch.cuda.Stream(device=device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        x.sum(0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = x.sum(0)
    torch.cuda.current_stream(device).wait_stream(s)
    for _ in range(replays):
        x.mul_(1.5)
        g.replay()
        if not torch.allclose(out, x.sum(0), rtol=1e-4, atol=1e-3):
            raise RuntimeError(
                "HIP graph replay of torch reductions is wrong in this process (ROCm CLR graph packet "
                "capture). Set DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 before the first GPU call -- importing "
                "exo_amd before touching the GPU does it -- or use VecTrainer(use_graphs=False).")
    return True


class CaptureForkError(RuntimeError):
    pass


def unjoined_streams(events, origin):
    """Fork/join audit of one capture.  events: in order, ("wait", waiter,
    waited) for every Stream.wait_stream and ("use", stream) when a
    `torch.cuda.stream(stream)` block ends (the last point work can have been
    enqueued there).  A branch is joined when its work up to its last use is
    ordered before the capture stream `origin`: a wait of the origin on it
    after that use, or of another branch that is itself joined after that
    wait.  Returns the branches (streams forked from the captured set) that
    are not -- the `hipErrorStreamCaptureUnjoined` of capture end."""
    def key(st):  # torch returns a new Stream object per current_stream() call: key by the raw handle
        return st.cuda_stream
    captured, last_use = {key(origin)}, {}
    joins = {}  # waited -> [(time, waiter)]
    objs = {}
    for t, ev in enumerate(events):
        if ev[0] == "wait":
            _, w, x = ev
            objs[key(w)], objs[key(x)] = w, x
            if key(x) in captured and key(w) not in captured:
                captured.add(key(w))
                last_use.setdefault(key(w), t)
            if key(x) in captured and key(x) != key(origin):
                joins.setdefault(key(x), []).append((t, key(w)))
        else:
            objs[key(ev[1])] = ev[1]
            if key(ev[1]) in captured:
                last_use[key(ev[1])] = t

    def ordered(s, t, seen=()):  # is s's work up to time t ordered before origin's end?
        if s == key(origin):
            return True
        return any(tj >= t and w not in seen and ordered(w, tj, seen + (s,)) for tj, w in joins.get(s, ()))

    return [objs[s] for s in captured if s != key(origin) and not ordered(s, last_use.get(s, 0))]


class ForkJoinAudit:
    """Records every Stream.wait_stream and stream-context exit while a graph is
    captured on `origin`; on exit raises CaptureForkError naming any branch not
    joined back (after joining it, so that capture end still succeeds)."""

    def __init__(self, origin):
        self.origin = origin
        self.events = []

    def __enter__(self):
        audit = self
        self._wait = torch.cuda.Stream.wait_stream
        self._exit = torch.cuda.StreamContext.__exit__

        def wait_stream(st, other):
            audit.events.append(("wait", st, other))
            return audit._wait(st, other)

        def ctx_exit(ctx, *a):
            if ctx.stream is not None:
                audit.events.append(("use", ctx.stream))
            return audit._exit(ctx, *a)

        torch.cuda.Stream.wait_stream = wait_stream
        torch.cuda.StreamContext.__exit__ = ctx_exit
        return self

    def __exit__(self, exc_type, exc, tb):
        torch.cuda.Stream.wait_stream = self._wait
        torch.cuda.StreamContext.__exit__ = self._exit
        if exc_type is not None:
            return False
        bad = unjoined_streams(self.events, self.origin)
        if bad:
            for st in bad:
                self.origin.wait_stream(st)
            raise CaptureForkError(f"{len(bad)} stream(s) forked from the capture stream were not joined back "
                                   "before capture end")
        return False


class VecTrainer:
    def __init__(self, env, agent, strata=None, use_graphs=True, warmup_eager=3, exploration="gaussian"):
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
        # two observation buffers used in alternation (iteration i reads obs[c]
        # and the env writes its next observation into obs[1 - c]): no copy of
        # the next observation per step.  A captured graph bakes in the pair it
        # was captured with, so graphs are keyed by (policy-update parity, c):
        # with policy_freq 2 and training_steps advanced only here the two
        # alternate in lockstep and 2 graphs are captured; otherwise (policy_freq
        # 1/3/4, or train() called in between) up to 4.
        o0 = env.reset()
        self._obs = [o0, torch.empty_like(o0)]
        outs = [env.new_outputs(True), env.new_outputs(True)]
        self._outs = [(self._obs[1], *outs[0][1:]), (self._obs[0], *outs[1][1:])]
        self._cur = 0
        # this step's active mask: the rollout ends by advancing the device step
        # counter k_dev and copying the NEXT step's row of the table
        # (exo_active_advance; an extra all-False row past the round's end, where
        # the counter saturates), so no host copy runs between graph replays
        self._table_ext = torch.cat([self.active_table, torch.zeros_like(self.active_table[:1])]).contiguous()
        self.active = self.active_table[0].clone()
        self.k = 0
        self.use_graphs = use_graphs
        self.warmup_eager = warmup_eager
        self.iters = 0
        self.resets = 0  # episode-round resets done by step()
        self.graphs = {}
        self.dp = agent.sync.active  # tests set it to exercise the 3-graph layout at world 1
        # the env step shares the GPU with the TD7 passes: packed into half the
        # CUs (512-thread workgroups) unless the caller chose a kernel variant.
        # Only where 'auto' runs the row-parallel kernel (N <= 16,384): above it
        # the two-lane kernel is the fast one (65,536 envs: 106 vs 291 us)
        if (getattr(env, "step_variant", None) == "auto" and env.n <= 16384
                and os.environ.get("EXO_TRAIN_STEP_SHARED", "1") == "1"):
            env.set_step_variant("rows_shared")
        self.last_actions = None
        # exploration: "gaussian" (TD7_multi_agent.py select_action) or "pink"
        # (TD7_multi_agent_Pink_noise.py: one coloured sequence per episode round)
        if exploration not in ("gaussian", "pink"):
            raise ValueError(f"exploration must be 'gaussian' or 'pink', not {exploration!r}")
        self.exploration = exploration
        self.k_dev = torch.zeros((1,), dtype=torch.int64, device=self.device)
        if exploration == "pink":
            agent.init_episode_noise_device(self.round_len)
        if use_graphs and os.environ.get("EXO_GRAPH_CHECK", "1") != "0":
            graph_reductions_ok(self.device)

    # ----------------------------------------------------------- pieces
    def _rollout(self):
        ag = self.agent
        obs = self.obs
        act = ag.select_action_batch(obs, timestep=self.k_dev if self.exploration == "pink" else None)
        nobs, rew, done, info = self.env.step(act, active=self.active, out=self._outs[self._cur])
        ag.replay_buffer.add_batch(obs, act, nobs, rew, done, self.strata, self.active)
        nat.check(nat.lib().exo_active_advance(nat.ptr(self._table_ext), self._table_ext.shape[0], self.n,
                                               nat.ptr(self.k_dev), nat.ptr(self.active), nat.stream_ptr(self.device)),
                  "exo_active_advance")
        self.last_actions = act

    @property
    def obs(self):
        """The current observation buffer."""
        return self._obs[self._cur]

    @property
    def out(self):
        """The env output buffers (obs, reward, done, info) of the current step."""
        return self._outs[self._cur]

    # The update samples its batch BEFORE this iteration's transitions are
    # stored (from iteration 1 on), which frees the rollout (batched actor
    # inference -> exo_step -> replay insert) to run on a side stream -- a
    # parallel branch of the captured graph -- concurrently with the TD7
    # gradients.  The branch joins before the priority update and the
    # optimiser steps, so the replay insert still precedes update_priority and
    # select_action still reads the weights of the previous update, as in the
    # serial order; the only change is the one-step lag between a transition's
    # insert and its first chance to be sampled (the reference trains in
    # bursts after each episode round anyway, Exoskeleton_agent_train.py:208).
    # EXO_ROLLOUT_OVERLAP=0 keeps the serial insert-then-sample order.
    overlap_rollout = os.environ.get("EXO_ROLLOUT_OVERLAP", "1") == "1"
    # With the rollout overlapped, iteration t+1's batch (which must follow
    # iteration t's inserts and priority update, and nothing else) is sampled
    # at the end of iteration t, on the priority branch, into the other of two
    # batch slots (slot = observation-buffer parity, so a captured graph keeps
    # reading the slot it was captured with): the sample leaves the head of the
    # iteration's critical path.  EXO_SAMPLE_PREFETCH=0 samples at the start.
    prefetch_sample = os.environ.get("EXO_SAMPLE_PREFETCH", "1") == "1"

    def _prefetching(self):
        return self.prefetch_sample and self.overlap_rollout

    def _pre(self):
        ag = self.agent
        # one GPU: the encoder's gradients and step stay on its branch, joined
        # at the end of the iteration (_join_prio)
        ag.learner.defer_side_join = ENC_STEP_BRANCH and not self.dp
        rb = ag.replay_buffer
        slot = self._cur if self._prefetching() else None
        if self.iters == 0 or not self.overlap_rollout:
            self._rollout()
            self._batch = rb.sample(slot)
            self._ind = rb.ind
            self._prio = ag.learner.phase_grads(*self._batch)
            return
        if self._prefetching():
            self._batch, self._ind = rb._slot(slot)  # sampled by the previous iteration
        else:
            self._batch = rb.sample()
            self._ind = rb.ind
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_rollout_stream", None) is None:
            self._rollout_stream = torch.cuda.Stream(device=self.device)
        br = self._rollout_stream
        br.wait_stream(cur)
        with torch.cuda.stream(br):
            self._rollout()
        self._prio = ag.learner.phase_grads(*self._batch)
        cur.wait_stream(br)

    # LAP.update_priority reads only the sampled indices and the new priorities
    # and writes only the sum trees, which nothing else in the iteration reads
    # after the sample: on one GPU it runs as its own graph branch beside the
    # optimiser steps and the actor update, joined at the end of the iteration
    # (before the next sample).  Data-parallel runs keep it in place (the MAX
    # all-reduce of max_priority follows it).  EXO_PRIO_BRANCH=0 serialises.
    prio_branch = os.environ.get("EXO_PRIO_BRANCH", "1") == "1"

    def _mid(self, update_actor, flat_grad=None, grad_scale=1.0):
        ag = self.agent
        self._pside = None
        if self.prio_branch and not self.dp:
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_prio_stream", None) is None:
                self._prio_stream = torch.cuda.Stream(device=self.device)
            self._pside = self._prio_stream
            self._pside.wait_stream(cur)
            with torch.cuda.stream(self._pside):
                ag.replay_buffer.update_priority(self._prio, self._ind)
                self._sample_next()
            ag.learner.phase_steps(flat_grad, grad_scale)
        else:
            ag.learner.phase_steps(flat_grad, grad_scale)
            ag.replay_buffer.update_priority(self._prio, self._ind)
            self._sample_next()
        if update_actor:
            ag.learner.phase_actor_grads(self._batch[0], self._batch[1])

    def _sample_next(self):
        if self._prefetching():
            self.agent.replay_buffer.sample(1 - self._cur)

    def _join_prio(self):
        if getattr(self, "_pside", None) is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._pside)
            self._pside = None
        self.agent.learner.join_side()  # the encoder branch's optimiser step

    def _post(self, update_actor, flat_grad=None, grad_scale=1.0):
        if update_actor:
            self.agent.learner.phase_actor_step(flat_grad, grad_scale)

    def _eager(self, update_actor):
        L = self.agent.learner
        self._pre()
        L.sync.allreduce_grads(L.grad_params())
        self._mid(update_actor)
        self.agent.sync.max_(self.agent.replay_buffer._maxp)
        if update_actor:
            L.sync.allreduce_grads(L.grad_params(actor=True))
        self._post(update_actor)
        self._join_prio()

    def _capture(self, update_actor):
        """Capture this parity's iteration; the capture itself performs one real iteration."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        pool = None  # one private pool per parity: the two parities replay in alternation
        parts = []
        with torch.cuda.stream(s):
            if not self.dp:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, stream=s), ForkJoinAudit(s):
                    self._pre()
                    self._mid(update_actor)
                    self._post(update_actor)
                    self._join_prio()
                parts = [g]
            else:
                # Each parity's graphs own their gradient buffers (set_to_none
                # grads are allocated inside the capture), so the all-reduces
                # work on flat buckets packed/unpacked inside the graphs.
                L, S = self.agent.learner, self.agent.sync
                g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1, pool=pool, stream=s), ForkJoinAudit(s):
                    self._pre()
                    flat_c = S.pack(L.grad_params())
                pool = g1.pool()
                flat_a = None
                scale = 1.0 / S.world
                with torch.cuda.graph(g2, pool=pool, stream=s), ForkJoinAudit(s):
                    self._mid(update_actor, flat_c, scale)   # the optimisers read the reduced bucket in place
                    if update_actor:
                        flat_a = S.pack(L.grad_params(actor=True))
                if update_actor:  # no actor step at this parity: nothing to capture
                    with torch.cuda.graph(g3, pool=pool, stream=s), ForkJoinAudit(s):
                        self._post(update_actor, flat_a, scale)
                else:
                    g3 = None
                parts = [g1, g2, g3, flat_c, flat_a]
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graphs[(update_actor, self._cur)] = parts
        # capture records but does not execute: run the iteration now
        self._replay(update_actor)

    def _replay(self, update_actor):
        parts = self.graphs[(update_actor, self._cur)]
        if not self.dp:
            parts[0].replay()
            return
        S = self.agent.sync
        g1, g2, g3, flat_c, flat_a = parts
        g1.replay()
        S.allreduce_flat(flat_c)
        g2.replay()
        S.max_(self.agent.replay_buffer._maxp)  # global max_priority after this step's updates
        if update_actor:
            S.allreduce_flat(flat_a)
            g3.replay()

    # ------------------------------------------------------------- step
    def step(self):
        """One training iteration; returns the number of active env-steps."""
        ag = self.agent
        L = ag.learner
        if self.k == self.round_len:
            self.env.reset(obs_out=self.obs)
            self.k = 0
            self.k_dev.zero_()
            self.active.copy_(self.active_table[0])
            self.resets += 1
            if self.exploration == "pink":
                ag.init_episode_noise_device(self.round_len)
        L.training_steps += 1
        update_actor = L.training_steps % ag.hp.policy_freq == 0
        L.prefetch_actor = update_actor  # phase_grads may start the actor forward early
        if not self.use_graphs or self.iters < self.warmup_eager:
            self._eager(update_actor)
        elif (update_actor, self._cur) not in self.graphs:
            self._capture(update_actor)
        else:
            self._replay(update_actor)
        if L.maybe_update_targets():
            ag.replay_buffer.reset_max_priority()
            ag.sync.max_(ag.replay_buffer._maxp)
        n_active = int(self.active_counts[self.k])
        self.k += 1
        self.iters += 1
        self._cur ^= 1  # the next observation is in the other buffer
        return n_active
