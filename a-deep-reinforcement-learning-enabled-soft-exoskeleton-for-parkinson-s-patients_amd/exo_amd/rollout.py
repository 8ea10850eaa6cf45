"""Vectorised TD7 training loop on one GPU, replayed from HIP graphs.

One iteration = the reference training script's per-step work for every env
(Simulation/Exoskeleton_agent_train.py:123-147: select_action, env.step,
replay_buffer.add) plus one Agent.train() step (:208 / TD7_multi_agent.py:211).
Episodes are synchronous like the script (:110-123): all envs reset together
and done envs stay idle until the longest motion ends.

Everything inside an iteration is device work with no host synchronisation,
so it is captured once into HIP graphs and replayed:
  * world == 1: one graph per policy-update parity (actor updated or not);
  * world  > 1 on RCCL: the same one graph with the collectives captured in
    it (VecTrainer._inline): the encoder's gradient bucket all-reduced on the
    encoder's branch, the critic's before its step, a MAX of max_priority
    after the priority update, the actor's bucket before its step;
  * world  > 1 on gloo (or EXO_DP_CAPTURE=0): the collectives run eagerly
    between three graphs: the encoder/critic gradient bucket after `pre`
    (rollout + grads), a MAX of max_priority after `mid` (optimiser steps +
    priorities + actor grads), the actor bucket before `post` (actor step).
Host-side bookkeeping left outside the graphs: the env reset at the end of a
round, the target-network refresh every 250 steps (:284-293).
"""
import contextlib
import os
import threading

import numpy as np
import torch

from . import _native as nat
from .graphs import capture, new_graph
from . import td7 as _td7
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
        g = new_graph()
        with capture(g, stream=s):
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


def retire_graphs(trainer):
    """Release a finished trainer's captured graphs: their execs and memory
    pools are freed and ballast streams replace the runtime streams they held
    (exo_amd.graphs.release_graphs; destroying execs without the ballast can
    leave the hardware-queue loads uneven, after which the ROCm 7.0 runtime's
    launch of a later exec reads past its stream vector -- DESIGN.md 4, "The
    graph-replay crash").  Synchronises the device.  Returns the number of
    graphs released."""
    from .graphs import release_graphs
    objs = []
    for name in ("graphs", "_round_graphs"):
        g = getattr(trainer, name, None)
        if isinstance(g, dict) and g:
            objs.append(dict(g))
            g.clear()
    if trainer.__dict__.get("_refresh_graph") is not None:
        objs.append(trainer._refresh_graph)
        trainer._refresh_graph = None
    return release_graphs(*objs)


def _np_median(x):
    """numpy's median of a 1-D tensor (the mean of the two middle values for
    an even count; torch.median returns the lower one)."""
    v = x.sort().values
    n = v.numel()
    return v[n // 2] if n % 2 else (v[n // 2 - 1] + v[n // 2]) / 2


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
    joined back (after joining it, so that capture end still succeeds).

    The two torch methods are patched once for all audits alive in the
    process (a depth count: nested audits unpatch when the outermost exits),
    and an audit records only the calls made on the thread that opened it --
    another thread's captures and waits stay out of its log."""

    _lock = threading.Lock()
    _depth = 0
    _orig = None
    _open = []  # audits currently entered (any thread)

    def __init__(self, origin):
        self.origin = origin
        self.events = []
        self._thread = None

    @classmethod
    def _record(cls, ev):
        me = threading.get_ident()
        for audit in list(cls._open):
            if audit._thread == me:
                audit.events.append(ev)

    def __enter__(self):
        cls = ForkJoinAudit
        self._thread = threading.get_ident()
        with cls._lock:
            if cls._depth == 0:
                wait0, exit0 = torch.cuda.Stream.wait_stream, torch.cuda.StreamContext.__exit__
                cls._orig = (wait0, exit0)

                def wait_stream(st, other):
                    cls._record(("wait", st, other))
                    return wait0(st, other)

                def ctx_exit(ctx, *a):
                    if ctx.stream is not None:
                        cls._record(("use", ctx.stream))
                    return exit0(ctx, *a)

                torch.cuda.Stream.wait_stream = wait_stream
                torch.cuda.StreamContext.__exit__ = ctx_exit
            cls._depth += 1
            cls._open.append(self)
        return self

    def __exit__(self, exc_type, exc, tb):
        cls = ForkJoinAudit
        with cls._lock:
            cls._open.remove(self)
            cls._depth -= 1
            if cls._depth == 0:
                torch.cuda.Stream.wait_stream, torch.cuda.StreamContext.__exit__ = cls._orig
                cls._orig = None
        if exc_type is not None:
            return False
        bad = unjoined_streams(self.events, self.origin)
        if bad:
            for st in bad:
                self.origin.wait_stream(st)
            raise CaptureForkError(f"{len(bad)} stream(s) forked from the capture stream were not joined back "
                                   "before capture end")
        return False


# r05: where the rollout branch (select_action -> env step -> replay insert)
# forks from the iteration.  The iteration's first ~90 us are CU-throughput
# bound (DESIGN.md 4 "TD7 fused", r05 schedule): EXO_ROLLOUT_AFTER="fixed"
# forks it after the fixed embeddings' pass instead of at the iteration start.
ROLLOUT_AFTER = os.environ.get("EXO_ROLLOUT_AFTER", "")
# r05, the captured order (bit-identical either way): EXO_TRAIN_FIRST (default
# on) captures the rollout branch after the target chain (still forked from
# the iteration's start), so the graph's first node -- which runs on the
# launch stream's queue, where the other queues' first nodes wait for a
# cross-queue start -- is the critical chain's target pass: 0.2535-0.2537 vs
# 0.2571-0.2577 ms per iteration (profiles/r05_sched/r05o);
# EXO_PAIR_CRITIC_AFTER_SELECT=1 makes an overlapped pair's second critic pass
# wait for that iteration's select_action: 0.2616-0.2618, off.
TRAIN_FIRST = os.environ.get("EXO_TRAIN_FIRST", "1") == "1"
EARLY_LAP = os.environ.get("EXO_EARLY_LAP", "1") == "1"
PAIR_CRITIC_AFTER_SELECT = os.environ.get("EXO_PAIR_CRITIC_AFTER_SELECT", "0") == "1"


class VecTrainer:
    def __init__(self, env, agent, strata=None, use_graphs=True, warmup_eager=3, exploration="gaussian",
                 shared_step=True, episodes=None):
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
        # envs running at this step = the script's select_action calls (:125-128),
        # written by exo_active_advance with the next step's mask
        self.active_count = torch.full((1,), int(self.active_counts[0]), dtype=torch.int32, device=self.device)
        self.k = 0
        self.use_graphs = use_graphs
        self.warmup_eager = warmup_eager
        self.iters = 0
        self.resets = 0  # episode-round resets done by step()
        self.graphs = {}
        self.dp = agent.sync.active  # tests set it to exercise the data-parallel layouts at world 1
        # data parallel on RCCL: the collectives run inside the iteration's one
        # graph (GradSync.graph_capturable; EXO_DP_CAPTURE=0 or gloo: three
        # graphs per iteration with eager all-reduces between them)
        self.dp_inline = bool(self.dp and use_graphs and agent.sync.graph_capturable(self.device))
        # the env step beside the TD7 passes: EXO_TRAIN_STEP_SHARED=1 packs it
        # into half the CUs (512-thread workgroups, r02: 306 vs 316 us per
        # iteration then).  Off since r05: with the overlapped pairs the second
        # iteration's env step is on the pair's critical chain, where the
        # 256-thread shape's own speed wins -- 0.2493-0.2496 vs 0.2526-0.2531 ms
        # per iteration (profiles/r05_sched/r05sh).  Only where 'auto' runs the
        # row-parallel kernel (N <= 16,384): above it the two-lane kernel is the
        # fast one (65,536 envs: 106 vs 291 us)
        if (shared_step and getattr(env, "step_variant", None) == "auto" and env.n <= 16384
                and os.environ.get("EXO_TRAIN_STEP_SHARED", "0") == "1"):
            env.set_step_variant("rows_shared")
        self.last_actions = None
        # exploration: "gaussian" (TD7_multi_agent.py select_action) or "pink"
        # (TD7_multi_agent_Pink_noise.py: one coloured sequence per episode round)
        if exploration not in ("gaussian", "pink"):
            raise ValueError(f"exploration must be 'gaussian' or 'pink', not {exploration!r}")
        self.exploration = exploration
        self.k_dev = torch.zeros((1,), dtype=torch.int64, device=self.device)
        # budgeted env steps (env.set_step_budget, BASELINE configs[3]): a stiff
        # env's solve spans launches; the step mask then comes from the device
        # (exo_budget_advance: episode not over and no solve pending) and a
        # round lasts until every env finished (`remaining` read by the host
        # once the round's round_len iterations are done)
        self.budget = int(getattr(env, "step_budget", 0))
        if self.budget:
            if exploration == "pink":
                raise ValueError("Pink exploration indexes its noise by the round's step: not with a step budget")
            self._remaining = torch.zeros((1,), dtype=torch.int32, device=self.device)
            self._steps_total = torch.zeros((1,), dtype=torch.int64, device=self.device)
        # episodes: "sync" -- the script's synchronous rounds (every env resets
        # when the longest motion ends, envs that finished early idle until
        # then) -- or "async" -- each env resets in place as soon as its own
        # episode ends (exo_episode_advance inside the iteration, no host work
        # between rounds), so every launch steps every env that has no
        # pending budgeted solve.  EXO_EPISODES picks the default.
        if episodes is None:
            episodes = os.environ.get("EXO_EPISODES", "sync")
        if episodes not in ("sync", "async"):
            raise ValueError(f"episodes must be 'sync' or 'async', not {episodes!r}")
        self.episodes = episodes
        if episodes == "async":
            if exploration == "pink":
                raise ValueError("Pink exploration indexes its noise by the round's step: not with async episodes")
            self.active.fill_(True)
            self.active_count.fill_(self.n)
            if not self.budget:
                self._steps_total = torch.zeros((1,), dtype=torch.int64, device=self.device)
        if exploration == "pink":
            agent.init_episode_noise_device(self.round_len)
        if use_graphs and os.environ.get("EXO_GRAPH_CHECK", "1") != "0":
            graph_reductions_ok(self.device)

    # ----------------------------------------------------------- pieces
    # select_action's workgroups per launch in this loop (td7f_select's cap):
    # here it runs beside the iteration's fused passes, off the critical
    # chain, so with fp32 operands it takes at most 128 CUs at a time (0.488-
    # 0.491 vs 0.493-0.499 ms per iteration at 4,096 envs, profiles/r04sc_raw);
    # EXO_LOOP_SELECT_CAP overrides (0: one launch)
    def _select_cap(self):
        env = os.environ.get("EXO_LOOP_SELECT_CAP")
        if env is not None:
            return int(env)
        return 128 if self.agent.learner.precision == "fp32" else None

    # select_action's row tiles in this loop (16-bit operands; fp32 keeps 16
    # rows): with overlapped pairs (below) the second iteration's select_action
    # is on the pair's critical chain beside the update's passes, where 32-row
    # tiles (half the workgroups, half the weight bytes) run it sooner: 0.249-
    # 0.255 vs 0.259-0.265 ms per iteration (profiles/r05_sched); unpaired they
    # measured even (r03).  Not bit-identical to 16-row tiles (another fp32
    # summation order: ~1 % of the actions differ in the last bf16 bits).
    # EXO_LOOP_SELECT_RT: 2 (default), 1, or 0 (the library's pick).
    loop_select_rt = int(os.environ.get("EXO_LOOP_SELECT_RT", "2"))

    def _select_rt(self):
        if self.agent.learner.precision == "fp32":
            return None
        return self.loop_select_rt or None

    # r06: in the overlapped pair's second iteration select_action's fixed-
    # encoder half (zs of the observations, td7f_select_part mode 1) runs from
    # the iteration's start; only its actor half waits for the first
    # iteration's actor step.  Bit-identical (the two halves are the one-launch
    # pass split at its zs image).  Same box, 3 / 2 alternations
    # (profiles/r06_split_select): fp32 0.4005-0.4107 vs 0.4222-0.4242 ms per
    # iteration -- on by default there; bf16 0.2504-0.2525 vs 0.2418-0.2459
    # (the zs half's 128 workgroups beside the second iteration's target chain
    # cost more than the shorter select saves) -- off.  EXO_SPLIT_SELECT:
    # "auto" (fp32 only), "1" (always), "0" (never).
    split_select = os.environ.get("EXO_SPLIT_SELECT", "auto")

    def _split_select_ok(self):
        L = self.agent.learner
        on = self.split_select == "1" or (self.split_select == "auto" and L.precision == "fp32")
        return on and L.fused is not None and self.exploration == "gaussian" and self.obs.is_cuda

    def _select_zs(self):
        """the zs half of this iteration's select_action (see split_select;
        EXO_SPLIT_ZS_CAP: its own workgroup cap, default the loop's)"""
        cap = os.environ.get("EXO_SPLIT_ZS_CAP")
        return self.agent.learner.fused.select_zs(self.obs, wg_cap=int(cap) if cap is not None else self._select_cap(),
                                                  rt=self._select_rt())

    def _rollout(self, zs_img=None):
        ag = self.agent
        obs = self.obs
        act = ag.select_action_batch(obs, timestep=self.k_dev if self.exploration == "pink" else None,
                                     dec_count=self.active_count, wg_cap=self._select_cap(), rt=self._select_rt(),
                                     zs_img=zs_img)
        if self._overlap_wait is not None and PAIR_CRITIC_AFTER_SELECT:
            self._select_done = torch.cuda.Event()
            self._select_done.record(torch.cuda.current_stream(self.device))
        nobs, rew, done, info = self.env.step(act, active=self.active, out=self._outs[self._cur],
                                              obs_cur=obs if self.budget else None)
        ag.replay_buffer.add_batch(obs, act, nobs, rew, done, self.strata, self.active)
        if self._early_on:  # the tree is current from here (see EARLY_LAP)
            self._ins_ev = torch.cuda.Event()
            self._ins_ev.record(torch.cuda.current_stream(self.device))
        self._advance()
        self.last_actions = act

    def _advance(self, rew=None, score=None):
        """The next step's active mask and count on the device (exo_active_advance);
        with rew / score: score += rew where the replaced mask is set, in the same
        launch (exo_active_advance_score).  Step budget: the mask from the
        envs' own progress (exo_budget_advance).  Async episodes: finished
        envs reset in place, into the observation buffer the step wrote
        (exo_episode_advance)."""
        if self.episodes == "async":
            self.env.episode_advance(self.active, self.active_count, self._outs[self._cur][0], self._steps_total)
            return
        if self.budget:
            self.env.budget_advance(self.active, self.active_count, self._remaining, self._steps_total)
            return
        if score is not None:
            nat.check(nat.lib().exo_active_advance_score(
                nat.ptr(self._table_ext), self._table_ext.shape[0], self.n, nat.ptr(self.k_dev), nat.ptr(self.active),
                nat.ptr(self.active_count), nat.ptr(rew), nat.ptr(score), nat.stream_ptr(self.device)),
                "exo_active_advance_score")
            return
        nat.check(nat.lib().exo_active_advance(nat.ptr(self._table_ext), self._table_ext.shape[0], self.n,
                                               nat.ptr(self.k_dev), nat.ptr(self.active), nat.ptr(self.active_count),
                                               nat.stream_ptr(self.device)), "exo_active_advance")

    def _round_start(self):
        """Device step counter, active mask and count back to the first step of a round."""
        self.k = 0
        self.k_dev.zero_()
        self.active.copy_(self.active_table[0])
        self.active_count.fill_(int(self.active_counts[0]))

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

    # r04 (EXO_TARGET_PREFETCH=1, off by default): with the next batch sampled
    # at the end of an iteration, its fixed embeddings and target heads are
    # computed right after it (beside the actor update of an actor iteration)
    # into one of two persistent slots (TD7Learner.prefetch_targets), and the
    # next iteration's critic pass starts at once.  Not before a target
    # refresh (the refresh changes those nets), not in the data-parallel
    # three-graph layout.  Bit-identical, but measured slower (0.37-0.46 vs
    # 0.30 ms per iteration, profiles/r04h_raw): the critic -> priority ->
    # sample -> targets chain is as long as before, and the graph's four
    # hardware queues put the actor passes behind the target chain instead of
    # beside it ("TD7 fused").
    prefetch_targets = os.environ.get("EXO_TARGET_PREFETCH", "0") == "1"
    _pre_in = _pre_out = False

    def _target_prefetch_flags(self):
        L = self.agent.learner
        ok = (self.prefetch_targets and self._prefetching() and L.fused_train and self.iters > 0
              and (not self.dp or self.dp_inline))
        pre_in = ok and L.prefetch_ready(self._cur)
        pre_out = ok and L.training_steps % L.hp.target_update_rate != 0
        return pre_in, pre_out

    def _pre(self, rollout=True):
        ag = self.agent
        self._early_on = False
        # one GPU: the encoder's gradients and step stay on its branch, joined
        # at the end of the iteration (_join_prio)
        ag.learner.defer_side_join = ENC_STEP_BRANCH and (not self.dp or self.dp_inline)
        rb = ag.replay_buffer
        if not rollout:  # a training step alone (Agent.train): sample, then the gradients
            if self._train_pin:  # sampled by the burst's previous step (RefScheduleTrainer)
                self._batch, self._ind = rb._slot(self._bslot)
            else:
                self._batch = rb.sample(self._bslot if self._train_pout else None)
                self._ind = rb.ind
            self._prio = ag.learner.phase_grads(*self._batch)
            return
        slot = self._cur if self._prefetching() else None
        if self.iters == 0 or not self.overlap_rollout:
            self._rollout()
            self._batch = rb.sample(slot)
            self._ind = rb.ind
            self._prio = ag.learner.phase_grads(*self._batch)
            return
        self._early_on = self._early_lap()
        if self._prefetching():
            self._batch, self._ind = rb._slot(slot)  # sampled by the previous iteration
            if self._pre_in:
                ag.learner.pre_in = slot  # and its critic inputs computed there too
        else:
            self._batch = rb.sample()
            self._ind = rb.ind
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_rollout_stream", None) is None:
            self._rollout_stream = torch.cuda.Stream(device=self.device)
        br = self._rollout_stream

        split = self._overlap_wait is not None and self._split_select_ok()  # (its image: _capture_pair)

        def rollout_branch(cur=cur, br=br):
            br.wait_stream(cur)
            zimg = None
            if split:  # select_action's zs half needs only the observations
                with torch.cuda.stream(br):
                    zimg = self._select_zs()
            if self._overlap_wait is not None:  # overlapped pair: after the previous actor step
                br.wait_stream(self._overlap_wait)
            with torch.cuda.stream(br):
                self._rollout(zs_img=zimg)
        L = ag.learner
        late = (ROLLOUT_AFTER == "fixed" and L.fused_train and L.pre_in is None and not self._pre_in
                and not _td7.TARGET_ON_MAIN)
        first = (TRAIN_FIRST and not late and L.fused_train and L.pre_in is None and not self._pre_in
                 and not _td7.TARGET_ON_MAIN and L.overlap)
        if late:
            # forked after the fixed pass (TD7Learner.after_fixed): see ROLLOUT_AFTER
            L.after_fixed = rollout_branch
        elif first:
            # forked from the iteration's start, captured after the target chain
            # (TD7Learner.after_target): see TRAIN_FIRST
            ev0 = torch.cuda.Event()
            ev0.record(cur)

            def rollout_from_start(ev0=ev0, br=br):
                br.wait_event(ev0)
                zimg = None
                if split:
                    with torch.cuda.stream(br):
                        zimg = self._select_zs()
                if self._overlap_wait is not None:
                    br.wait_stream(self._overlap_wait)
                with torch.cuda.stream(br):
                    self._rollout(zs_img=zimg)
            L.after_target = rollout_from_start
        else:
            rollout_branch()
        if self._overlap_wait is not None and PAIR_CRITIC_AFTER_SELECT:
            # overlapped pair, second iteration: its critic pass after its
            # select_action (which is on the pair's critical chain)
            def critic_after_select():
                torch.cuda.current_stream(self.device).wait_event(self._select_done)
            L.before_critic = critic_after_select
        self._us_done = False
        if self._us_after_critic():
            # the priority update + next sample on its branch as soon as the
            # critic pass has written |td| (beside the weight gradients and the
            # optimiser steps); it also needs this iteration's inserts
            def fork(td, cur=cur, br=br):
                L = ag.learner
                ps = self._prio_stream_get()
                ps.wait_stream(cur)
                ps.wait_stream(br)
                with torch.cuda.stream(ps):
                    ag.replay_buffer.update_priority_and_sample_td(td, L.hp.alpha, L.hp.min_priority, self._ind,
                                                                   1 - self._cur)
                self._pside = ps
                self._us_done = True
            ag.learner.after_critic = fork
        self._prio = ag.learner.phase_grads(*self._batch)
        ag.learner.after_critic = None
        if ag.learner.after_fixed is not None or ag.learner.after_target is not None:
            raise RuntimeError("VecTrainer: the rollout branch was not forked (no fixed / target pass in phase_grads)")
        ag.learner.before_critic = None
        if self._early_on:
            self._br_pending = br  # joined by the sample's gather / the actor passes / the iteration's end
        else:
            cur.wait_stream(br)

    # LAP.update_priority reads only the sampled indices and the new priorities
    # and writes only the sum trees, which nothing else in the iteration reads
    # after the sample: on one GPU it runs as its own graph branch beside the
    # optimiser steps and the actor update, joined at the end of the iteration
    # (before the next sample).  Data-parallel runs keep it in place (the MAX
    # all-reduce of max_priority follows it).  EXO_PRIO_BRANCH=0 serialises.
    prio_branch = os.environ.get("EXO_PRIO_BRANCH", "1") == "1"
    # r03: only when this iteration also updates the actor (the branch then
    # runs beside the actor's passes); otherwise the update and the next
    # sample follow the critic's weight gradients on the iteration's stream,
    # with no cross-queue hand-off on the critical path (EXO_PRIO_BRANCH_ALL=1:
    # the branch in every iteration, the r02 layout)
    prio_branch_all = os.environ.get("EXO_PRIO_BRANCH_ALL", "0") == "1"

    # r04: the priority update + next sample from the critic pass's |td|
    # (LAP.update_priority_and_sample_td) right after the critic pass, on its
    # branch, instead of after the weight-gradient launch; one GPU, prefetching
    # trainer only.  Off until measured (EXO_US_AFTER_CRITIC=1: on).
    us_after_critic = os.environ.get("EXO_US_AFTER_CRITIC", "0") == "1"
    _us_done = False

    def _us_after_critic(self):
        L = self.agent.learner
        rb = self.agent.replay_buffer
        return (self.us_after_critic and not self.dp and self._prefetching() and not self._pre_out
                and L.fused_train and rb.device_rng and rb.batch_size <= 1024)

    def _prio_stream_get(self):
        if getattr(self, "_prio_stream", None) is None:
            self._prio_stream = torch.cuda.Stream(device=self.device)
        return self._prio_stream

    # r05: in a critic-only iteration the priority update + next sample's
    # indices wait only for this iteration's insert (the tree current: its
    # rank launch), not for the row copies, the episode advance and the
    # resets after it; the rows are gathered once the rollout branch has
    # joined.  Bit-identical (lap_update_sample_idx + lap_gather_rows).  An
    # actor iteration joins the rollout before its actor passes (select_action
    # reads the actor they update).  EXO_EARLY_LAP=0: the whole rollout first.
    _early_on = False
    _br_pending = None
    _ins_ev = None

    def _early_lap(self):
        rb = self.agent.replay_buffer
        return (EARLY_LAP and not self.dp and self._prefetching() and not self._us_after_critic()
                and not self._pre_out and rb.device_rng and rb.fuse_update_sample and rb.batch_size <= 1024)

    def _join_rollout(self):
        if self._br_pending is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._br_pending)
            self._br_pending = None

    def _mid(self, update_actor, flat_grad=None, grad_scale=1.0, rollout=True):
        ag = self.agent
        self._mid_rollout = rollout
        if update_actor:
            self._join_rollout()
        if self._us_done:  # the priority update already runs on its branch (_pre)
            self._us_done = False
            ag.learner.phase_steps(flat_grad, grad_scale)
            if update_actor:
                with self._actor_ctx():
                    ag.learner.phase_actor_grads(self._batch[0], self._batch[1])
            return
        self._pside = None
        if update_actor and self._actor_stream is not None:
            # overlapped pair, first iteration: the actor branch captured before
            # the priority update's, so the graph's stream assignment (first
            # child inherits its parent's queue) keeps the actor passes off the
            # queue the next iteration's update chain inherits from the sample
            ag.learner.phase_steps(flat_grad, grad_scale)
            with self._actor_ctx():
                ag.learner.phase_actor_grads(self._batch[0], self._batch[1])
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_prio_stream", None) is None:
                self._prio_stream = torch.cuda.Stream(device=self.device)
            self._pside = self._prio_stream
            self._pside.wait_stream(cur)
            with torch.cuda.stream(self._pside):
                self._update_and_sample_next()
            return
        if self.prio_branch and not self.dp and (update_actor or self.prio_branch_all):
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_prio_stream", None) is None:
                self._prio_stream = torch.cuda.Stream(device=self.device)
            self._pside = self._prio_stream
            self._pside.wait_stream(cur)
            with torch.cuda.stream(self._pside):
                self._update_and_sample_next()
            ag.learner.phase_steps(flat_grad, grad_scale)
        else:
            ag.learner.phase_steps(flat_grad, grad_scale)
            self._update_and_sample_next()
        if update_actor:
            with self._actor_ctx():
                ag.learner.phase_actor_grads(self._batch[0], self._batch[1])

    # overlapped pairs (below): the first iteration's actor passes on a stream
    # of their own, which the next iteration's rollout and critic step wait for
    _actor_stream = None
    _overlap_wait = None

    def _actor_ctx(self):
        st = self._actor_stream
        cur = torch.cuda.current_stream(self.device)
        if st is None or cur.cuda_stream == st.cuda_stream:  # (already on it: no self-wait in the capture)
            return contextlib.nullcontext()
        st.wait_stream(cur)
        return torch.cuda.stream(st)

    def _update_and_sample_next(self):
        """LAP.update_priority of this iteration's batch, then (prefetching) the
        next iteration's batch into the other slot -- one launch
        (LAP.update_priority_and_sample).  The MAX all-reduce of max_priority
        (data parallel) follows; the sample does not read it."""
        rb = self.agent.replay_buffer
        if not self._mid_rollout and self._train_pout:
            # a burst step with another after it: the next batch now, beside
            # this step's optimiser steps (RefScheduleTrainer.train_step)
            rb.update_priority_and_sample(self._prio, self._ind, 1 - self._bslot)
        elif self._prefetching() and self._mid_rollout:
            if self._br_pending is not None and self._ins_ev is not None:
                torch.cuda.current_stream(self.device).wait_event(self._ins_ev)
                rb.update_priority_and_sample(self._prio, self._ind, 1 - self._cur, before_gather=self._join_rollout)
            else:
                self._join_rollout()
                rb.update_priority_and_sample(self._prio, self._ind, 1 - self._cur)
            if self._pre_out:
                b = rb._slot(1 - self._cur)[0]
                self.agent.learner.prefetch_targets(b[0], b[1], b[2], 1 - self._cur)
        else:
            rb.update_priority(self._prio, self._ind)

    def _join_prio(self):
        self._join_rollout()
        if getattr(self, "_pside", None) is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._pside)
            self._pside = None
        L = self.agent.learner
        L.join_side()  # the encoder branch's optimiser step
        L.join_prefetch()  # the next batch's fixed pass
        # the deferred-join mode belongs to this iteration only: an update()
        # called later (Agent.train) must not leave work on the branch
        L.defer_side_join = False

    def _post(self, update_actor, flat_grad=None, grad_scale=1.0):
        if update_actor:
            with self._actor_ctx():
                self.agent.learner.phase_actor_step(flat_grad, grad_scale)

    def _inline(self, update_actor, rollout=True):
        """One iteration with the data-parallel collectives in line (RCCL,
        captured into the iteration's graph like every other launch): the
        encoder bucket's AVG all-reduce on the encoder's branch (inside
        phase_grads), the critic bucket's before the optimiser steps, the MAX
        of max_priority after the priority update, the actor bucket's before
        the actor's step.  All ranks capture the collectives in this one
        order, each on the process group's stream."""
        ag, L, S = self.agent, self.agent.learner, self.agent.sync
        L.dp_inline = True
        try:
            self._pre(rollout)
            self._mid_rollout = rollout
            # the priority update and the next sample on a branch beside the
            # critic bucket's all-reduce and step; its MAX of max_priority is
            # captured after the critic bucket's all-reduce (one collective
            # stream: capture order is execution order on every rank)
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_prio_stream", None) is None:
                self._prio_stream = torch.cuda.Stream(device=self.device)
            self._pside = self._prio_stream
            if update_actor and self._actor_stream is not None:
                # overlapped pair, first iteration: the critic bucket, the
                # actor branch (its bucket's all-reduce and step on it), then
                # the priority update + sample and its MAX -- the actor branch
                # captured before the priority update's (see _mid); the
                # collectives' capture order is still one order on every rank
                flat_c = L.allreduce_phase_grads(self._batch[0].shape[0])
                L.phase_steps(flat_c, 1.0)
                with self._actor_ctx():
                    L.phase_actor_grads(self._batch[0], self._batch[1])
                    flat_a = L.allreduce_actor_grads()
                    self._post(update_actor, flat_a, 1.0)
                self._pside.wait_stream(cur)
                with torch.cuda.stream(self._pside):
                    self._update_and_sample_next()
                    S.max_(ag.replay_buffer._maxp)
                self._join_prio()
                return
            self._pside.wait_stream(cur)
            with torch.cuda.stream(self._pside):
                self._update_and_sample_next()
            flat_c = L.allreduce_phase_grads(self._batch[0].shape[0])
            with torch.cuda.stream(self._pside):
                S.max_(ag.replay_buffer._maxp)
            L.phase_steps(flat_c, 1.0)
            flat_a = None
            if update_actor:
                L.phase_actor_grads(self._batch[0], self._batch[1])
                flat_a = L.allreduce_actor_grads()
            self._post(update_actor, flat_a, 1.0)
            self._join_prio()
        finally:
            L.dp_inline = False

    def _eager(self, update_actor, rollout=True):
        if self.dp_inline:
            self._inline(update_actor, rollout)
            return
        L = self.agent.learner
        self._pre(rollout)
        L.sync.allreduce_grads(L.grad_params())
        self._mid(update_actor, rollout=rollout)
        self.agent.sync.max_(self.agent.replay_buffer._maxp)
        if update_actor:
            L.sync.allreduce_grads(L.grad_params(actor=True))
        self._post(update_actor)
        self._join_prio()

    def _key(self, update_actor, rollout):
        if rollout:
            return update_actor, self._cur, self._pre_in, self._pre_out
        if self._train_pin or self._train_pout:
            return "train", update_actor, self._train_pin, self._train_pout, self._bslot
        return "train", update_actor

    # burst steps (RefScheduleTrainer.train_step): the next step's batch sampled
    # at the end of the current one, into the other of two slots, when the
    # burst has another step -- the sample leaves the head of every step
    # (r04; bit-identical: the same update-then-sample order)
    _train_pin = _train_pout = False
    _bslot = 0

    def _capture(self, update_actor, rollout=True):
        """Capture this parity's iteration (rollout=False: a training step
        alone), then run it (a capture records, it does not execute)."""
        self._capture_graph(update_actor, rollout)
        self._replay(update_actor, rollout)

    def _capture_graph(self, update_actor, rollout=True):
        """Record this parity's iteration graph(s) under its key; nothing runs."""
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        pool = None  # one private pool per parity: the two parities replay in alternation
        parts = []
        with torch.cuda.stream(s):
            if not self.dp or self.dp_inline:
                g = new_graph()
                with capture(g, pool=pool, stream=s), ForkJoinAudit(s):
                    if self.dp_inline:
                        self._inline(update_actor, rollout)
                    else:
                        self._pre(rollout)
                        self._mid(update_actor, rollout=rollout)
                        self._post(update_actor)
                        self._join_prio()
                parts = [g]
            else:
                # Each parity's graphs own their gradient buffers (set_to_none
                # grads are allocated inside the capture), so the all-reduces
                # work on flat buckets packed/unpacked inside the graphs.
                L, S = self.agent.learner, self.agent.sync
                g1, g2, g3 = new_graph(), new_graph(), new_graph()
                with capture(g1, pool=pool, stream=s), ForkJoinAudit(s):
                    self._pre(rollout)
                    flat_c = S.pack(L.grad_params())
                pool = g1.pool()
                flat_a = None
                scale = 1.0 / S.world
                with capture(g2, pool=pool, stream=s), ForkJoinAudit(s):
                    self._mid(update_actor, flat_c, scale, rollout)  # the optimisers read the reduced bucket in place
                    if update_actor:
                        flat_a = S.pack(L.grad_params(actor=True))
                if update_actor:  # no actor step at this parity: nothing to capture
                    with capture(g3, pool=pool, stream=s), ForkJoinAudit(s):
                        self._post(update_actor, flat_a, scale)
                else:
                    g3 = None
                parts = [g1, g2, g3, flat_c, flat_a]
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graphs[self._key(update_actor, rollout)] = parts
        if self._graph_refresh() and self._refresh_graph is None:
            self._capture_refresh()

    def _replay(self, update_actor, rollout=True):
        parts = self.graphs[self._key(update_actor, rollout)]
        if not self.dp or self.dp_inline:
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

    # Two iterations per graph replay (r04, EXO_PAIR_GRAPHS=1, one GPU): the
    # iteration and the next one captured back to back into one graph (each
    # joins all its branches before the next starts), so the GPU pays one
    # graph launch per two iterations.  Only where no host work falls between
    # them: no target refresh, no episode-round reset, no prefetch flags.
    pair_graphs = os.environ.get("EXO_PAIR_GRAPHS", "0") == "1"
    # r05, overlapped pairs (EXO_OVERLAP_PAIRS=1; one GPU, fused update, policy
    # freq 2): an actor iteration and the critic-only iteration after it as one
    # graph in which the second iteration's target chain, fixed embeddings and
    # encoder update start as soon as the first one's priority update + next
    # sample (their batch) and encoder step are in -- beside the first one's
    # actor passes -- while its rollout (select_action reads the new actor and
    # the priority update's max_priority) and its critic step (the actor
    # passes read the critic's weights) wait for the actor branch.  The same
    # launches on the same inputs: bit-identical to the unpaired graphs.
    # On by default since r05: 0.249-0.269 vs 0.287-0.288 ms per iteration
    # (profiles/r05_sched); EXO_OVERLAP_PAIRS=0 turns it off.
    overlap_pairs = os.environ.get("EXO_OVERLAP_PAIRS", "1") == "1"
    _pair_second = False

    def _pair_ok(self):
        L = self.agent.learner
        if self.overlap_pairs and not self.pair_graphs:
            # overlapped pairs start at an actor iteration (fused update only)
            if not (L.fused_train and L.training_steps % L.hp.policy_freq == 0 and L.hp.policy_freq == 2):
                return False
        elif not self.pair_graphs:
            return False
        return (self.use_graphs and (not self.dp or (self.dp_inline and self.overlap_pairs and not self.pair_graphs))
                and self.iters >= self.warmup_eager
                and not (self._pre_in or self._pre_out)
                and L.training_steps % L.hp.target_update_rate != 0
                and (self.episodes == "async" or self.k + 1 < self.round_len))

    def _pair_key(self, ua, ua2, overlap=False):
        return ("pair", ua, ua2, self._cur) + (("overlap",) if overlap else ())

    def _run_pair(self, ua, ua2, overlap=False):
        """This iteration and the next as one graph (captured on first use per
        policy-update parities and observation buffer).  overlap (an actor
        iteration, then a critic-only one; see overlap_pairs): the first
        iteration's actor passes on a branch of their own that only the second
        iteration's rollout and critic step wait for."""
        g = self.graphs.get(self._pair_key(ua, ua2, overlap))
        if g is None:
            g = self._capture_pair(ua, ua2, overlap)
        g.replay()

    def _capture_pair(self, ua, ua2, overlap=False):
        """Record the pair graph of _run_pair under its key; nothing runs."""
        L = self.agent.learner
        key = self._pair_key(ua, ua2, overlap)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = new_graph()
        cur0 = self._cur
        keep = []
        if overlap and getattr(self, "_astream", None) is None:
            self._astream = torch.cuda.Stream(device=self.device)
        if overlap and self._split_select_ok():
            L.fused.zs_image(self.n)  # the split select's zs image, allocated before the capture
        try:
            with torch.cuda.stream(s):
                with capture(g, stream=s), ForkJoinAudit(s):
                    for i, u in enumerate((ua, ua2)):
                        L.prefetch_actor = u
                        if overlap and i == 0:
                            self._actor_stream = self._astream
                        if overlap and i == 1:
                            self._actor_stream = None
                            self._overlap_wait = self._astream
                            L.before_critic_step = lambda st=self._astream: (
                                torch.cuda.current_stream(self.device).wait_stream(st))
                        if self.dp_inline:
                            self._inline(u, True)
                        else:
                            self._pre(True)
                            self._mid(u, rollout=True)
                            self._post(u)
                            self._join_prio()
                        if i == 0:
                            # the first iteration's tensors its actor branch
                            # still reads stay allocated through the capture
                            keep.append(L._fixed_zs)
                            self._cur ^= 1
                            self.iters += 1  # the second half is never iteration 0
                    if overlap:
                        s.wait_stream(self._astream)
        finally:
            self._actor_stream = self._overlap_wait = None
            L.before_critic_step = None
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._cur = cur0
        self.iters -= 1
        L.prefetch_actor = ua
        self.graphs[key] = g
        self._pair_keep = getattr(self, "_pair_keep", []) + keep
        return g

    # ------------------------------------------------------------- step
    def next_step_resets(self):
        """Whether the next step() starts a new episode round: after round_len
        iterations, and with a step budget once no env is left unfinished (a
        host read of the device count)."""
        if self.episodes == "async" or self.k < self.round_len:
            return False
        return not self.budget or int(self._remaining.item()) == 0

    def env_steps_total(self):
        """Step budget / async episodes: the env-steps taken so far (device
        counter, host sync)."""
        return int(self._steps_total.item())

    # Pair graphs run two iterations' GPU work at the first one's step(): only
    # inside a run the caller announced (plan), so no step() ever does work
    # past the last call the caller makes.
    _horizon = None

    def plan(self, n):
        """Announce that step() will be called n more times in a row (None:
        unknown, every step() one iteration's work).  Pair graphs -- the
        overlapped pairs, on by default -- start only where at least two
        announced calls remain."""
        self._horizon = None if n is None else int(n)

    def prepare(self):
        """Record, without running them, the graphs the announced steps (plan)
        replay: the next two iterations' graphs and, where they will run as an
        overlapped pair, the pair graph (r06, VERDICT r5 item 2: the pair was
        captured on first use, inside the caller's timed window).  A capture
        records and does not execute, so the trainer's state and every tensor
        stay as they were; only host-side capture bookkeeping is done here.
        Needs the eager warm-up iterations done (their buffers) and no pair
        half pending.  Returns the number of graphs recorded."""
        L = self.agent.learner
        if (not self.use_graphs or self.iters < self.warmup_eager or self._pair_second
                or self.prefetch_targets):
            return 0
        pf = L.hp.policy_freq
        saved = (L.training_steps, L.prefetch_actor, self._pre_in, self._pre_out, self._cur, self.iters, self.k)
        made = 0
        try:
            self._pre_in = self._pre_out = False
            for _ in range(2):  # the next two iterations alone (the pair's halves)
                L.training_steps += 1
                ua = L.training_steps % pf == 0
                L.prefetch_actor = ua
                if self._key(ua, True) not in self.graphs:
                    self._capture_graph(ua)
                    made += 1
                self._cur ^= 1
                self.iters += 1
            L.training_steps, self._cur, self.iters = saved[0], saved[4], saved[5]
            L.training_steps += 1
            ua, ua2 = L.training_steps % pf == 0, (L.training_steps + 1) % pf == 0
            if self._horizon is not None and self._horizon >= 2 and self._pair_ok():
                overlap = self.overlap_pairs and ua and not ua2 and L.fused_train
                if self._pair_key(ua, ua2, overlap) not in self.graphs:
                    L.prefetch_actor = ua
                    self._capture_pair(ua, ua2, overlap)
                    made += 1
        finally:
            (L.training_steps, L.prefetch_actor, self._pre_in, self._pre_out, self._cur, self.iters,
             self.k) = saved
        return made

    def step(self):
        """One training iteration; returns the number of active env-steps (with
        a step budget: 0, the count stays on the device, env_steps_total();
        async episodes without a budget: every env, N)."""
        ag = self.agent
        L = ag.learner
        horizon = self._horizon
        if horizon is not None:
            self._horizon = horizon - 1
        if self._pair_second:  # its GPU work ran with the previous step's pair graph
            self._pair_second = False
            L.training_steps += 1
            return self._step_tail()
        if self.next_step_resets():
            self.env.reset(obs_out=self.obs)
            self._round_start()
            self.resets += 1
            if self.exploration == "pink":
                ag.init_episode_noise_device(self.round_len)
        L.training_steps += 1
        update_actor = L.training_steps % ag.hp.policy_freq == 0
        L.prefetch_actor = update_actor  # phase_grads may start the actor forward early
        self._pre_in, self._pre_out = self._target_prefetch_flags()
        if not self.use_graphs or self.iters < self.warmup_eager:
            self._eager(update_actor)
        elif (horizon is not None and horizon >= 2 and self._pair_ok() and self._key(update_actor, True) in self.graphs
              and ((L.training_steps + 1) % ag.hp.policy_freq == 0, 1 - self._cur, False, False) in self.graphs):
            # (both halves captured alone first: their warm-up created every
            # buffer the pair capture needs)
            ua2 = (L.training_steps + 1) % ag.hp.policy_freq == 0
            self._run_pair(update_actor, ua2,
                           overlap=self.overlap_pairs and update_actor and not ua2 and L.fused_train)
            self._pair_second = True
        elif self._key(update_actor, True) not in self.graphs:
            self._capture(update_actor)
        else:
            self._replay(update_actor)
        # the prefetch slots' state after this iteration (a replay runs no host code)
        if self._pre_in or self._pre_out:
            if not isinstance(L._pre_ready, list):
                L._pre_ready = [False, False]
            if self._pre_in:
                L._pre_ready[self._cur] = False
            if self._pre_out:
                L._pre_ready[1 - self._cur] = True
        L.pre_in = None
        return self._step_tail()

    # The target refresh every target_update_rate steps (:284-293, plus the LAP
    # max_priority reset, :119-120) with the collectives of data parallelism
    # (the Q bounds and max_priority MAX-reduced): on RCCL with the collectives
    # captured in the iteration graphs it is itself replayed from a graph
    # captured at the first refresh, so no eager collective follows the
    # captured ones -- the first such eager all-reduce of a process cost 96 ms
    # (31-35 ms in later processes) of host time, GPU idle, at training step
    # 250: the first RCCL process's slow mode of r04 (profiles/r05rccl_raw).
    # One GPU as well (r05): the eager refresh's first run inside a timed
    # window cost ~8 ms of one-time host work (0.277 vs 0.256 ms per iteration
    # over a 400-iteration window on a fresh box, profiles/r05_sched/r05x);
    # the graph is captured with the first iteration graphs.  Eager-collective
    # data parallelism (gloo) keeps the eager refresh.
    _refresh_graph = None

    def _graph_refresh(self):
        return self.use_graphs and (not self.dp or self.dp_inline)

    def _refresh_targets(self):
        ag = self.agent
        L = ag.learner
        if L.training_steps % L.hp.target_update_rate != 0:
            return False
        if not self._graph_refresh():
            L.maybe_update_targets()
            ag.replay_buffer.reset_max_priority()
            ag.sync.max_(ag.replay_buffer._maxp)
            return True
        L.drop_prefetch()
        if self._refresh_graph is None:
            self._capture_refresh()
        self._refresh_graph.replay()
        return True

    def _capture_refresh(self):
        """Record (not run) the refresh graph.  Captured with the first
        iteration graphs, not at the first refresh inside a timed window: the
        capture of its collectives itself cost ~60 ms there (r05).  Thread-
        local capture mode: the process group's watchdog thread queries its
        events meanwhile (a global-mode capture failed it once with
        hipErrorStreamCaptureUnsupported)."""
        ag, L = self.agent, self.agent.learner
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = new_graph()
        with torch.cuda.stream(s):
            with capture(g, stream=s, capture_error_mode="thread_local"), ForkJoinAudit(s):
                L.update_targets_device()
                ag.replay_buffer.reset_max_priority()
                ag.sync.max_(ag.replay_buffer._maxp)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._refresh_graph = g

    def _step_tail(self):
        """Host bookkeeping after an iteration's GPU work."""
        ag = self.agent
        L = ag.learner
        self._refresh_targets()
        if self.budget:
            n_active = 0
        elif self.episodes == "async":
            n_active = self.n
        else:
            n_active = int(self.active_counts[self.k])
        self.k += 1
        self.iters += 1
        self._cur ^= 1  # the next observation is in the other buffer
        return n_active


class RefScheduleTrainer(VecTrainer):
    """The reference training script's schedule on N device envs
    (Simulation/Exoskeleton_agent_train.py:110-211), where VecTrainer trains one
    step per vectorised env step:

    * per episode round every env resets (:111-113) and the score starts at
      the reset's second value (counts = 2); the envs step synchronously until
      the longest motion ends (:123), done envs idle (:126, :140);
    * actions are uniform in [-1, 1) until the warm-up has passed, then
      select_action with Gaussian exploration (:125-131) -- noise scale
      decremented once per running env (:207);
    * every running env's transition goes to the replay in env order with the
      reference's shared pointer (LAP.add_batch_ref; ref_replay=False: the
      per-stratum rings of add_batch) -- no training during the rollout;
    * after the round, agent.maybe_train_and_checkpoint(round(mean(ep_len)),
      mean(score)) (:208): its train_and_reset runs that many TD7 steps as a
      burst, each a HIP-graph replay of Agent.train (sample, update, priority
      update, target refresh every 250 steps), and refreshes the policy
      checkpoint by the reference's rule (TD7_multi_agent.py:296-325);
    * the warm-up switch after the round (:210-211): steps_count counts active
      env-steps over all data-parallel ranks;
    * save_prefix (the script's agent.save("AGENT_NNS/test_agent") after every
      round, :290): Agent.save(save_prefix) once per round, its 8 files, on
      rank 0 of a data-parallel run (the replicas are identical); the host
      time it takes is summed in save_seconds.  None (the default): no save.

    One rollout step = select / uniform actions -> exo_step -> score -> replay
    insert -> next active mask, replayed from a captured graph per (random,
    observation buffer).  Parity hooks (eager rollout):
    action_source(trainer, random) -> [N, 7] actions of this step on the host
    (rows of idle envs ignored) instead of the device draws / batched
    select_action -- e.g. the script's own per-env np.random.uniform and
    select_action calls; reset_source(round, obs_out) resets every env (e.g.
    from injected draw streams) instead of exo_reset."""

    def __init__(self, env, agent, warmup=25_000, strata=None, use_graphs=True, ref_replay=True,
                 action_source=None, reset_source=None, warmup_eager=2, round_graph=None, stats=None,
                 save_prefix=None):
        if getattr(env, "step_budget", 0):
            raise ValueError("RefScheduleTrainer steps the script's synchronous episodes: no step budget")
        super().__init__(env, agent, strata=strata, use_graphs=use_graphs, warmup_eager=warmup_eager,
                         shared_step=False, episodes="sync")
        # the rollout runs alone (no TD7 pass beside it): the env step's own fast shape
        if getattr(env, "step_variant", None) == "rows_shared":
            env.set_step_variant("auto")
        self.warmup = int(warmup)
        self.ref_replay = ref_replay
        self.action_source, self.reset_source = action_source, reset_source
        self.world = agent.sync.world
        self.steps_count = 0      # :146, over every rank's envs
        self.allow_train = False  # :87, :210-211
        self.rounds = 0
        self.updates = 0
        dev = self.device
        self.score = torch.zeros(self.n, dtype=torch.float64, device=dev)
        self._rand_act = torch.zeros((self.n, 7), dtype=torch.float32, device=dev)  # injected actions
        # the warm-up's uniform actions, one buffer per observation parity: in
        # the overlapped round graph step k's replay insert (on its branch)
        # still reads step k's actions while step k+1 draws its own
        self._rand_acts = torch.zeros((2, self.n, 7), dtype=torch.float32, device=dev)
        Ls = env.lengths_host
        self.ep_len = Ls - 2  # starts at 1 (:115), +1 per step (:145) for L-3 steps
        self.round_env_steps = int((Ls - 3).sum())
        self.active_host = np.stack([Ls - 3 > k for k in range(self.round_len)])
        self._train_iters = 0
        self._roll_iters = 0
        self.trace = []
        # one graph per rollout round (round_graph): the round's steps replayed
        # as one graph, each step's replay insert on a branch beside the next
        # step's select_action (joined before that step's env step, which
        # overwrites the observation buffer the insert reads); the insert's
        # active mask comes from a per-parity copy (the step's own mask is
        # advanced in place for the next step)
        # off by default: measured no faster (40.0-40.4 vs 39.4-39.5 ms per
        # 4,096-env rollout round, profiles/r03_refsched_raw): the select_action
        # workgroups hold every CU, so the overlapped insert kernels wait for
        # CUs (lap_add 9 -> 34 us) and the next env step waits for them
        # EXO_REF_ROUND_GRAPH=2 (round_graph="serial", the default since r04):
        # the round graph with each step's insert in line (no branch), so the
        # only change from the per-step replays is one graph launch per round
        # instead of one per step -- with the one-launch insert + mask advance
        # 28.80 vs 29.19-29.27 ms per 4,096-env rollout round
        # (profiles/r04v_raw); EXO_REF_ROUND_GRAPH=0: per-step replays
        if round_graph is None:  # EXO_REF_ROUND_GRAPH=1: the branch-overlapped round graph
            round_graph = {"1": True, "2": "serial"}.get(os.environ.get("EXO_REF_ROUND_GRAPH", "2"), False)
        self.round_graph = bool(round_graph)
        self.round_overlap = round_graph != "serial"
        self._ins_stream = None
        self._ins_pending = False
        self._act_prev = torch.zeros((2, self.n), dtype=torch.bool, device=dev)
        self._round_graphs = {}
        self._eager_kinds = set()
        # the episode scores (:144) accumulated inside the mask advance launch;
        # EXO_REF_FUSED_SCORE=0: torch's where + add_ (2 launches per step)
        self.fused_score = os.environ.get("EXO_REF_FUSED_SCORE", "1") == "1"
        # r04: that advance inside the replay insert's launch (its last
        # workgroup out); EXO_REF_INSERT_ADVANCE=0: its own launch
        self.insert_advance = os.environ.get("EXO_REF_INSERT_ADVANCE", "1") == "1"
        # the burst steps' next-batch prefetch (VecTrainer._key): 74.7 vs
        # 75.3-75.7 ms per 283-step burst (profiles/r04v_raw), bit-identical,
        # but OFF: with it on, the full default bench segfaulted in the first
        # graph replay of the trainer that runs after this one (sync_rounds,
        # host side, inside hipGraphLaunch; profiles/r04seg_raw); off, the same
        # bench runs clean.  EXO_BURST_PREFETCH=1 turns it on.
        self.burst_prefetch = os.environ.get("EXO_BURST_PREFETCH", "0") == "1"
        self._burst_i = 0
        # the script's per-step tremor statistics (:149-205: exo_tremor_metrics
        # into a [round_len, N, 16] device record + per-env counters, 2
        # launches per step) and its per-round outputs (:213-317, round_stats()
        # -> self.round_stats); stats=None: EXO_REF_STATS=1 turns them on
        self.stats = (os.environ.get("EXO_REF_STATS", "0") == "1") if stats is None else bool(stats)
        self.round_stats = []
        self._stat_bufs = None
        self.save_prefix = save_prefix
        self.saves = 0
        self.save_seconds = 0.0
        # r05: the round's inserts planned at its start (LAP.ref_plan: the
        # steps' envs come from the mask table, so every add's slot follows
        # from the pointer at the round start), one elementwise launch per
        # step (LAP.ref_step: rows, scores, next mask) and the tree updated
        # once at the end (LAP.ref_commit) -- bit for bit the per-step fused
        # inserts (the branch-overlapped round graph, EXO_REF_ROUND_GRAPH=1,
        # keeps those).  EXO_REF_PLANNED=0: the per-step inserts.
        self.planned = os.environ.get("EXO_REF_PLANNED", "1") == "1" and ref_replay
        if self.planned:
            rows = self._table_ext.shape[0]
            counts = self._table_ext.sum(1).to(torch.int64)
            self._offs = torch.cumsum(counts, 0) - counts           # adds before each row
            self._plan_total = int(counts.sum())
            self._counts_tab = counts.to(torch.int32)
            self._plan = torch.full((rows, self.n), -1, dtype=torch.int32, device=dev)
            self._kk = torch.zeros((2,), dtype=torch.int64, device=dev)

    # ------------------------------------------------------------ rollout
    def _use_plan(self):
        """The planned inserts (ref_plan / ref_step / ref_commit) this round:
        the reference pointer with the score in the insert launch, not the
        branch-overlapped round graph."""
        return (self.planned and self.ref_replay and self.fused_score and self.active.dtype == torch.bool
                and not (self.round_graph and self.round_overlap))

    def _seen_eager(self, random):
        """A round graph is captured only after a per-step round of the same
        kind (random / policy) allocated its buffers."""
        return (bool(random), self.stats) in self._eager_kinds

    def _stats_buffers(self):
        if self._stat_bufs is None:
            f32 = dict(dtype=torch.float32, device=self.device)
            self._stat_bufs = (torch.zeros((self.n, 16), **f32), torch.zeros((self.round_len, self.n, 16), **f32),
                               torch.zeros((self.n, 6), **f32))
            self._pct_hist = []
        return self._stat_bufs

    def _step_stats(self, info):
        """:149-200 for this step: the envs running at this step (the mask
        before its advance) into row k of the round record, the counters
        accumulated."""
        step, rec, ctr = self._stats_buffers()
        self.env.tremor_metrics(info, stepped=self.active, counters=ctr, out=step)
        rec.index_copy_(0, self.k_dev, step.unsqueeze(0))

    @torch.no_grad()
    def compute_round_stats(self):
        """The training script's per-round outputs (:213-317) from the round's
        device record, over all N envs (the script's 8): per env the mean and
        median of the non-zero torque suppressions within its first
        max_length rows (:233-247), then the global line (:292-317).  One host
        sync.  Returns a dict of floats."""
        step, rec, ctr = self._stats_buffers()
        dev = self.device
        Ls = torch.as_tensor(self.env.lengths_host, device=dev)
        T = self.round_len
        inlen = torch.arange(T, device=dev)[:, None] < Ls[None, :]            # tred[:max_lengths[i], i]
        tred = rec[..., 0:7].double()
        ared = rec[..., 7:14].double()
        tot = rec[..., 14].double()
        v = torch.where(inlen[..., None] & (tred != 0), tred, torch.nan)      # [T, N, 7]
        v = v.permute(1, 0, 2).reshape(self.n, -1)
        cnt = (~v.isnan()).sum(1)
        sup_avg = v.nansum(1) / cnt                                           # NaN for an env with none
        srt = torch.sort(torch.where(v.isnan(), torch.inf, v), dim=1).values
        lo = ((cnt - 1).clamp(min=0) // 2)[:, None]
        hi = (cnt // 2).clamp(max=v.shape[1] - 1)[:, None]
        sup_med = torch.where(cnt > 0, (srt.gather(1, lo)[:, 0] + srt.gather(1, hi)[:, 0]) / 2, torch.nan)
        ep_len = torch.as_tensor(self.ep_len, device=dev, dtype=torch.float64)
        gotten = self.score - 2.0                                             # score - initial_score (:215)
        pct = gotten / ep_len * 100
        self._pct_hist = (self._pct_hist + [pct])[-100:]
        avg_r = torch.stack(self._pct_hist).mean(0)                           # mean of agent_rew[-100:] (:219)
        nz_a, nz_t = ared[ared != 0], tot[tot != 0]
        c = ctr.double().sum(0)
        vals = torch.stack([
            gotten.mean(), pct.mean(), avg_r.mean(), _np_median(avg_r),
            c[1] / (c[0] + c[1]) * 100, c[2] / float(Ls.sum()) * 100,
            sup_avg.nanmean(), sup_med.nanmean(),
            nz_a.mean() if nz_a.numel() else torch.zeros((), dtype=torch.float64, device=dev),
            c[4] / (c[3] + c[4]) * 100,
            nz_t.mean() if nz_t.numel() else torch.zeros((), dtype=torch.float64, device=dev)]).cpu().tolist()
        keys = ("avg_reward", "reward_pct", "avg_rewards_pct", "median_rewards_pct", "tremor_reduction_occurrence",
                "any_axis_reduction_pct", "overall_suppression_avg", "overall_suppression_median",
                "angle_suppression", "amplitude_reduction_occurrence", "total_amplitude_suppression")
        out = dict(zip(keys, vals))
        out["suppression_avg_per_env"] = sup_avg.cpu().numpy()
        out["suppression_median_per_env"] = sup_med.cpu().numpy()
        return out

    def _rollout_ref(self, random, injected=False, overlap=False):
        ag = self.agent
        obs = self.obs
        if injected:
            act = self._rand_act
        elif random:
            act = self._rand_acts[self._cur].uniform_(-1.0, 1.0)
        else:
            act = ag.select_action_batch(obs, dec_count=self.active_count)
        cur = torch.cuda.current_stream(self.device) if overlap else None
        if self._ins_pending:  # the previous step's insert reads the buffer this step overwrites
            cur.wait_stream(self._ins_stream)
            self._ins_pending = False
        nobs, rew, done, info = self.env.step(act, active=self.active, out=self._outs[self._cur])
        if self.stats:
            self._step_stats(info)
        if not self.fused_score:
            self.score.add_(rew.where(self.active, 0.0))  # :144 (float32 into the float64 score, 2 launches)
        add = ag.replay_buffer.add_batch_ref if self.ref_replay else ag.replay_buffer.add_batch
        rb = ag.replay_buffer
        if self._use_plan():  # the round's planned slots; score, next mask and count in the same launch
            rb.ref_step(self._plan, self._table_ext, self._kk, self._cur, obs, act, nobs, rew, done, self.strata,
                        self.active, k_dev=self.k_dev, count=self.active_count, counts_table=self._counts_tab,
                        score=self.score)
            self.last_actions = act
            return
        if (self.insert_advance and self.fused_score and self.ref_replay and not overlap and rb.ref_insert_fused
                and self.active.dtype == torch.bool):
            # the insert's last workgroup out advances the mask and adds the
            # scores (:144), one launch for both (lap_store_batch_ref_fused_adv)
            rb.add_batch_ref(obs, act, nobs, rew, done, self.strata, self.active,
                             advance=(self._table_ext, self.k_dev, self.active_count, self.score))
            self.last_actions = act
            return
        if overlap:
            mask = self._act_prev[self._cur]
            mask.copy_(self.active)
            if self._ins_stream is None:
                self._ins_stream = torch.cuda.Stream(device=self.device)
            self._ins_stream.wait_stream(cur)
            with torch.cuda.stream(self._ins_stream):
                add(obs, act, nobs, rew, done, self.strata, mask)  # :142
            self._ins_pending = True
        else:
            add(obs, act, nobs, rew, done, self.strata, self.active)  # :142
        if self.fused_score:  # :144 in the mask advance (the insert above read the mask first)
            self._advance(rew, self.score)
        else:
            self._advance()
        self.last_actions = act

    def _roll_round(self, random):
        """The whole rollout of a round (round_len steps) as one graph replay,
        captured on first use per (random, starting observation parity)."""
        key = ("round", bool(random), self._cur, self.stats)
        g = self._round_graphs.get(key)
        if g is None:
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            g = new_graph()
            cur0 = self._cur
            with torch.cuda.stream(s):
                with capture(g, stream=s), ForkJoinAudit(s):
                    for _ in range(self.round_len):
                        self._rollout_ref(random, overlap=self.round_overlap)
                        self._cur ^= 1
                    if self._ins_pending:
                        s.wait_stream(self._ins_stream)
                        self._ins_pending = False
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._cur = cur0
            self._round_graphs[key] = g
        g.replay()
        self._roll_iters += self.round_len
        self.k += self.round_len
        self._cur ^= self.round_len & 1

    def _roll_step(self, random):
        if self.action_source is not None:
            a = np.asarray(self.action_source(self, random), dtype=np.float32).reshape(self.n, -1)
            self._rand_act.copy_(torch.as_tensor(a, device=self.device))
            self._rollout_ref(random, injected=True)
        elif not self.use_graphs or self._roll_iters < self.warmup_eager:
            self._rollout_ref(random)
        else:
            key = ("roll", bool(random), self._cur, self.stats)
            g = self.graphs.get(key)
            if g is None:
                s = torch.cuda.Stream(device=self.device)
                s.wait_stream(torch.cuda.current_stream(self.device))
                g = new_graph()
                with torch.cuda.stream(s):
                    with capture(g, stream=s), ForkJoinAudit(s):
                        self._rollout_ref(random)
                torch.cuda.current_stream(self.device).wait_stream(s)
                self.graphs[key] = g
            g.replay()
        self._roll_iters += 1
        self.k += 1
        self._cur ^= 1

    # ----------------------------------------------------------- training
    def _burst_flags(self, burst):
        """The step's burst-prefetch flags (read the batch the previous step
        sampled / sample the next one) and batch slot."""
        self._train_pin = self.burst_prefetch and self._burst_i > 0
        self._train_pout = self.burst_prefetch and self._burst_i + 1 < burst
        if self._train_pin:
            self._bslot ^= 1

    # r05: overlapped pairs inside the update bursts too -- an actor step and
    # the critic-only step after it as one graph, the second's passes beside
    # the first's actor passes (VecTrainer.overlap_pairs; with burst prefetch
    # only: the second step's batch is then sampled by the first into the
    # other slot, and the slot it samples into itself is the first's, written
    # after its critic step, which waits for the first's actor branch)
    _tpair_second = False

    def train_step(self):
        """One Agent.train() (TD7_multi_agent.py:211-293 with the LAP sample and
        priority update, TD7_buffer_multi_agent.py:65-117) as a graph replay."""
        ag, L = self.agent, self.agent.learner
        L.training_steps += 1
        if self._tpair_second:  # its GPU work ran with the previous step's pair graph
            self._tpair_second = False
            self._burst_i += 1
            self._refresh_targets()
            self._train_iters += 1
            return
        update_actor = L.training_steps % ag.hp.policy_freq == 0
        L.prefetch_actor = update_actor
        self._pre_in = self._pre_out = False
        L.drop_prefetch()
        # the burst's position (maybe_train_and_checkpoint runs
        # timesteps_since_update steps back to back, run_round zeroes _burst_i)
        burst = int(ag.timesteps_since_update)
        bslot0 = self._bslot
        self._burst_flags(burst)
        # both policy-update parities run eagerly once before their capture
        if not self.use_graphs or self._train_iters < max(2, self.warmup_eager):
            self._eager(update_actor, rollout=False)
        elif self._key(update_actor, False) not in self.graphs:
            self._capture(update_actor, rollout=False)
        elif self._train_pair_ok(update_actor, burst):
            key_a = self._key(True, False)
            self._bslot = bslot0
            self._run_train_pair(key_a, burst)
            self._tpair_second = True
        else:
            self._replay(update_actor, rollout=False)
        L.prefetch_actor = False
        self._burst_i += 1
        self._train_pin = self._train_pout = False
        self._refresh_targets()
        self._train_iters += 1

    def _train_pair_ok(self, update_actor, burst):
        L = self.agent.learner
        if not (self.overlap_pairs and update_actor and self.burst_prefetch and self._train_pout
                and self._burst_i + 2 <= burst and L.fused_train and L.hp.policy_freq == 2
                and L.training_steps % L.hp.target_update_rate != 0 and (not self.dp or self.dp_inline)):
            return False
        # the second step's own graph exists (its warm-up allocated what the pair reads)
        pin2, pout2 = True, self._burst_i + 2 < burst
        return ("train", False, pin2, pout2, 1 - self._bslot) in self.graphs

    def _run_train_pair(self, key_a, burst):
        """Steps _burst_i (actor) and _burst_i + 1 (critic only) of the burst as
        one graph; the flags and slot of each set as train_step sets them."""
        L = self.agent.learner
        i0, b0 = self._burst_i, self._bslot

        def half(i):  # the host state train_step sets for step i0 + i
            self._bslot = b0
            self._burst_i = i0
            self._burst_flags(burst)
            if i == 1:
                self._burst_i = i0 + 1
                self._burst_flags(burst)

        key = ("tpair",) + key_a + (i0 + 2 < burst,)
        g = self.graphs.get(key)
        if g is None:
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            g = new_graph()
            keep = []
            if getattr(self, "_astream", None) is None:
                self._astream = torch.cuda.Stream(device=self.device)
            try:
                with torch.cuda.stream(s):
                    with capture(g, stream=s), ForkJoinAudit(s):
                        for i, u in enumerate((True, False)):
                            half(i)
                            L.prefetch_actor = u
                            self._actor_stream = self._astream if i == 0 else None
                            if i == 1:
                                L.before_critic_step = lambda st=self._astream: (
                                    torch.cuda.current_stream(self.device).wait_stream(st))
                            if self.dp_inline:
                                self._inline(u, False)
                            else:
                                self._pre(False)
                                self._mid(u, rollout=False)
                                self._post(u)
                                self._join_prio()
                            if i == 0:
                                keep.append(L._fixed_zs)  # read by the actor branch
                        s.wait_stream(self._astream)
            finally:
                self._actor_stream = None
                L.before_critic_step = None
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.graphs[key] = g
            self._pair_keep = getattr(self, "_pair_keep", []) + keep
        g.replay()
        half(1)  # the host state after both steps: the second's slot
        self._burst_i = i0

    # -------------------------------------------------------------- round
    def save_round(self):
        """:290 -- agent.save(prefix) after the round (rank 0 only when data
        parallel).  Agent.save copies every tensor to the host, which orders it
        after the round's burst on the device."""
        import time
        if self.agent.sync.rank != 0:
            return
        t = time.perf_counter()
        self.agent.save(self.save_prefix)
        self.save_seconds += time.perf_counter() - t
        self.saves += 1

    def run_round(self):
        """One episode round (:111-211); returns (active env-steps of this
        rank, training steps of the burst)."""
        ag, L = self.agent, self.agent.learner
        if self.reset_source is not None:
            self.reset_source(self.rounds, self.obs)
        else:
            self.env.reset(obs_out=self.obs)
        self.score.fill_(2.0)  # reset() returns (obs, counts = 2) into score[i] (:112)
        self._round_start()
        if self.stats:
            self._stats_buffers()[2].zero_()  # the round's counters (:117-121)
        plan = self._use_plan()
        if plan:
            self._kk.zero_()
            ag.replay_buffer.ref_plan(self._table_ext, self.strata, self._offs, self._plan_total, self._plan)
        random = not self.allow_train
        if (self.round_graph and self.use_graphs and self.action_source is None
                and self._roll_iters >= max(self.warmup_eager, 1) and self._seen_eager(random)):
            self._roll_round(random)
        else:
            for _ in range(self.round_len):
                self._roll_step(random)
                self._eager_kinds.add((bool(random), self.stats))
        if plan:
            ag.replay_buffer.ref_commit(self._plan, self.strata, self._plan_total)
        self.resets += 1
        # :208 -- the host sees one value per round: the mean episode return
        ep_return = float(np.mean(self.score.cpu().numpy()))
        ep_timesteps = round(np.mean(self.ep_len))
        before, refreshed = L.training_steps, ag.checkpoint_refreshes
        self._burst_i = 0
        ag.maybe_train_and_checkpoint(ep_timesteps, ep_return, train=self.train_step)
        burst = L.training_steps - before
        self.updates += burst
        self.steps_count += self.round_env_steps * self.world
        if self.steps_count > self.warmup:  # :210-211
            self.allow_train = True
        if self.stats:
            self.round_stats.append(self.compute_round_stats())
        if self.save_prefix is not None:
            self.save_round()
        self.rounds += 1
        self.trace.append(dict(round=self.rounds, random_actions=random, ep_return=ep_return,
                               ep_timesteps=ep_timesteps, training_steps=L.training_steps,
                               eps_since_update=ag.eps_since_update, best_min_return=ag.best_min_return,
                               min_return=ag.min_return, max_eps_before_update=ag.max_eps_before_update,
                               checkpoint_refreshed=ag.checkpoint_refreshes > refreshed,
                               steps_count=self.steps_count))
        return self.round_env_steps, burst
