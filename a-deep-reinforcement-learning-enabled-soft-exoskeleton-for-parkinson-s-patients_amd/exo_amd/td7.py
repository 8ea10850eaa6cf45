"""TD7 (SALE encoder, twin critic, actor, LAP) on PyTorch-ROCm.

Mirrors Agent/TD7_multi_agent.py (nets, losses, schedules, checkpoint policy,
save/load suffixes) with three MI355X-first changes:

* no host synchronisation inside train(): the running Q-target bounds
  (:245-246) and max_priority live in device tensors, the target policy noise
  scale is a device scalar, and LAP sampling/priority updates are HIP sum-tree
  kernels (exo_amd.replay.LAP, csrc/lap.hip);
* optional bf16 / fp16 MFMA operands in the dense layers (BASELINE.json
  configs[1] "TD7 bf16", configs[4] "fp16 MFMA"); activations, losses,
  optimiser state and master weights stay fp32;
* data-parallel training: gradients of encoder/critic/actor are flattened into
  one bucket per update and all-reduced over RCCL; the scalar bounds are
  MAX-reduced.

The update math lives in TD7Learner, which is device-agnostic torch code (the
CPU parity tests run it against the reference's golden train() steps); Agent
adds the replay buffer, the checkpoint policy and data parallelism.
"""
import copy
import ctypes
import os
import sys
import warnings
from dataclasses import dataclass, field
from typing import Callable

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from . import _native as nat
from . import ops
from .graphs import capture, new_graph
from .ops import avg_l1_norm

# fused schedule variant (r03, off): the critic target chain on the update's
# own stream and the fixed embeddings on a branch, so the critic's join waits
# on a branch that finished early -- measured 307 vs 304 us per iteration
# (profiles/r03_sched_raw/ab.txt); EXO_TD7_TARGET_ON_MAIN=1 turns it on
TARGET_ON_MAIN = os.environ.get("EXO_TD7_TARGET_ON_MAIN", "0") == "1"
# r05: the fused critic pass as two launches, the forward (Q, which needs only
# the batch and the fixed embeddings) on the fixed embeddings' stream beside
# the target chain, the loss and backward once the target heads are in
# (td7f_critic_phase, bit-identical to one launch).  Measured slower, so off:
# 0.318-0.319 vs 0.296-0.303 ms per bf16 iteration, 0.510-0.513 vs 0.487-0.491
# fp32 (profiles/r05m_raw) -- its 128 workgroups take CUs from the target chain
# it runs beside.  EXO_CRITIC_SPLIT=1 turns it on.
CRITIC_SPLIT = os.environ.get("EXO_CRITIC_SPLIT", "0") == "1"
# r05: when the encoder update's branch starts.  The iteration's first ~90 us
# are CU-throughput bound (select_action 256 workgroups x ~40 us, fixed, the
# target chain's first pass and the encoder pass 64 x ~50 / ~48 / ~108 us:
# ~23 k CU-us on 256 CUs, and target_a -- the critical chain -- ends when that
# work drains, wherever it starts); the encoder pass has the most slack (only
# its own step at the iteration's end reads it).  EXO_ENC_AFTER: "fixed" (the
# default) forks it after the fixed embeddings' pass: 0.2946-0.3003 vs
# 0.2976-0.3083 ms per iteration over 3 same-box A/B runs (profiles/r05_sched,
# target_a 78 -> 55 us in the loop's trace); "target" after the target chain
# (0.3064-0.3066: no gain); "0" at the iteration start (r04 layout).
ENC_AFTER = os.environ.get("EXO_ENC_AFTER", "fixed")
if ENC_AFTER == "0":
    ENC_AFTER = ""
# fused optimiser step + weight repack (td7f_adam_pack); EXO_ADAM_PACK=0: two launches
ADAM_PACK = os.environ.get("EXO_ADAM_PACK", "1") != "0"
# graph-replayed trainer on one GPU, fused: the encoder's weight gradients and
# step on the encoder's graph branch (TD7Learner.defer_side_join);
# EXO_ENC_STEP_BRANCH=0 joins the branch before the gradients
ENC_STEP_BRANCH = os.environ.get("EXO_ENC_STEP_BRANCH", "1") != "0"
# ...and every optimiser step (encoder, critic, actor) inside its weight-gradient
# launch (td7f_wgrad_adam); EXO_WGRAD_ADAM=0: separate td7f_adam_pack launches
WGRAD_ADAM = os.environ.get("EXO_WGRAD_ADAM", "1") != "0"


@dataclass
class Hyperparameters:
    # Generic (Agent/TD7_multi_agent.py:10-50)
    batch_size: int = 128
    buffer_size: int = 2.5e5
    discount: float = 0.99
    target_update_rate: int = 250
    exploration_noise: float = 0.1
    # TD3
    target_policy_noise: float = 0.2
    noise_clip: float = 0.5
    policy_freq: int = 2
    # LAP
    alpha: float = 0.4
    min_priority: float = 1
    # TD3+BC
    lmbda: float = 0.1
    # Checkpointing
    max_eps_when_checkpointing: int = 20
    steps_before_checkpointing: int = 75e4
    reset_weight: float = 0.9
    # Encoder Model
    zs_dim: int = 300
    enc_hdim: int = 300
    enc_activ: Callable = field(default=F.elu)
    encoder_lr: float = 3e-4
    # Critic Model
    critic_hdim: int = 320
    critic_activ: Callable = field(default=F.elu)
    critic_lr: float = 3e-4
    # Actor Model
    actor_hdim: int = 320
    actor_activ: Callable = field(default=F.relu)
    actor_lr: float = 3e-4
    # Pink noise (Agent/TD7_multi_agent_Pink_noise.py:21-24)
    beta: float = 1
    noise_scale: float = 0.3


def AvgL1Norm(x, eps=1e-8):
    """Agent/TD7_multi_agent.py:53-54 (one fused HIP kernel each way on the GPU)."""
    return avg_l1_norm(x, eps)


def LAP_huber(x, min_priority=1):
    return torch.where(x < min_priority, 0.5 * x.pow(2), min_priority * x).sum(1).mean()


class Actor(nn.Module):
    """Agent/TD7_multi_agent.py:61-77 (same parameter names: state_dicts interchange)."""

    def __init__(self, state_dim, action_dim, zs_dim=286, hdim=286, activ=F.relu):
        super().__init__()
        self.activ = activ
        self.l0 = nn.Linear(state_dim, hdim)
        self.l1 = nn.Linear(zs_dim + hdim, hdim)
        self.l2 = nn.Linear(hdim, hdim)
        self.l3 = nn.Linear(hdim, action_dim)

    def forward(self, state, zs):
        act = ops.act_code(self.activ)
        if act is None:  # an activation the fused kernels do not know: plain torch
            a = AvgL1Norm(self.l0(state))
            a = torch.cat([a, zs], 1)
            a = self.activ(self.l1(a))
            a = self.activ(self.l2(a))
            return torch.tanh(self.l3(a))
        # inference at the wide configuration's sizes: l0's norm, l1's and
        # l2's outputs handed on as the 16-bit values l1 / l2 / l3 round them
        # to (ops.dense_norm / dense half_out; zs too when the caller asked
        # Encoder.zs for it)
        a = ops.dense_norm([state], self.l0.weight, self.l0.bias, half_out=True)
        a = ops.dense_cat([a, zs], self.l1.weight, self.l1.bias, act, half_out=True)
        a = ops.dense(a, self.l2.weight, self.l2.bias, act, half_out=True)
        return ops.dense(a, self.l3.weight, self.l3.bias, ops.ACT_CODES["tanh"])


class Encoder(nn.Module):
    """Agent/TD7_multi_agent.py:80-106"""

    def __init__(self, state_dim, action_dim, zs_dim=286, hdim=286, activ=F.elu):
        super().__init__()
        self.activ = activ
        self.zs1 = nn.Linear(state_dim, hdim)
        self.zs2 = nn.Linear(hdim, hdim)
        self.zs3 = nn.Linear(hdim, zs_dim)
        self.zsa1 = nn.Linear(zs_dim + action_dim, hdim)
        self.zsa2 = nn.Linear(hdim, hdim)
        self.zsa3 = nn.Linear(hdim, zs_dim)

    def zs(self, state, half_out=False):
        """half_out: at the large-layer inference sizes zs may come back as
        16-bit values (for Actor.forward's [a | zs], select_action)."""
        act = ops.act_code(self.activ)
        if act is None:
            zs = self.activ(self.zs1(state))
            zs = self.activ(self.zs2(zs))
            return AvgL1Norm(self.zs3(zs))
        zs = ops.dense(state, self.zs1.weight, self.zs1.bias, act, half_out=True)  # see Actor.forward
        zs = ops.dense(zs, self.zs2.weight, self.zs2.bias, act, half_out=True)
        return ops.dense_norm([zs], self.zs3.weight, self.zs3.bias, half_out=half_out)

    def zsa(self, zs, action):
        act = ops.act_code(self.activ)
        if act is None:
            zsa = self.activ(self.zsa1(torch.cat([zs, action], 1)))
            zsa = self.activ(self.zsa2(zsa))
            return self.zsa3(zsa)
        zsa = ops.dense_cat([zs, action], self.zsa1.weight, self.zsa1.bias, act)
        zsa = ops.dense(zsa, self.zsa2.weight, self.zsa2.bias, act)
        return ops.dense(zsa, self.zsa3.weight, self.zsa3.bias)


class Critic(nn.Module):
    """Agent/TD7_multi_agent.py:109-140.  The two Q heads share their input, so
    their parameters are stored stacked ([2, out, in]) and each layer of both
    heads runs as ONE batched GEMM.  state_dict()/load_state_dict() use the
    reference's per-head names (q01, q1, q2, q3 / q02, q4, q5, q6), so
    checkpoints interchange with the reference; seeded initialisation draws
    in the reference's layer order."""

    HEADS = (("q01", "q02"), ("q1", "q4"), ("q2", "q5"), ("q3", "q6"))

    def __init__(self, state_dim, action_dim, zs_dim=286, hdim=286, activ=F.elu):
        super().__init__()
        self.activ = activ
        self.hdim, self.zs_dim = hdim, zs_dim
        dims = [(state_dim + action_dim, hdim), (2 * zs_dim + hdim, hdim), (hdim, hdim), (hdim, 1)]
        heads = [[nn.Linear(i, o) for i, o in dims] for _ in range(2)]  # reference creation order
        for k, (i, o) in enumerate(dims):
            self.register_parameter(f"w{k}", nn.Parameter(torch.stack([heads[0][k].weight.data,
                                                                       heads[1][k].weight.data])))
            self.register_parameter(f"b{k}", nn.Parameter(torch.stack([heads[0][k].bias.data,
                                                                       heads[1][k].bias.data])))
        self._register_state_dict_hook(Critic._to_reference_keys)
        self._register_load_state_dict_pre_hook(Critic._from_reference_keys)

    @staticmethod
    def _to_reference_keys(module, sd, prefix, local_metadata):
        for k, names in enumerate(Critic.HEADS):
            w, b = sd.pop(prefix + f"w{k}"), sd.pop(prefix + f"b{k}")
            for h, name in enumerate(names):
                sd[prefix + name + ".weight"] = w[h].clone()
                sd[prefix + name + ".bias"] = b[h].clone()
        return sd

    @staticmethod
    def _from_reference_keys(sd, prefix, local_metadata, strict, missing, unexpected, errors):
        for k, names in enumerate(Critic.HEADS):
            if prefix + names[0] + ".weight" in sd:
                sd[prefix + f"w{k}"] = torch.stack([sd.pop(prefix + n + ".weight") for n in names])
                sd[prefix + f"b{k}"] = torch.stack([sd.pop(prefix + n + ".bias") for n in names])

    @staticmethod
    def optimizer_layout():
        """Where each stacked parameter (w0, b0, ..., w3, b3) sits in the
        reference Critic's parameter order (q01.weight, q01.bias, q1.weight, ...,
        q3.bias, q02.weight, ..., q6.bias; :109-121): for parameter j, head h is
        reference parameter h * 8 + j."""
        return [[(h * 8 + j, h) for h in range(2)] for j in range(8)]

    def forward(self, state, action, zsa, zs):
        act = ops.act_code(self.activ)
        if act is not None and state.is_cuda:
            # both heads per layer as one grouped td7_dense launch: [2, B, *]
            # the concatenations [state, action] and [q, zsa, zs] are read in
            # place by the kernels (zsa, zs shared by the two heads)
            q = ops.dense_norm([state, action], self.w0, self.b0)  # -> [2, B, h]
            x = ops.dense_cat([q, zsa, zs], self.w1, self.b1, act)
            x = ops.dense(x, self.w2, self.b2, act)
            return ops.dense(x, self.w3, self.b3).squeeze(2).t()             # [B, 2]
        B, h = state.shape[0], self.hdim
        sa = torch.cat([state, action], 1)
        embeddings = torch.cat([zsa, zs], 1)
        # layer 0 of both heads as one GEMM: [B, in0] x [2h, in0]^T -> [B, 2, h]
        q = F.linear(sa, self.w0.view(2 * h, -1), self.b0.view(2 * h)).view(B, 2, h)
        q = AvgL1Norm(q)
        x = torch.cat([q.transpose(0, 1), embeddings.unsqueeze(0).expand(2, B, embeddings.shape[1])], 2)
        x = self.activ(torch.baddbmm(self.b1.unsqueeze(1), x, self.w1.transpose(1, 2)))
        x = self.activ(torch.baddbmm(self.b2.unsqueeze(1), x, self.w2.transpose(1, 2)))
        x = torch.baddbmm(self.b3.unsqueeze(1), x, self.w3.transpose(1, 2))  # [2, B, 1]
        return x.squeeze(2).t()


def flatten_params(module):
    """Re-seat every parameter of `module` as a view of one contiguous fp32
    buffer (parameter order) and return the buffer."""
    params = list(module.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in params])
    off = 0
    for p in params:
        n = p.numel()
        p.data = flat[off:off + n].view_as(p)
        off += n
    return flat


class FlatAdam(torch.optim.Adam):
    """torch.optim.Adam (same hyper-parameters, same state_dict layout:
    per-parameter step / exp_avg / exp_avg_sq) whose parameters, moments and
    step count live in flat device buffers; step() is one gradient concat and
    one td7_adam_step launch (csrc/td7_ops.hip) instead of PyTorch's
    multi-tensor kernels.  step(flat_grad=g) takes an already flat (e.g.
    all-reduced) gradient, scaled by grad_scale inside the kernel."""

    def __init__(self, module, lr, weight_decay=0.0, betas=(0.9, 0.999), eps=1e-8, layout=None):
        self.flat = flatten_params(module)
        params = list(module.parameters())
        # layout (Critic.optimizer_layout): the reference module's parameters
        # are slices of ours; state_dict() writes, load_state_dict() reads the
        # reference's per-parameter layout so optimizer checkpoints interchange
        self.layout = layout
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self._step = torch.zeros((), dtype=torch.float32, device=self.flat.device)
        self._ticket = torch.zeros((1,), dtype=torch.int32, device=self.flat.device)
        self._bind_state()

    def _params(self):
        return self.param_groups[0]["params"]

    def _bind_state(self):
        off = 0
        for p in self._params():
            n = p.numel()
            self.state[p] = {"step": self._step, "exp_avg": self.m[off:off + n].view_as(p),
                             "exp_avg_sq": self.v[off:off + n].view_as(p)}
            off += n

    def state_dict(self):
        sd = super().state_dict()
        if self.layout is None:
            return sd
        n_ref = sum(len(parts) for parts in self.layout)
        state = {}
        for j, parts in enumerate(self.layout):
            st = sd["state"].get(j)
            if st is None:
                continue
            for ref, sl in parts:
                state[ref] = {"step": st["step"].clone() if torch.is_tensor(st["step"]) else st["step"],
                              "exp_avg": st["exp_avg"][sl].clone(), "exp_avg_sq": st["exp_avg_sq"][sl].clone()}
        groups = [dict(g, params=list(range(n_ref))) for g in sd["param_groups"]]
        return {"state": state, "param_groups": groups}

    def _from_reference_layout(self, sd):
        n_ref = sum(len(parts) for parts in self.layout)
        if len(sd["param_groups"][0]["params"]) != n_ref:
            return sd  # already in this module's own layout
        state = {}
        for j, parts in enumerate(self.layout):
            refs = [sd["state"].get(ref) for ref, _ in parts]
            if any(r is None for r in refs):
                continue
            state[j] = {"step": refs[0]["step"], "exp_avg": torch.stack([r["exp_avg"] for r in refs]),
                        "exp_avg_sq": torch.stack([r["exp_avg_sq"] for r in refs])}
        groups = [dict(g, params=list(range(len(self.layout)))) for g in sd["param_groups"]]
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, state_dict):
        if self.layout is not None:
            state_dict = self._from_reference_layout(state_dict)
        super().load_state_dict(state_dict)
        off, step = 0, None
        with torch.no_grad():
            for p in self._params():
                n = p.numel()
                st = self.state.get(p, {})
                if "exp_avg" in st:
                    self.m[off:off + n].copy_(st["exp_avg"].reshape(-1))
                    self.v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
                    step = st["step"]
                off += n
            self._step.fill_(float(step) if step is not None else 0.0)
        self._bind_state()

    @torch.no_grad()
    def step(self, closure=None, flat_grad=None, grad_scale=1.0):
        g = flat_grad if flat_grad is not None else torch.cat([p.grad.reshape(-1) for p in self._params()])
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        nat.check(nat.lib().td7_adam_step(nat.ptr(self.flat), nat.ptr(g), nat.ptr(self.m), nat.ptr(self.v),
                                          nat.ptr(self._step), nat.ptr(self._ticket), self.flat.numel(),
                                          float(grp["lr"]), float(b1), float(b2), float(grp["eps"]),
                                          float(grp["weight_decay"]), float(grad_scale),
                                          nat.stream_ptr(self.flat.device)), "td7_adam_step")


    MAX_OPT, MAX_SEG = 3, 40  # include/exo_amd.h TD7_ADAM_MAX_*

    @staticmethod
    @torch.no_grad()
    def step_many(opts):
        """The steps of several FlatAdams (GPU, grad_scale 1) as ONE
        td7_adam_step_multi launch reading each parameter's gradient where
        autograd left it -- no concatenation into a flat gradient buffer.
        Parameters without a gradient are skipped (torch.optim.Adam)."""
        segs = FlatAdam.segments(opts)
        if not segs:
            return
        if len(opts) > FlatAdam.MAX_OPT or len(segs) > FlatAdam.MAX_SEG:
            for o in opts:
                o.step()
            return
        nat.check(nat.lib().td7_adam_step_multi(*FlatAdam.multi_args(opts, segs)), "td7_adam_step_multi")

    @staticmethod
    def segments(opts):
        """[(grad, flat offset, numel, optimiser index)] of every parameter with a gradient."""
        segs = []
        for k, o in enumerate(opts):
            off = 0
            for p in o._params():
                if p.grad is not None:
                    segs.append((p.grad.contiguous(), off, p.numel(), k))
                off += p.numel()
        return segs

    @staticmethod
    def multi_args(opts, segs, extra=()):
        """The arguments of td7_adam_step_multi (td7f_adam_pack: `extra` goes
        between the segments and the ticket)."""
        dev = opts[0].flat.device
        # the first optimiser's ticket: launches over disjoint optimiser sets
        # may run concurrently (graph branches), each with its own counter
        ticket = opts[0]._ticket
        n = len(opts)
        P = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
        F32 = lambda vs: (ctypes.c_float * n)(*[float(v) for v in vs])  # noqa: E731
        grps = [o.param_groups[0] for o in opts]
        ns = len(segs)
        return (n, P([o.flat for o in opts]), P([o.m for o in opts]), P([o.v for o in opts]),
                P([o._step for o in opts]), F32([g["lr"] for g in grps]), F32([g["betas"][0] for g in grps]),
                F32([g["betas"][1] for g in grps]), F32([g["eps"] for g in grps]),
                F32([g["weight_decay"] for g in grps]), ns,
                (ctypes.c_void_p * ns)(*[sg[0].data_ptr() for sg in segs]),
                (ctypes.c_int64 * ns)(*[sg[1] for sg in segs]), (ctypes.c_int32 * ns)(*[sg[2] for sg in segs]),
                (ctypes.c_int32 * ns)(*[sg[3] for sg in segs])) + tuple(extra) + (nat.ptr(ticket),
                                                                                   nat.stream_ptr(dev))


class GradSync:
    """Data-parallel gradient exchange: one flat fp32 bucket per module set,
    one all-reduce (AVG) per optimiser step (RCCL over xGMI; gloo on CPU)."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if group is not None else 1
        self.rank = dist.get_rank(group) if group is not None else 0
        self.backend = dist.get_backend(group) if group is not None else None
        # EXO_FORCE_DIST=1 (bench.py under torchrun with one rank): the
        # data-parallel layout and its collectives at world 1, so a one-GPU box
        # runs the RCCL path the multi-GPU runs take
        self.forced = group is not None and os.environ.get("EXO_FORCE_DIST") == "1"
        self._capture_ok = None

    @property
    def active(self):
        return self.world > 1 or self.forced

    def avg_(self, flat):
        """In-place average over the ranks (RCCL: one ncclAvg all-reduce; gloo:
        SUM then 1/world).  A no-op on one process."""
        if not self.active:
            return flat
        if self.backend == "nccl":
            dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
            flat.mul_(1.0 / self.world)
        return flat

    def graph_capturable(self, device):
        """Whether the collectives can run INSIDE the trainers' captured HIP
        graphs (RCCL stream capture): the nccl backend, EXO_DP_CAPTURE != 0,
        and a captured AVG / MAX all-reduce pair that replays correctly on
        every rank -- checked once, the ranks' verdicts MIN-reduced so all of
        them take the same layout.  gloo collectives run on the host and
        cannot be captured."""
        if not self.active or self.backend != "nccl":
            return False
        if self._capture_ok is None:
            ok = os.environ.get("EXO_DP_CAPTURE", "1") != "0"
            if ok:
                try:
                    ok = self._capture_selftest(device)
                except Exception:  # capture refused by the runtime / RCCL: the eager layout
                    ok = False
            flag = torch.tensor([1.0 if ok else 0.0], device=device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            self._capture_ok = bool(float(flag) == 1.0)
        return self._capture_ok

    def _capture_selftest(self, device, replays=3):
        """The training graphs' collective pattern captured and replayed at
        this world size, before any training graph is captured -- so a
        cross-stream ordering the runtime or RCCL mishandles at world > 1
        shows here.  Iteration 1 (VecTrainer._inline): an AVG on a forked
        branch (the encoder bucket), an AVG on the capture stream (the critic
        bucket), a MAX on a second branch forked after it (max_priority), and
        -- the overlapped pair's order (r06) -- the actor
        bucket's AVG on a third branch beside iteration 2's encoder AVG on a
        fourth; iteration 2's critic AVG after the actor branch; every branch
        joined at the end.  Every collective goes through the process group's
        one stream, so the graph orders them as captured, the same order on
        every rank.  Bounded: if the capture or the replays have not finished
        after EXO_DP_SELFTEST_TIMEOUT seconds (default 120) the process exits
        (status 3) with a message instead of hanging the job -- EXO_DP_CAPTURE=0
        skips the self-test and runs the eager-collective layout."""
        import threading
        xe = torch.zeros(4096, device=device)
        xc = torch.zeros(1024, device=device)
        xa = torch.zeros(256, device=device)
        xe2 = torch.zeros(4096, device=device)
        xc2 = torch.zeros(1024, device=device)
        y = torch.zeros(1, device=device)
        self.avg_(xe)  # eager first: communicator set up outside the capture
        dist.all_reduce(y, op=dist.ReduceOp.MAX, group=self.group)
        torch.cuda.synchronize(device)
        limit = float(os.environ.get("EXO_DP_SELFTEST_TIMEOUT", "120"))

        def _hung():
            sys.stderr.write(f"[exo_amd] rank {self.rank}: the captured-collective self-test (GradSync."
                             f"_capture_selftest) did not finish within {limit:.0f} s at world {self.world}; "
                             "exiting. EXO_DP_CAPTURE=0 runs the eager-collective layout instead.\n")
            sys.stderr.flush()
            os._exit(3)
        timer = threading.Timer(limit, _hung)
        timer.daemon = True
        timer.start()
        try:
            cur = torch.cuda.current_stream(device)
            s = torch.cuda.Stream(device=device)
            side, prio = torch.cuda.Stream(device=device), torch.cuda.Stream(device=device)
            abr, side2 = torch.cuda.Stream(device=device), torch.cuda.Stream(device=device)
            s.wait_stream(cur)
            g = new_graph()
            captured = True
            try:
                with torch.cuda.stream(s):
                    with capture(g, stream=s):
                        try:
                            side.wait_stream(s)
                            with torch.cuda.stream(side):
                                xe.mul_(2.0)
                                self.avg_(xe)
                            xc.add_(1.0)
                            self.avg_(xc)
                            prio.wait_stream(s)
                            with torch.cuda.stream(prio):
                                dist.all_reduce(y, op=dist.ReduceOp.MAX, group=self.group)
                            abr.wait_stream(s)
                            with torch.cuda.stream(abr):  # iteration 1's actor bucket on its branch
                                xa.mul_(3.0)
                                self.avg_(xa)
                            side2.wait_stream(s)
                            with torch.cuda.stream(side2):  # beside it, iteration 2's encoder bucket
                                xe2.add_(xc[:1])
                                self.avg_(xe2)
                            s.wait_stream(abr)  # iteration 2's critic step waits for the actor branch
                            xc2.add_(xa[:1])
                            self.avg_(xc2)
                        finally:  # every branch joined, also when the capture failed: the capture ends
                            for b in (side, prio, abr, side2):
                                s.wait_stream(b)
            except Exception as e:  # noqa: BLE001 -- any refusal: the eager layout, said why
                warnings.warn(f"GradSync: the captured-collective self-test could not capture ({e!r}); "
                              "the eager-collective layout will run")
                captured = False
            cur.wait_stream(s)
            # a replay runs the collectives: only if EVERY rank captured them
            flag = torch.tensor([1.0 if captured else 0.0], device=device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            if float(flag) != 1.0:
                return False
            ok = True
            for k in range(replays):
                r = float(self.rank + 1 + k)
                for t in (xe, xc, xa, xe2, xc2):
                    t.fill_(r)
                y.fill_(float(self.rank + 2 * k))
                g.replay()
                torch.cuda.synchronize(device)
                want = (self.world + 1) / 2.0 + k  # the mean of rank + 1 + k
                # xe2 = mean(r + (r + 1) averaged) = want + want + 1; xc2 = mean(r + 3 want)
                checks = ((xe, 2 * want), (xc, want + 1), (xa, 3 * want), (xe2, 2 * want + 1), (xc2, 4 * want))
                ok = ok and all(bool((t - v).abs().max() <= 2e-5 * v) for t, v in checks)
                ok = ok and float(y) == self.world - 1 + 2 * k
            del g
            return ok
        finally:
            timer.cancel()

    def allreduce_grads(self, params):
        if not self.active:
            return
        grads = [p.grad for p in params if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        flat /= self.world
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    # Graph-friendly split of allreduce_grads: pack/unpack are captured inside
    # the HIP graphs around an eager all-reduce of the static flat bucket, so
    # the collective always sees the gradient buffers the graph wrote.
    @staticmethod
    def pack(params):
        return torch.cat([p.grad.reshape(-1) for p in params if p.grad is not None])

    def unpack(self, flat, params):
        off = 0
        for p in params:
            if p.grad is None:
                continue
            n = p.grad.numel()
            torch.mul(flat[off:off + n].view_as(p.grad), 1.0 / self.world, out=p.grad)
            off += n

    def allreduce_flat(self, flat):
        if self.active:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)

    def max_(self, t):
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def broadcast_module(self, m, src=0):
        if self.active:
            with torch.no_grad():
                for p in list(m.parameters()) + list(m.buffers()):
                    dist.broadcast(p.data, src, group=self.group)


class TD7Learner:
    """Nets, optimisers and one TD7 update (Agent/TD7_multi_agent.py:211-293)."""

    def __init__(self, state_dim, action_dim, hp=None, learning_steps=500000, offline=False, device="cpu",
                 precision="fp32", sync=None, fused_adam=None, graph_safe=False):
        self.hp = hp if hp is not None else Hyperparameters()
        hp = self.hp
        self.device = torch.device(device)
        self.precision = precision
        self.sync = sync if sync is not None else GradSync(None)
        self.actor = Actor(state_dim, action_dim, hp.zs_dim, hp.actor_hdim, hp.actor_activ).to(self.device)
        self.critic = Critic(state_dim, action_dim, hp.zs_dim, hp.critic_hdim, hp.critic_activ).to(self.device)
        self.encoder = Encoder(state_dim, action_dim, hp.zs_dim, hp.enc_hdim, hp.enc_activ).to(self.device)
        for m in (self.actor, self.critic, self.encoder):
            self.sync.broadcast_module(m)
        if fused_adam is None:
            fused_adam = self.device.type == "cuda"
        if fused_adam:
            # one flat parameter buffer per net, one td7_adam_step launch per step
            self.actor_optimizer = FlatAdam(self.actor, lr=hp.actor_lr, weight_decay=1e-7)
            self.critic_optimizer = FlatAdam(self.critic, lr=hp.critic_lr, weight_decay=1e-7,
                                             layout=Critic.optimizer_layout())
            self.encoder_optimizer = FlatAdam(self.encoder, lr=hp.encoder_lr, weight_decay=1e-7)
        else:
            kw = dict(weight_decay=1e-7)
            self.actor_optimizer = torch.optim.Adam(self.actor.parameters(), lr=hp.actor_lr, **kw)
            self.critic_optimizer = torch.optim.Adam(self.critic.parameters(), lr=hp.critic_lr, **kw)
            self.encoder_optimizer = torch.optim.Adam(self.encoder.parameters(), lr=hp.encoder_lr, **kw)
        self.actor_target = copy.deepcopy(self.actor)
        self.critic_target = copy.deepcopy(self.critic)
        self.fixed_encoder = copy.deepcopy(self.encoder)
        self.fixed_encoder_target = copy.deepcopy(self.encoder)
        self.pair_fixed_encoders()
        self.checkpoint_actor = copy.deepcopy(self.actor)
        self.checkpoint_encoder = copy.deepcopy(self.encoder)
        self.offline = offline
        self.training_steps = 0
        # True: gradients are freed and re-created by each backward (no zeroing
        # kernels); False keeps persistent buffers zeroed in place
        self.grads_to_none = True
        # device-resident scalars (:183-186, :236-237)
        f32 = dict(device=self.device, dtype=torch.float32)
        self.max = torch.tensor(-1e8, **f32)
        self.min = torch.tensor(1e8, **f32)
        self.max_target = torch.tensor(0.0, **f32)
        self.min_target = torch.tensor(0.0, **f32)
        self.target_policy_noise = torch.tensor(float(hp.target_policy_noise), **f32)
        self.policy_noise_decrease = hp.target_policy_noise / learning_steps
        self.action_noise_decrease = hp.exploration_noise / learning_steps
        self.exploration_noise_t = torch.tensor(float(hp.exploration_noise), **f32)
        # target-policy and exploration noise drawn inside their kernels on the
        # GPU (ops.DeviceRNG); EXO_DEVICE_RNG=0: torch.randn_like
        self._device_rng = os.environ.get("EXO_DEVICE_RNG", "1") != "0"
        self._noise_rng = ops.DeviceRNG(self.device, 1) if self.device.type == "cuda" else None
        self._explore_rng = ops.DeviceRNG(self.device, 2) if self.device.type == "cuda" else None
        # on the GPU: whole-network fused launches (exo_amd/fused.py,
        # csrc/td7_fused.hip) over packed weight copies in the operand type
        # (bf16 / fp16 / fp32); EXO_TD7_FUSED=0 keeps the per-layer kernels
        self.fused = None
        if os.environ.get("EXO_TD7_FUSED", "1") != "0" and self._device_rng:
            from . import fused as _fused
            if _fused.supported(self):
                try:
                    self.fused = _fused.FusedNets(self)
                except _fused.PlanError as e:  # the per-layer kernels run this shape
                    warnings.warn(f"{e}; the per-layer kernels run this network")

    ENC_LAYERS = ("zs1", "zs2", "zs3", "zsa1", "zsa2", "zsa3")

    def pair_fixed_encoders(self):
        """Store the fixed encoder's and the fixed target encoder's weights as
        one stacked [2, out, in] tensor per layer (the two modules' parameters
        become views of slices 0 / 1, so loads, target refreshes and
        checkpoints are unchanged).  Their passes in the critic update -- zs of
        the state (fixed) and of the next state (target), then zsa -- are
        independent and equal in shape, so on the GPU each layer of both runs
        as ONE grouped td7_dense launch (Agent/TD7_multi_agent.py:236-251)."""
        self._pair = {}
        with torch.no_grad():
            for name in self.ENC_LAYERS:
                fa, fb = getattr(self.fixed_encoder, name), getattr(self.fixed_encoder_target, name)
                W = torch.stack([fa.weight.data, fb.weight.data])
                B = torch.stack([fa.bias.data, fb.bias.data])
                fa.weight.data, fb.weight.data = W[0], W[1]
                fa.bias.data, fb.bias.data = B[0], B[1]
                self._pair[name] = (W, B)

    def _paired(self):
        return (self.device.type == "cuda" and getattr(self, "_pair", None) is not None
                and ops.act_code(self.fixed_encoder.activ) is not None
                and self._pair["zs1"][0].data_ptr() == self.fixed_encoder.zs1.weight.data_ptr())

    def _pair_dense(self, x, name, act):
        W, B = self._pair[name]
        return ops.dense(x, W, B, act)

    def _pair_zs(self, state, next_state):
        """[fixed_encoder.zs(state), fixed_encoder_target.zs(next_state)] as [2, B, zs_dim]."""
        act = ops.act_code(self.fixed_encoder.activ)
        x = ops.pair_rows(state, next_state)
        x = self._pair_dense(x, "zs1", act)
        x = self._pair_dense(x, "zs2", act)
        W, B = self._pair["zs3"]
        return ops.dense_norm([x], W, B)

    def _pair_zsa(self, zs2, actions2):
        act = ops.act_code(self.fixed_encoder.activ)
        W, B = self._pair["zsa1"]
        x = ops.dense_cat([zs2, actions2], W, B, act)
        x = self._pair_dense(x, "zsa2", act)
        return self._pair_dense(x, "zsa3", 0)

    @property
    def exploration_noise(self):
        return float(self.exploration_noise_t)

    def _autocast(self):
        """fp32 (default): exact f32 MFMA.  bf16 / fp16: the dense layers'
        GEMMs take MFMA operands rounded to bf16 / fp16 (fp32 storage,
        accumulation, activations, norms, losses and optimiser state)."""
        if self.precision not in ops.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(ops.PRECISIONS)}, not {self.precision!r}")
        return ops.matrix_precision(self.precision)

    # One TD7 update (:211-293) is split into phases so a data-parallel step
    # needs only two collectives and every phase can be captured in a HIP
    # graph.  Encoder and critic gradients are independent (the critic only
    # sees fixed_encoder / fixed_encoder_target, :233-251), so both are
    # computed before either optimiser steps -- the same arithmetic as the
    # reference's encoder-then-critic order.
    # The encoder's loss and gradients (:219-228) depend on nothing the critic
    # computes and the critic never reads the live encoder (only the fixed
    # encoders), so on the GPU they run on a side stream -- a parallel branch
    # of the captured iteration graph -- concurrently with the critic's
    # target / fixed-embedding passes and its loss and gradients; the branch
    # joins before the optimiser steps (and the data-parallel all-reduce).
    # The small GEMMs of each branch fill a fraction of the 256 CUs, so the
    # two overlap: 0.965 vs 1.095 ms per bench iteration
    # (profiles/r01b_raw/overlap_ab.txt; also measured there and not kept:
    # the encoder's Adam step on the branch -- no gain -- and LAP.update_priority
    # on a third branch -- slower).  EXO_TD7_OVERLAP=0 serialises.
    overlap = os.environ.get("EXO_TD7_OVERLAP", "1") == "1"
    # the actor forward of an actor-update iteration on its own branch during the
    # critic update (set per iteration by the trainer through prefetch_actor)
    actor_branch = os.environ.get("EXO_TD7_ACTOR_BRANCH", "1") == "1"
    prefetch_actor = False
    # True (one GPU, set by the graph-replayed trainer): the fused update leaves
    # the encoder's weight gradients and optimiser step on the encoder's branch
    # and the caller joins it (join_side, end of iteration); False: phase_grads
    # returns with every gradient ordered on the current stream
    defer_side_join = False
    # True (data parallel, collectives inside the iteration, set per iteration
    # by the trainer): the fused update all-reduces the encoder's gradient
    # bucket on the encoder's branch, between its weight-gradient launch and
    # its optimiser step, like the one-GPU layout keeps that step there
    dp_inline = False

    def _encoder_grads(self, state, action, next_state):
        """:219-228 -- loss and gradients of the live encoder."""
        with self._autocast():
            # zs(state) and zs(next_state) of the live encoder as one pass; the
            # next-state half is detached (it is computed under no_grad at :220)
            B = state.shape[0]
            enc = self.encoder
            act = ops.act_code(enc.activ)
            if state.is_cuda and act is not None and state.dtype == torch.float32 and not state.requires_grad:
                # one launch per layer over both halves, backward over the first only
                zs, next_zs = ops.encoder_zs_half_grad(ops.pair_rows(state, next_state).view(2 * B, -1), B, act,
                                                       [(l.weight, l.bias) for l in (enc.zs1, enc.zs2, enc.zs3)])
            else:
                zs_all = enc.zs(torch.cat([state, next_state], 0))
                zs, next_zs = zs_all[:B], zs_all[B:].detach()
            pred_zs = self.encoder.zsa(zs, action)
        self.encoder_optimizer.zero_grad(set_to_none=self.grads_to_none)
        if pred_zs.is_cuda and pred_zs.dtype == torch.float32:
            # d mse / d pred_zs from one kernel, back-propagated from pred_zs
            # (the loss value itself is not used by the update)
            torch.autograd.backward(pred_zs, ops.mse_grad(pred_zs, next_zs.detach()))
        else:
            encoder_loss = ops.mse_loss(pred_zs.float(), next_zs.float())
            encoder_loss.backward()

    @property
    def fused_train(self):
        """The update's passes run fused (FusedNets.train_ok: every gradient
        pass's plan fits; a learner whose actor pass does not -- e.g. the Pink
        agent's 300-wide actor -- keeps the fused select_action and trains on
        the per-layer kernels)."""
        return self.fused is not None and self.fused.train_ok

    def phase_grads(self, state, action, next_state, reward, not_done, noise=None):
        if self.fused_train and state.is_cuda:
            return self._phase_grads_fused(state, action, next_state, reward, not_done, noise)
        hp = self.hp
        # ---- encoder (:219-228)
        side = None
        if self.overlap and self.device.type == "cuda":
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_side", None) is None:
                self._side = torch.cuda.Stream(device=self.device)
            side = self._side
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._encoder_grads(state, action, next_state)
        else:
            self._encoder_grads(state, action, next_state)
        # ---- critic (:233-257)
        if noise is None and not (action.is_cuda and self._device_rng):
            noise = torch.randn_like(action)  # on the GPU: drawn inside the noisy-action kernel
        split = side is not None and os.environ.get("EXO_TD7_TARGET_BRANCH", "1") == "1"
        with torch.no_grad():
            with self._autocast():
                paired = self._paired()
                if paired:  # fixed (state) and fixed target (next state) encoders, one launch per layer
                    zs2 = self._pair_zs(state, next_state)
                    fixed_zs, fixed_target_zs = zs2[0], zs2[1]
                else:
                    fixed_target_zs = self.fixed_encoder_target.zs(next_state)
                    fixed_zs = self.fixed_encoder.zs(state)
        if split and self.prefetch_actor and self.actor_branch:
            # this iteration also updates the actor (:268-277): its forward and
            # the fixed encoder's zsa of its actions read no weight the critic /
            # encoder steps change, so they run now on a fourth branch, under
            # the critic's backward; only the critic pass of the actor loss
            # waits for the new critic weights (phase_actor_grads)
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_aside", None) is None:
                self._aside = torch.cuda.Stream(device=self.device)
            self._aside.wait_stream(cur)
            with torch.cuda.stream(self._aside), self._autocast():
                actor = self.actor(state, fixed_zs)
                self._actor_pre = (actor, self.fixed_encoder.zsa(fixed_zs, actor))
        if split:
            # the target chain (actor_target -> zsa -> critic_target -> Q_target,
            # :236-246) as a third branch, concurrent with the online critic's
            # forward on the current stream; they meet at the loss
            cur = torch.cuda.current_stream(self.device)
            if getattr(self, "_tside", None) is None:
                self._tside = torch.cuda.Stream(device=self.device)
            self._tside.wait_stream(cur)
            with torch.cuda.stream(self._tside):
                Q_target = self._target_chain(next_state, reward, not_done, noise, fixed_target_zs, None)
            with torch.no_grad(), self._autocast():
                fixed_zsa = self.fixed_encoder.zsa(fixed_zs, action)
            with self._autocast():
                Q = self.critic(state, action, fixed_zsa, fixed_zs)
            cur.wait_stream(self._tside)
        else:
            fixed_zsa = None
            if paired:
                Q_target, fixed_zsa = self._target_chain(next_state, reward, not_done, noise, fixed_target_zs,
                                                         (zs2, action))
            else:
                Q_target = self._target_chain(next_state, reward, not_done, noise, fixed_target_zs, None)
                with torch.no_grad(), self._autocast():
                    fixed_zsa = self.fixed_encoder.zsa(fixed_zs, action)
            with self._autocast():
                Q = self.critic(state, action, fixed_zsa, fixed_zs)
        # LAP_huber critic loss and the new priorities (:257-262): one
        # td7_critic_loss launch forward, one multiply backward
        self.critic_optimizer.zero_grad(set_to_none=self.grads_to_none)
        if Q.is_cuda and Q.dtype == torch.float32:
            # dloss/dQ from the loss kernel, back-propagated from Q directly
            critic_loss, priority, dQ = ops.critic_loss_and_grad(Q, Q_target, hp.alpha, hp.min_priority)
            torch.autograd.backward(Q, dQ)
        else:
            critic_loss, priority = ops.critic_loss(Q.float(), Q_target, hp.alpha, hp.min_priority)
            critic_loss.backward()
        if side is not None:
            self.join_side()
        if getattr(self, "_actor_pre", None) is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._aside)
        self._fixed_zs = fixed_zs
        return priority

    def _phase_grads_fused(self, state, action, next_state, reward, not_done, noise=None):
        """phase_grads as fused launches (exo_amd/fused.py, csrc/td7_fused*.hip):
        the encoder update (one launch) on a side branch, the critic target
        chain (two launches) on a second, fixed_zs / fixed_zsa (one) and -- in
        an actor-update iteration -- the actor's forward (one) on a third; the
        critic's forward, loss and backward as one launch once the target heads
        are in, then every encoder and critic weight gradient plus the LAP
        priorities as one grouped launch.  The gradients land in the
        optimisers' flat gradient buffers (the parameters' .grad are views)."""
        hp, fz = self.hp, self.fused
        B = state.shape[0]
        tr = fz.train(B)
        state, action, next_state = state.contiguous(), action.contiguous(), next_state.contiguous()
        reward, not_done = reward.contiguous(), not_done.contiguous()
        cur = torch.cuda.current_stream(self.device)
        branch = self.overlap

        def stream(name):
            st = getattr(self, name, None)
            if st is None:
                st = torch.cuda.Stream(device=self.device)
                setattr(self, name, st)
            st.wait_stream(cur)
            return st

        # one GPU: the encoder's weight gradients and optimiser step stay on
        # its branch (nothing else in the update reads them); data parallel
        # with the collectives inside the iteration: the same, with the
        # encoder bucket's all-reduce between them on the branch (the step is
        # then a td7f_adam_pack launch); eager data parallel: all-reduced with
        # the critic's
        inline = self.sync.active and self.dp_inline
        enc_step = (branch and ADAM_PACK and self.defer_side_join and (not self.sync.active or inline)
                    and isinstance(self.encoder_optimizer, FlatAdam))
        wg_adam = enc_step and WGRAD_ADAM and tr.fuses_adam() and not self.sync.active
        self._enc_step_pending = False
        self._actor_fused_pre = False
        critic_phase = 0
        pre = self.pre_in
        self.pre_in = None
        if pre is not None:
            # the fixed embeddings and the target heads of this batch were
            # computed at the end of the previous iteration (prefetch_targets)
            if not self._pre_ready[pre]:
                raise RuntimeError("phase_grads: no prefetched targets in slot %d" % pre)
            self._pre_ready[pre] = False
            zs, zsa, qt = self._pre_bufs[pre]
            if branch:
                side = stream("_side")
                with torch.cuda.stream(side):
                    tr.encoder(state, action, next_state)
                    if enc_step:
                        tr.wgrad_encoder(adam=wg_adam)
                        if inline:
                            self.sync.avg_(tr.enc_grad)
                if self.prefetch_actor and self.actor_branch:
                    aside = stream("_aside")
                    with torch.cuda.stream(aside):
                        tr.actor(0, state, zs)
                    self._actor_fused_pre = True
            else:
                tr.encoder(state, action, next_state)
        elif branch and TARGET_ON_MAIN:
            # the critic target chain (target_a -> target_b, the longest branch
            # before the critic) on the iteration's own stream, the fixed
            # embeddings beside it: the critic's join then waits on a branch
            # that finished long before (a satisfied cross-queue wait) instead
            # of putting a cross-queue hand-off on the critical path
            side, fside = stream("_side"), stream("_fside")
            with torch.cuda.stream(side):
                tr.encoder(state, action, next_state)
                if enc_step:
                    tr.wgrad_encoder(adam=wg_adam)
                    if inline:
                        self.sync.avg_(tr.enc_grad)
            with torch.cuda.stream(fside):
                zs, zsa = fz.fixed(state, action)
            if self.prefetch_actor and self.actor_branch:
                aside = stream("_aside")
                aside.wait_stream(fside)
                with torch.cuda.stream(aside):
                    tr.actor(0, state, zs)
                self._actor_fused_pre = True
            qt = fz.target_heads(next_state, noise)
            cur.wait_stream(fside)
        else:
            def encoder_branch():
                side = stream("_side")
                with torch.cuda.stream(side):
                    tr.encoder(state, action, next_state)
                    if enc_step:
                        tr.wgrad_encoder(adam=wg_adam)
                        if inline:
                            self.sync.avg_(tr.enc_grad)
                return side

            if branch:
                if not ENC_AFTER:
                    side = encoder_branch()
                tside = stream("_tside")
                with torch.cuda.stream(tside):
                    qt = fz.target_heads(next_state, noise)
                hook, self.after_target = self.after_target, None
                if hook is not None:  # the trainer's rollout branch (VecTrainer._pre, EXO_TRAIN_FIRST)
                    hook()
            else:
                tr.encoder(state, action, next_state)
                qt = fz.target_heads(next_state, noise)
            zs, zsa = fz.fixed(state, action)
            hook, self.after_fixed = self.after_fixed, None
            if hook is not None:  # the trainer's rollout branch (VecTrainer._pre, EXO_ROLLOUT_AFTER)
                hook()
            if branch and self.prefetch_actor and self.actor_branch:
                aside = stream("_aside")
                with torch.cuda.stream(aside):
                    tr.actor(0, state, zs)
                self._actor_fused_pre = True
            if branch and ENC_AFTER == "fixed":
                side = encoder_branch()  # forks from the iteration's stream after the fixed pass
            elif branch and ENC_AFTER:
                cur.wait_stream(tside)
                side = encoder_branch()  # ... after the target chain (and the fixed pass)
            if branch and CRITIC_SPLIT:
                # the critic's forward now, beside the target chain
                tr.critic(state, action, zs, zsa, qt, reward, not_done, phase=1)
                critic_phase = 2
            if branch:
                cur.wait_stream(tside)
        hook, self.before_critic = self.before_critic, None
        if hook is not None:  # the trainer's overlapped pairs (EXO_PAIR_CRITIC_AFTER_SELECT)
            hook()
        tr.critic(state, action, zs, zsa, qt, reward, not_done, phase=critic_phase)
        hook, self.after_critic = self.after_critic, None
        if hook is not None:  # the trainer's priority update, from |td| (VecTrainer._fork_update_sample)
            hook(tr.td)
        hook, self.before_critic_step = self.before_critic_step, None
        if hook is not None:  # the trainer's overlapped pairs: the previous actor passes read the critic
            hook()
        if enc_step:
            priority = tr.wgrad_critic(adam=wg_adam)
            self._enc_step_pending = True
            self._steps_in_wgrad = wg_adam
        else:
            if branch:
                cur.wait_stream(side)
            priority = tr.wgrad_encoder_critic()
        if self._actor_fused_pre:
            cur.wait_stream(self._aside)
        self._fixed_zs = zs
        return priority

    @torch.no_grad()
    def _target_chain(self, next_state, reward, not_done, noise, fixed_target_zs, pair):
        """:236-246: target action with clipped noise, the target critic's heads
        and Q_target with the running bounds.  pair = (zs2, action): the fixed
        encoder's zsa rides along in the grouped zsa launches and is returned."""
        hp = self.hp
        with self._autocast():
            # (noise * sigma).clamp(+-noise_clip); sigma -= decrease; (a + noise).clamp(-1, 1)
            next_action = ops.noisy_action(self.actor_target(next_state, fixed_target_zs).float(), noise,
                                           self.target_policy_noise, self.policy_noise_decrease,
                                           clip=hp.noise_clip, rng=self._noise_rng)
            fixed_zsa = None
            if pair is not None:
                zs2, action = pair
                zsa2 = self._pair_zsa(zs2, torch.stack([action, next_action]))
                fixed_zsa, fixed_target_zsa = zsa2[0], zsa2[1]
            else:
                fixed_target_zsa = self.fixed_encoder_target.zsa(fixed_target_zs, next_action)
            Q_heads = self.critic_target(next_state, next_action, fixed_target_zsa, fixed_target_zs).float()
        # Q_target and the running bounds (:240-246; bounds kept per rank,
        # MAX-reduced when the targets refresh): one td7_q_target launch
        Q_target = ops.q_target(Q_heads, reward, not_done, hp.discount, self.min_target, self.max_target,
                                self.max, self.min)
        return Q_target if pair is None else (Q_target, fixed_zsa)

    # Cross-iteration prefetch of the critic's inputs (r04).  The fixed
    # embeddings fixed_encoder.zs/zsa(s, a) and the target heads
    # critic_target(s', actor_target(s') + noise, ...) of a batch read only the
    # batch and nets that change at a target refresh (:284-293), so the
    # trainer computes them for the NEXT batch right after sampling it, at the
    # end of the current iteration -- beside that iteration's actor update --
    # into one of two persistent slots; the next iteration's critic pass then
    # starts at once.  The same launches on the same inputs in the same order
    # (the target-noise stream included): bit-identical.  Never across a target
    # refresh (the trainer does not prefetch before one; the refresh drops any
    # prefetched slot), and Agent.train()'s own updates drop them too.
    pre_in = None  # slot whose prefetched inputs the next phase_grads reads (set by the trainer)
    after_critic = None  # called with the critic pass's |td| right after it (set by the trainer)
    after_fixed = None  # called right after the fixed pass is captured (set by the trainer)
    after_target = None  # called right after the target chain is captured (set by the trainer)
    before_critic = None  # called before the critic pass is captured (set by the trainer)
    before_critic_step = None  # called before the critic's weight-gradient + step launch (set by the trainer)

    def _pre_slot(self, slot, B):
        bufs = getattr(self, "_pre_bufs", None)
        if bufs is None or bufs[0][0].shape[0] != B:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("prefetch_targets: run once eagerly before graph capture")
            Z = self.hp.zs_dim
            f32 = dict(dtype=torch.float32, device=self.device)
            self._pre_bufs = bufs = [(torch.empty((B, Z), **f32), torch.empty((B, Z), **f32),
                                      torch.empty((B, 2), **f32)) for _ in range(2)]
        return bufs[slot]

    _pre_ready = (False, False)

    def prefetch_ready(self, slot):
        return bool(self._pre_ready[slot])

    def drop_prefetch(self):
        self._pre_ready = [False, False]

    def prefetch_targets(self, state, action, next_state, slot):
        """fixed(s, a) and the target heads of (s') for the batch in `slot`, on
        the current stream (fixed on a branch beside the target chain)."""
        if not self.fused_train:
            raise RuntimeError("prefetch_targets: the fused TD7 path only")
        fz = self.fused
        zs, zsa, qt = self._pre_slot(slot, state.shape[0])
        # the fixed pass on a branch of its own beside the target chain, joined
        # by the trainer at the end of the iteration (join_prefetch) -- not back
        # into this stream: a fork joined inside a forked branch made
        # hipStreamEndCapture crash (r04, tools/seg_bisect.py)
        cur = torch.cuda.current_stream(self.device)
        st = getattr(self, "_pfside", None)
        if st is None:
            st = self._pfside = torch.cuda.Stream(device=self.device)
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            fz.fixed(state, action, out=(zs, zsa))
        fz.target_heads(next_state, None, out=qt)
        self._pf_open = True
        if not isinstance(self._pre_ready, list):
            self._pre_ready = [False, False]
        self._pre_ready[slot] = True

    _pf_open = False

    def join_prefetch(self):
        """Order the current stream after prefetch_targets' fixed-pass branch."""
        if self._pf_open:
            torch.cuda.current_stream(self.device).wait_stream(self._pfside)
            self._pf_open = False

    def join_side(self):
        """Order the current stream after the encoder branch (end of an update)."""
        side = getattr(self, "_side", None)
        if side is not None and self.device.type == "cuda":
            torch.cuda.current_stream(self.device).wait_stream(side)

    def phase_steps(self, flat_grad=None, grad_scale=1.0):
        """Encoder and critic optimiser steps; flat_grad: their gradients packed
        in grad_params() order (the data-parallel all-reduce bucket), consumed
        in place by FlatAdam."""
        if flat_grad is not None and isinstance(self.encoder_optimizer, FlatAdam):
            if getattr(self, "_enc_step_pending", False):
                raise RuntimeError("phase_steps: a flat gradient bucket with the encoder step on its branch")
            ne = self.encoder_optimizer.flat.numel()
            self.encoder_optimizer.step(flat_grad=flat_grad[:ne], grad_scale=grad_scale)
            self.critic_optimizer.step(flat_grad=flat_grad[ne:], grad_scale=grad_scale)
            if self.fused is not None:
                self.fused.pack("encoder", "critic")
            return
        if isinstance(self.encoder_optimizer, FlatAdam) and self.device.type == "cuda":
            if getattr(self, "_enc_step_pending", False):
                # the encoder's step on its branch (after its weight gradients),
                # the critic's on the update's chain
                self._enc_step_pending = False
                if self._steps_in_wgrad:  # already applied by the weight-gradient launches
                    return
                with torch.cuda.stream(self._side):
                    self.fused.adam_pack([self.encoder_optimizer], "encoder")
                self.fused.adam_pack([self.critic_optimizer], "critic")
                return
            if self.fused is not None and ADAM_PACK:
                self.fused.adam_pack([self.encoder_optimizer, self.critic_optimizer], "encoder", "critic")
                return
            FlatAdam.step_many([self.encoder_optimizer, self.critic_optimizer])
            if self.fused is not None:
                self.fused.pack("encoder", "critic")
            return
        self.encoder_optimizer.step()
        self.critic_optimizer.step()

    def phase_actor_grads(self, state, action):
        """:268-277 with the just-updated critic."""
        if self.fused_train and state.is_cuda and not self.offline:
            # fused: actor forward (unless prefetched on its branch), the critic
            # heads back to the action / zsa inputs, the zsa and actor backward,
            # then the actor's weight gradients (one grouped launch)
            tr = self.fused.train(state.shape[0])
            st = state.contiguous()
            if not getattr(self, "_actor_fused_pre", False):
                tr.actor(0, st, self._fixed_zs)
            self._actor_fused_pre = False
            tr.actor(1, st, self._fixed_zs)
            tr.actor(2, st, self._fixed_zs)
            # graph-replayed trainer on one GPU: the actor's optimiser step and
            # repack in the weight-gradient launch (phase_actor_step has nothing left)
            self._actor_step_done = (self.defer_side_join and WGRAD_ADAM and ADAM_PACK and not self.sync.active
                                     and isinstance(self.actor_optimizer, FlatAdam) and tr.fuses_adam())
            tr.wgrad_actor(adam=self._actor_step_done)
            self._actor_bucket = tr.actor_grad
            return
        self._actor_bucket = None
        fixed_zs = self._fixed_zs
        pre, self._actor_pre = getattr(self, "_actor_pre", None), None
        with self._autocast():
            if pre is not None:  # computed on the actor branch of phase_grads
                actor, fixed_zsa = pre
            else:
                actor = self.actor(state, fixed_zs)
                fixed_zsa = self.fixed_encoder.zsa(fixed_zs, actor)
            Q = self.critic(state, actor, fixed_zsa, fixed_zs)
        self.actor_optimizer.zero_grad(set_to_none=self.grads_to_none)
        # gradients of the actor's parameters only: the reference's backward()
        # also accumulates critic / fixed-encoder gradients that its next
        # zero_grad() discards (:275-277) -- skipping them skips their GEMMs
        params = list(self.actor.parameters())
        if Q.is_cuda and Q.dtype == torch.float32 and not self.offline:
            # d(-Q.mean())/dQ is the constant -1/Q.numel(): back-propagated from
            # Q directly (a cached tensor in Q's strides, no loss kernels)
            grads = torch.autograd.grad(Q, params, grad_outputs=self._neg_mean_grad(Q))
        else:
            actor_loss = -Q.float().mean()
            if self.offline:
                actor_loss = actor_loss + self.hp.lmbda * Q.float().abs().mean().detach() * F.mse_loss(actor.float(),
                                                                                                   action)
            grads = torch.autograd.grad(actor_loss, params)
        for p, g in zip(params, grads):
            if p.grad is None:
                p.grad = g
            else:
                p.grad.add_(g)

    def _neg_mean_grad(self, Q):
        key = (tuple(Q.shape), Q.stride(), Q.device)
        cache = getattr(self, "_nmg", None)
        if cache is None or cache[0] != key:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("actor update: run once eagerly before graph capture")
            g = torch.empty_strided(Q.shape, Q.stride(), dtype=torch.float32, device=Q.device)
            g.fill_(-1.0 / Q.numel())
            self._nmg = cache = (key, g)
        return cache[1]

    def phase_actor_step(self, flat_grad=None, grad_scale=1.0):
        if getattr(self, "_actor_step_done", False):
            self._actor_step_done = False
            if flat_grad is not None:
                raise RuntimeError("phase_actor_step: a flat gradient bucket after the fused actor step")
            return
        if flat_grad is not None and isinstance(self.actor_optimizer, FlatAdam):
            self.actor_optimizer.step(flat_grad=flat_grad, grad_scale=grad_scale)
        elif isinstance(self.actor_optimizer, FlatAdam) and self.device.type == "cuda":
            if self.fused is not None and ADAM_PACK:
                self.fused.adam_pack([self.actor_optimizer], "actor")  # select_action reads the packed actor
                return
            FlatAdam.step_many([self.actor_optimizer])
        else:
            self.actor_optimizer.step()
        if self.fused is not None:
            self.fused.pack("actor")  # select_action reads the packed actor

    # Data parallel with the collectives inside the iteration (the trainers'
    # one-graph layout): each optimiser phase's gradients are averaged in
    # place between the weight-gradient launches and the optimiser steps.
    def allreduce_phase_grads(self, B):
        """After phase_grads: the encoder + critic gradients averaged over the
        ranks.  Fused with the encoder's step on its branch: its bucket was
        reduced there, the critic's flat gradient buffer is reduced here and
        None is returned (phase_steps reads the gradients in place); otherwise
        one packed bucket of both is reduced and returned for
        phase_steps(flat_grad=...)."""
        if getattr(self, "_enc_step_pending", False):
            self.sync.avg_(self.fused.train(B).critic_grad)
            return None
        flat = GradSync.pack(self.grad_params())
        self.sync.avg_(flat)
        return flat

    def allreduce_actor_grads(self):
        """After phase_actor_grads: the actor's gradients averaged over the
        ranks (the fused flat gradient buffer in place -> None; otherwise a
        packed bucket for phase_actor_step(flat_grad=...))."""
        if getattr(self, "_actor_bucket", None) is not None:
            self.sync.avg_(self._actor_bucket)
            return None
        flat = GradSync.pack(self.grad_params(actor=True))
        self.sync.avg_(flat)
        return flat

    def grad_params(self, actor=False):
        if actor:
            return list(self.actor.parameters())
        return list(self.encoder.parameters()) + list(self.critic.parameters())

    def update(self, state, action, next_state, reward, not_done, noise=None, update_actor=None):
        """One TD7 gradient step on a sampled batch.  Returns the per-sample
        priorities |td|max.clamp(min_priority)^alpha (:262)."""
        self.training_steps += 1
        self.drop_prefetch()  # prefetched inputs belong to the trainer's next batch, not this one
        self.pre_in = None
        if update_actor is None:
            update_actor = self.training_steps % self.hp.policy_freq == 0
        # an eager update is self-contained: every branch it forks is joined
        # before it returns and an actor forward is prefetched only for an
        # update that consumes it (the graph-replayed trainers set both flags
        # per iteration and join themselves)
        self.defer_side_join = False
        self.prefetch_actor = bool(update_actor)
        priority = self.phase_grads(state, action, next_state, reward, not_done, noise)
        self.sync.allreduce_grads(self.grad_params())
        self.phase_steps()
        if update_actor:
            self.phase_actor_grads(state, action)
            self.sync.allreduce_grads(self.grad_params(actor=True))
            self.phase_actor_step()
        self.prefetch_actor = False
        self.join_side()
        return priority

    def sync_bounds(self):
        """Global running Q-target bounds = MAX over ranks of the local ones."""
        if self.sync.active:
            b = torch.stack([self.max, -self.min])
            self.sync.max_(b)
            self.max.copy_(b[0])
            self.min.copy_(-b[1])

    def maybe_update_targets(self):
        """:284-293; returns True when the targets were refreshed."""
        if self.training_steps % self.hp.target_update_rate != 0:
            return False
        self.drop_prefetch()  # computed with the nets this refresh replaces
        self.update_targets_device()
        return True

    def update_targets_device(self):
        """The refresh's device work (:284-293): the target and fixed nets
        copied, repacked, the Q bounds MAX-reduced over data-parallel ranks
        and made the new target bounds -- no host synchronisation, so a
        trainer can capture it into a graph (VecTrainer._refresh_targets)."""
        for dst, src in ((self.actor_target, self.actor), (self.critic_target, self.critic),
                         (self.fixed_encoder_target, self.fixed_encoder), (self.fixed_encoder, self.encoder)):
            with torch.no_grad():
                torch._foreach_copy_(list(dst.parameters()), list(src.parameters()))
        if self.fused is not None:
            self.fused.pack("actor_target", "critic_target", "fixed_encoder_target", "fixed_encoder")
        self.sync_bounds()
        self.max_target.copy_(self.max)
        self.min_target.copy_(self.min)

    @torch.no_grad()
    def act(self, state, use_checkpoint=False):
        with self._autocast():
            if use_checkpoint:
                zs = self.checkpoint_encoder.zs(state, half_out=True)
                a = self.checkpoint_actor(state, zs)
            else:
                zs = self.fixed_encoder.zs(state, half_out=True)
                a = self.actor(state, zs)
        return a.float()


class Agent:
    """Drop-in for Agent/TD7_multi_agent.py:143 (and the batched select_action of
    TD7_multi_agent_Pink_noise.py:209-228), backed by the HIP LAP replay."""

    def __init__(self, state_dim, action_dim, max_action, learning_steps=500000, offline=False, hp=None,
                 env_num=15, ep_length=300, device=None, precision="fp32", n_envs=None, process_group=None,
                 buffer_size=None, graph_safe=False):
        from . import _native as nat
        from .replay import LAP
        self.device = nat.require_gpu(device)
        self.hp = hp if hp is not None else Hyperparameters()
        self.sync = GradSync(process_group)
        self.learner = TD7Learner(state_dim, action_dim, self.hp, learning_steps, offline, self.device, precision,
                                  self.sync, graph_safe=graph_safe)
        self.env_num = env_num
        self.ep_length = ep_length
        self.action_dim = action_dim
        size = int(buffer_size if buffer_size is not None else self.hp.buffer_size)
        self.replay_buffer = LAP(state_dim, action_dim, self.device, env_num, size, self.hp.batch_size, max_action,
                                 normalize_actions=True, prioritized=True)
        if self.sync.world > 1:
            # data parallel: every rank explores and samples its own replay shard
            # with its own streams (the weights are rank 0's broadcast)
            for rng in (self.learner._explore_rng, self.replay_buffer._rng):
                if rng is not None:
                    rng.fold(self.sync.rank)
        self.max_action = max_action
        self.offline = offline
        self._init_checkpointing()
        self.noise = None

    def _init_checkpointing(self):
        """Checkpointing tracked values (:175-180)."""
        self.eps_since_update = 0
        self.timesteps_since_update = 0
        self.max_eps_before_update = 1
        self.min_return = 1e8
        self.best_min_return = -1e8
        self.checkpoint_refreshes = 0  # policy checkpoints taken (:307-310), for traces

    # the reference exposes the nets and counters on the agent itself
    def __getattr__(self, name):
        learner = self.__dict__.get("learner")
        if learner is not None and hasattr(learner, name):
            return getattr(learner, name)
        raise AttributeError(name)

    # ----------------------------------------------------------- acting
    # Exploration-noise schedule: every select_action call decrements
    # exploration_noise once, as both reference variants do
    # (TD7_multi_agent.py:207, TD7_multi_agent_Pink_noise.py:225) -- the
    # training script calls it once per env with a 1-D state, the Pink
    # evaluation once per step with the batch.  select_action_batch stands in
    # for the training script's per-env calls of one vectorised step, so its
    # Gaussian branch decrements once per env; its Pink branch is the batched
    # Pink select_action and decrements once per call.
    def select_action(self, state, timestep=None, first_step=True, use_checkpoint=False, use_exploration=True):
        """Accepts one state (80,) or a batch (N, 80) as numpy; returns numpy."""
        s = np.asarray(state, dtype=np.float32)
        single = s.ndim == 1
        st = torch.as_tensor(s.reshape(-1, s.shape[-1]), device=self.device)
        a = self.learner.act(st, use_checkpoint)
        a = a.cpu().numpy()
        if use_exploration:
            if timestep is not None:
                # Pink-noise variant (TD7_multi_agent_Pink_noise.py:218-226): one coloured
                # noise sequence per episode, scaled by exploration_noise
                if first_step or self.noise is None:
                    self.init_episode_noise()
                a = a + self.noise[:, timestep]
            else:
                a = a + np.random.randn(*a.shape).astype(np.float32) * self.learner.exploration_noise
            self.learner.exploration_noise_t -= self.learner.action_noise_decrease
        a = np.clip(a, -1, 1) * self.max_action
        return a[0] if single else a

    # source of the per-episode coloured-noise generator (the reference's
    # ColoredNoiseProcess creates np.random.default_rng() per episode,
    # Agent/Pink_noise.py:57 -> colorednoise.py:104); tests inject seeded ones
    noise_rng_factory = staticmethod(np.random.default_rng)

    def init_episode_noise(self):
        """TD7_multi_agent_Pink_noise.py:203-206: a fresh [action_dim, ep_length]
        power-law sequence, peak-normalised, times the current exploration noise."""
        from .pink import powerlaw_psd_gaussian
        buf = powerlaw_psd_gaussian(self.hp.beta, (self.action_dim, self.ep_length), rng=self.noise_rng_factory())
        self.noise = buf / np.max(np.abs(buf)) * self.learner.exploration_noise

    @torch.no_grad()
    def init_episode_noise_device(self, n_steps=None, generator=None, spectrum=None):
        """Device Pink-noise sequence for a new episode round (the batched
        TD7_multi_agent_Pink_noise.py:203-207 on the GPU): [action_dim, L],
        peak-normalised and scaled by the current exploration noise; written
        into a persistent buffer so captured graphs keep reading it.
        spectrum = (sr, si): given scaled Gaussian spectra instead of device
        draws (parity tests)."""
        from .pink import powerlaw_psd_gaussian_device
        L = int(n_steps or self.ep_length)
        buf = powerlaw_psd_gaussian_device(self.hp.beta, self.action_dim, L, self.device, generator, spectrum)
        buf = buf / buf.abs().max() * self.learner.exploration_noise_t
        if getattr(self, "noise_dev", None) is None or self.noise_dev.shape != buf.shape:
            self.noise_dev = torch.empty_like(buf)
        self.noise_dev.copy_(buf)
        return self.noise_dev

    @torch.no_grad()
    def select_action_batch(self, obs, use_checkpoint=False, use_exploration=True, timestep=None, dec_count=None,
                            wg_cap=None, rt=None, zs_img=None):
        """Device-resident batched actions for the vectorised loop (no host sync).
        timestep (int64 device tensor [1]): Pink-noise exploration -- column
        `timestep` of the episode's noise (init_episode_noise_device) is added
        to every env's action, as the reference's batched Pink select_action
        does (:218-226), and exploration_noise decreases once per call (:225);
        otherwise Gaussian noise per env (TD7_multi_agent.py:205-207), one
        decrement per env (the training script's per-env calls; under data
        parallelism per env of every rank: the ranks' envs are the script's
        envs, and every rank's replica takes all of their decrements) -- dec_count
        (int32 device scalar): one per env counted there, the envs still
        running at this step of a synchronous round (the script calls
        select_action only for envs that are not done, :125-128)."""
        fz = self.learner.fused
        if fz is not None and use_exploration and timestep is None and not use_checkpoint and obs.is_cuda:
            # zs, actor and the noise in one launch
            return fz.select(obs, scale=self.max_action, dec_count=dec_count, world=self.sync.world, wg_cap=wg_cap,
                             rt=rt, zs_img=zs_img)
        if zs_img is not None:
            raise ValueError("select_action_batch: zs_img needs the fused Gaussian-exploration path")
        a = self.learner.act(obs, use_checkpoint)
        if use_exploration and timestep is not None:
            col = self.noise_dev.index_select(1, timestep).t()           # [1, action_dim]
            self.learner.exploration_noise_t -= self.learner.action_noise_decrease
            return (a + col).clamp(-1, 1) * self.max_action
        if use_exploration:
            L = self.learner
            noise = None if (a.is_cuda and L._device_rng) else torch.randn_like(a)
            dec = L.action_noise_decrease * self.sync.world
            if dec_count is not None:
                return ops.noisy_action(a, noise, L.exploration_noise_t, dec, scale=self.max_action,
                                        rng=L._explore_rng, dec_count=dec_count)
            return ops.noisy_action(a, noise, L.exploration_noise_t, dec * a.shape[0],
                                    scale=self.max_action, rng=L._explore_rng)
        return a.clamp(-1, 1) * self.max_action

    # ---------------------------------------------------------- training
    def train(self):
        state, action, next_state, reward, not_done = self.replay_buffer.sample()
        priority = self.learner.update(state, action, next_state, reward, not_done)
        self.replay_buffer.update_priority(priority)
        self.sync.max_(self.replay_buffer._maxp)  # global max_priority (:116)
        if self.learner.maybe_update_targets():
            self.replay_buffer.reset_max_priority()
            self.sync.max_(self.replay_buffer._maxp)  # :120 over every rank's leaves

    def maybe_train_and_checkpoint(self, ep_timesteps, ep_return, train=None):
        """:296-312 (the episode return is MIN-reduced over data-parallel ranks).
        train: the callable one training step runs (default self.train; the
        vectorised reference-schedule trainer passes its graph-replayed step)."""
        self.eps_since_update += 1
        self.timesteps_since_update += ep_timesteps
        r = float(ep_return)
        if self.sync.active:
            t = torch.tensor([-r], device=self.device, dtype=torch.float64)
            self.sync.max_(t)
            r = -float(t)
        self.min_return = min(self.min_return, r)
        if self.min_return < self.best_min_return:
            self.train_and_reset(train)
        elif self.eps_since_update == self.max_eps_before_update:
            self.best_min_return = self.min_return
            self.learner.checkpoint_actor.load_state_dict(self.learner.actor.state_dict())
            self.learner.checkpoint_encoder.load_state_dict(self.learner.fixed_encoder.state_dict())
            self.checkpoint_refreshes += 1
            self.train_and_reset(train)

    def train_and_reset(self, train=None):
        """:315-325"""
        train = self.train if train is None else train
        for _ in range(self.timesteps_since_update):
            if self.learner.training_steps == self.hp.steps_before_checkpointing:
                self.best_min_return *= self.hp.reset_weight
                self.max_eps_before_update = self.hp.max_eps_when_checkpointing
            train()
        self.eps_since_update = 0
        self.timesteps_since_update = 0
        self.min_return = 1e8

    def reset_buffer(self):
        self.replay_buffer.reset_buffer()

    # ------------------------------------------------------- checkpoints
    SUFFIXES = ["_critic", "_critic_optimizer", "_actor", "_actor_optimizer", "_encoder", "_encoder_optimizer",
                "_checkpoint_actor", "_checkpoint_encoder"]

    def save(self, filename):
        """:330-345 (same 8 files)."""
        L = self.learner
        torch.save(L.critic.state_dict(), filename + "_critic")
        torch.save(L.critic_optimizer.state_dict(), filename + "_critic_optimizer")
        torch.save(L.actor.state_dict(), filename + "_actor")
        torch.save(L.actor_optimizer.state_dict(), filename + "_actor_optimizer")
        torch.save(L.encoder.state_dict(), filename + "_encoder")
        torch.save(L.encoder_optimizer.state_dict(), filename + "_encoder_optimizer")
        torch.save(L.checkpoint_actor.state_dict(), filename + "_checkpoint_actor")
        torch.save(L.checkpoint_encoder.state_dict(), filename + "_checkpoint_encoder")

    def load(self, filename, load_optimizers=True):
        """:347-366.  weights_only loading; optimizer files are optional (the
        shipped checkpoints lack _critic_optimizer)."""
        import os
        L = self.learner
        ld = lambda suffix: torch.load(filename + suffix, map_location=self.device, weights_only=True)  # noqa: E731
        L.critic.load_state_dict(ld("_critic"))
        L.actor.load_state_dict(ld("_actor"))
        L.encoder.load_state_dict(ld("_encoder"))
        if load_optimizers:
            for suffix, opt in (("_critic_optimizer", L.critic_optimizer), ("_actor_optimizer", L.actor_optimizer),
                                ("_encoder_optimizer", L.encoder_optimizer)):
                if os.path.exists(filename + suffix):
                    opt.load_state_dict(ld(suffix))
        L.critic_target = copy.deepcopy(L.critic)
        L.actor_target = copy.deepcopy(L.actor)
        L.fixed_encoder = copy.deepcopy(L.encoder)
        L.fixed_encoder_target = copy.deepcopy(L.encoder)
        L.pair_fixed_encoders()
        if L.fused is not None:
            L.fused.rebuild()
        L.checkpoint_actor.load_state_dict(ld("_checkpoint_actor"))
        L.checkpoint_encoder.load_state_dict(ld("_checkpoint_encoder"))


def smoke():
    """One TD7 train() step through the HIP LAP kernels on cuda:0."""
    hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16)
    agent = Agent(80, 7, 1, hp=hp, env_num=8, device="cuda:0", buffer_size=1024)
    n = 64
    obs = torch.randn(n, 80, device="cuda:0")
    act = torch.rand(n, 7, device="cuda:0") * 2 - 1
    strata = torch.arange(n, device="cuda:0", dtype=torch.int32) % 8
    for _ in range(4):
        nobs = torch.randn(n, 80, device="cuda:0")
        agent.replay_buffer.add_batch(obs, act, nobs, torch.rand(n, device="cuda:0"),
                                      torch.zeros(n, dtype=torch.bool, device="cuda:0"), strata)
        obs = nobs
    agent.train()
    agent.train()
    torch.cuda.synchronize()
    assert torch.isfinite(agent.learner.max)
