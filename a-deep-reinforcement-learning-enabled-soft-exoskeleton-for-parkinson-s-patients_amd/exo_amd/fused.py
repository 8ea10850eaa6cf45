"""Row-tile-fused TD7 networks on the GPU (csrc/td7_fused.hip): the host side.

With bf16 / fp16 MFMA operands -- and exact fp32 ones (v_mfma_f32_16x16x4_f32,
the reference's precision; EXO_FUSED_F32=0 keeps fp32 per layer) -- the TD7 nets of
Agent/TD7_multi_agent.py:61-140 run as whole-network launches (one workgroup
per 16 rows, activations in LDS) instead of one launch per Linear.  Their
weights are read from packed copies in MFMA-fragment order (PackedLinear),
refreshed by td7f_pack after every change of the fp32 master weights
(optimiser steps, target refreshes, loads).

FusedNets owns the packed copies of every net the update reads and the
launch wrappers; TD7Learner routes its passes here when `fused` is on.
"""
import ctypes
import os

import torch

from . import _native as nat
from . import ops

PD = 5  # include/exo_amd.h TD7F_PD
NW = 4  # waves per fused workgroup (csrc/td7_fused.h)
MAX_PACK = 32
MAX_ADAM_PACK = 16  # include/exo_amd.h TD7F_MAX_ADAM_PACK
PREC = {"bf16": 1, "fp16": 2, "fp32": 3}
# inputs per k-step (64 bytes of a row): 32 16-bit or 16 fp32 operands
KD = {1: 32, 2: 32, 3: 16}
# the fp32 fused path (csrc/td7_fused.h Ty<PREC_F32>): 0.50 vs 0.79 ms per
# configs[1] iteration per layer, parity-tested against the reference golden at
# the fp32 bounds (tests/test_td7_full.py); EXO_FUSED_F32=0 runs fp32 per layer
FUSED_F32 = os.environ.get("EXO_FUSED_F32", "1") == "1"


TD7FLin, TD7FPackJob, TD7FNoise = nat.TD7FLin, nat.TD7FPackJob, nat.TD7FNoise


def _ks(k, kd=32):
    """k-steps of a packed operand: ceil(k / kd) rounded up to TD7F_PD."""
    return -(-(-(-k // kd)) // PD) * PD


def _etype(prec):
    """torch dtype of an operand-type buffer (bit storage)."""
    return torch.float32 if prec == 3 else torch.int16


def _tiles(n):
    """16-wide tiles of a packed operand: exact up to NW, else a multiple of NW."""
    t = -(-n // 16)
    return t if t <= NW else -(-t // NW) * NW


class PackedLinear:
    """The packed operands of one Linear W [N, K] (a view of the fp32 master
    weight; one head of a stacked critic layer is a slice) in the operand type
    of prec: the forward operand and, with bwd=True, the dX operand (16 bytes
    per lane per 64-lane block either way)."""

    def __init__(self, weight, bias, bwd, prec=1):
        N, K = weight.shape
        dev = weight.device
        kd = KD[prec]
        self.weight, self.bias = weight, bias
        self.N, self.K = N, K
        self.ksf, self.ntf = _ks(K, kd), _tiles(N)
        self.wf = torch.zeros(self.ntf * self.ksf * 64 * 8, dtype=torch.int16, device=dev)
        self.ksb = _ks(N, kd) if bwd else 0
        self.ntb = -(-(-(-K // 16)) // NW) * NW if bwd else 0
        self.wb = torch.zeros(self.ntb * self.ksb * 64 * 8, dtype=torch.int16, device=dev) if bwd else None
        assert weight.stride(1) == 1
        self.lin = TD7FLin(self.wf.data_ptr(), self.wb.data_ptr() if bwd else None, bias.data_ptr(), N, K, self.ksf,
                           self.ksb, weight.data_ptr(), weight.stride(0))

    def job(self):
        w = self.weight
        assert w.stride(1) == 1
        return TD7FPackJob(w.data_ptr(), w.stride(0), self.N, self.K, self.wf.data_ptr(),
                           self.wb.data_ptr() if self.wb is not None else None, self.ksf, self.ntf, self.ksb, self.ntb)


def _lin_array(lins):
    return (TD7FLin * len(lins))(*[pl.lin for pl in lins])


class PackedNet:
    """Packed copies of a set of Linears, refreshed together by one td7f_pack launch."""

    def __init__(self, layers, prec, bwd=False):
        self.layers = [PackedLinear(w, b, bwd, prec) for w, b in layers]
        self.prec = prec
        self.array = _lin_array(self.layers)

    def pack(self, stream=None):
        jobs = [pl.job() for pl in self.layers]
        dev = self.layers[0].wf.device
        st = stream if stream is not None else nat.stream_ptr(dev)
        for i in range(0, len(jobs), MAX_PACK):
            part = jobs[i:i + MAX_PACK]
            nat.check(nat.lib().td7f_pack(self.prec, len(part), (TD7FPackJob * len(part))(*part), st), "td7f_pack")
        self._ver = self._versions()

    def _versions(self):
        return tuple(t._version for pl in self.layers for t in (pl.weight, pl.bias))

    def refresh(self):
        """Repack when a master weight changed through torch since the last
        pack (load_state_dict, copy_: their version counters moved); the HIP
        optimiser steps write the masters in place, and their callers repack
        explicitly (TD7Learner.phase_actor_step, maybe_update_targets)."""
        if self._versions() != self._ver:
            self.pack()


def encoder_layers(enc):
    return [(getattr(enc, n).weight, getattr(enc, n).bias) for n in ("zs1", "zs2", "zs3", "zsa1", "zsa2", "zsa3")]


def actor_layers(actor):
    return [(getattr(actor, n).weight, getattr(actor, n).bias) for n in ("l0", "l1", "l2", "l3")]


def critic_layers(critic):
    """[layer][head] order: w_k[h] of the stacked critic (the reference's q01/q02, q1/q4, q2/q5, q3/q6)."""
    out = []
    for k in range(4):
        w, b = getattr(critic, f"w{k}"), getattr(critic, f"b{k}")
        for h in range(2):
            out.append((w[h], b[h]))
    return out


def supported(learner):
    """The fused path applies: GPU, bf16/fp16/fp32 operands (fp32 unless
    EXO_FUSED_F32=0), the reference's activations, and every hidden width
    (zs_dim, enc_hdim, critic_hdim, actor_hdim) a multiple of 4 in 241..320 --
    16-wide tiles per wave of 4 or 5 (NW = 4 waves), all widths in the same
    tile class.  Anything else (the wide configuration, widths below 241)
    runs the per-layer kernels."""
    hp = learner.hp
    if learner.device.type != "cuda" or learner.precision not in PREC:
        return False
    if learner.precision == "fp32" and not FUSED_F32:
        return False
    acts = [ops.act_code(f) for f in (hp.enc_activ, hp.actor_activ, hp.critic_activ)]
    if any(a is None or a == ops.ACT_CODES["tanh"] for a in acts):
        return False
    widths = (hp.zs_dim, hp.enc_hdim, hp.critic_hdim, hp.actor_hdim)
    th = {_tiles(w) // NW for w in widths}
    return all(49 <= w <= 320 and w % 4 == 0 for w in widths) and len(th) == 1 and th <= {4, 5}


class PlanError(RuntimeError):
    """A network shape the fused passes' shared-memory plan cannot hold."""


class FusedNets:
    """Packed copies of every TD7 net plus the fused launches of one learner."""

    def __init__(self, learner):
        L = learner
        self.L = L
        self.prec = PREC[L.precision]
        self.dev = L.device
        hp = L.hp
        self.act = (ctypes.c_int32 * 3)(ops.act_code(hp.enc_activ), ops.act_code(hp.actor_activ),
                                        ops.act_code(hp.critic_activ))
        self._build()
        self.probe()

    @torch.no_grad()
    def probe(self):
        """Every fused pass once in plan-only mode (td7f_probe: arguments and
        the LDS plan checked, nothing launched) at the row counts whose plans
        differ (select's 16- and 32-row tiles), when the learner builds its
        passes instead of at the first call of a pass that cannot run (ADVICE
        r4: fp32 with zs_dim well above actor_hdim).  An inference pass
        (select_action, the target heads, the fixed embeddings) that does not
        fit raises PlanError: the learner keeps the per-layer kernels.  A
        gradient pass that does not (the actor passes need hidden widths in
        multiples of 16: the Pink agent's 300-wide actor) leaves train_ok
        False: fused inference, per-layer update (TD7Learner.fused_train)."""
        L, dev = self.L, self.dev
        S, A = L.actor.l0.in_features, L.actor.l3.out_features
        B = 16
        # FusedTrain points the parameters' .grad at its own buffers: restored after
        params = [p for m in (L.encoder, L.critic, L.actor) for p in m.parameters()]
        grads = [p.grad for p in params]
        f32 = dict(dtype=torch.float32, device=dev)
        lib = nat.lib()
        lib.td7f_probe(1)
        self.train_ok = False
        try:
            s, a = torch.zeros((B, S), **f32), torch.zeros((B, A), **f32)
            try:
                for n in (B, 8200):
                    self.select(torch.zeros((n, S), **f32))
                self.target_heads(s, noise=torch.zeros((B, A), **f32))
                zs, zsa = self.fixed(s, a)
            except RuntimeError as e:
                raise PlanError(f"fused TD7 passes: {e}") from e
            try:
                t = FusedTrain(self, B)
                one = torch.zeros((B, 1), **f32)
                t.encoder(s, a, s)
                for ph in (0, 1, 2):
                    t.critic(s, a, zs, zsa, torch.zeros((B, 2), **f32), one, one, phase=ph)
                for ph in (0, 1, 2):
                    t.actor(ph, s, zs)
                self.train_ok = True
            except RuntimeError as e:  # inference fused, the update per layer
                self.train_error = str(e)
        finally:
            lib.td7f_probe(0)
            for p, g in zip(params, grads):
                p.grad = g

    def _build(self):
        L, p = self.L, self.prec
        self.nets = {
            "fixed_encoder": PackedNet(encoder_layers(L.fixed_encoder), p, bwd=True),
            "fixed_encoder_target": PackedNet(encoder_layers(L.fixed_encoder_target), p),
            "actor": PackedNet(actor_layers(L.actor), p, bwd=True),
            "actor_target": PackedNet(actor_layers(L.actor_target), p),
            "critic_target": PackedNet(critic_layers(L.critic_target), p),
            "encoder": PackedNet(encoder_layers(L.encoder), p, bwd=True),
            "critic": PackedNet(critic_layers(L.critic), p, bwd=True),
        }
        self.pack_all()
        self._train = {}

    def train(self, B):
        """The gradient passes for batches of B rows (buffers made on first use)."""
        t = self._train.get(B)
        if t is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedNets.train: run once eagerly before graph capture")
            t = self._train[B] = FusedTrain(self, B)
        return t

    def rebuild(self):
        """After the learner re-created nets (Agent.load): new views, repacked."""
        self._build()

    def pack(self, *names):
        """Repack the named nets in as few td7f_pack launches as their layers fit
        (TD7F_MAX_PACK jobs each)."""
        nets = [self.nets[n] for n in names]
        jobs = [pl.job() for net in nets for pl in net.layers]
        st = nat.stream_ptr(self.dev)
        for i in range(0, len(jobs), MAX_PACK):
            part = jobs[i:i + MAX_PACK]
            nat.check(nat.lib().td7f_pack(self.prec, len(part), (TD7FPackJob * len(part))(*part), st), "td7f_pack")
        for net in nets:
            net._ver = net._versions()

    def pack_all(self):
        self.pack(*self.nets)

    def adam_pack(self, opts, *names):
        """FlatAdam.step_many(opts) followed by pack(*names), as one
        td7f_adam_pack launch: the thread that updates a weight writes its
        packed copies.  Every packed weight must be a parameter (or a head of
        one) of one of the optimisers; one without a gradient is not stepped
        and keeps its packed copy."""
        from .td7 import FlatAdam
        segs = FlatAdam.segments(opts)
        if not segs:
            return
        nets = [self.nets[n] for n in names]
        jobs, jseg = [], []
        for net in nets:
            for pl in net.layers:
                ptr = pl.weight.data_ptr()
                for k, o in enumerate(opts):
                    e = (ptr - o.flat.data_ptr()) // 4
                    if 0 <= e < o.flat.numel():
                        break
                else:
                    raise ValueError("adam_pack: a packed weight outside the optimisers' parameters")
                hit = [i for i, sg in enumerate(segs) if sg[3] == k and sg[1] <= e < sg[1] + sg[2]]
                if hit:
                    jobs.append(pl.job())
                    jseg.append(hit[0])
        if (len(opts) > FlatAdam.MAX_OPT or len(segs) > FlatAdam.MAX_SEG or len(jobs) > MAX_ADAM_PACK
                or not all(pl.weight.is_contiguous() for net in nets for pl in net.layers)):
            FlatAdam.step_many(opts)
            self.pack(*names)
            return
        nj = len(jobs)
        extra = (nj, (TD7FPackJob * nj)(*jobs), (ctypes.c_int32 * nj)(*jseg))
        nat.check(nat.lib().td7f_adam_pack(self.prec, *FlatAdam.multi_args(opts, segs, extra)), "td7f_adam_pack")
        for net in nets:
            net._ver = net._versions()

    def refresh(self, *names):
        for n in names:
            self.nets[n].refresh()

    # ------------------------------------------------------------- noise
    def _noise(self, rng, sigma, dec, clip, scale, z=None, dec_count=None):
        return TD7FNoise(rng.seed, rng.tag, 0, rng.counter_ptr, rng.ticket_ptr, sigma.data_ptr(), float(dec),
                         float(clip), float(scale), 0, z.data_ptr() if z is not None else None,
                         dec_count.data_ptr() if dec_count is not None else None)

    # ------------------------------------------------------------- passes
    def zs_image(self, n):
        """the [n][zs_dim] operand-type buffer select_zs fills (allocated on the
        first call, which must come before any graph capture that uses it)"""
        Z = self.L.hp.zs_dim
        buf = getattr(self, "_zs_img", None)
        if buf is None or buf.shape[0] < n:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedNets.zs_image: allocate it eagerly before graph capture")
            buf = self._zs_img = torch.empty((n, Z), dtype=_etype(self.prec), device=self.dev)
        return buf[:n]

    @torch.no_grad()
    def select_zs(self, obs, wg_cap=None, rt=None):
        """The fixed encoder's half of select (td7f_select_part mode 1):
        fixed_encoder.zs(obs) (TD7_multi_agent.py:93-97), normalised, into
        zs_image(n) -- no actor, no noise, no exploration-state change.  The
        fixed encoder changes only at target refreshes, so a training loop can
        run this as soon as the observations exist and the actor half, select
        (..., zs_img=), after the actor step: the pair is select bit for bit
        (same rt)."""
        self.refresh("fixed_encoder")
        obs = obs.contiguous()
        n = obs.shape[0]
        img = self.zs_image(n)
        fe = self.nets["fixed_encoder"].layers
        nat.check(nat.lib().td7f_select_part(self.prec, self.act, _lin_array(fe[:3]), self.nets["actor"].array,
                                             nat.ptr(obs), n, None, None, int(wg_cap or 0), int(rt or 0),
                                             nat.ptr(img), 1, nat.stream_ptr(obs.device)), "td7f_select_part")
        return img

    @torch.no_grad()
    def select(self, obs, scale=1.0, dec_count=None, world=1, wg_cap=None, rt=None, zs_img=None):
        """select_action_batch with Gaussian exploration (one launch): actor(obs,
        fixed_encoder.zs(obs)) + N(0, exploration_noise) per element, clamped,
        times max_action; exploration_noise decreases once per env (dec_count:
        an int32 device scalar -- once per env counted there, the active envs
        of a vectorised step; times `world`, the data-parallel ranks stepping
        as many envs each)."""
        L = self.L
        self.refresh(*(("actor",) if zs_img is not None else ("fixed_encoder", "actor")))
        obs = obs.contiguous()
        n = obs.shape[0]
        out = torch.empty((n, L.actor.l3.out_features), dtype=torch.float32, device=obs.device)
        dec = L.action_noise_decrease * world
        if dec_count is not None:
            nz = self._noise(L._explore_rng, L.exploration_noise_t, dec, 0.0, scale, dec_count=dec_count)
        else:
            nz = self._noise(L._explore_rng, L.exploration_noise_t, dec * n, 0.0, scale)
        fe, ac = self.nets["fixed_encoder"].layers, self.nets["actor"].layers
        # wg_cap: at most this many workgroups per launch (None / 0: one launch);
        # rt: rows per tile / 16 (None / 0: the library's pick)
        if zs_img is not None:  # the actor half after select_zs (td7f_select_part mode 2)
            nat.check(nat.lib().td7f_select_part(self.prec, self.act, _lin_array(fe[:3]), self.nets["actor"].array,
                                                 nat.ptr(obs), n, ctypes.byref(nz), nat.ptr(out), int(wg_cap or 0),
                                                 int(rt or 0), nat.ptr(zs_img), 2, nat.stream_ptr(obs.device)),
                      "td7f_select_part")
            return out
        nat.check(nat.lib().td7f_select(self.prec, self.act, _lin_array(fe[:3]), self.nets["actor"].array,
                                        nat.ptr(obs), n, ctypes.byref(nz), nat.ptr(out), int(wg_cap or 0),
                                        int(rt or 0), nat.stream_ptr(obs.device)), "td7f_select")
        return out

    def _img(self, B):
        Z = self.L.hp.zs_dim
        A = self.L.actor.l3.out_features
        buf = getattr(self, "_tgt_img", None)
        if buf is None or buf.shape[0] < B:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedNets.target: run once eagerly before graph capture")
            buf = self._tgt_img = torch.empty((B, -(-(2 * Z + A) // 8) * 8), dtype=_etype(self.prec), device=self.dev)
        return buf

    @torch.no_grad()
    def target_heads(self, next_state, noise=None, out=None):
        """Both heads of critic_target(s', a'(s'), zsa', zs') [B, 2] with a' the
        noisy target action (:233-241); two launches.  noise: given standard
        normals [B, A] (parity tests) instead of the device stream.  out: a
        [B, 2] fp32 buffer to write (else a new tensor)."""
        L = self.L
        self.refresh("fixed_encoder_target", "actor_target", "critic_target")
        ns = next_state.contiguous()
        B = ns.shape[0]
        qt = out if out is not None else torch.empty((B, 2), dtype=torch.float32, device=ns.device)
        z = noise.to(device=ns.device, dtype=torch.float32).contiguous() if noise is not None else None
        nz = self._noise(L._noise_rng, L.target_policy_noise, L.policy_noise_decrease, L.hp.noise_clip, 1.0, z)
        nat.check(nat.lib().td7f_target(self.prec, self.act, self.nets["fixed_encoder_target"].array,
                                        self.nets["actor_target"].array, self.nets["critic_target"].array,
                                        nat.ptr(ns), B, ctypes.byref(nz), nat.ptr(self._img(B)), nat.ptr(qt),
                                        nat.stream_ptr(ns.device)), "td7f_target")
        return qt

    @torch.no_grad()
    def fixed(self, state, action, out=None):
        """(fixed_encoder.zs(state), fixed_encoder.zsa(zs, action)), one launch
        (:248-249); out: a (zs, zsa) pair of [B, Z] fp32 buffers to write."""
        self.refresh("fixed_encoder")
        s, a = state.contiguous(), action.contiguous()
        B = s.shape[0]
        Z = self.L.hp.zs_dim
        if out is not None:
            zs, zsa = out
        else:
            zs = torch.empty((B, Z), dtype=torch.float32, device=s.device)
            zsa = torch.empty((B, Z), dtype=torch.float32, device=s.device)
        nat.check(nat.lib().td7f_fixed(self.prec, self.act, self.nets["fixed_encoder"].array, nat.ptr(s), nat.ptr(a),
                                       B, nat.ptr(zs), nat.ptr(zsa), nat.stream_ptr(s.device)), "td7f_fixed")
        return zs, zsa


class XTBuffers:
    """The transposed weight-gradient operands of one Linear in the operand
    type (include/exo_amd.h td7f_xt)."""

    def __init__(self, N, K, B, ld, dev, prec=1):
        r64 = lambda n: -(-n // 64) * 64  # noqa: E731
        self.N, self.K = N, K
        self.x = torch.zeros((r64(K), ld), dtype=_etype(prec), device=dev)
        self.dp = torch.zeros((r64(N), ld), dtype=_etype(prec), device=dev)
        self.part = torch.zeros((-(-B // 16), N), dtype=torch.float32, device=dev)
        self.c = nat.TD7FXT(self.x.data_ptr(), self.dp.data_ptr(), self.part.data_ptr())


def _grad_views(opt):
    """Persistent gradient tensors of a FlatAdam's parameters: views of one flat
    buffer in parameter order (the fused weight-gradient launch writes them;
    the optimiser step and the data-parallel all-reduce read them)."""
    g = torch.zeros_like(opt.flat)
    off = 0
    for p in opt._params():
        n = p.numel()
        p.grad = g[off:off + n].view_as(p)
        off += n
    return g


class FusedTrain:
    """The gradient passes of one TD7 update as fused launches (csrc/td7_fused_train.hip)
    for a batch of B rows: buffers are allocated on the first call (outside graph capture)."""

    def __init__(self, nets, B):
        self.nets, self.L, self.B = nets, nets.L, B
        L, dev = self.L, nets.dev
        hp = L.hp
        # row stride of the transposed operands = the weight-gradient reduction
        # length: the batch padded to 256 rows (zero columns; td7f_wgrad's k-loop)
        self.ld = -(-B // 256) * 256
        Z, He, Hc, Ha = hp.zs_dim, hp.enc_hdim, hp.critic_hdim, hp.actor_hdim
        A = L.actor.l3.out_features
        S = L.actor.l0.in_features
        self.S, self.A = S, A
        f32 = dict(dtype=torch.float32, device=dev)
        p = nets.prec
        self.xt_enc = [XTBuffers(pl.N, pl.K, B, self.ld, dev, p) for pl in nets.nets["encoder"].layers]
        self.xt_critic = [XTBuffers(pl.N, pl.K, B, self.ld, dev, p) for pl in nets.nets["critic"].layers]
        self.xt_actor = [XTBuffers(pl.N, pl.K, B, self.ld, dev, p) for pl in nets.nets["actor"].layers]
        self.y_enc = [torch.empty((B, He), **f32) for _ in range(4)]
        self.y_critic = [torch.empty((2, B, Hc), **f32) for _ in range(2)]
        self.td = torch.zeros((B, 2), **f32)
        self.q = torch.zeros((B, 2), **f32)
        # the critic pass split in two launches (critic(phase=1 / 2)): the
        # forward's state for the backward -- Q, q0's pre-norm output, row means
        bp = -(-B // 16) * 16
        self.crit_q = torch.zeros((2, bp), **f32)
        self.crit_h0 = torch.zeros((2, bp, Hc), **f32)
        self.crit_mean = torch.zeros((2, bp), **f32)
        self.prio = torch.zeros((B,), **f32)
        self.act_out = torch.zeros((B, A), **f32)
        self.zsa_out = torch.zeros((B, Z), **f32)
        self.h0 = torch.zeros((B, Ha), **f32)
        self.mean0 = torch.zeros((B,), **f32)
        self.ya = [torch.zeros((B, Ha), **f32) for _ in range(2)]
        self.yz = [torch.zeros((B, He), **f32) for _ in range(2)]
        self.yc = [torch.zeros((2, B, Hc), **f32) for _ in range(2)]
        self.da = torch.zeros((2, B, A), **f32)
        self.dzsa = torch.zeros((2, B, Z), **f32)
        P = ctypes.c_void_p
        self.actor_bufs = nat.TD7FActorBufs(self.act_out.data_ptr(), self.zsa_out.data_ptr(), self.h0.data_ptr(),
                                            self.mean0.data_ptr(), (P * 2)(*[t.data_ptr() for t in self.ya]),
                                            (P * 2)(*[t.data_ptr() for t in self.yz]),
                                            (P * 2)(*[t.data_ptr() for t in self.yc]), self.da.data_ptr(),
                                            self.dzsa.data_ptr())
        self.enc_grad = _grad_views(L.encoder_optimizer)
        self.critic_grad = _grad_views(L.critic_optimizer)
        self.actor_grad = _grad_views(L.actor_optimizer)
        # weight-gradient jobs: [layer] (encoder), [layer][head] (critic), [layer] (actor)
        rt = -(-B // 16)
        enc_p = list(L.encoder.parameters())
        jobs = []
        for i, xb in enumerate(self.xt_enc):
            jobs.append(self._job(xb, enc_p[2 * i].grad, enc_p[2 * i + 1].grad, rt))
        for k in range(4):
            gw, gb = getattr(L.critic, f"w{k}").grad, getattr(L.critic, f"b{k}").grad
            for h in range(2):
                jobs.append(self._job(self.xt_critic[2 * k + h], gw[h], gb[h], rt))
        self.jobs_ec = (nat.TD7FWgJob * len(jobs))(*jobs)
        ne = len(self.xt_enc)
        self.jobs_e = (nat.TD7FWgJob * ne)(*jobs[:ne])
        self.jobs_c = (nat.TD7FWgJob * (len(jobs) - ne))(*jobs[ne:])
        # td7f_wgrad_adam: where each job's layer sits in its optimiser (None
        # when the jobs do not cover every parameter of that optimiser)
        self.adam_e = self._adam_descs(L.encoder_optimizer, nets.nets["encoder"].layers)
        self.adam_c = self._adam_descs(L.critic_optimizer, nets.nets["critic"].layers)
        self.adam_a = self._adam_descs(L.actor_optimizer, nets.nets["actor"].layers)
        act_p = list(L.actor.parameters())
        ajobs = [self._job(xb, act_p[2 * i].grad, act_p[2 * i + 1].grad, rt) for i, xb in enumerate(self.xt_actor)]
        self.jobs_a = (nat.TD7FWgJob * len(ajobs))(*ajobs)
        self.ptrs_y_enc = (P * 4)(*[t.data_ptr() for t in self.y_enc])
        # the encoder pass with zs(s') on its own workgroup row (r04, EXO_ENC_SPLIT=1).
        # Off by default: alone the split pass is shorter, but inside the training
        # iteration its extra 64 workgroups take CUs from the concurrent target /
        # fixed passes on the critical chain (0.320 vs 0.299 ms per iteration,
        # profiles/r04b_raw/bench_ab_*.log)
        self.enc_split = os.environ.get("EXO_ENC_SPLIT", "0") == "1"
        self.enc_nz = torch.zeros((rt * 16, Z), **f32)
        self.enc_flag = torch.zeros((rt,), dtype=torch.int32, device=dev)

    @staticmethod
    def _adam_descs(opt, layers):
        flat = getattr(opt, "flat", None)
        if flat is None:
            return None
        base, descs, covered = flat.data_ptr(), [], 0
        for pl in layers:
            w, b = pl.weight, pl.bias
            descs.append(nat.TD7FWgAdam(0, (w.data_ptr() - base) // 4, (b.data_ptr() - base) // 4, pl.wf.data_ptr(),
                                        pl.wb.data_ptr() if pl.wb is not None else None, pl.ksf, pl.ksb))
            covered += w.numel() + b.numel()
        return (nat.TD7FWgAdam * len(descs))(*descs) if covered == flat.numel() else None

    def fuses_adam(self):
        """The weight-gradient launches can carry the optimiser steps (every
        parameter of the encoder / critic / actor optimisers is one of their layers)."""
        return all(d is not None for d in (self.adam_e, self.adam_c, self.adam_a))

    def _wgrad(self, jobs, descs, opt, adam, td=None, prio=None, B=0):
        fz, hp = self.nets, self.L.hp
        if adam and descs is None:
            raise RuntimeError("td7f_wgrad_adam: the layers do not cover the optimiser's parameters")
        st = nat.stream_ptr(fz.dev)
        alpha, minp = (float(hp.alpha), float(hp.min_priority)) if prio is not None else (0.0, 0.0)
        if not adam:
            nat.check(nat.lib().td7f_wgrad(fz.prec, len(jobs), jobs, self.ld, self.ld, td, prio, B, alpha, minp, st),
                      "td7f_wgrad")
            return
        g = opt.param_groups[0]
        P1 = lambda t: (ctypes.c_void_p * 1)(t.data_ptr())  # noqa: E731
        F1 = lambda x: (ctypes.c_float * 1)(float(x))  # noqa: E731
        nat.check(nat.lib().td7f_wgrad_adam(fz.prec, len(jobs), jobs, self.ld, self.ld, td, prio, B, alpha, minp, 1,
                                            P1(opt.flat), P1(opt.m), P1(opt.v), P1(opt._step), F1(g["lr"]),
                                            F1(g["betas"][0]), F1(g["betas"][1]), F1(g["eps"]),
                                            F1(g["weight_decay"]), descs, nat.ptr(opt._ticket), st), "td7f_wgrad_adam")

    @staticmethod
    def _job(xb, gw, gb, rt):
        assert gw.is_contiguous() and gb.is_contiguous()
        return nat.TD7FWgJob(xb.dp.data_ptr(), xb.x.data_ptr(), xb.part.data_ptr(), gw.data_ptr(), gb.data_ptr(),
                             xb.N, xb.K, rt)

    @staticmethod
    def _xts(bufs):
        return (nat.TD7FXT * len(bufs))(*[b.c for b in bufs])

    def encoder(self, state, action, next_state):
        fz = self.nets
        fz.refresh("encoder")
        nz, fl = (self.enc_nz, self.enc_flag) if self.enc_split else (None, None)
        nat.check(nat.lib().td7f_encoder(fz.prec, fz.act, fz.nets["encoder"].array, nat.ptr(state), nat.ptr(action),
                                         nat.ptr(next_state), self.B, self.ptrs_y_enc, self._xts(self.xt_enc), self.ld,
                                         nat.ptr(nz), nat.ptr(fl), nat.stream_ptr(state.device)), "td7f_encoder")

    def critic(self, state, action, zs, zsa, qt, reward, not_done, phase=0):
        """td7f_critic_phase: 0 the whole critic pass; 1 its forward alone (needs
        no qt: it runs beside the target chain); 2 the loss and the backward
        from phase 1's stored state -- phases 1 + 2 == phase 0 bit for bit."""
        fz, L = self.nets, self.L
        if phase != 2:
            fz.refresh("critic")
        nat.check(nat.lib().td7f_critic_phase(
            int(phase), fz.prec, fz.act, fz.nets["critic"].array, nat.ptr(state), nat.ptr(action), nat.ptr(zs),
            nat.ptr(zsa), nat.ptr(qt), nat.ptr(reward), nat.ptr(not_done), float(L.hp.discount),
            nat.ptr(L.min_target), nat.ptr(L.max_target), nat.ptr(L.max), nat.ptr(L.min), self.B, self.S, self.A,
            nat.ptr(self.td), nat.ptr(self.q), nat.ptr(self.y_critic[0]), nat.ptr(self.y_critic[1]),
            self._xts(self.xt_critic), self.ld, nat.ptr(self.crit_q), nat.ptr(self.crit_h0), nat.ptr(self.crit_mean),
            nat.stream_ptr(state.device)), "td7f_critic_phase")

    def wgrad_encoder_critic(self):
        """Every encoder and critic weight/bias gradient (one launch) and the LAP priorities."""
        fz, hp = self.nets, self.L.hp
        nat.check(nat.lib().td7f_wgrad(fz.prec, len(self.jobs_ec), self.jobs_ec, self.ld, self.ld, nat.ptr(self.td),
                                       nat.ptr(self.prio), self.B, float(hp.alpha), float(hp.min_priority),
                                       nat.stream_ptr(fz.dev)), "td7f_wgrad")
        return self.prio

    def wgrad_encoder(self, adam=False):
        """The encoder's weight/bias gradients alone (its branch of the update);
        adam: with the encoder's optimiser step and repack (td7f_wgrad_adam)."""
        L = self.L
        self._wgrad(self.jobs_e, self.adam_e, L.encoder_optimizer, adam)

    def wgrad_critic(self, adam=False):
        """The critic's weight/bias gradients and the LAP priorities; adam: with
        the critic's optimiser step and repack."""
        L = self.L
        self._wgrad(self.jobs_c, self.adam_c, L.critic_optimizer, adam, nat.ptr(self.td),
                    nat.ptr(self.prio), self.B)
        return self.prio

    def actor(self, phase, state, zs):
        fz = self.nets
        fz.refresh("actor", "fixed_encoder", "critic")
        nat.check(nat.lib().td7f_actor(fz.prec, phase, fz.act, fz.nets["actor"].array, fz.nets["fixed_encoder"].array,
                                       fz.nets["critic"].array, nat.ptr(state), nat.ptr(zs), self.B,
                                       ctypes.byref(self.actor_bufs), self._xts(self.xt_actor), self.ld,
                                       nat.stream_ptr(state.device)), f"td7f_actor[{phase}]")

    def wgrad_actor(self, adam=False):
        self._wgrad(self.jobs_a, self.adam_a, self.L.actor_optimizer, adam)
