"""td7f_adam_pack (csrc/td7_fused.hip): the optimiser step fused with the
repack of the weights it changes must leave exactly the state of the two
launches it replaces -- td7_adam_step_multi (FlatAdam.step_many) then td7f_pack
(FusedNets.pack) -- bit for bit: parameters, both moments, the step counts
and every packed forward / dX operand.  The two-launch path is itself pinned
to torch.optim.Adam (tests/test_td7_ops_gpu.py) and to the fused passes'
per-layer references (tests/test_fused_gpu.py).

Shapes: the bench's nets (zs / enc 300, critic / actor 320: inputs 80, 87,
307, 620, 920 -- rows that are not 16-byte aligned take the scalar path, 300
leaves a 4-wide last chunk) and the 256-wide alias in fp16."""
import ctypes

import pytest
import torch

from exo_amd import _native as nat
from exo_amd.fused import TD7FPackJob
from exo_amd.td7 import FlatAdam, Hyperparameters, TD7Learner

pytestmark = pytest.mark.gpu


def _learner(precision, width):
    torch.manual_seed(7)
    hp = Hyperparameters() if width is None else Hyperparameters(zs_dim=width, enc_hdim=width, critic_hdim=width,
                                                                 actor_hdim=width)
    L = TD7Learner(80, 7, hp, device="cuda", precision=precision)
    assert L.fused is not None
    return L


def _state(opts, nets):
    out = []
    for o in opts:
        out += [o.flat.clone(), o.m.clone(), o.v.clone(), o._step.clone()]
    for net in nets:
        for pl in net.layers:
            out.append(pl.wf.clone())
            if pl.wb is not None:
                out.append(pl.wb.clone())
    return out


def _restore(opts, nets, st):
    it = iter(st)
    for o in opts:
        for t in (o.flat, o.m, o.v, o._step):
            t.copy_(next(it))
    for net in nets:
        for pl in net.layers:
            pl.wf.copy_(next(it))
            if pl.wb is not None:
                pl.wb.copy_(next(it))


def _grads(modules, seed, skip=None):
    g = torch.Generator(device="cuda").manual_seed(seed)
    for m in modules:
        for name, p in m.named_parameters():
            p.grad = None if name == skip else torch.randn(p.shape, device="cuda", generator=g) * 0.1


@pytest.mark.parametrize("precision,width", [("bf16", None), ("fp16", 256)])
@pytest.mark.parametrize("which", ["critic", "actor"])
def test_adam_pack_matches_step_then_pack(precision, width, which):
    L = _learner(precision, width)
    F = L.fused
    if which == "critic":
        opts, names, mods = [L.encoder_optimizer, L.critic_optimizer], ("encoder", "critic"), [L.encoder, L.critic]
    else:
        opts, names, mods = [L.actor_optimizer], ("actor",), [L.actor]
    nets = [F.nets[n] for n in names]
    with torch.no_grad():
        for step in range(3):  # moments and bias corrections away from their first-step values
            _grads(mods, 11 + step)
            before = _state(opts, nets)
            FlatAdam.step_many(opts)
            F.pack(*names)
            ref = _state(opts, nets)
            _restore(opts, nets, before)
            F.adam_pack(opts, *names)
            got = _state(opts, nets)
            for k, (a, b) in enumerate(zip(got, ref)):
                assert torch.equal(a, b), f"step {step}: tensor {k} differs"
        assert all(float(o._step) == 3.0 for o in opts)


def test_adam_pack_skips_parameters_without_gradient():
    """A weight without a gradient is neither stepped nor repacked (torch.optim.Adam
    skips it); the other weights still match the two-launch path."""
    L = _learner("bf16", None)
    F = L.fused
    opts, names = [L.actor_optimizer], ("actor",)
    nets = [F.nets[n] for n in names]
    with torch.no_grad():
        _grads([L.actor], 3, skip="l2.weight")
        before = _state(opts, nets)
        FlatAdam.step_many(opts)
        F.pack(*names)
        ref = _state(opts, nets)
        _restore(opts, nets, before)
        F.adam_pack(opts, *names)
        got = _state(opts, nets)
    for k, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f"tensor {k} differs"


def test_adam_pack_rejects_partial_segment_cover():
    """A segment must be covered exactly by its jobs or by none."""
    L = _learner("bf16", None)
    o = L.critic_optimizer
    _grads([L.critic], 1)
    segs = FlatAdam.segments([o])
    pl = L.fused.nets["critic"].layers[0]  # head 0 of w0 only: half of w0's segment
    k = next(i for i, sg in enumerate(segs) if sg[1] <= (pl.weight.data_ptr() - o.flat.data_ptr()) // 4 < sg[1] + sg[2])
    jobs = (TD7FPackJob * 1)(pl.job())
    rc = nat.lib().td7f_adam_pack(1, *FlatAdam.multi_args([o], segs, (1, jobs, (ctypes.c_int32 * 1)(k))))
    assert rc == -22  # EXO_EINVAL


def _batch(B, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    s = torch.randn(B, 80, device="cuda", generator=g)
    a = torch.rand(B, 7, device="cuda", generator=g) * 2 - 1
    ns = torch.randn(B, 80, device="cuda", generator=g)
    r = torch.randn(B, 1, device="cuda", generator=g)
    nd = torch.ones(B, 1, device="cuda")
    return s, a, ns, r, nd


@pytest.mark.parametrize("precision,width,B", [("bf16", None, 1024), ("fp16", 256, 1000)])
def test_wgrad_adam_matches_wgrad_then_adam_pack(precision, width, B):
    """td7f_wgrad_adam == td7f_wgrad + td7f_adam_pack bit for bit (gradients,
    parameters, moments, step counts, packed operands, LAP priorities) for the
    encoder, critic and actor launches of one update, three steps running."""
    L = _learner(precision, width)
    F = L.fused
    tr = F.train(B)
    assert tr.fuses_adam()
    cases = [("encoder", [L.encoder_optimizer], tr.wgrad_encoder, tr.enc_grad),
             ("critic", [L.critic_optimizer], tr.wgrad_critic, tr.critic_grad),
             ("actor", [L.actor_optimizer], tr.wgrad_actor, tr.actor_grad)]
    with torch.no_grad():
        for step in range(3):
            batch = _batch(B, step)
            L.phase_grads(*batch)  # fills the transposed operands of every layer
            L.phase_actor_grads(batch[0], batch[1])
            for name, opts, wgrad, grad in cases:
                nets = [F.nets[name]]
                before = _state(opts, nets)
                wgrad(adam=False)
                F.adam_pack(opts, name)
                ref = _state(opts, nets) + [grad.clone(), tr.prio.clone()]
                _restore(opts, nets, before)
                grad.zero_()
                wgrad(adam=True)
                got = _state(opts, nets) + [grad.clone(), tr.prio.clone()]
                for k, (a, b) in enumerate(zip(got, ref)):
                    assert torch.equal(a, b), f"step {step} {name}: tensor {k} differs"
    assert all(float(o._step) == 3.0 for _, opts, _, _ in cases for o in opts)
