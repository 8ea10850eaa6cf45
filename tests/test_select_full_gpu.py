"""select_action at the bench's widths against the reference:
tests/golden/select_action_full.npz holds the Pink agent's batched
select_action (Agent/TD7_multi_agent_Pink_noise.py:209-228, exploration off)
for 256 real observations, checkpoint and live nets, at zs / enc 300, critic
320 and actor 300 (the Pink agent's and the shipped checkpoints' shapes) and
actor 320 (the bench's).  The nets are rebuilt from the fixture's seeds (the
build's seeded init is bit-exact) plus the generator's perturbation of the
live actor / fixed encoder.

Paths checked on the MI355X:
* fp32: Agent.select_action (1-D and batched) and select_action_batch --
  exact fp32 MFMA, bound 2e-5 (fp32 summation order only);
* bf16: the per-layer kernels (act(), bf16 operands) and the bench's fused
  td7f_select kernel (exploration noise scale set to 0 so the launch returns
  the deterministic action).  Bound: the bf16 rounding model.  The test runs
  the same forward on the CPU with every Linear's operands rounded to bf16
  (x.bfloat16() @ W.bfloat16()^T + b, fp32 accumulation, everything else
  fp32 -- what the kernels do); the GPU result must stay within
  1.5x the emulation's own distance to the reference + 5e-4, and within 2e-3
  of the emulation itself (intermediate activations that sit on a bf16
  rounding boundary can round the other way after an fp32 summation-order
  difference)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import GOLDEN, SELECT_FULL, select_full_perturb

pytestmark = pytest.mark.gpu


def _golden():
    return np.load(f"{GOLDEN}/select_action_full.npz", allow_pickle=False)


def _cases():
    return SELECT_FULL


def _agent(name, kw, seed, precision):
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(seed)
    hp = Hyperparameters(**kw)
    hp.actor_hdim = kw.get("actor_hdim", 300)  # the Pink agent's default actor width
    ag = Agent(80, 7, 1, hp=hp, env_num=8, device="cuda", buffer_size=64, precision=precision)
    L = ag.learner
    _perturb_on_device(L.actor, 1000 * seed, select_full_perturb)
    _perturb_on_device(L.fixed_encoder, 1000 * seed + 500, select_full_perturb)
    return ag


def _perturb_on_device(module, seed, fn):
    """select_full_perturb on a CPU copy of `module`'s parameters, copied back."""
    params = [p for _, p in module.named_parameters()]
    cpu = [torch.nn.Parameter(p.detach().cpu().clone()) for p in params]
    holder = torch.nn.Module()
    for k, p in enumerate(cpu):
        holder.register_parameter(f"p{k:03d}", p)  # named_parameters keeps this order
    fn(holder, seed)
    with torch.no_grad():
        for p, c in zip(params, cpu):
            p.copy_(c)


def _bf(x):
    return x.bfloat16().float()


def _emulate_bf16(ag, st, checkpoint):
    """CPU forward with bf16-rounded Linear operands (fp32 accumulation)."""
    L = ag.learner
    enc = L.checkpoint_encoder if checkpoint else L.fixed_encoder
    act = L.checkpoint_actor if checkpoint else L.actor
    P = lambda lin: (lin.weight.detach().cpu().float(), lin.bias.detach().cpu().float())  # noqa: E731

    def lin(x, layer):
        w, b = P(layer)
        return _bf(x) @ _bf(w).t() + b

    def norm(x):
        return x / x.abs().mean(-1, keepdim=True).clamp(min=1e-8)
    s = torch.as_tensor(st)
    zs = F.elu(lin(s, enc.zs1))
    zs = F.elu(lin(zs, enc.zs2))
    zs = norm(lin(zs, enc.zs3))
    a = norm(lin(s, act.l0))
    a = F.relu(lin(torch.cat([a, zs], 1), act.l1))
    a = F.relu(lin(a, act.l2))
    return torch.tanh(lin(a, act.l3)).clamp(-1, 1).numpy()


@pytest.mark.parametrize("case", [0, 1])
def test_select_full_fp32(case):
    g = _golden()
    name, kw, seed = _cases()[case]
    ag = _agent(name, kw, seed, "fp32")
    L = ag.learner
    sums = [float(sum(p.detach().double().sum() for p in m.parameters())) for m in (L.actor, L.fixed_encoder)]
    np.testing.assert_allclose(sums, g[f"{name}.live_sum"], rtol=0, atol=1e-9)  # the rebuild is the reference's
    st = g["state"]
    for ckpt, key in ((True, "ckpt"), (False, "live")):
        want = g[f"{name}.{key}"]
        a = ag.select_action(st, use_checkpoint=ckpt, use_exploration=False)
        np.testing.assert_allclose(a, want, rtol=0, atol=2e-5, err_msg=f"{name}.{key} batched")
        a1 = np.stack([ag.select_action(s, use_checkpoint=ckpt, use_exploration=False) for s in st[:16]])
        np.testing.assert_allclose(a1, want[:16], rtol=0, atol=2e-5, err_msg=f"{name}.{key} 1-D")
        b = ag.select_action_batch(torch.as_tensor(st, device="cuda"), use_checkpoint=ckpt, use_exploration=False)
        np.testing.assert_allclose(b.cpu().numpy(), want, rtol=0, atol=2e-5, err_msg=f"{name}.{key} device")


@pytest.mark.parametrize("case", [0, 1])
def test_select_full_bf16_per_layer_and_fused(case):
    g = _golden()
    name, kw, seed = _cases()[case]
    ag = _agent(name, kw, seed, "bf16")
    L = ag.learner
    assert L.fused is not None, "the bench's fused path must apply at these widths"
    st = g["state"]
    obs = torch.as_tensor(st, device="cuda")
    report = {}
    for ckpt, key in ((True, "ckpt"), (False, "live")):
        want = g[f"{name}.{key}"]
        emu = _emulate_bf16(ag, st, ckpt)
        e_emu = float(np.abs(emu - want).max())
        bound = 1.5 * e_emu + 5e-4
        got = {"per_layer": ag.select_action_batch(obs, use_checkpoint=ckpt, use_exploration=False).cpu().numpy()}
        if not ckpt:  # the bench's launch: actor(obs, fixed_encoder.zs(obs)) + sigma * z with sigma = 0
            L.exploration_noise_t.fill_(0.0)
            got["fused_select"] = L.fused.select(obs).cpu().numpy()
            L.exploration_noise_t.fill_(float(ag.hp.exploration_noise))
        for path, a in got.items():
            e_ref, e_to_emu = float(np.abs(a - want).max()), float(np.abs(a - emu).max())
            report[f"{key}.{path}"] = (e_ref, e_to_emu, e_emu)
            assert e_ref <= bound, f"{name}.{key} {path}: |gpu - ref| {e_ref:.3g} > {bound:.3g} (emulation {e_emu:.3g})"
            assert e_to_emu <= 2e-3, f"{name}.{key} {path}: |gpu - bf16 emulation| {e_to_emu:.3g}"
    print(name, {k: tuple(f"{x:.2e}" for x in v) for k, v in report.items()})
