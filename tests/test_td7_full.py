"""The TD7 update at the bench's own shape (BASELINE configs[1]: zs/enc 300,
critic/actor 320, 8 strata x 128 = 1,024 rows) against three golden
Agent.train() steps of the reference (tests/golden/td7_full.npz, made by
tests/golden/make_golden.py --only td7_full from Agent/TD7_multi_agent.py:211-293;
step 2 updates the actor), and configs[4]'s wide TD7 (every MLP and zs 1,024
wide) against two reference steps (tests/golden/td7_wide.npz).

Compared per step: the gradient every optimiser step consumes (sampled at 512
fixed indices per tensor, plus the float64 sum / L2 norm of the whole tensor),
the parameter change since initialisation (same samples), the LAP priorities
(:262) and the running Q-target bounds (:245-246).

Error measure: ``rel = ||x - ref||_2 / ||ref||_2`` over a tensor's samples.

Two yardsticks per gradient:
* the reference golden (trajectory level).  Some gradients are
  ill-conditioned -- the actor's are means of per-row terms that largely
  cancel, and the reference's own fp32 actor.l0.weight is 2e-3 away from the
  exact update -- so bounds scale with ``noise`` = rel(golden, an fp64
  restatement run freely from the same initial weights and batches:
  TD7Learner on torch-CPU in float64, test infrastructure);
* the fp64 restatement of THIS step, teacher-forced from the GPU learner's own
  state (weights, running bounds) with the GPU's operand rounding: every
  GEMM's operands rounded to bf16 / fp16 as the kernels load them (dP = dY
  act'(Y) rounded, bias gradients from the unrounded dP -- pinned per layer by
  tests/test_td7_dense_gpu.py).  What is left is fp32 accumulation order.
Bounds:
* fp32: both yardsticks max(1e-4, 4 noise); priorities 1e-5 elementwise;
  parameter changes (Adam: ~ +-lr per element, a sign test for small
  gradients) max(1e-3, 4 noise) where |g| > 0.02 rms(g).
* bf16 (the bench) / fp16 (configs[4]): this step's rounded restatement
  max(1e-2, 4 noise sqrt(u / 1e-7)).  Each layer alone equals the fp64 GEMM of
  its rounded operands to ~1e-6 (tests/test_td7_dense_gpu.py, 1e-4 bound);
  through a chain, the activations re-rounded to u = 2^-9 / 2^-11 at every
  layer turn fp32-level forward differences into one-ulp flips (a
  perturbation ~ sqrt(1e-7 u)) that saturating activations amplify in the
  backward (tanh near +-1 through 1 - y^2, ReLU at 0): measured up to 4e-3 on
  the wide actor's first layer in fp16 (tools/diag_actor_fp16.py).  The
  golden: max(3e-2, 4 noise, 1.5 x the rounded restatement's own distance
  from the golden) (unit roundoff 2^-9: ~3e-3 per
  rounded dot product, up to 7 GEMMs in a gradient chain, x3.5 margin; the
  ill-conditioned actor.l0.weight moves 3.7e-2 under bf16 rounding alone),
  priorities 3e-2; parameter changes 0.15 where |g| > 0.1 rms(g) (a
  trajectory sanity check: Adam's sign-like early steps follow the rounding
  noise of small gradients; the per-step gradients above are the real test).
"""
import numpy as np
import pytest
import torch

from helpers import (GOLDEN, TD7_FULL_LEARNING_STEPS, TD7_FULL_QBOUNDS, TD7_GOLDENS, td7_full_batch,
                     td7_full_sample_index)
from exo_amd.td7 import Critic, Hyperparameters, TD7Learner

TOL = {"fp32": dict(grad=1e-4, delta=1e-3, prio=1e-5, bound=1e-5, mask=0.02),
       "bf16": dict(grad=1e-2, golden=3e-2, delta=0.15, prio=1e-3, bound=1e-3, mask=0.1),
       "fp16": dict(grad=1e-2, golden=3e-2, delta=0.15, prio=1e-3, bound=1e-3, mask=0.1)}
COND = 4.0  # bounds scale with the reference's own fp32 deviation from fp64 ("noise")
# sqrt(u / eps32) with eps32 = 1e-7 (fp32-level perturbation): bf16 u = 2^-9, fp16 u = 2^-11
AMP = {"fp32": 1.0, "bf16": (2.0 ** -9 / 1e-7) ** 0.5, "fp16": (2.0 ** -11 / 1e-7) ** 0.5}
ROUND = {"fp32": None, "bf16": torch.bfloat16, "fp16": torch.float16}


def _golden(name="td7_full"):
    return np.load(f"{GOLDEN}/{name}.npz", allow_pickle=False)


def _cpu_learner(name="td7_full"):
    hp = Hyperparameters(**TD7_GOLDENS[name][0])
    torch.manual_seed(0)
    return TD7Learner(80, 7, hp, learning_steps=TD7_FULL_LEARNING_STEPS, device="cpu", fused_adam=False)


def _learner(device, precision="fp32", golden="td7_full", fused_f32=False):
    L = _cpu_learner(golden)
    if device == "cpu":
        L2 = L
    else:
        from exo_amd import fused
        f0 = fused.FUSED_F32
        fused.FUSED_F32 = fused_f32  # read when the learner builds its fused nets
        try:
            L2 = TD7Learner(80, 7, L.hp, learning_steps=TD7_FULL_LEARNING_STEPS, device=device, precision=precision)
        finally:
            fused.FUSED_F32 = f0
        assert (L2.fused is not None) == (fused_f32 or precision != "fp32") or golden != "td7_full"
        for name in ("actor", "critic", "encoder", "actor_target", "critic_target", "fixed_encoder",
                     "fixed_encoder_target"):
            getattr(L2, name).load_state_dict(getattr(L, name).state_dict())
    L2.min_target.fill_(TD7_FULL_QBOUNDS[0])
    L2.max_target.fill_(TD7_FULL_QBOUNDS[1])
    return L2


def _named(mod, mname, grad=False):
    """Reference-named flat tensors of a module (the critic's stacked heads split)."""
    out = {}
    if isinstance(mod, Critic):
        for k, names in enumerate(Critic.HEADS):
            for what in ("weight", "bias"):
                p = getattr(mod, f"{'w' if what == 'weight' else 'b'}{k}")
                t = p.grad if grad else p
                for h, n in enumerate(names):
                    out[f"{mname}.{n}.{what}"] = None if t is None else t[h]
        return out
    for n, p in mod.named_parameters():
        out[f"{mname}.{n}"] = p.grad if grad else p
    return out


def _sample(name, t):
    v = t.detach().float().cpu().numpy().reshape(-1)
    return v[td7_full_sample_index(name, v.size)], v


def _rel(x, ref):
    d = np.linalg.norm(ref.astype(np.float64))
    return np.linalg.norm((x - ref).astype(np.float64)) / max(d, 1e-30)


def _check_grads(g, step, L, mnames, precision, report, free, forced):
    """L's gradients vs the reference golden (trajectory level, bound scaled by
    the golden's own distance from exact arithmetic) and vs `forced`, the fp64
    restatement of this one step from L's own state with L's operand rounding."""
    tol = TOL[precision]
    worst, bad = 0.0, []
    for mname in mnames:
        for name, t in _named(getattr(L, mname), mname, grad=True).items():
            key = f"step{step}_grad.{name}"
            assert t is not None, f"no gradient for {name}"
            xs, _ = _sample(name, t)
            noise = free["noise"][key]
            r = _rel(xs, g[key])
            r_x = _rel(xs, forced[key])
            report[f"step{step}.grad.{name}"] = (r, r_x)
            worst = max(worst, r)
            # reduced precision: operands re-rounded to 8/11 bits turn the fp32-level
            # differences between this GPU step and its fp64 restatement into
            # occasional one-ulp flips, a perturbation ~ sqrt(eps32 * u) instead of
            # eps32 -- x sqrt(u / eps32) on the conditioning-scaled bound
            b_x = max(tol["grad"], COND * noise * AMP[precision])
            # reduced precision: the rounding's own effect on this tensor -- the
            # rounded restatement's distance from the golden -- x1.5 is allowed too
            b_g = b_x if precision == "fp32" else max(tol["golden"], COND * noise, 1.5 * _rel(forced[key], g[key]))
            if r > b_g or r_x > b_x:
                bad.append(f"{name}: vs golden {r:.3g} (bound {b_g:.3g}), vs this step's fp64 restatement "
                           f"{r_x:.3g} (bound {b_x:.3g})")
    assert not bad, f"step {step} gradients ({precision}): " + "; ".join(bad)
    return worst


class _RoundedGemm(torch.autograd.Function):
    """y = x @ w^T (+ b) with x, w rounded to `dt` (batched if 3-D); backward
    with dY rounded for both GEMMs (fp16: after scaling by 2^10), the bias
    gradient from the unrounded dY -- the reduced-precision td7_dense kernels'
    arithmetic, in float64."""

    @staticmethod
    def forward(ctx, x, w, b, dt):
        r = lambda t: t.to(dt).to(t.dtype)  # noqa: E731
        ctx.save_for_backward(x, w)
        ctx.dt, ctx.has_b = dt, b is not None
        y = r(x) @ r(w).transpose(-1, -2)
        return y + b.unsqueeze(-2) if b is not None else y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        r = lambda t: t.to(ctx.dt).to(t.dtype)  # noqa: E731
        gs = 1024.0 if ctx.dt == torch.float16 else 1.0  # fp16: dP scaled by 2^10 before rounding (grad_scale)
        rdy = (dy * gs).to(ctx.dt).to(dy.dtype) / gs
        dx = rdy @ r(w)
        xx = x if x.dim() == dy.dim() else x.unsqueeze(0).expand(dy.shape[0], *x.shape)
        dw = rdy.transpose(-1, -2) @ r(xx)
        if dw.dim() > w.dim():
            dw = dw.sum(0)
        if dx.dim() > x.dim():
            dx = dx.sum(0)
        db = dy.sum(-2) if ctx.has_b else None
        if db is not None and db.dim() > 1 and w.dim() == 2:
            db = db.sum(0)
        return dx, dw, db, None


class _rounded_matmuls:
    """Route the CPU path's F.linear / torch.baddbmm / torch.bmm through _RoundedGemm."""

    def __init__(self, dt):
        self.dt = dt

    def __enter__(self):
        import torch.nn.functional as F
        self.saved = (F.linear, torch.baddbmm, torch.bmm)
        dt = self.dt
        F.linear = lambda x, w, b=None: _RoundedGemm.apply(x, w, b, dt)
        torch.baddbmm = lambda b, x, wt: _RoundedGemm.apply(x, wt.transpose(1, 2), b.squeeze(1), dt)
        torch.bmm = lambda x, wt: _RoundedGemm.apply(x, wt.transpose(1, 2), None, dt)

    def __exit__(self, *a):
        import torch.nn.functional as F
        F.linear, torch.baddbmm, torch.bmm = self.saved


_EXACT = {}
NETS = ("actor", "critic", "encoder", "actor_target", "critic_target", "fixed_encoder", "fixed_encoder_target")


def _f64_learner(golden):
    """A float64 TD7Learner on the CPU (torch.optim.Adam, scalar state in fp64)."""
    L = _cpu_learner(golden)
    for name in NETS:
        getattr(L, name).double()
    L.actor_optimizer = torch.optim.Adam(L.actor.parameters(), lr=L.hp.actor_lr, weight_decay=1e-7)
    L.critic_optimizer = torch.optim.Adam(L.critic.parameters(), lr=L.hp.critic_lr, weight_decay=1e-7)
    L.encoder_optimizer = torch.optim.Adam(L.encoder.parameters(), lr=L.hp.encoder_lr, weight_decay=1e-7)
    f64 = dict(dtype=torch.float64)
    L.max, L.min = torch.tensor(-1e8, **f64), torch.tensor(1e8, **f64)
    L.min_target, L.max_target = torch.tensor(TD7_FULL_QBOUNDS[0], **f64), torch.tensor(TD7_FULL_QBOUNDS[1], **f64)
    L.target_policy_noise = L.target_policy_noise.double()
    return L


def _copy_state(dst, src):
    """dst (fp64 CPU learner) <- src's weights and running scalars."""
    with torch.no_grad():
        for name in NETS:
            for p, q in zip(getattr(dst, name).parameters(), getattr(src, name).parameters()):
                p.copy_(q.detach().double().cpu())
        for k in ("max", "min", "min_target", "max_target", "target_policy_noise"):
            getattr(dst, k).copy_(getattr(src, k).detach().double().cpu())
    dst.training_steps = src.training_steps


def _grads(L, mnames, step):
    out = {}
    for mname in mnames:
        for name, t in _named(getattr(L, mname), mname, grad=True).items():
            out[f"step{step}_grad.{name}"] = _sample(name, t.double())[0]
    return out


def _free_run(golden):
    """The unrounded fp64 restatement run freely from the golden's initial
    weights: its gradients per step, and noise[key] = rel(golden, it) -- how far
    the reference's own fp32 trajectory is from exact arithmetic."""
    if golden in _EXACT:
        return _EXACT[golden]
    g = _golden(golden)
    L = _f64_learner(golden)
    out = {}
    for step in range(TD7_GOLDENS[golden][1]):
        s, a, s2, r, nd, nz = td7_full_batch(step)
        b = [torch.tensor(x, dtype=torch.float64) for x in (s, a, s2, r, nd)]
        L.training_steps += 1
        L.phase_grads(*b, noise=torch.tensor(nz, dtype=torch.float64))
        out.update(_grads(L, ("encoder", "critic"), step))
        L.phase_steps()
        if L.training_steps % L.hp.policy_freq == 0:
            L.phase_actor_grads(b[0], b[1])
            out.update(_grads(L, ("actor",), step))
            L.phase_actor_step()
    _EXACT[golden] = {"grads": out, "noise": {k: _rel(g[k], v) for k, v in out.items()}}
    return _EXACT[golden]


def _run(device, precision="fp32", golden="td7_full", fused_f32=False):
    g = _golden(golden)
    free = _free_run(golden)
    tol = TOL[precision]
    L = _learner(device, precision, golden, fused_f32)
    X = _f64_learner(golden)  # teacher-forced restatement, reloaded from L before every phase
    rounding = _rounded_matmuls(ROUND[precision]) if ROUND[precision] is not None else None
    init = {}
    for mname in ("actor", "critic", "encoder"):
        for name, t in _named(getattr(L, mname), mname).items():
            init[name] = _sample(name, t)[0]
    report = {}

    def on_x(fn):
        if rounding:
            rounding.__enter__()
        try:
            fn()
        finally:
            if rounding:
                rounding.__exit__()

    for step in range(TD7_GOLDENS[golden][1]):
        s, a, s2, r, nd, nz = td7_full_batch(step)
        sums = np.array([x.astype(np.float64).sum() for x in (s, a, s2, r, nd, nz)])
        np.testing.assert_array_equal(sums, g[f"batch{step}_sum"])  # regenerated batch == the golden's
        b = [torch.tensor(x, device=device) for x in (s, a, s2, r, nd)]
        bx = [torch.tensor(x, dtype=torch.float64) for x in (s, a, s2, r, nd)]
        _copy_state(X, L)
        L.training_steps += 1
        X.training_steps += 1
        prio = L.phase_grads(*b, noise=torch.tensor(nz, device=device))
        on_x(lambda: X.phase_grads(*bx, noise=torch.tensor(nz, dtype=torch.float64)))
        forced = _grads(X, ("encoder", "critic"), step)
        report[f"grad{step}"] = _check_grads(g, step, L, ("encoder", "critic"), precision, report, free, forced)
        L.phase_steps()
        updated = ["critic", "encoder"]
        if L.training_steps % L.hp.policy_freq == 0:
            _copy_state(X, L)  # the just-updated critic
            L.phase_actor_grads(b[0], b[1])

            def actor_x():
                X._fixed_zs = X.fixed_encoder.zs(bx[0]).detach()
                X.phase_actor_grads(bx[0], bx[1])
            on_x(actor_x)
            forced = _grads(X, ("actor",), step)
            report[f"grad{step}_actor"] = _check_grads(g, step, L, ("actor",), precision, report, free, forced)
            L.phase_actor_step()
            updated.append("actor")
        assert sorted(updated) == sorted(g[f"step{step}_updated"].tolist())
        p = prio.detach().float().cpu().numpy().reshape(-1)
        if precision == "fp32":
            np.testing.assert_allclose(p, g[f"priority{step}"], rtol=tol["prio"], atol=tol["prio"])
        else:
            assert _rel(p - 1, g[f"priority{step}"] - 1) <= tol["golden"]
        for key, val in (("max", L.max), ("min", L.min)):
            ref = float(g[f"step{step}_{key}"])
            bnd = tol["bound"] if precision == "fp32" else tol["golden"]
            assert abs(float(val) - ref) <= bnd * max(1.0, abs(ref)), (key, float(val), ref)
        assert abs(float(L.target_policy_noise) - float(g[f"step{step}_target_policy_noise"])) < 1e-7
        worst, bad = 0.0, []
        for mname in ("actor", "critic", "encoder"):
            for name, t in _named(getattr(L, mname), mname).items():
                xs, _ = _sample(name, t)
                d, dref = xs - init[name], g[f"step{step}.{name}"] - g[f"init.{name}"]
                last = [k for k in range(step + 1) if f"step{k}_grad.{name}" in g.files]
                if last:  # entries whose latest gradient is well above the rounding noise
                    gr = g[f"step{last[-1]}_grad.{name}"].astype(np.float64)
                    keep = np.abs(gr) > tol["mask"] * np.sqrt(np.mean(gr ** 2))
                    d, dref = d[keep], dref[keep]
                noise_d = max([free["noise"].get(f"step{k}_grad.{name}", 0.0) for k in range(step + 1)])
                bound = max(tol["delta"], COND * noise_d)
                r = _rel(d, dref)
                worst = max(worst, r)
                if r > bound:
                    bad.append(f"{name}: rel {r:.3g} > {bound:.3g}")
        assert not bad, f"step {step} parameter changes ({precision}): " + "; ".join(bad)
        report[f"delta{step}"] = worst
    return report


@pytest.mark.parametrize("golden", ["td7_full", "td7_wide"])
def test_seeded_init_matches_reference_at_bench_shape(golden):
    """torch.manual_seed(0) initialisation at 300/320 (and 1,024) widths is bit-exact."""
    g = _golden(golden)
    L = _cpu_learner(golden)
    for mname in ("actor", "critic", "encoder"):
        for name, t in _named(getattr(L, mname), mname).items():
            xs, full = _sample(name, t)
            np.testing.assert_array_equal(xs, g[f"init.{name}"], err_msg=name)
            assert full.astype(np.float64).sum() == g[f"init.{name}.sum"], name


def test_three_train_steps_at_bench_shape_cpu():
    """The update math (TD7Learner on torch-CPU fp32) vs the reference."""
    _run("cpu")


def test_wide_train_steps_cpu():
    _run("cpu", golden="td7_wide")


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_three_train_steps_at_bench_shape_gpu(precision):
    """The HIP path (td7_dense kernels, loss / Adam kernels) at the bench's
    shape, exact fp32 MFMA and the bench's bf16 operands."""
    rep = _run("cuda", precision)
    print(precision, {k: f"{v:.2e}" for k, v in rep.items() if not isinstance(v, tuple)})


@pytest.mark.gpu
def test_three_train_steps_at_bench_shape_gpu_fused_fp32():
    """The row-tile-fused passes with exact fp32 operands (EXO_FUSED_F32,
    csrc/td7_fused.h Ty<PREC_F32>: v_mfma_f32_16x16x4_f32, fp32 images and
    weight-gradient operands) against the same golden at the fp32 bounds."""
    rep = _run("cuda", "fp32", fused_f32=True)
    print("fp32 fused", {k: f"{v:.2e}" for k, v in rep.items() if not isinstance(v, tuple)})


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_wide_train_steps_gpu(precision):
    """configs[4]'s wide TD7 (1,024-wide MLPs and zs; tests/golden/td7_wide.npz,
    2 reference steps, the second updating the actor) in exact fp32 and in
    the configuration's fp16 MFMA operands (unit roundoff 2^-11: the bf16
    bounds above hold with margin)."""
    rep = _run("cuda", precision, golden="td7_wide")
    print(precision, {k: f"{v:.2e}" for k, v in rep.items() if not isinstance(v, tuple)})
