"""Fused HIP AvgL1Norm (csrc/td7_ops.hip) vs the plain PyTorch fp32 expression
of Agent/TD7_multi_agent.py:53-54, forward and backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(1, 7), (1024, 300), (2048, 320), (3, 1000), (4096, 64)])
def test_avgl1norm_matches_torch(rows, cols):
    from exo_amd.ops import avg_l1_norm
    g = torch.Generator(device="cuda").manual_seed(rows * 7 + cols)
    x = torch.randn(rows, cols, device="cuda", generator=g)
    x[0, : cols // 2] = 0.0
    gy = torch.randn(rows, cols, device="cuda", generator=g)
    xa = x.clone().requires_grad_(True)
    ya = avg_l1_norm(xa)
    ya.backward(gy)
    xb = x.clone().requires_grad_(True)
    yb = xb / xb.abs().mean(-1, keepdim=True).clamp(min=1e-8)
    yb.backward(gy)
    torch.testing.assert_close(ya, yb, rtol=2e-6, atol=1e-6)
    torch.testing.assert_close(xa.grad, xb.grad, rtol=2e-5, atol=2e-5)


def test_avgl1norm_clamped_rows_and_3d():
    from exo_amd.ops import avg_l1_norm
    x = torch.zeros(2, 5, 16, device="cuda")
    x[1, 2] = torch.linspace(-1, 1, 16, device="cuda")
    xa = x.clone().requires_grad_(True)
    avg_l1_norm(xa).sum().backward()
    xb = x.clone().requires_grad_(True)
    (xb / xb.abs().mean(-1, keepdim=True).clamp(min=1e-8)).sum().backward()
    torch.testing.assert_close(xa.grad, xb.grad, rtol=1e-5, atol=1e-5)


def test_q_target_and_critic_loss_match_reference_expressions():
    """td7_q_target / td7_critic_loss vs the reference's torch expressions
    (Agent/TD7_multi_agent.py:240-262) on the same inputs."""
    from exo_amd import ops
    torch.manual_seed(3)
    B = 1024
    qt = torch.randn(2, B, device="cuda").t() * 5          # [B,2] view of [2,B], like Critic.forward's output
    reward = torch.randn(B, 1, device="cuda")
    not_done = (torch.rand(B, 1, device="cuda") > 0.1).float()
    lo, hi = torch.tensor(-3.0, device="cuda"), torch.tensor(4.0, device="cuda")
    rmax, rmin = torch.tensor(-1e8, device="cuda"), torch.tensor(1e8, device="cuda")
    out = ops.q_target(qt, reward, not_done, 0.99, lo, hi, rmax, rmin)
    ref = reward + not_done * 0.99 * qt.min(1, keepdim=True)[0].clamp(lo, hi)
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)
    assert float(rmax) == float(ref.max()) and float(rmin) == float(ref.min())

    q = (torch.randn(2, B, device="cuda").t() * 2).requires_grad_(True)
    q_ref = q.detach().clone().requires_grad_(True)
    loss, prio = ops.critic_loss(q, out, 0.4, 1.0)
    td = (q_ref - out).abs()
    loss_ref = torch.where(td < 1, 0.5 * td.pow(2), 1 * td).sum(1).mean()
    prio_ref = td.detach().max(1)[0].clamp(min=1.0).pow(0.4)
    torch.testing.assert_close(loss, loss_ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(prio, prio_ref, rtol=1e-6, atol=1e-6)
    loss.backward()
    loss_ref.backward()
    torch.testing.assert_close(q.grad, q_ref.grad, rtol=1e-6, atol=1e-8)


def test_noisy_action_and_mse_match_torch():
    from exo_amd import ops
    torch.manual_seed(4)
    a = torch.tanh(torch.randn(1024, 7, device="cuda") * 2)
    noise = torch.randn(1024, 7, device="cuda")
    for clip, scale in ((0.5, 1.0), (0.0, 2.0)):
        sig = torch.tensor(0.3, device="cuda")
        out = ops.noisy_action(a, noise, sig, 1e-3, clip=clip, scale=scale)
        e = noise * 0.3
        if clip > 0:
            e = e.clamp(-clip, clip)
        torch.testing.assert_close(out, (a + e).clamp(-1, 1) * scale, rtol=0, atol=1e-7)
        assert abs(float(sig) - (0.3 - 1e-3)) < 1e-7
    x = torch.randn(1024, 300, device="cuda", requires_grad=True)
    y = torch.randn(1024, 300, device="cuda")
    x2 = x.detach().clone().requires_grad_(True)
    l1 = ops.mse_loss(x, y)
    l2 = torch.nn.functional.mse_loss(x2, y)
    torch.testing.assert_close(l1, l2, rtol=1e-5, atol=1e-7)
    (3 * l1).backward()
    (3 * l2).backward()
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-6, atol=1e-9)


def test_critic_loss_and_grad_writes_dq_in_q_strides():
    """ops.critic_loss_and_grad: the same loss / priorities / dq as the
    autograd path, dq laid out like q (the [B,2] view of the heads' [2,B])."""
    from exo_amd import ops
    torch.manual_seed(4)
    B = 1000
    target = torch.randn(B, 1, device="cuda")
    q = torch.randn(2, B, device="cuda").t() * 2
    loss, prio, dq = ops.critic_loss_and_grad(q, target, 0.4, 1.0)
    assert dq.stride() == q.stride()
    qr = q.clone().requires_grad_(True)
    loss_r, prio_r = ops.critic_loss(qr, target, 0.4, 1.0)
    loss_r.backward()
    torch.testing.assert_close(loss, loss_r, rtol=0, atol=0)
    torch.testing.assert_close(prio, prio_r, rtol=0, atol=0)
    torch.testing.assert_close(dq, qr.grad, rtol=0, atol=0)


def test_flat_adam_step_many_matches_separate_steps():
    """FlatAdam.step_many (one td7_adam_step_multi launch over per-parameter
    gradients of several optimisers) == each optimiser's own step; a
    parameter without gradient is left alone."""
    import copy

    import torch.nn.functional as F
    from exo_amd.td7 import Critic, Encoder, FlatAdam
    torch.manual_seed(5)
    nets = [Encoder(80, 7, 300, 300, F.elu).cuda(), Critic(80, 7, 300, 320, F.elu).cuda()]
    twins = [copy.deepcopy(n) for n in nets]
    opts = [FlatAdam(nets[0], lr=3e-4, weight_decay=1e-7), FlatAdam(nets[1], lr=1e-3, weight_decay=1e-7)]
    refs = [FlatAdam(twins[0], lr=3e-4, weight_decay=1e-7), FlatAdam(twins[1], lr=1e-3, weight_decay=1e-7)]
    for it in range(3):
        for a, b in zip(nets, twins):
            for i, (p, q) in enumerate(zip(a.parameters(), b.parameters())):
                g = torch.randn_like(p)
                p.grad, q.grad = g.clone(), g.clone()
        skip = list(nets[0].parameters())[1]
        skip_before = skip.detach().clone()
        skip.grad = None
        FlatAdam.step_many(opts)
        # reference: the same update with the skipped parameter's gradient zero
        # and its value / moments restored afterwards
        rskip = list(twins[0].parameters())[1]
        keep = (rskip.detach().clone(), refs[0].state[rskip]["exp_avg"].clone(), refs[0].state[rskip]["exp_avg_sq"].clone())
        rskip.grad = torch.zeros_like(rskip)
        for o in refs:
            o.step()
        with torch.no_grad():
            rskip.copy_(keep[0])
            refs[0].state[rskip]["exp_avg"].copy_(keep[1])
            refs[0].state[rskip]["exp_avg_sq"].copy_(keep[2])
        torch.testing.assert_close(skip.detach(), skip_before, rtol=0, atol=0)
        for a, b in zip(nets, twins):
            for p, q in zip(a.parameters(), b.parameters()):
                torch.testing.assert_close(p.detach(), q.detach(), rtol=0, atol=0)
        for o, r in zip(opts, refs):
            assert float(o._step) == float(r._step) == it + 1


@pytest.mark.parametrize("cols", [300, 1000, 1024])
def test_avgl1norm_register_kernel_is_bit_identical(cols, monkeypatch):
    """avgl1_fwd_reg_kernel (r03d: rows of 257-1,024 kept in registers, one
    read) adds each lane's elements in the same order as avgl1_fwd_kernel."""
    from exo_amd.ops import avg_l1_norm
    torch.manual_seed(cols)
    x = torch.randn(4099, cols, device="cuda") * torch.rand(4099, 1, device="cuda") ** 4
    x[7] = 0.0  # a clamped row (mean < eps)
    with torch.no_grad():
        y_reg = avg_l1_norm(x)
        monkeypatch.setenv("EXO_AVGL1_REG", "0")
        y_old = avg_l1_norm(x)
    assert torch.equal(y_reg, y_old)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_avgl1norm_16bit_output_is_the_rounded_fp32_norm(prec):
    """td7_avgl1norm_fwd_h (r03d, select_action's AvgL1Norm outputs at the
    wide sizes): the fp32 kernel's values rounded to nearest even, bit for
    bit; outside 256 < cols <= 1,024 it answers EXO_ERANGE (None)."""
    from exo_amd import ops
    p = ops.PRECISIONS[prec]
    half = torch.bfloat16 if prec == "bf16" else torch.float16
    torch.manual_seed(3)
    for cols in (1024, 520):
        x = torch.randn(3001, cols, device="cuda") * torch.rand(3001, 1, device="cuda") ** 4
        x[5] = 0.0
        with torch.no_grad():
            y = ops.avg_l1_norm(x)
            h = ops.avg_l1_norm_h(x, p)
        assert h.dtype == half and torch.equal(h, y.to(half))
    assert ops.avg_l1_norm_h(torch.randn(64, 256, device="cuda"), p) is None
