"""td7_dense kernels (csrc/td7_dense.hip) against a plain PyTorch fp32
reference of the same layer: forward, input gradient, weight and bias
gradients, for every activation and the grouped (Q-head) layouts, at the TD7
shapes (K = 80, 87, 307, 620, 920; N = 300, 7, 1) and ragged M."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ACTS = {0: lambda y: y, 1: torch.relu, 2: torch.nn.functional.elu, 3: torch.tanh}


def _ref(x, w, b, act):
    if w.dim() == 3:
        xx = x if x.dim() == 3 else x.unsqueeze(0).expand(w.shape[0], *x.shape)
        y = torch.baddbmm(b.unsqueeze(1), xx, w.transpose(1, 2))
    else:
        y = torch.nn.functional.linear(x, w, b)
    return ACTS[act](y)


@pytest.fixture(params=["torch_fwd", "kernel_fwd"])
def fwd_mode(request):
    from exo_amd import ops
    old = ops._DenseFn.fwd_kernel_max_rows
    ops._DenseFn.fwd_kernel_max_rows = (1 << 30) if request.param == "kernel_fwd" else 0
    yield request.param
    ops._DenseFn.fwd_kernel_max_rows = old


def _check(x, w, b, act, tol=2e-5):
    from exo_amd import ops
    xs = [x.clone().requires_grad_(True) for _ in range(2)]
    ws = [w.clone().requires_grad_(True) for _ in range(2)]
    bs = [b.clone().requires_grad_(True) for _ in range(2)]
    y0 = ops._DenseFn.apply(xs[0], ws[0], bs[0], act)
    y1 = _ref(xs[1].double(), ws[1].double(), bs[1].double(), act)
    torch.testing.assert_close(y0.double(), y1, rtol=tol, atol=tol)
    g = torch.randn_like(y0)
    y0.backward(g)
    y1.backward(g.double())
    for a, r, n in ((xs[0].grad, xs[1].grad, "dx"), (ws[0].grad, ws[1].grad, "dW"), (bs[0].grad, bs[1].grad, "db")):
        scale = max(1.0, float(r.abs().max()))
        torch.testing.assert_close(a.double(), r.double(), rtol=tol, atol=tol * scale, msg=n)


@pytest.mark.parametrize("act", [0, 1, 2, 3])
@pytest.mark.parametrize("m,n,k", [(1024, 300, 80), (1000, 300, 307), (1024, 7, 300), (37, 300, 87), (4096, 300, 300),
                                   (3, 5, 4), (130, 6, 9), (1023, 65, 130)])
def test_dense_plain(act, m, n, k, fwd_mode):
    torch.manual_seed(m + n + k + act)
    x = torch.randn(m, k, device="cuda")
    w = torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(n, device="cuda")
    _check(x, w, b, act)


@pytest.mark.parametrize("shared", [True, False])
@pytest.mark.parametrize("n,k", [(320, 87), (320, 920), (1, 320)])
def test_dense_grouped(shared, n, k, fwd_mode):
    torch.manual_seed(n + k)
    m = 1024
    x = torch.randn(m, k, device="cuda") if shared else torch.randn(2, m, k, device="cuda")
    w = torch.randn(2, n, k, device="cuda") / k ** 0.5
    b = torch.randn(2, n, device="cuda")
    _check(x, w, b, 2)


def test_dense_strided_input_rows(fwd_mode):
    """A column slice of a wider buffer (row stride > K) is read in place."""
    from exo_amd import ops
    torch.manual_seed(5)
    big = torch.randn(512, 400, device="cuda")
    x = big[:, 50:350]
    w = torch.randn(64, 300, device="cuda") / 300 ** 0.5
    b = torch.randn(64, device="cuda")
    y = ops._DenseFn.apply(x, w, b, 2)
    torch.testing.assert_close(y, _ref(x, w, b, 2), rtol=2e-5, atol=2e-5)


def test_nets_fused_match_torch_layers():
    """Actor / Encoder / Critic forward + backward: fused kernels vs the
    reference's nn.Linear expression (activation codes unknown -> torch path)."""
    import copy

    import torch.nn.functional as F
    from exo_amd.td7 import Actor, Critic, Encoder
    torch.manual_seed(0)
    B = 256
    state, action = torch.randn(B, 80, device="cuda"), torch.rand(B, 7, device="cuda") * 2 - 1
    enc = Encoder(80, 7, 300, 300, F.elu).cuda()
    actor = Actor(80, 7, 300, 320, F.relu).cuda()
    critic = Critic(80, 7, 300, 320, F.elu).cuda()
    outs = []
    for fused in (True, False):
        e, a, c = copy.deepcopy(enc), copy.deepcopy(actor), copy.deepcopy(critic)
        if not fused:  # wrap the activations so act_code() does not recognise them
            e.activ = lambda t: F.elu(t)
            a.activ = lambda t: F.relu(t)
            c.activ = lambda t: F.elu(t)
        zs = e.zs(state)
        zsa = e.zsa(zs, action)
        pi = a(state, zs)
        q = c(state, pi, zsa, zs)
        loss = q.mean() + zsa.square().mean()
        loss.backward()
        outs.append((q.detach(), pi.detach(), [p.grad.clone() for m in (e, a, c) for p in m.parameters()]))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-4, atol=1e-5)
    for g0, g1 in zip(outs[0][2], outs[1][2]):
        torch.testing.assert_close(g0, g1, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("c0,c1,shared", [(0, 320, False), (0, 620, False), (320, 620, False), (80, 87, True),
                                         (1, 919, False)])
def test_dense_bwd_data_column_window(c0, c1, shared):
    """td7_dense_bwd_data_cols writes exactly the input columns [c0, c1) of dX,
    equal to the full input gradient there."""
    from exo_amd import _native as nat
    torch.manual_seed(c0 + c1)
    m, n, k = 1000, 320, 87 if shared else 920
    c1 = min(c1, k)
    dy = torch.randn(2, m, n, device="cuda")
    y = torch.randn(2, m, n, device="cuda")
    w = torch.randn(2, n, k, device="cuda") / k ** 0.5
    shape = (m, k) if shared else (2, m, k)
    full = torch.zeros(shape, device="cuda")
    win = torch.full(shape, 7.0, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for out, (a, b) in ((full, (0, k)), (win, (c0, c1))):
        nat.check(nat.lib().td7_dense_bwd_data_cols(nat.ptr(dy), m * n, n, nat.ptr(y), m * n, n, nat.ptr(w),
                                                    nat.ptr(out), m * k, k, 2, int(shared), m, n, k, a, b, 2, s),
                  "td7_dense_bwd_data_cols")
    torch.cuda.synchronize()
    torch.testing.assert_close(win[..., c0:c1], full[..., c0:c1], rtol=0, atol=0)
    assert (win[..., :c0] == 7.0).all() and (win[..., c1:] == 7.0).all()
    bad = nat.lib().td7_dense_bwd_data_cols(nat.ptr(dy), m * n, n, nat.ptr(y), m * n, n, nat.ptr(w), nat.ptr(full),
                                            m * k, k, 2, int(shared), m, n, k, 5, 5, 2, s)
    assert bad != 0


@pytest.mark.parametrize("case", ["plain2", "grouped3", "grouped_shared2", "pairs"])
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_dense_cat_matches_concatenation(case, prec):
    """td7_dense_fwd_cat / bwd_weight_cat / per-part bwd_data against the same
    layer on torch.cat of the parts: forward, every part's gradient (only for
    parts that require one), dW and db."""
    from exo_amd import ops
    torch.manual_seed(hash(case) % 1000)
    M = 777
    mk = lambda *s: torch.randn(*s, device="cuda")
    if case == "plain2":      # Encoder.zsa1: [zs | action]
        parts, w, b, need = [mk(M, 300), mk(M, 7)], mk(300, 307) / 17, mk(300), [True, True]
    elif case == "grouped3":  # critic layer 1: [q (per head) | zsa | zs (shared)]
        parts, w, b, need = [mk(2, M, 320), mk(M, 300), mk(M, 300)], mk(2, 320, 920) / 30, mk(2, 320), [True, True, False]
    elif case == "grouped_shared2":  # critic layer 0: [state | action], both shared
        parts, w, b, need = [mk(M, 80), mk(M, 7)], mk(2, 320, 87) / 9, mk(2, 320), [False, True]
    else:                     # paired fixed encoders' zsa1: [zs2 | actions2] per group
        parts, w, b, need = [mk(2, M, 300), mk(2, M, 7)], mk(2, 300, 307) / 17, mk(2, 300), [True, False]
    outs = []
    for fused in (True, False):
        ps = [p.clone().requires_grad_(r) for p, r in zip(parts, need)]
        ww, bb = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        with ops.matrix_precision(prec):
            if fused:
                y = ops.dense_cat(ps, ww, bb, 2)
            else:
                if w.dim() == 3 and any(p.dim() == 3 for p in ps):
                    full = torch.cat([p if p.dim() == 3 else p.unsqueeze(0).expand(w.shape[0], *p.shape)
                                      for p in ps], -1)
                else:
                    full = torch.cat(ps, -1)
                y = ops.dense(full, ww, bb, 2)
        torch.manual_seed(7)  # the same output gradient for both
        y.backward(torch.randn_like(y))
        outs.append((y.detach(), ww.grad, bb.grad, [p.grad for p in ps]))
    tol = 1e-5 if prec == "fp32" else 2e-3
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=tol, atol=tol)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=tol, atol=tol * 30)
    torch.testing.assert_close(outs[0][2], outs[1][2], rtol=tol, atol=tol * 30)
    for a, r, n in zip(outs[0][3], outs[1][3], need):
        if n:
            torch.testing.assert_close(a, r, rtol=tol, atol=tol * 10)
        else:
            assert a is None and r is None


def test_dense_cat_rejects_bad_layouts():
    from exo_amd import _native as nat
    import ctypes
    x = torch.zeros(8, 6, device="cuda")
    w = torch.zeros(4, 12, device="cuda")
    y = torch.zeros(8, 4, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    P = (ctypes.c_void_p * 2)(x.data_ptr(), x.data_ptr())
    sg, ld = (ctypes.c_long * 2)(0, 0), (ctypes.c_long * 2)(6, 6)
    assert nat.lib().td7_dense_fwd_cat(2, P, sg, ld, (ctypes.c_int32 * 2)(6, 6), nat.ptr(w), None, nat.ptr(y), 32, 4,
                                       1, 8, 4, 0, s) != 0  # interior width 6 not a multiple of 4
    assert nat.lib().td7_dense_fwd_cat(2, P, sg, ld, (ctypes.c_int32 * 2)(8, 2), nat.ptr(w), None, nat.ptr(y), 32, 4,
                                       1, 8, 4, 0, s) != 0  # last part narrower than 4
    assert nat.lib().td7_dense_fwd_cat(5, P, sg, ld, (ctypes.c_int32 * 2)(4, 4), nat.ptr(w), None, nat.ptr(y), 32, 4,
                                       1, 8, 4, 0, s) != 0  # too many parts


def test_critic_actor_update_gradients_with_partial_inputs():
    """The actor-update pattern: the critic's zs and the encoder's zs are
    constants, only the action path needs input gradients (column windows)."""
    import copy

    import torch.nn.functional as F
    from exo_amd.td7 import Actor, Critic, Encoder
    torch.manual_seed(1)
    B = 300
    state = torch.randn(B, 80, device="cuda")
    enc = Encoder(80, 7, 300, 300, F.elu).cuda()
    actor = Actor(80, 7, 300, 320, F.relu).cuda()
    critic = Critic(80, 7, 300, 320, F.elu).cuda()
    with torch.no_grad():
        zs = enc.zs(state)
    outs = []
    for fused in (True, False):
        e, a, c = copy.deepcopy(enc), copy.deepcopy(actor), copy.deepcopy(critic)
        if not fused:
            e.activ = lambda t: F.elu(t)
            a.activ = lambda t: F.relu(t)
            c.activ = lambda t: F.elu(t)
        pi = a(state, zs)
        q = c(state, pi, e.zsa(zs, pi), zs)
        (-q.mean()).backward()
        outs.append([p.grad.clone() for p in a.parameters()])
    for g0, g1 in zip(*outs):
        torch.testing.assert_close(g0, g1, rtol=1e-3, atol=1e-6)


# ------------------------------------------------------------ bf16 / fp16 MFMA
_ROUND = {"bf16": torch.bfloat16, "fp16": torch.float16}
# the backward's gradient operand dP is rounded after scaling by 2^10 in fp16
# (csrc/td7_dense_kernels.h grad_scale: keeps small gradients out of fp16's
# subnormal range); exact power of two, so this is the rounding model
_GSCALE = {"bf16": 1.0, "fp16": 1024.0}


def _rd_grad(t, prec):
    return (t * _GSCALE[prec]).to(_ROUND[prec]).double() / _GSCALE[prec]
_GRAD = {0: lambda y: torch.ones_like(y), 1: lambda y: (y > 0).to(y.dtype), 2: lambda y: torch.where(y > 0, 1.0, y + 1),
         3: lambda y: 1 - y * y}


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("act", [0, 2, 3])
@pytest.mark.parametrize("m,n,k,g,shared", [(1024, 300, 80, 0, False), (1000, 300, 307, 0, False),
                                            (4096, 300, 300, 0, False), (37, 7, 87, 0, False),
                                            (1024, 320, 920, 2, False), (1024, 320, 87, 2, True),
                                            (1024, 1, 320, 2, False),
                                            # configs[4] (wide TD7, 1,024 x 4): hidden layers, the critic's
                                            # [q|zsa|zs] layer, the shared first layer, 8 x 1,024 rows
                                            (1024, 1024, 1024, 0, False), (1024, 1024, 3072, 2, False),
                                            (1024, 1024, 87, 2, True), (8192, 1024, 1024, 0, False),
                                            (8192, 1024, 3072, 2, False)])
def test_dense_reduced_precision_is_the_gemm_of_rounded_operands(prec, act, m, n, k, g, shared):
    """bf16 / fp16 operand mode: each GEMM equals the fp64 GEMM of the
    operands rounded to nearest even (dP = dY * act'(Y) rounded as loaded);
    the bias gradient is the fp32 column sum of the unrounded dP.  Covers the
    TD7 default widths and the wide configuration (forward, bwd-data and
    wgrad at 1,024 / 3,072)."""
    from exo_amd import ops
    torch.manual_seed(m + n + k + act)
    rd = lambda t: t.to(_ROUND[prec]).double()  # noqa: E731
    x = torch.randn(m, k, device="cuda") if (g == 0 or shared) else torch.randn(g, m, k, device="cuda")
    w = (torch.randn(n, k, device="cuda") if g == 0 else torch.randn(g, n, k, device="cuda")) / k ** 0.5
    b = torch.randn(n, device="cuda") if g == 0 else torch.randn(g, n, device="cuda")
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    with ops.matrix_precision(prec):
        y = ops._DenseFn.apply(xr, wr, br, act)
    xx = rd(x) if (g == 0 or not shared) else rd(x).unsqueeze(0).expand(g, m, k)
    pre = (xx @ rd(w).transpose(-1, -2)) + b.double().unsqueeze(-2)
    ref = ACTS[act](pre)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    dp32 = dy * _GRAD[act](y.detach())
    dp = _rd_grad(dp32, prec)
    dx = dp @ rd(w)
    if g and shared:
        dx = dx.sum(0)
    dw = dp.transpose(-1, -2) @ xx
    db = dp32.double().sum(-2)
    # tanh: the kernel forms 1 - y*y with one fused multiply-add, torch with two
    # roundings; near |y| = 1 that ulp-level difference flips the rounding of
    # some dP elements to 16 bits
    tg = 1e-3 if act == 3 else 1e-4
    for got, r, name, tol in ((xr.grad, dx, "dx", tg), (wr.grad, dw, "dW", tg), (br.grad, db, "db", 1e-5)):
        scale = max(1.0, float(r.abs().max()))
        torch.testing.assert_close(got.double(), r, rtol=tol, atol=tol * scale, msg=name)


def test_reduced_precision_rejects_bad_codes():
    from exo_amd import _native as nat
    x = torch.randn(4, 4, device="cuda")
    y = torch.empty(4, 4, device="cuda")
    rc = nat.lib().td7_dense_fwd(nat.ptr(x), 0, 4, nat.ptr(x), None, nat.ptr(y), 16, 4, 1, 4, 4, 4, 3 << 8,
                                 nat.stream_ptr(x.device))
    assert rc == -22


def test_encoder_zs_half_grad_matches_autograd_slices():
    """ops.encoder_zs_half_grad (forward over 2B rows, backward over the first
    B) == the reference expression zs(cat)[:B] / [B:].detach() under autograd."""
    import copy

    import torch.nn.functional as F
    from exo_amd import ops
    from exo_amd.td7 import Encoder
    torch.manual_seed(9)
    B = 300
    sn = torch.randn(2, B, 80, device="cuda")
    enc = Encoder(80, 7, 300, 300, F.elu).cuda()
    ref = copy.deepcopy(enc)
    x = ops.pair_rows(sn[0], sn[1])
    assert x.data_ptr() == sn.data_ptr()
    zs, nxt = ops.encoder_zs_half_grad(x.view(2 * B, 80), B, 2, [(l.weight, l.bias) for l in (enc.zs1, enc.zs2, enc.zs3)])
    allr = ref.zs(torch.cat([sn[0], sn[1]], 0))
    zr, nr = allr[:B], allr[B:].detach()
    torch.testing.assert_close(zs, zr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(nxt, nr, rtol=1e-5, atol=1e-5)
    assert not nxt.requires_grad
    g = torch.randn_like(zs)
    zs.backward(g)
    zr.backward(g)
    for p, q in zip(enc.parameters(), ref.parameters()):
        if p.grad is None:
            assert q.grad is None or not q.grad.any()
            continue
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("case", ["plain", "pair3d", "critic_cat", "ragged"])
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_dense_norm_matches_separate_ops(case, prec):
    """ops.dense_norm (td7_dense_fwd_norm[_cat]: GEMM + bias + AvgL1Norm in one
    launch) == AvgL1Norm(dense(...)) forward and backward."""
    from exo_amd import ops
    torch.manual_seed(len(case))
    mk = lambda *s: torch.randn(*s, device="cuda")
    if case == "plain":        # Actor.l0 / Encoder.zs3
        parts, w, b = [mk(1024, 80)], mk(320, 80) / 9, mk(320)
    elif case == "pair3d":     # paired fixed encoders' zs3
        parts, w, b = [mk(2, 1024, 300)], mk(2, 300, 300) / 17, mk(2, 300)
    elif case == "critic_cat":  # critic q = AvgL1Norm(Linear([state | action])), both heads
        parts, w, b = [mk(1024, 80), mk(1024, 7)], mk(2, 320, 87) / 9, mk(2, 320)
    else:                      # ragged rows and columns
        parts, w, b = [mk(37, 19)], mk(45, 19) / 4, mk(45)
    outs = []
    for fused in (True, False):
        ps = [p.clone().requires_grad_(True) for p in parts]
        ww, bb = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        with ops.matrix_precision(prec):
            if fused:
                y = ops.dense_norm(ps, ww, bb)
            else:
                y = ops.avg_l1_norm(ops.dense_cat(ps, ww, bb, 0) if len(ps) > 1 else ops.dense(ps[0], ww, bb, 0))
        torch.manual_seed(3)
        y.backward(torch.randn_like(y))
        outs.append((y.detach(), ww.grad, bb.grad, [p.grad for p in ps]))
    tol = 2e-5 if prec == "fp32" else 2e-3
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=tol, atol=tol)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=tol, atol=tol * 20)
    torch.testing.assert_close(outs[0][2], outs[1][2], rtol=tol, atol=tol * 20)
    for a, r in zip(outs[0][3], outs[1][3]):
        torch.testing.assert_close(a, r, rtol=tol, atol=tol * 20)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("g,m,n,k,cat", [(1, 1100, 130, 333, False), (2, 1024, 320, 920, True), (1, 4096, 300, 300, False),
                                         (1, 1031, 70, 259, True), (2, 2048, 1024, 1027, False)])
def test_lds_forward_kernel_is_the_gemm_of_rounded_operands(prec, g, m, n, k, cat):
    """The LDS-tiled forward (td7_dense_fwd / _fwd_cat with 16-bit operands at
    >= 1,024 rows and K >= 256): ragged edges, groups, concatenated inputs."""
    from exo_amd import ops
    torch.manual_seed(m + n + k)
    dt = _ROUND[prec]
    w = torch.randn(g, n, k, device="cuda") / k ** 0.5 if g > 1 else torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(g, n, device="cuda") if g > 1 else torch.randn(n, device="cuda")
    if cat:  # [q (per group) | e (shared)] with a 4-aligned boundary
        k0 = (k // 3) // 4 * 4
        parts = [torch.randn(g, m, k0, device="cuda") if g > 1 else torch.randn(m, k0, device="cuda"),
                 torch.randn(m, k - k0, device="cuda")]
        with ops.matrix_precision(prec):
            y = ops.dense_cat(parts, w, b, 2)
        x = torch.cat([parts[0], parts[1].expand(g, m, k - k0) if g > 1 else parts[1]], -1)
    else:
        x = torch.randn(g, m, k, device="cuda") if g > 1 else torch.randn(m, k, device="cuda")
        with ops.matrix_precision(prec):
            y = ops.dense(x, w, b, 2)
    ref = torch.nn.functional.elu(x.to(dt).float() @ w.to(dt).float().transpose(-1, -2) + b.unsqueeze(-2))
    torch.testing.assert_close(y, ref.reshape(y.shape), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("m", [1024, 8192])
def test_wide_critic_concat_layer_fp16(m):
    """configs[4]'s critic layer 1 as the model runs it: [q | zsa | zs] read in
    place (q per head [2,M,1024], zsa and zs shared), W [2, 1024, 3072], fp16
    operands: forward, every part's gradient and dW / db against the fp64 GEMM
    of the rounded operands."""
    from exo_amd import ops
    torch.manual_seed(m)
    rd = lambda t: t.to(torch.float16).double()  # noqa: E731
    q = torch.randn(2, m, 1024, device="cuda")
    zsa, zs = torch.randn(m, 1024, device="cuda"), torch.randn(m, 1024, device="cuda")
    w = torch.randn(2, 1024, 3072, device="cuda") / 3072 ** 0.5
    b = torch.randn(2, 1024, device="cuda")
    parts = [t.clone().requires_grad_(True) for t in (q, zsa, zs)]
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    with ops.matrix_precision("fp16"):
        y = ops.dense_cat(parts, wr, br, 2)
    x = torch.cat([rd(q), rd(zsa).unsqueeze(0).expand(2, m, 1024), rd(zs).unsqueeze(0).expand(2, m, 1024)], -1)
    ref = torch.nn.functional.elu(x @ rd(w).transpose(-1, -2) + b.double().unsqueeze(-2))
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    dp32 = dy * _GRAD[2](y.detach())
    dp = _rd_grad(dp32, "fp16")
    dx = dp @ rd(w)                                       # [2, M, 3072]
    want = {"q": dx[..., :1024], "zsa": dx[..., 1024:2048].sum(0), "zs": dx[..., 2048:].sum(0),
            "dW": dp.transpose(-1, -2) @ x, "db": dp32.double().sum(-2)}
    got = {"q": parts[0].grad, "zsa": parts[1].grad, "zs": parts[2].grad, "dW": wr.grad, "db": br.grad}
    for name, r in want.items():
        scale = max(1.0, float(r.abs().max()))
        tol = 1e-5 if name == "db" else 1e-4
        torch.testing.assert_close(got[name].double(), r, rtol=tol, atol=tol * scale, msg=name)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("g,m,n,k,cat", [(1, 8200, 1000, 1032, False), (2, 8192, 1024, 3072, True),
                                         (1, 16384, 1024, 2048, True), (1, 8192, 1024, 1000, True),
                                         (2, 4100, 520, 1024, False)])
def test_big_forward_kernel_is_the_gemm_of_rounded_operands(prec, g, m, n, k, cat):
    """The 256 x 128-tile forward (dense_fwd_big_kernel: >= 256 such tiles, K %
    8 == 0; the wide configuration's update at 8 x 1,024 rows and its policy
    over 65,536 envs): ragged M, N and K (K = 1,032: a partial 64-deep slice),
    two groups, concatenated inputs with 64-aligned boundaries ([q | zsa | zs],
    [a | zs]) and one with a boundary at 384 + 616 (k = 1,000: not 64-aligned,
    the dispatcher keeps the LDS kernel) -- the GEMM of the operands rounded
    to 16 bits with fp32 accumulation, ELU epilogue."""
    from exo_amd import ops
    torch.manual_seed(m + n + k + g)
    dt = _ROUND[prec]
    w = torch.randn(g, n, k, device="cuda") / k ** 0.5 if g > 1 else torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(g, n, device="cuda") if g > 1 else torch.randn(n, device="cuda")
    if cat:
        widths = [k // 3] * 3 if k == 3072 else ([k // 2] * 2 if k == 2048 else [384, k - 384])
        parts = [torch.randn(g, m, widths[0], device="cuda") if g > 1 else torch.randn(m, widths[0], device="cuda")]
        parts += [torch.randn(m, wd, device="cuda") for wd in widths[1:]]
        with ops.matrix_precision(prec):
            y = ops.dense_cat(parts, w, b, 2)
        x = torch.cat([parts[0]] + [p.expand(g, m, p.shape[-1]) if g > 1 else p for p in parts[1:]], -1)
    else:
        x = torch.randn(g, m, k, device="cuda") if g > 1 else torch.randn(m, k, device="cuda")
        with ops.matrix_precision(prec):
            y = ops.dense(x, w, b, 2)
    ref = torch.nn.functional.elu(x.to(dt).float() @ w.to(dt).float().transpose(-1, -2) + b.unsqueeze(-2))
    torch.testing.assert_close(y, ref.reshape(y.shape), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("g,m,n,k,cat", [(1, 8200, 1000, 1032, False), (2, 8192, 1024, 3072, True),
                                         (1, 16384, 1024, 2048, True), (2, 8192, 520, 1024, False)])
def test_big_forward_with_16bit_weights_is_bit_identical(prec, g, m, n, k, cat):
    """td7_dense_fwd*_w16 (r03d): the large-layer kernel reading W already
    rounded to bf16 / fp16 (W.to(dtype), one conversion per call) returns
    exactly what it returns rounding the fp32 W itself (RNE both ways)."""
    from exo_amd import ops
    torch.manual_seed(g + m + n + k)
    w = torch.randn(g, n, k, device="cuda") / k ** 0.5 if g > 1 else torch.randn(n, k, device="cuda") / k ** 0.5
    w[..., 0, :4] = torch.tensor([1.0 + 2.0 ** -9, -3.0e-8, 65504.0, 1.0e-30])  # ties, tiny, fp16 max, bf16-only
    b = torch.randn(g, n, device="cuda") if g > 1 else torch.randn(n, device="cuda")
    if cat:
        widths = [k // 3] * 3 if k == 3072 else [k // 2] * 2
        parts = [torch.randn(g, m, widths[0], device="cuda") if g > 1 else torch.randn(m, widths[0], device="cuda")]
        parts += [torch.randn(m, wd, device="cuda") for wd in widths[1:]]
        run = lambda: ops.dense_cat(parts, w, b, 2)  # noqa: E731
    else:
        x = torch.randn(g, m, k, device="cuda") if g > 1 else torch.randn(m, k, device="cuda")
        run = lambda: ops.dense(x, w, b, 2)  # noqa: E731
    old = ops.W16_MIN_ROWS
    try:
        with ops.matrix_precision(prec):
            ops.W16_MIN_ROWS = 1 << 62
            y32 = run()
            ops.W16_MIN_ROWS = 8192
            y16 = run()
    finally:
        ops.W16_MIN_ROWS = old
    assert torch.equal(y16, y32)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_inference_chain_with_16bit_activations_is_bit_identical(prec):
    """ops.dense / dense_cat half_out (r03d, td7_dense_fwd_h / _cat_h): the
    wide configuration's select chain -- zs1 -> zs2 (16-bit out) -> zs3 +
    AvgL1Norm and l0 -> l1 = [a | zs] (16-bit out) -> l2 -> l3 -- under no_grad
    equals the fp32-activation chain bit for bit (every consumer rounds its
    input to the same 16-bit values); with autograd on nothing is 16-bit."""
    from exo_amd import ops
    from exo_amd.td7 import Actor, Encoder
    torch.manual_seed(5)
    enc = Encoder(80, 7, 1024, 1024).cuda()
    actor = Actor(80, 7, 1024, 1024).cuda()
    state = torch.randn(8192, 80, device="cuda")

    def chain(half_zs=False):
        zs = enc.zs(state, half_out=half_zs)
        return zs, actor(state, zs)

    old = ops.W16_MIN_ROWS
    try:
        with ops.matrix_precision(prec), torch.no_grad():
            ops.W16_MIN_ROWS = 1 << 62
            zs32, a32 = chain()
            ops.W16_MIN_ROWS = 8192
            zs16, a16 = chain()
            # r03d: the AvgL1Norm outputs as 16-bit (td7_avgl1norm_fwd_h) and
            # l1 reading both segments of [a | zs] as 16-bit (select_action)
            zsh, ah = chain(half_zs=True)
            h = ops.dense(state, enc.zs1.weight, enc.zs1.bias, 2)
            assert ops.dense(h, enc.zs2.weight, enc.zs2.bias, 2, half_out=True).dtype != torch.float32
        with ops.matrix_precision(prec):
            h = ops.dense(state, enc.zs1.weight, enc.zs1.bias, 2)
            assert ops.dense(h, enc.zs2.weight, enc.zs2.bias, 2, half_out=True).dtype == torch.float32
    finally:
        ops.W16_MIN_ROWS = old
    assert zs16.dtype == a16.dtype == torch.float32
    assert torch.equal(zs16, zs32) and torch.equal(a16, a32)
    half = torch.bfloat16 if prec == "bf16" else torch.float16
    assert zsh.dtype == half and torch.equal(zsh, zs32.to(half))
    assert ah.dtype == torch.float32 and torch.equal(ah, a32)


@pytest.fixture(params=[2, 1], ids=["xl8", "xl"])
def xl_variant(request):
    """The 256 x 256-tile forward's kernel (td7_dense_set_xl): 2 the two-slice
    LDS-DMA kernel (r05, the default where K % 64 == 0), 1 the register-staged
    one (any K % 8 == 0)."""
    from exo_amd import _native as nat
    prev = nat.lib().td7_dense_set_xl(request.param)
    yield request.param
    nat.lib().td7_dense_set_xl(prev)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("m,n,k,cat,half_out", [(16384, 1024, 1024, False, True), (16500, 1000, 1024, False, True),
                                                (16384, 1024, 1024, False, False), (16384, 1024, 1032, False, True),
                                                (16400, 1024, 1024, True, True), (16384, 520, 2048, False, True),
                                                (65536, 256, 64, False, True), (16384, 1024, 320, True, True)])
def test_xl_forward_kernel_is_the_gemm_of_rounded_operands(prec, m, n, k, cat, half_out, xl_variant):
    """The 256 x 256-tile forward of 16-bit inference chains (r05:
    dense_fwd_xl8_kernel, LDS-DMA staging, at >= 256 such tiles and K % 64 ==
    0; dense_fwd_xl_kernel otherwise -- K = 1,032 here -- and for every shape
    through td7_dense_set_xl; K = 64 and 320: one and five slices): 16-bit X (and
    16-bit [a | zs] segments), ragged M and N (16,500 x 1,000: partial tiles
    both ways), 16-bit or fp32 output -- the GEMM of the rounded operands with
    fp32 accumulation + ELU, to fp32 summation-order tolerance (1e-4; the
    16-bit output to one rounding of it).  Unlike the 256 x 128 kernel it is
    not bit-identical to the fp32-activation chain (32x32x16 MFMAs sum in
    another order)."""
    from exo_amd import ops
    torch.manual_seed(m + n + k)
    dt = _ROUND[prec]
    w = torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(n, device="cuda")
    if cat:
        parts = [torch.randn(m, 256, device="cuda").to(dt), torch.randn(m, k - 256, device="cuda").to(dt)]
        with ops.matrix_precision(prec), torch.no_grad():
            y = ops.dense_cat(parts, w, b, 2, half_out=half_out)
        x = torch.cat(parts, -1)
    else:
        x = torch.randn(m, k, device="cuda").to(dt)
        with ops.matrix_precision(prec), torch.no_grad():
            y = ops.dense(x, w, b, 2, half_out=half_out)
    assert y.dtype == (dt if half_out else torch.float32)
    ref = torch.nn.functional.elu(x.float() @ w.to(dt).float().t() + b)
    if half_out:
        # within one 16-bit rounding of the fp32 result
        ulp = 2.0 ** -8 if prec == "bf16" else 2.0 ** -11
        excess = (y.float() - ref).abs() - ulp * ref.abs()
        assert float(excess.max()) <= 1e-4, float(excess.max())
    else:
        torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("m,n,k", [(8192, 7, 1024), (65536, 7, 1024), (8200, 7, 1000), (9000, 20, 260)])
def test_small_head_reading_16bit_x_is_bit_identical(prec, m, n, k):
    """r05: a 16-bit X into a layer the fp32 path runs on dense_fwd_kernel
    (the actor's 7-wide tanh head l3 after a 16-bit l2 on the wide select
    chain) takes its AH variant -- 8-byte loads of the values the fp32 path
    rounds to: bit-identical to feeding the same values as fp32, at both
    tilings (16 x 16 below 2,048 tiles, 32 x 32 above), K with a 16-wide
    tail (1,000) and a 20-wide head."""
    from exo_amd import ops
    torch.manual_seed(m + n + k)
    dt = _ROUND[prec]
    x16 = torch.randn(m, k, device="cuda").to(dt)
    w = torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(n, device="cuda")
    with ops.matrix_precision(prec), torch.no_grad():
        y16 = ops._dense_h(x16, w, b, ops.ACT_CODES["tanh"], False)  # the kernel itself (None = EXO_ERANGE)
        y32 = ops.dense(x16.float(), w, b, ops.ACT_CODES["tanh"])
        y_op = ops.dense(x16, w, b, ops.ACT_CODES["tanh"])
    assert y16 is not None and y16.dtype == torch.float32
    assert torch.equal(y16, y32) and torch.equal(y_op, y32)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_xl_forward_grouped_through_the_abi(prec):
    """td7_dense_fwd_h with two groups (W [2, N, K], X [2, M, K], both 16-bit)
    at the 256 x 256-tile sizes: each group's output equals that group's GEMM
    of the rounded operands (the grid's z = group; ops never sends groups
    here, the C ABI allows it)."""
    from exo_amd import _native as nat
    from exo_amd import ops
    torch.manual_seed(11)
    dt = _ROUND[prec]
    G, m, n, k = 2, 16400, 1024, 1024
    x16 = torch.randn(G, m, k, device="cuda").to(dt)
    w = torch.randn(G, n, k, device="cuda") / k ** 0.5
    b = torch.randn(G, n, device="cuda")
    w16 = w.to(dt)
    y16 = torch.empty(G, m, n, device="cuda", dtype=dt)
    rc = nat.lib().td7_dense_fwd_h(None, nat.ptr(x16), m * k, k, nat.ptr(w), nat.ptr(b), None, nat.ptr(y16), m * n, n,
                                   G, m, n, k, 2 | ops.PRECISIONS[prec] << 8, nat.ptr(w16),
                                   nat.stream_ptr(x16.device))
    assert rc == 0
    ref = torch.nn.functional.elu(x16.float() @ w16.float().transpose(-1, -2) + b.unsqueeze(-2))
    ulp = 2.0 ** -8 if prec == "bf16" else 2.0 ** -11
    excess = (y16.float() - ref).abs() - ulp * ref.abs()
    assert float(excess.max()) <= 1e-4, float(excess.max())
