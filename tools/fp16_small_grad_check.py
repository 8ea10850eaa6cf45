"""fp16-operand backward at gradient scales down to the wide encoder's
(d mse / d pred ~ 2 (pred - target) / (B zs_dim) ~ 1e-6): bwd-data, wgrad and
the bias gradient of an ELU layer against the fp64 GEMM of the fp16-rounded
operands (the kernels round dP = dY act'(Y) after scaling it by 2^10,
csrc/td7_dense_kernels.h grad_scale) and against exact arithmetic, and the
encoder's fused zs pass (ops.encoder_zs_half_grad) against the rounded
restatement.  Without the scale the rounding of dP ~ 1e-6 as an fp16
subnormal cost 2 % of the gradient (profiles/r02_fp16_grad_scale.txt)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import conftest  # noqa: E402,F401
from exo_amd import ops  # noqa: E402

torch.manual_seed(0)
rd = lambda t: t.to(torch.float16).double()  # noqa: E731
rg = lambda t: (t * 1024).to(torch.float16).double() / 1024  # noqa: E731  (the kernels' dP rounding)
rel = lambda a, b: float((a.detach().double() - b).norm() / b.norm())  # noqa: E731
m, n, k = 1024, 1024, 1024
x = torch.randn(m, k, device="cuda")
w = torch.randn(n, k, device="cuda") / k ** 0.5
b = torch.randn(n, device="cuda") * 0.1
for scale in (1.0, 1e-5, 1e-6, 1e-7):
    xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    with ops.matrix_precision("fp16"):
        y = ops._DenseFn.apply(xr, wr, br, 2)
    dy = torch.randn_like(y) * scale
    y.backward(dy)
    dp32 = dy * torch.where(y.detach() > 0, 1.0, y.detach() + 1)
    dp = rg(dp32)
    print(f"scale {scale:g}: vs rounded model dX {rel(xr.grad, dp @ rd(w)):.2e} dW {rel(wr.grad, dp.t() @ rd(x)):.2e}"
          f" db {rel(br.grad, dp32.double().sum(0)):.2e};  vs exact dX "
          f"{rel(xr.grad, dp32.double() @ w.double()):.2e} dW {rel(wr.grad, dp32.double().t() @ x.double()):.2e}")

# the encoder's zs over [state; next_state] at the wide widths
B = 1024
xs = torch.randn(2 * B, 80, device="cuda")
W = [torch.randn(1024, 80, device="cuda") / 9, torch.randn(1024, 1024, device="cuda") / 32,
     torch.randn(1024, 1024, device="cuda") / 32]
Bs = [torch.randn(1024, device="cuda") * 0.1 for _ in range(3)]
params = [t.clone().requires_grad_(True) for pair in zip(W, Bs) for t in pair]
with ops.matrix_precision("fp16"):
    zs, nxt = ops.encoder_zs_half_grad(xs, B, 2, [(params[0], params[1]), (params[2], params[3]), (params[4], params[5])])
gz = torch.randn_like(zs) * 2e-6
zs.backward(gz)


class RG(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, w_, b_):
        ctx.save_for_backward(a, w_)
        return rd(a) @ rd(w_).t() + b_

    @staticmethod
    def backward(ctx, g):
        a, w_ = ctx.saved_tensors
        return rg(g) @ rd(w_), rg(g).t() @ rd(a), g.sum(0)


ref = [t.detach().double().clone().requires_grad_(True) for t in params]
h = xs.double()[:B]
h = torch.nn.functional.elu(RG.apply(h, ref[0], ref[1]))
h = torch.nn.functional.elu(RG.apply(h, ref[2], ref[3]))
h = RG.apply(h, ref[4], ref[5])
z = h / h.abs().mean(-1, keepdim=True).clamp(min=1e-8)
z.backward(gz.double())
print("zs fwd", f"{rel(zs, z):.2e}", " ".join(f"{nm} {rel(p.grad, r.grad):.2e}" for nm, p, r in
                                        zip(["w1", "b1", "w2", "b2", "w3", "b3"], params, ref)))
