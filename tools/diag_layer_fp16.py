"""One layer's fp16 backward vs the fp64 GEMM of the rounded operands (dP
scaled by 2^10 before rounding), per shape / activation / gradient scale."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import conftest  # noqa: E402,F401
from exo_amd import ops  # noqa: E402

G = {0: lambda y: torch.ones_like(y), 1: lambda y: (y > 0).to(y.dtype), 2: lambda y: torch.where(y > 0, 1.0, y + 1),
     3: lambda y: 1 - y * y}
ACT = {0: lambda x: x, 1: torch.relu, 2: torch.nn.functional.elu, 3: torch.tanh}
rd = lambda t: t.to(torch.float16).double()  # noqa: E731
rg = lambda t: (t * 1024).to(torch.float16).double() / 1024  # noqa: E731
rel = lambda a, b: float((a.detach().double() - b).norm() / b.norm())  # noqa: E731
torch.manual_seed(0)
for (m, n, k, act) in ((1024, 7, 1024, 3), (1024, 7, 320, 3), (1024, 1024, 1024, 1), (1024, 320, 620, 1),
                       (1024, 1024, 2048, 1)):
    for scale in (1.0, 1e-2, 1e-5):
        x = torch.randn(m, k, device="cuda")
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda") * 0.1
        xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
        with ops.matrix_precision("fp16"):
            y = ops._DenseFn.apply(xr, wr, br, act)
        ref = ACT[act](rd(x) @ rd(w).t() + b.double())
        dy = torch.randn_like(y) * scale
        y.backward(dy)
        dp32 = dy * G[act](y.detach())
        dp = rg(dp32)
        print(f"m{m} n{n} k{k} act{act} scale {scale:g}: fwd {rel(y, ref):.2e} dX {rel(xr.grad, dp @ rd(w)):.2e} "
              f"dW {rel(wr.grad, dp.t() @ rd(x)):.2e} db {rel(br.grad, dp32.double().sum(0)):.2e}", flush=True)
