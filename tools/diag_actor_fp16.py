"""Wide actor (1,024) backward in fp16 vs the fp64 restatement with the same
operand rounding (tests/test_td7_full.py's _RoundedGemm), isolated from the
critic: loss = sum(actor(s, zs) * c) with c ~ scale."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import conftest  # noqa: E402,F401
import test_td7_full as t  # noqa: E402
from exo_amd import ops  # noqa: E402
from exo_amd.td7 import Actor  # noqa: E402

torch.manual_seed(0)
for prec, width in (("fp16", 1024), ("bf16", 320), ("fp16", 320)):
    for scale in (1e-2, 1e-5):
        a_gpu = Actor(80, 7, width if width == 1024 else 300, width).cuda()
        a_ref = Actor(80, 7, width if width == 1024 else 300, width).double()
        a_ref.load_state_dict(a_gpu.state_dict())
        B = 1024
        s = torch.randn(B, 80, device="cuda")
        zs = torch.randn(B, width if width == 1024 else 300, device="cuda")
        zs = zs / zs.abs().mean(-1, keepdim=True)
        c = torch.randn(B, 7, device="cuda") * scale
        with ops.matrix_precision(prec):
            out = a_gpu(s, zs)
        (out * c).sum().backward()
        with t._rounded_matmuls(t.ROUND[prec]):
            o2 = a_ref(s.double().cpu(), zs.double().cpu())
            (o2 * c.double().cpu()).sum().backward()
        rel = lambda x, y: float((x.double().cpu() - y).norm() / y.norm())  # noqa: E731
        print(prec, width, f"scale {scale:g}", f"fwd {rel(out, o2.detach()):.2e}",
              " ".join(f"{n} {rel(p.grad, q.grad):.2e}" for (n, p), q in zip(a_gpu.named_parameters(),
                                                                               a_ref.parameters())), flush=True)
