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
