"""Fused TD7 net ops backed by csrc/td7_ops.hip (GPU) with the reference's
torch expression on CPU tensors (the CPU path exists for the learner's parity
tests; on a GPU the HIP kernels are mandatory -- a missing library raises)."""
import torch

from . import _native as nat


class _AvgL1NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y = torch.empty_like(x2)
        m = torch.empty((x2.shape[0],), dtype=torch.float32, device=x.device)
        nat.check(nat.lib().td7_avgl1norm_fwd(nat.ptr(x2), nat.ptr(y), nat.ptr(m), x2.shape[0], x2.shape[1],
                                              float(eps), nat.stream_ptr(x.device)), "td7_avgl1norm_fwd")
        ctx.save_for_backward(x2, m)
        ctx.eps = float(eps)
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, gy):
        x2, m = ctx.saved_tensors
        g2 = gy.reshape(-1, x2.shape[1]).contiguous()
        gx = torch.empty_like(x2)
        nat.check(nat.lib().td7_avgl1norm_bwd(nat.ptr(x2), nat.ptr(m), nat.ptr(g2), nat.ptr(gx), x2.shape[0],
                                              x2.shape[1], ctx.eps, nat.stream_ptr(gy.device)), "td7_avgl1norm_bwd")
        return gx.view(ctx.shape), None


def avg_l1_norm(x, eps=1e-8):
    """AvgL1Norm (Agent/TD7_multi_agent.py:53-54)."""
    if x.device.type != "cuda":
        return x / x.abs().mean(-1, keepdim=True).clamp(min=eps)
    if x.dtype != torch.float32:
        return _AvgL1NormFn.apply(x.float(), eps).to(x.dtype)
    return _AvgL1NormFn.apply(x, eps)
