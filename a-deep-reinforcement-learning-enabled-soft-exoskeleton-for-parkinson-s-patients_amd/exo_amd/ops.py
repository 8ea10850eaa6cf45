"""Fused TD7 net ops backed by csrc/td7_ops.hip (GPU) with the reference's
torch expression on CPU tensors (the CPU path exists for the learner's parity
tests; on a GPU the HIP kernels are mandatory -- a missing library raises)."""
import contextlib
import ctypes
import os

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


# ---------------------------------------------------------------- dense layers
ACT_CODES = {None: 0, "none": 0, "relu": 1, "elu": 2, "tanh": 3}

# MFMA operand precision of the td7_dense kernels (csrc/td7_dense_kernels.h
# Prec; bits 8-15 of the act argument): "fp32" exact f32 MFMA; "bf16" / "fp16"
# round the fp32 operands to nearest even as they are loaded (fp32 memory,
# accumulation, epilogues and bias gradients).
PRECISIONS = {"fp32": 0, "bf16": 1, "fp16": 2}
_matrix_prec = 0


@contextlib.contextmanager
def matrix_precision(name):
    """Dense layers created inside the block run their GEMMs (forward and the
    matching backward) with `name` MFMA operands."""
    global _matrix_prec
    old, _matrix_prec = _matrix_prec, PRECISIONS[name]
    try:
        yield
    finally:
        _matrix_prec = old


def act_code(fn):
    """Activation function of the reference nets -> td7_dense act code (None if unsupported)."""
    import torch.nn.functional as F
    return {F.relu: 1, torch.relu: 1, F.elu: 2, torch.tanh: 3}.get(fn)


def _engine_needs(ctx, i):
    """False when the running backward (e.g. torch.autograd.grad with explicit
    inputs) will not use input i's gradient -- its GEMM is then skipped."""
    fn = ctx.next_functions[i][0]
    if fn is None:
        return False
    try:
        return torch._C._will_engine_execute_node(fn)
    except (AttributeError, RuntimeError):
        return True


# the large-layer forward kernel reads W already rounded to 16 bits (one
# conversion per call, ~2 MB at 1,024 x 1,024) when M reaches this many rows
# at bf16 / fp16 operands (r03d: configs[4]'s select over 65,536 envs and the
# update at 8 x 1,024); EXO_FWD_W16=0 keeps the in-kernel rounding
W16_MIN_ROWS = 8192 if os.environ.get("EXO_FWD_W16", "1") != "0" else 1 << 62


def _w16(w, prec, M, K):
    """W rounded to the MFMA operand type for td7_dense_fwd*_w16, or None."""
    if prec == 0 or M < W16_MIN_ROWS or K < 64:
        return None
    return w.to(torch.bfloat16 if prec == PRECISIONS["bf16"] else torch.float16)


_HALF = {PRECISIONS["bf16"]: torch.bfloat16, PRECISIONS["fp16"]: torch.float16}
EXO_ERANGE = -34
# EXO_FWD_HALF=0: inference chains keep fp32 activations (half_out ignored)
HALF_CHAIN = os.environ.get("EXO_FWD_HALF", "1") != "0"


def _half_ok(M, K, grouped):
    """An inference-chain layer (no autograd) at the large-layer sizes: its
    input / output may be 16-bit (td7_dense_fwd_h; the C side answers
    EXO_ERANGE where no 16-bit-capable kernel runs)."""
    return (HALF_CHAIN and _matrix_prec in _HALF and not grouped and not torch.is_grad_enabled() and M >= W16_MIN_ROWS
            and K >= 64 and not torch.is_autocast_enabled())


def _dense_h(x, w, b, act, half_out):
    """td7_dense_fwd_h: x fp32 or 16-bit (the matrix precision's type), y fp32
    or 16-bit; None where the large-layer kernel does not apply."""
    prec = _matrix_prec
    M, K, N = x.shape[-2], x.shape[-1], w.shape[-2]
    w = w.contiguous()
    x, ldx = _rows(x)
    x16 = x.dtype != torch.float32
    y = torch.empty((M, N), dtype=_HALF[prec] if half_out else torch.float32, device=x.device)
    bb = b.contiguous() if b is not None else None
    rc = nat.lib().td7_dense_fwd_h(None if x16 else nat.ptr(x), nat.ptr(x) if x16 else None, 0, ldx, nat.ptr(w),
                                   nat.ptr(bb), None if half_out else nat.ptr(y), nat.ptr(y) if half_out else None,
                                   M * N, N, 1, M, N, K, act | prec << 8, nat.ptr(_w16(w, prec, M, K)),
                                   nat.stream_ptr(x.device))
    if rc == EXO_ERANGE:
        return None
    nat.check(rc, "td7_dense_fwd_h")
    return y


def _rows(t):
    """(tensor with unit column stride, row stride)."""
    if t.stride(-1) != 1:
        t = t.contiguous()
    return t, t.stride(-2)


class _DenseFn(torch.autograd.Function):
    """act(x W^T + b).  Shapes: plain x [M,K], W [N,K], b [N]; grouped W
    [G,N,K], b [G,N] with x [G,M,K] (one input per group) or x [M,K] (shared by
    the groups) -> y [G,M,N].

    Forward: td7_dense_fwd (one launch: GEMM + bias + activation) for up to
    fwd_kernel_max_rows rows, hipBLASLt + the activation above; backward: the
    td7_dense kernels -- act'(Y) folded into the
    operand loads, the bias gradient as the GEMM against a ones column: two
    launches where autograd issues the activation backward, two GEMMs, a
    column reduction and a fill."""

    # td7_dense_fwd (fused bias + activation) up to this many rows, hipBLASLt + the
    # activation above it (profiles/r01_dense_bench.txt: 6.7 vs 9.8 us at
    # 1,024x300x300, 22 vs 18 us at 4,096 rows); EXO_DENSE_FWD=0/1 forces a side
    fwd_kernel_max_rows = {"0": 0, "1": 1 << 30}.get(os.environ.get("EXO_DENSE_FWD", ""), 2048)

    @staticmethod
    def forward(ctx, x, w, b, act, dx_cols=None):
        grouped = w.dim() == 3
        G = w.shape[0] if grouped else 1
        N, K = w.shape[-2], w.shape[-1]
        shared = grouped and x.dim() == 2
        x, ldx = _rows(x)
        M = x.shape[-2]
        xsg = 0 if (shared or not grouped) else x.stride(0)
        w = w.contiguous()
        bb = b.contiguous() if b is not None else None
        prec = _matrix_prec
        if prec or M <= _DenseFn.fwd_kernel_max_rows:
            y = torch.empty((G, M, N) if grouped else (M, N), dtype=torch.float32, device=x.device)
            w16 = _w16(w, prec, M, K)
            nat.check(nat.lib().td7_dense_fwd_w16(nat.ptr(x), xsg, ldx, nat.ptr(w), nat.ptr(bb), nat.ptr(y),
                                                  M * N, N, G, M, N, K, act | prec << 8, nat.ptr(w16),
                                                  nat.stream_ptr(x.device)), "td7_dense_fwd")
        else:
            y = _torch_dense(x, w, bb, act)
        ctx.save_for_backward(x, w, y)
        ctx.meta = (grouped, shared, G, M, N, K, act | prec << 8, xsg, ldx, b is not None)
        ctx.dx_cols = dx_cols
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        grouped, shared, G, M, N, K, act, xsg, ldx, has_b = ctx.meta
        dy = dy.contiguous()
        s = nat.stream_ptr(dy.device)
        dx = dw = db = None
        need = [ctx.needs_input_grad[i] and _engine_needs(ctx, i) for i in range(3)]
        if need[0]:
            dx = torch.empty((G, M, K) if (grouped and not shared) else (M, K), dtype=torch.float32, device=dy.device)
            c0, c1 = ctx.dx_cols if ctx.dx_cols is not None else (0, K)
            # columns outside [c0, c1) belong to concatenated inputs that need no
            # gradient: left unwritten, never read
            nat.check(nat.lib().td7_dense_bwd_data_cols(nat.ptr(dy), M * N, N, nat.ptr(y), M * N, N, nat.ptr(w),
                                                        nat.ptr(dx), M * K, K, G, int(shared), M, N, K, c0, c1, act,
                                                        s), "td7_dense_bwd_data")
        if need[1] or (has_b and need[2]):
            dw = torch.empty_like(w)
            db = torch.empty((G, N) if grouped else (N,), dtype=torch.float32, device=dy.device) if has_b else None
            nat.check(nat.lib().td7_dense_bwd_weight(nat.ptr(dy), M * N, N, nat.ptr(y), M * N, N, nat.ptr(x), xsg,
                                                     ldx, nat.ptr(dw), nat.ptr(db), G, M, N, K, act, s),
                      "td7_dense_bwd_weight")
        return dx, dw, db, None, None


class _DenseCatFn(torch.autograd.Function):
    """act(torch.cat(parts, -1) W^T + b) without materialising the
    concatenation: td7_dense_fwd_cat / td7_dense_bwd_weight_cat read the parts
    in place, and each part that needs a gradient gets its own td7_dense_bwd_data
    launch over its column window, written straight into its gradient tensor.
    With grouped W [G,N,K] a part is [G,M,k] (one per group) or [M,k] (shared
    by the groups: its gradient sums over them)."""

    @staticmethod
    def forward(ctx, w, b, act, *parts):
        grouped = w.dim() == 3
        G = w.shape[0] if grouped else 1
        N, K = w.shape[-2], w.shape[-1]
        parts = [_rows(p)[0] for p in parts]
        M = parts[0].shape[-2]
        n = len(parts)
        widths = [p.shape[-1] for p in parts]
        sgs = [p.stride(0) if (grouped and p.dim() == 3) else 0 for p in parts]
        lds = [p.stride(-2) for p in parts]
        w = w.contiguous()
        bb = b.contiguous() if b is not None else None
        prec = _matrix_prec
        seg = ((ctypes.c_void_p * n)(*[p.data_ptr() for p in parts]), (ctypes.c_long * n)(*sgs),
               (ctypes.c_long * n)(*lds), (ctypes.c_int32 * n)(*widths))
        y = torch.empty((G, M, N) if grouped else (M, N), dtype=torch.float32, device=w.device)
        w16 = _w16(w, prec, M, K)
        nat.check(nat.lib().td7_dense_fwd_cat_w16(n, *seg, nat.ptr(w), nat.ptr(bb), nat.ptr(y), M * N, N, G, M, N,
                                                  act | prec << 8, nat.ptr(w16), nat.stream_ptr(w.device)),
                  "td7_dense_fwd_cat")
        ctx.save_for_backward(w, y, *parts)
        ctx.meta = (grouped, G, M, N, K, act | prec << 8, b is not None, widths, sgs, lds)
        # ctx.next_functions has one entry per TENSOR input: argument index -> entry
        args = (w, b, act, *parts)
        ctx.edge = {i: sum(isinstance(t, torch.Tensor) for t in args[:i]) for i in range(len(args))}
        return y

    @staticmethod
    def backward(ctx, dy):
        w, y, *parts = ctx.saved_tensors
        return _parts_backward(ctx, dy, w, y, parts, ctx.meta)


def _seg_arrays(parts, sgs, lds, widths):
    n = len(parts)
    return ((ctypes.c_void_p * n)(*[p.data_ptr() for p in parts]), (ctypes.c_long * n)(*sgs),
            (ctypes.c_long * n)(*lds), (ctypes.c_int32 * n)(*widths))


def _parts_backward(ctx, dy, w, y, parts, meta):
    """Backward of act(cat(parts) W^T + b) (y: the layer's output, for act'):
    (dW, db, None, grad of each part) -- see _DenseCatFn."""
    grouped, G, M, N, K, act, has_b, widths, sgs, lds = meta
    dy = dy.contiguous()
    s = nat.stream_ptr(dy.device)
    n = len(parts)
    dw = db = None
    if (ctx.needs_input_grad[0] and _engine_needs(ctx, ctx.edge[0])) or \
            (has_b and ctx.needs_input_grad[1] and _engine_needs(ctx, ctx.edge[1])):
        dw = torch.empty_like(w)
        db = torch.empty((G, N) if grouped else (N,), dtype=torch.float32, device=dy.device) if has_b else None
        nat.check(nat.lib().td7_dense_bwd_weight_cat(nat.ptr(dy), M * N, N, nat.ptr(y), M * N, N, n,
                                                     *_seg_arrays(parts, sgs, lds, widths), nat.ptr(dw),
                                                     nat.ptr(db), G, M, N, act, s), "td7_dense_bwd_weight_cat")
    grads = []
    c0 = 0
    for i, p in enumerate(parts):
        k = widths[i]
        g = None
        if ctx.needs_input_grad[3 + i] and _engine_needs(ctx, ctx.edge[3 + i]):
            shared = grouped and p.dim() == 2
            g = torch.empty(p.shape, dtype=torch.float32, device=dy.device)
            # C = dx + c0 is the part's own gradient buffer (row stride k)
            nat.check(nat.lib().td7_dense_bwd_data_cols(nat.ptr(dy), M * N, N, nat.ptr(y), M * N, N, nat.ptr(w),
                                                        g.data_ptr() - 4 * c0, M * k, k, G, int(shared), M, N, K,
                                                        c0, c0 + k, act, s), "td7_dense_bwd_data")
        grads.append(g)
        c0 += k
    return (dw, db, None, *grads)


def _parts_meta(w, parts):
    grouped = w.dim() == 3
    widths = [p.shape[-1] for p in parts]
    sgs = [p.stride(0) if (grouped and p.dim() == 3) else 0 for p in parts]
    lds = [p.stride(-2) for p in parts]
    return grouped, widths, sgs, lds


class _DenseNormFn(torch.autograd.Function):
    """AvgL1Norm(cat(parts) W^T + b) (no activation) as ONE td7_dense_fwd_norm
    launch (the row mean reduced inside the GEMM's workgroup); the backward is
    td7_avgl1norm_bwd from the saved pre-norm h and mean, then the layer's
    backward as _DenseCatFn.  N <= 320."""

    @staticmethod
    def forward(ctx, w, b, train, *parts):
        parts = [_rows(p)[0] for p in parts]
        grouped, widths, sgs, lds = _parts_meta(w, parts)
        G = w.shape[0] if grouped else 1
        N, K = w.shape[-2], w.shape[-1]
        M = parts[0].shape[-2]
        w = w.contiguous()
        bb = b.contiguous() if b is not None else None
        prec = _matrix_prec
        shape = (G, M, N) if grouped else (M, N)
        y = torch.empty(shape, dtype=torch.float32, device=w.device)
        h = torch.empty(shape, dtype=torch.float32, device=w.device) if train else None
        mean = torch.empty((G * M,), dtype=torch.float32, device=w.device) if train else None
        st = nat.stream_ptr(w.device)
        if len(parts) == 1:
            nat.check(nat.lib().td7_dense_fwd_norm(nat.ptr(parts[0]), sgs[0], lds[0], nat.ptr(w), nat.ptr(bb),
                                                   nat.ptr(y), nat.ptr(h), nat.ptr(mean), M * N, N, G, M, N, K, prec,
                                                   1e-8, st), "td7_dense_fwd_norm")
        else:
            nat.check(nat.lib().td7_dense_fwd_norm_cat(len(parts), *_seg_arrays(parts, sgs, lds, widths), nat.ptr(w),
                                                       nat.ptr(bb), nat.ptr(y), nat.ptr(h), nat.ptr(mean), M * N, N,
                                                       G, M, N, prec, 1e-8, st), "td7_dense_fwd_norm_cat")
        if train:
            ctx.save_for_backward(w, h, mean, *parts)
        ctx.meta = (grouped, G, M, N, K, prec << 8, b is not None, widths, sgs, lds)
        args = (w, b, train, *parts)
        ctx.edge = {i: sum(isinstance(t, torch.Tensor) for t in args[:i]) for i in range(len(args))}
        return y

    @staticmethod
    def backward(ctx, gy):
        w, h, mean, *parts = ctx.saved_tensors
        meta = ctx.meta
        G, M, N = meta[1], meta[2], meta[3]
        gy = gy.contiguous()
        gh = torch.empty_like(h)
        nat.check(nat.lib().td7_avgl1norm_bwd(nat.ptr(h), nat.ptr(mean), nat.ptr(gy), nat.ptr(gh), G * M, N, 1e-8,
                                              nat.stream_ptr(gy.device)), "td7_avgl1norm_bwd")
        return _parts_backward(ctx, gh, w, h, parts, meta)


_NORM = os.environ.get("EXO_TD7_NORM_FUSED", "1") != "0"
# fuse below 2,048 rows too (A/B switch)
_NORM_SMALL = os.environ.get("EXO_TD7_NORM_SMALL", "1") != "0"


def dense_norm(parts, w, b, half_out=False):
    """AvgL1Norm(dense(torch.cat(parts, -1), w, b)) -- one fused launch on the
    GPU where it applies (N <= 320, the concatenated-input rules of
    dense_cat); the two ops otherwise.  half_out: as dense (an inference chain
    at the large-layer sizes gets the norm as 16-bit values, avg_l1_norm_h)."""
    ok = (_NORM and w.is_cuda and w.dtype == torch.float32 and not torch.is_autocast_enabled()
          and w.shape[-2] <= 320 and (_matrix_prec or parts[0].shape[-2] <= _DenseFn.fwd_kernel_max_rows)
          and (_NORM_SMALL or parts[0].shape[-2] >= 2048))
    if ok and len(parts) > 1:
        ok = _CAT and _cat_ok(parts, w)
    elif ok:
        p = parts[0]
        ok = (p.is_cuda and p.dtype == torch.float32 and p.shape[-1] >= 4
              and (p.dim() == 2 or (w.dim() == 3 and p.shape[0] == w.shape[0])))
    if ok:
        # h and the mean are kept only when this call records a backward
        train = torch.is_grad_enabled() and (w.requires_grad or (b is not None and b.requires_grad)
                                             or any(p.requires_grad for p in parts))
        return _DenseNormFn.apply(w, b, train, *parts)
    y = dense_cat(parts, w, b, 0) if len(parts) > 1 else dense(parts[0], w, b, 0)
    if half_out and y.is_cuda and y.dtype == torch.float32 and y.dim() == 2 \
            and _half_ok(y.shape[0], w.shape[-1], w.dim() == 3):
        h = avg_l1_norm_h(y, _matrix_prec)
        if h is not None:
            return h
    return avg_l1_norm(y)


def avg_l1_norm_h(y, prec, eps=1e-8):
    """AvgL1Norm of fp32 rows as 16-bit values of the MFMA operand type
    (td7_avgl1norm_fwd_h, no autograd), or None outside its width range."""
    y = y.contiguous()
    out = torch.empty(y.shape, dtype=_HALF[prec], device=y.device)
    rc = nat.lib().td7_avgl1norm_fwd_h(nat.ptr(y), nat.ptr(out), None, y.shape[0], y.shape[1], float(eps), prec,
                                       nat.stream_ptr(y.device))
    if rc == EXO_ERANGE:
        return None
    nat.check(rc, "td7_avgl1norm_fwd_h")
    return out


def _cat_ok(parts, w):
    """The concatenated-input kernels apply: <= 4 parts, interior widths
    multiples of 4, the last >= 4 wide, N >= 4, fp32 on the GPU."""
    if not (1 < len(parts) <= 4) or w.shape[-2] < 4:
        return False
    widths = [p.shape[-1] for p in parts]
    if any(k % 4 for k in widths[:-1]) or widths[-1] < 4:
        return False
    grouped = w.dim() == 3
    rows = parts[0].shape[-2]
    for p in parts:
        if p.dtype != torch.float32 or not p.is_cuda or p.shape[-2] != rows:
            return False
        if p.dim() == 3 and not (grouped and p.shape[0] == w.shape[0]):
            return False
    return True


def dense_cat(parts, w, b, act=0, half_out=False):
    """dense(torch.cat(parts, -1), w, b, act) reading the parts in place (parts
    of a grouped layer may be [G,M,k] or shared [M,k]).  Falls back to the
    concatenation where the fused kernels do not apply.  half_out: as dense."""
    if w.dtype == torch.float32 and any(p.dtype in (torch.bfloat16, torch.float16) for p in parts):
        # 16-bit parts (avg_l1_norm_h outputs on an inference chain): all of
        # them read as 16-bit by the large-layer kernel, else as fp32 -- the same
        # values, the consumer rounds them to the same type
        if all(p.dtype == _HALF.get(_matrix_prec) for p in parts) and half_out \
                and _half_ok(parts[0].shape[-2], w.shape[-1], w.dim() == 3):
            y = _dense_cat_h(parts, w, b, act, xs16=True)
            if y is not None:
                return y
        parts = [p.float() if p.dtype in (torch.bfloat16, torch.float16) else p for p in parts]
    if _CAT and w.is_cuda and w.dtype == torch.float32 and not torch.is_autocast_enabled() and _cat_ok(parts, w) \
            and (_matrix_prec or parts[0].shape[-2] <= _DenseFn.fwd_kernel_max_rows):
        if half_out and _half_ok(parts[0].shape[-2], w.shape[-1], w.dim() == 3):
            y = _dense_cat_h(parts, w, b, act)
            if y is not None:
                return y
        return _DenseCatFn.apply(w, b, act, *parts)
    grouped = w.dim() == 3
    if grouped and any(p.dim() == 3 for p in parts):
        G = w.shape[0]
        parts = [p if p.dim() == 3 else p.unsqueeze(0).expand(G, *p.shape) for p in parts]
    return dense(torch.cat(parts, -1), w, b, act, concat_grad_cols(parts))


def _dense_cat_h(parts, w, b, act, xs16=False):
    """td7_dense_fwd_cat_h: the concatenated layer with a 16-bit output (and
    16-bit parts when xs16), or None."""
    prec = _matrix_prec
    N, K = w.shape[-2], w.shape[-1]
    w = w.contiguous()
    parts = [_rows(p)[0] for p in parts]
    M, n = parts[0].shape[-2], len(parts)
    seg = ((ctypes.c_void_p * n)(*[p.data_ptr() for p in parts]), (ctypes.c_long * n)(*([0] * n)),
           (ctypes.c_long * n)(*[p.stride(-2) for p in parts]), (ctypes.c_int32 * n)(*[p.shape[-1] for p in parts]))
    y = torch.empty((M, N), dtype=_HALF[prec], device=w.device)
    bb = b.contiguous() if b is not None else None
    rc = nat.lib().td7_dense_fwd_cat_h(n, seg[0], int(xs16), *seg[1:], nat.ptr(w), nat.ptr(bb), nat.ptr(y), M * N, N, 1, M, N,
                                       act | prec << 8, nat.ptr(_w16(w, prec, M, K)), nat.stream_ptr(w.device))
    if rc == EXO_ERANGE:
        return None
    nat.check(rc, "td7_dense_fwd_cat_h")
    return y


_CAT = os.environ.get("EXO_TD7_CAT", "1") != "0"


def pair_rows(a, b):
    """torch.stack([a, b]) for two equally shaped row-major tensors -- a view
    without a copy when b directly follows a in memory (the replay batch's
    state / next_state, exo_amd/replay.py); else the stack."""
    if (a.dim() == 2 and a.shape == b.shape and a.dtype == b.dtype and a.device == b.device and a.is_contiguous()
            and b.is_contiguous() and b.data_ptr() == a.data_ptr() + a.numel() * a.element_size()
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()  # adjacent in ONE allocation
            and not (a.requires_grad or b.requires_grad)):
        return a.as_strided((2, *a.shape), (a.numel(), *a.stride()))
    return torch.stack([a, b])


def _dense_raw(x, w, b, act):
    """Forward of one fused layer outside autograd -> y (x [M,K] row-major)."""
    x, ldx = _rows(x)
    M, N, K = x.shape[0], w.shape[0], w.shape[1]
    y = torch.empty((M, N), dtype=torch.float32, device=x.device)
    nat.check(nat.lib().td7_dense_fwd(nat.ptr(x), 0, ldx, nat.ptr(w), nat.ptr(b), nat.ptr(y), M * N, N, 1, M, N, K,
                                      act | _matrix_prec << 8, nat.stream_ptr(x.device)), "td7_dense_fwd")
    return y


class _ZsHalfGradFn(torch.autograd.Function):
    """The encoder's zs = AvgL1Norm(L3(act(L2(act(L1(x)))))) over 2B rows whose
    first B rows need gradients and the last B do not (Agent/TD7_multi_agent.py:
    220-223: zs(state) trained, zs(next_state) under no_grad): one launch per
    layer forward over all 2B rows, the backward over the first B rows only --
    no zero-padded gradient for the detached half (autograd's slice backward
    would fill and copy one)."""

    @staticmethod
    def forward(ctx, x, B, act, w1, b1, w2, b2, w3, b3):
        prec = _matrix_prec
        w1, w2, w3 = w1.contiguous(), w2.contiguous(), w3.contiguous()
        h1 = _dense_raw(x, w1, b1, act)
        h2 = _dense_raw(h1, w2, b2, act)
        M2, N3, K3 = h2.shape[0], w3.shape[0], w3.shape[1]
        mean = torch.empty((M2,), dtype=torch.float32, device=h2.device)
        st = nat.stream_ptr(h2.device)
        if _NORM and N3 <= 320:  # last layer + AvgL1Norm in one launch
            h3 = torch.empty((M2, N3), dtype=torch.float32, device=h2.device)
            zs = torch.empty_like(h3)
            nat.check(nat.lib().td7_dense_fwd_norm(nat.ptr(h2), 0, K3, nat.ptr(w3), nat.ptr(b3), nat.ptr(zs),
                                                   nat.ptr(h3), nat.ptr(mean), M2 * N3, N3, 1, M2, N3, K3, prec, 1e-8,
                                                   st), "td7_dense_fwd_norm")
        else:
            h3 = _dense_raw(h2, w3, b3, 0)
            zs = torch.empty_like(h3)
            nat.check(nat.lib().td7_avgl1norm_fwd(nat.ptr(h3), nat.ptr(zs), nat.ptr(mean), M2, N3, 1e-8, st),
                      "td7_avgl1norm_fwd")
        ctx.save_for_backward(x, h1, h2, h3, mean, w1, w2, w3)
        ctx.meta = (B, act, prec)
        nxt = zs[B:]
        ctx.mark_non_differentiable(nxt)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the detached half
        return zs[:B], nxt

    @staticmethod
    def backward(ctx, gzs, _gnext):
        x, h1, h2, h3, mean, w1, w2, w3 = ctx.saved_tensors
        B, act, prec = ctx.meta
        if gzs is None:
            return (None,) * 9
        s = nat.stream_ptr(gzs.device)
        L = nat.lib()
        gzs = gzs.contiguous()
        g3 = torch.empty((B, h3.shape[1]), dtype=torch.float32, device=gzs.device)
        nat.check(L.td7_avgl1norm_bwd(nat.ptr(h3), nat.ptr(mean), nat.ptr(gzs), nat.ptr(g3), B, h3.shape[1], 1e-8, s),
                  "td7_avgl1norm_bwd")
        grads = []
        x1, ldx1 = _rows(x)
        # (dY, Y, act, W, X, row stride of X, need dX) per layer, last first
        layers = ((h3, 0, w3, h2, h2.shape[1], True), (h2, act, w2, h1, h1.shape[1], True),
                  (h1, act, w1, x1, ldx1, False))
        dy = g3
        for y, a, w, xin, ldx, need_dx in layers:
            N, K = w.shape
            code = a | prec << 8
            dw = torch.empty_like(w)
            db = torch.empty((N,), dtype=torch.float32, device=w.device)
            nat.check(L.td7_dense_bwd_weight(nat.ptr(dy), B * N, N, nat.ptr(y), B * N, N, nat.ptr(xin), 0, ldx,
                                             nat.ptr(dw), nat.ptr(db), 1, B, N, K, code, s), "td7_dense_bwd_weight")
            dx = None
            if need_dx:
                dx = torch.empty((B, K), dtype=torch.float32, device=w.device)
                nat.check(L.td7_dense_bwd_data(nat.ptr(dy), B * N, N, nat.ptr(y), B * N, N, nat.ptr(w), nat.ptr(dx),
                                               B * K, K, 1, 0, B, N, K, code, s), "td7_dense_bwd_data")
            grads.append((dw, db))
            dy = dx
        (dw3, db3), (dw2, db2), (dw1, db1) = grads
        return None, None, None, dw1, db1, dw2, db2, dw3, db3


def encoder_zs_half_grad(x, B, act, layers):
    """(zs(x[:B]) with gradients, zs(x[B:]) without) -- see _ZsHalfGradFn.
    layers: the three (weight, bias) pairs."""
    if x.requires_grad:
        raise ValueError("encoder_zs_half_grad: the input rows take no gradient")
    (w1, b1), (w2, b2), (w3, b3) = layers
    return _ZsHalfGradFn.apply(x, B, act, w1, b1, w2, b2, w3, b3)


def _torch_dense(x, w, b, act):
    if w.dim() == 3:
        xx = x if x.dim() == 3 else x.unsqueeze(0).expand(w.shape[0], *x.shape)
        y = torch.baddbmm(b.unsqueeze(1), xx, w.transpose(1, 2)) if b is not None else torch.bmm(xx, w.transpose(1, 2))
    else:
        y = torch.nn.functional.linear(x, w, b)
    if act == 1:
        return torch.relu_(y)
    if act == 2:
        return torch.nn.functional.elu_(y)
    if act == 3:
        return torch.tanh_(y)
    return y


def dense(x, w, b, act=0, dx_cols=None, half_out=False):
    """Linear + activation (act code, see ACT_CODES) -- td7_dense kernels on a
    GPU for fp32 tensors; the reference's torch expression otherwise.
    dx_cols = (c0, c1): only input columns [c0, c1) need a gradient (x is a
    concatenation whose other parts do not require one).
    Inference chains (r03d): half_out=True asks for y as the 16-bit values
    the next layer rounds its input to (returned where the large-layer kernel
    runs, fp32 otherwise), and a 16-bit x (such a y) is read as it is --
    bit-identical to the fp32 chain."""
    if x.device.type == "cuda" and x.dtype in (torch.bfloat16, torch.float16) and w.dtype == torch.float32:
        if x.dtype == _HALF.get(_matrix_prec) and _half_ok(x.shape[-2], x.shape[-1], w.dim() == 3):
            y = _dense_h(x, w, b, act, half_out)
            if y is not None:
                return y
        x = x.float()
    if x.device.type == "cuda" and x.dtype == torch.float32 and w.dtype == torch.float32 \
            and not torch.is_autocast_enabled():
        if half_out and _half_ok(x.shape[-2], x.shape[-1], w.dim() == 3):
            y = _dense_h(x, w, b, act, True)
            if y is not None:
                return y
        return _DenseFn.apply(x, w, b, act, dx_cols)
    return _torch_dense(x, w, b, act)


# ---------------------------------------------------------------- critic tail
def q_target(qt, reward, not_done, discount, min_target, max_target, run_max, run_min):
    """Q_target (Agent/TD7_multi_agent.py:240-246) from the target critic's
    two heads qt [B,2]; updates the running bounds run_max / run_min in place.
    One td7_q_target launch on a GPU; the reference expression on a CPU."""
    if not qt.is_cuda:
        q = qt.min(1, keepdim=True)[0]
        out = reward + not_done * discount * q.clamp(min_target, max_target)
        torch.maximum(run_max, out.max(), out=run_max)
        torch.minimum(run_min, out.min(), out=run_min)
        return out
    B = qt.shape[0]
    out = torch.empty((B, 1), dtype=torch.float32, device=qt.device)
    nat.check(nat.lib().td7_q_target(nat.ptr(qt), qt.stride(0), qt.stride(1), nat.ptr(reward.contiguous()),
                                     nat.ptr(not_done.contiguous()), float(discount), nat.ptr(min_target),
                                     nat.ptr(max_target), nat.ptr(run_max), nat.ptr(run_min), nat.ptr(out), B,
                                     nat.stream_ptr(qt.device)), "td7_q_target")
    return out


class _CriticLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, q_target, alpha, min_priority):
        B = q.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=q.device)
        prio = torch.empty((B,), dtype=torch.float32, device=q.device)
        dq = torch.empty((B, 2), dtype=torch.float32, device=q.device)
        nat.check(nat.lib().td7_critic_loss(nat.ptr(q), q.stride(0), q.stride(1), nat.ptr(q_target.contiguous()),
                                            nat.ptr(loss), nat.ptr(prio), nat.ptr(dq), float(alpha),
                                            float(min_priority), B, nat.stream_ptr(q.device)), "td7_critic_loss")
        ctx.save_for_backward(dq)
        ctx.mark_non_differentiable(prio)
        return loss, prio

    @staticmethod
    def backward(ctx, gloss, gprio):
        (dq,) = ctx.saved_tensors
        return dq * gloss, None, None, None


def critic_loss(q, q_target, alpha, min_priority):
    """(LAP_huber(|q - q_target|), priority) of Agent/TD7_multi_agent.py:257-262
    for the critic's two heads q [B,2] -- one td7_critic_loss launch forward,
    one multiply backward on a GPU; the reference expressions on a CPU."""
    if not q.is_cuda:
        td = (q - q_target).abs()
        loss = torch.where(td < 1, 0.5 * td.pow(2), 1 * td).sum(1).mean()
        return loss, td.detach().max(1)[0].clamp(min=min_priority).pow(alpha)
    return _CriticLossFn.apply(q, q_target, alpha, min_priority)


def critic_loss_and_grad(q, q_target, alpha, min_priority):
    """GPU: (loss, priority, dloss/dq) in one td7_critic_loss launch with dq in
    q's own strides -- the caller back-propagates dq from q directly
    (torch.autograd.backward(q, dq)): no ones-seed fill, no dq * dloss
    multiply, and for the critic's [2,B] head layout viewed as [B,2] no copy
    before the last layer's backward."""
    B = q.shape[0]
    loss = torch.empty((), dtype=torch.float32, device=q.device)
    prio = torch.empty((B,), dtype=torch.float32, device=q.device)
    dq = torch.empty_strided(q.shape, q.stride(), dtype=torch.float32, device=q.device)
    nat.check(nat.lib().td7_critic_loss_strided(nat.ptr(q), q.stride(0), q.stride(1), nat.ptr(q_target.contiguous()),
                                                nat.ptr(loss), nat.ptr(prio), nat.ptr(dq), dq.stride(0), dq.stride(1),
                                                float(alpha), float(min_priority), B, nat.stream_ptr(q.device)),
              "td7_critic_loss")
    return loss, prio, dq


# ---------------------------------------------------------------- small fusions
class DeviceRNG:
    """A counter-based (Philox4x32-10) random stream consumed INSIDE the kernels
    that need random numbers (td7_noisy_action_rng, lap_sample_gather_rng):
    key = seed, counter = (draw index, call number, tag).  The call number lives
    on the device and each launch advances it, so a captured HIP graph draws
    fresh numbers on every replay with no generator kernel and no host value.
    The seed follows torch.initial_seed(), so torch.manual_seed reproduces runs;
    each consumer (tag) has its own stream (concurrent graph branches never
    share a counter)."""

    def __init__(self, device, tag):
        self.tag = int(tag) & 0xFFFFFFFF
        self.seed = (torch.initial_seed() * 0x9E3779B97F4A7C15 + (self.tag + 1) * 0xD1B54A32D192ED03) & (2 ** 64 - 1)
        # [call number, ticket (uint32 in the low half)]
        self.state = torch.zeros((2,), dtype=torch.int64, device=device)

    def fold(self, rank):
        """A rank's own stream (data parallel): the key mixed with the rank."""
        if rank:
            self.seed = (self.seed ^ ((int(rank) * 0x94D049BB133111EB) & (2 ** 64 - 1))) & (2 ** 64 - 1)
        return self

    @property
    def counter_ptr(self):
        return self.state.data_ptr()

    @property
    def ticket_ptr(self):
        return self.state.data_ptr() + 8


def noisy_action(a, noise, sigma, sigma_dec, clip=0.0, scale=1.0, rng=None, dec_count=None):
    """clamp(a + c(noise * sigma), -1, 1) * scale with c = clamp(+-clip) when
    clip > 0, then sigma -= sigma_dec in place (sigma: device scalar tensor).
    One td7_noisy_action launch on a GPU; the reference expressions on a CPU.
    noise=None: standard normal noise -- drawn inside the kernel from `rng`
    (a DeviceRNG) on a GPU, torch.randn_like on a CPU.  dec_count (int32
    device scalar): sigma -= sigma_dec * dec_count instead (in the noise
    kernel with the device RNG; one more small launch with given / host noise)."""
    if noise is None and a.is_cuda:
        if rng is None:
            raise ValueError("noisy_action: noise=None needs a DeviceRNG on the GPU")
        a = a.contiguous()
        out = torch.empty_like(a)
        nat.check(nat.lib().td7_noisy_action_rng(nat.ptr(a), rng.seed, rng.tag, rng.counter_ptr, rng.ticket_ptr,
                                                 nat.ptr(sigma),
                                                 float(sigma_dec), float(clip), float(scale), nat.ptr(out), a.numel(),
                                                 nat.ptr(dec_count), nat.stream_ptr(a.device)), "td7_noisy_action_rng")
        return out
    if noise is None:
        noise = torch.randn_like(a)
    if not a.is_cuda:
        e = noise * sigma
        if clip > 0:
            e = e.clamp(-clip, clip)
        out = (a + e).clamp(-1, 1) * scale
        if dec_count is not None:
            sigma -= sigma_dec * dec_count.to(sigma.dtype).reshape(sigma.shape)
        else:
            sigma -= sigma_dec
        return out
    a = a.contiguous()
    out = torch.empty_like(a)
    nat.check(nat.lib().td7_noisy_action(nat.ptr(a), nat.ptr(noise.contiguous()), nat.ptr(sigma),
                                         0.0 if dec_count is not None else float(sigma_dec),
                                         float(clip), float(scale), nat.ptr(out), a.numel(),
                                         nat.stream_ptr(a.device)), "td7_noisy_action")
    if dec_count is not None:
        sigma.sub_(dec_count.to(sigma.dtype).reshape(sigma.shape) * sigma_dec)
    return out


TD7_MSE_WS = 257  # include/exo_amd.h
_mse_ws = {}


def _mse_workspace(device):
    """Zeroed block-partials + ticket buffer of td7_mse_fwd, one per device (the
    encoder loss never runs on two streams at once)."""
    key = torch.device(device)
    ws = _mse_ws.get(key)
    if ws is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("mse_loss: run once eagerly on this stream before graph capture")
        ws = _mse_ws[key] = torch.zeros(TD7_MSE_WS, dtype=torch.float32, device=device)
    return ws


class _MSEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        x, y = x.contiguous(), y.contiguous()
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        nat.check(nat.lib().td7_mse_fwd(nat.ptr(x), nat.ptr(y), x.numel(), nat.ptr(loss),
                                        nat.ptr(_mse_workspace(x.device)), nat.stream_ptr(x.device)),
                  "td7_mse_fwd")
        ctx.save_for_backward(x, y)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        dx = torch.empty_like(x)
        nat.check(nat.lib().td7_mse_bwd(nat.ptr(x), nat.ptr(y), nat.ptr(g.contiguous()), x.numel(), nat.ptr(dx),
                                        nat.stream_ptr(x.device)), "td7_mse_bwd")
        return dx, None


_ones = {}


def mse_grad(x, y):
    """d F.mse_loss(x, y) / dx = 2 (x - y) / n as one td7_mse_bwd launch (the
    caller back-propagates it from x directly: no loss value, no seed fill)."""
    key = torch.device(x.device)
    one = _ones.get(key)
    if one is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("mse_grad: run once eagerly on this device before graph capture")
        one = _ones[key] = torch.ones((), dtype=torch.float32, device=x.device)
    x, y = x.contiguous(), y.contiguous()
    dx = torch.empty_like(x)
    nat.check(nat.lib().td7_mse_bwd(nat.ptr(x), nat.ptr(y), nat.ptr(one), x.numel(), nat.ptr(dx),
                                    nat.stream_ptr(x.device)), "td7_mse_bwd")
    return dx


def mse_loss(x, y):
    """F.mse_loss(x, y) for a target without gradient: one launch each way on a GPU."""
    if x.is_cuda and x.dtype == torch.float32 and y.dtype == torch.float32:
        return _MSEFn.apply(x, y.detach())
    return torch.nn.functional.mse_loss(x, y)


_DX_COLS = os.environ.get("EXO_TD7_DX_COLS", "1") != "0"


def concat_grad_cols(parts):
    """dx_cols hint for a dense layer whose input is torch.cat(parts, -1): the
    contiguous column range of the parts that require a gradient, or None
    (all columns) when they are not contiguous."""
    if not _DX_COLS:
        return None
    widths = [p.shape[-1] for p in parts]
    need = [p.requires_grad for p in parts]
    if not any(need):
        return None
    first = need.index(True)
    last = len(need) - 1 - need[::-1].index(True)
    if not all(need[first:last + 1]):
        return None
    c0 = sum(widths[:first])
    return (c0, c0 + sum(widths[first:last + 1]))
