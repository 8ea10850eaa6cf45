"""The wide configuration's select-path GEMM (65,536 x 1,024 x 1,024, fp16
operands, fp32 accumulation) three ways, us per launch (HIP events): the
build's dense_fwd_big_kernel through ops.dense (fp32 activations in and out,
bias + ELU fused), torch.nn.functional.linear on fp16 tensors (hipBLASLt,
fp16 out, bias fused) alone and followed by ELU.  What a library GEMM would buy
the wide select.  Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from exo_amd import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda")
    out = {}
    for m, n, k in ((65536, 1024, 1024), (65536, 1024, 2048)):
        flop = 2.0 * m * n * k
        x = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.03
        b = torch.randn(n, device=dev)
        xh, wh, bh = x.half(), w.half(), b.half()

        def ours():
            with ops.matrix_precision("fp16"):
                return ops.dense(x, w, b, 2)
        t_ours = timed(ours)
        def chain():
            with ops.matrix_precision("fp16"), torch.no_grad():
                return ops.dense(xh, w, b, 2, half_out=True)
        t_chain = timed(chain)
        y = chain()
        ref = F.elu(F.linear(xh.float(), wh.float(), b))
        err = ((y.float() - ref).abs() / (ref.abs() + 1.0)).max().item()
        t_lin = timed(lambda: F.linear(xh, wh, bh))
        t_lin_elu = timed(lambda: F.elu(F.linear(xh, wh, bh)))
        key = f"{m}x{n}x{k}"
        out[key] = {"ours_us": t_ours, "ours_tflops": flop / t_ours / 1e6,
                    "chain16_us": t_chain, "chain16_tflops": flop / t_chain / 1e6,
                    "chain16_dtype": str(y.dtype), "chain16_max_rel_err": err,
                    "hipblaslt_us": t_lin, "hipblaslt_tflops": flop / t_lin / 1e6,
                    "hipblaslt_elu_us": t_lin_elu}
    out["EXO_FWD_XL"] = os.environ.get("EXO_FWD_XL", "")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
