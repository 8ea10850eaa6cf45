"""Same-process A/B of the 256 x 256-tile 16-bit forward kernels (r06):
td7_dense_fwd_h at 65,536 x 1,024 x K (fp16 X, W and Y, bias + ELU), the
kernel switched with td7_dense_set_xl (2: dense_fwd_xl8_kernel, 3:
dense_fwd_xl9_kernel), interleaved rounds, HIP events around `reps`
back-to-back launches on the launch stream; plus hipBLASLt (F.linear fp16,
bias, no ELU) for scale.  Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from exo_amd import _native as nat  # noqa: E402
from exo_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    rounds, reps = int(os.environ.get("AB_ROUNDS", "5")), int(os.environ.get("AB_REPS", "20"))
    variants = [int(v) for v in os.environ.get("AB_VARIANTS", "2,3").split(",")]
    out = {}
    lib = nat.lib()
    stream = nat.stream_ptr(dev)
    for m, n, k in ((65536, 1024, 1024), (65536, 1024, 2048)):
        flop = 2.0 * m * n * k
        torch.manual_seed(0)
        xh = (torch.rand(m, k, device=dev) * 2 - 1).half()  # uniform [-1, 1): the guide's random-data rule
        w = (torch.rand(n, k, device=dev) * 2 - 1) * k ** -0.5
        b = torch.rand(n, device=dev) * 2 - 1
        wh = w.half()
        y = torch.empty(m, n, dtype=torch.float16, device=dev)
        prec = ops.PRECISIONS["fp16"]

        def call():
            rc = lib.td7_dense_fwd_h(None, nat.ptr(xh), 0, k, nat.ptr(w), nat.ptr(b), None, nat.ptr(y), m * n, n, 1,
                                     m, n, k, 2 | prec << 8, nat.ptr(wh), stream)
            assert rc == 0, rc
        ref = F.elu(F.linear(xh.float(), wh.float(), b))
        res = {v: [] for v in variants}
        errs = {}
        for r in range(rounds):
            for v in variants:
                lib.td7_dense_set_xl(v)
                call()
                torch.cuda.synchronize()
                if r == 0:
                    errs[v] = float(((y.float() - ref).abs() / (ref.abs() + 1.0)).max())
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / reps * 1e3)
        bh = b.half()
        for _ in range(3):
            F.linear(xh, wh, bh)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            F.linear(xh, wh, bh)
        e1.record()
        torch.cuda.synchronize()
        t_lib = e0.elapsed_time(e1) / reps * 1e3
        key = f"{m}x{n}x{k}"
        out[key] = {f"v{v}": {"us_rounds": [round(t, 2) for t in res[v]], "us_min": min(res[v]),
                              "tflops_best": flop / min(res[v]) / 1e6, "max_rel_err": errs[v]} for v in variants}
        out[key]["hipblaslt_us"] = t_lib
    lib.td7_dense_set_xl(2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
