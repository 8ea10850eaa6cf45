"""Large-layer forward GEMMs of the wide configuration (configs[4]) through
ops.dense / ops.dense_cat at fp16: us per launch (HIP events, 20 launches
after 3 warm-ups) and TFLOP/s.  Run twice -- EXO_FWD_BIG=0 keeps the
dense_fwd_lds_kernel, the default dispatches dense_fwd_big_kernel -- and
compare.  Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402

from exo_amd import ops  # noqa: E402

CASES = {  # name: (groups, rows, N, segment widths)
    "select zs2/zs3/l2 65536x1024x1024": (1, 65536, 1024, [1024]),
    "select actor l1 [a|zs] 65536x1024x2048": (1, 65536, 1024, [1024, 1024]),
    "update critic l1 [q|zsa|zs] 2x8192x1024x3072": (2, 8192, 1024, [1024, 1024, 1024]),
    "update 8192x1024x1024": (1, 8192, 1024, [1024]),
}


def main():
    dev = torch.device("cuda")
    out = {"EXO_FWD_BIG": os.environ.get("EXO_FWD_BIG", "1")}
    for name, (g, m, n, widths) in CASES.items():
        k = sum(widths)
        w = torch.randn(g, n, k, device=dev) if g > 1 else torch.randn(n, k, device=dev)
        b = torch.randn(g, n, device=dev) if g > 1 else torch.randn(n, device=dev)
        parts = [torch.randn(g, m, widths[0], device=dev) if g > 1 else torch.randn(m, widths[0], device=dev)]
        parts += [torch.randn(m, wd, device=dev) for wd in widths[1:]]

        def run():
            with ops.matrix_precision("fp16"):
                return ops.dense_cat(parts, w, b, 2) if len(parts) > 1 else ops.dense(parts[0], w, b, 2)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        out[name] = {"us": round(us, 1), "tflops": round(2 * g * m * n * k / us / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
