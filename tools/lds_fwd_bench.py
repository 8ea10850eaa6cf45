"""td7_dense_fwd at large shapes with bf16 operands: time per launch (graph
replayed) and max error against the fp32 GEMM of the bf16-rounded operands.
Run twice: EXO_FWD_LDS=0 (register-streaming kernel) and =1 (LDS-tiled
kernel wherever it applies)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dense_bench import timeit  # noqa: E402
import torch  # noqa: E402
from exo_amd import _native as nat  # noqa: E402

ACT = 2 | 1 << 8  # ELU, bf16


def main():
    L = nat.lib()
    dev = torch.device("cuda")
    mode = os.environ.get("EXO_FWD_LDS", "1")
    for (g, m, n, k) in [(1, 4096, 300, 80), (1, 4096, 300, 300), (1, 4096, 320, 320), (1, 4096, 7, 320),
                         (2, 1024, 320, 920), (1, 65536, 1024, 80), (1, 65536, 1024, 1024), (1, 65536, 1024, 2048),
                         (2, 1024, 1024, 3072), (1, 1000, 100, 77)]:
        torch.manual_seed(m + n + k)
        x = torch.randn(g, m, k, device=dev) if g > 1 else torch.randn(m, k, device=dev)
        w = torch.randn(g, n, k, device=dev) / k ** 0.5 if g > 1 else torch.randn(n, k, device=dev) / k ** 0.5
        b = torch.randn(g, n, device=dev) if g > 1 else torch.randn(n, device=dev)
        y = torch.empty(g, m, n, device=dev)
        xsg = m * k if g > 1 else 0
        f = lambda: L.td7_dense_fwd(nat.ptr(x), xsg, k, nat.ptr(w), nat.ptr(b), nat.ptr(y), m * n, n, g, m, n, k, ACT,
                                    nat.stream_ptr(dev))
        us = timeit(f, reps=10, replays=5)
        f()
        torch.cuda.synchronize()
        xr, wr = x.bfloat16().float(), w.bfloat16().float()
        ref = torch.nn.functional.elu((xr @ wr.transpose(-1, -2)) + b.unsqueeze(-2)).reshape(g, m, n)
        err = float((y - ref).abs().max())
        print(f"EXO_FWD_LDS={mode} {g}x{m:6d} {n:5d} {k:5d} | {us:9.2f} us | {2 * g * m * n * k / us / 1e6:8.1f} TF/s"
              f" | max err {err:.2e}")


if __name__ == "__main__":
    main()
