"""td7_dense_fwd_cat (parts read in place) vs td7_dense_fwd on the
concatenation, at the TD7 concatenated-input shapes; graph-replayed launches
(tools/dense_bench.py timing)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dense_bench import timeit  # noqa: E402
import torch  # noqa: E402
from exo_amd import _native as nat  # noqa: E402

ACT = 2 | 1 << 8  # ELU, bf16 operands


def main():
    L = nat.lib()
    dev = torch.device("cuda")
    s = nat.stream_ptr(dev)
    M = int(os.environ.get("CB_ROWS", "1024"))
    cases = {"critic1 [q(2)|zsa|zs] 920": ([(2, 320), (1, 300), (1, 300)], 2, 320),
             "critic0 [state|action] 87": ([(1, 80), (1, 7)], 2, 320),
             "zsa1 [zs|action] 307": ([(1, 300), (1, 7)], 1, 300),
             "actor1 [a|zs] 620": ([(1, 320), (1, 300)], 1, 320),
             "aligned [a|b] 640": ([(1, 320), (1, 320)], 1, 320),
             "wide critic1 [q(2)|zsa|zs] 3072": ([(2, 1024), (1, 1024), (1, 1024)], 2, 1024),
             "wide actor1 [a|zs] 2048": ([(1, 1024), (1, 1024)], 1, 1024)}
    for name, (segs, G, N) in cases.items():
        parts = [torch.randn(M, k, device=dev) if g == 1 else torch.randn(g, M, k, device=dev) for g, k in segs]
        K = sum(k for _, k in segs)
        w = torch.randn(G, N, K, device=dev) if G > 1 else torch.randn(N, K, device=dev)
        b = torch.randn(G, N, device=dev) if G > 1 else torch.randn(N, device=dev)
        y = torch.empty(G, M, N, device=dev)
        n = len(parts)
        P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in parts])
        SG = (ctypes.c_long * n)(*[p.stride(0) if p.dim() == 3 else 0 for p in parts])
        LD = (ctypes.c_long * n)(*[p.stride(-2) for p in parts])
        WD = (ctypes.c_int32 * n)(*[p.shape[-1] for p in parts])
        t_cat = timeit(lambda: L.td7_dense_fwd_cat(n, P, SG, LD, WD, nat.ptr(w), nat.ptr(b), nat.ptr(y), M * N, N, G, M,
                                                   N, ACT, nat.stream_ptr(dev)))
        full = torch.cat([p if p.dim() == 3 or G == 1 else p.unsqueeze(0).expand(G, M, p.shape[-1]) for p in parts], -1) \
            if any(p.dim() == 3 for p in parts) else torch.cat(parts, -1)
        xsg = full.stride(0) if full.dim() == 3 else 0
        t_plain = timeit(lambda: L.td7_dense_fwd(nat.ptr(full), xsg, K, nat.ptr(w), nat.ptr(b), nat.ptr(y), M * N, N, G,
                                                 M, N, K, ACT, nat.stream_ptr(dev)))
        t_copy = timeit(lambda: torch.cat(parts if G == 1 or not any(p.dim() == 3 for p in parts) else
                                          [p if p.dim() == 3 else p.unsqueeze(0).expand(G, M, p.shape[-1])
                                           for p in parts], -1))
        print(f"M={M} {name:34s} cat-kernel {t_cat:7.2f} us | plain kernel {t_plain:7.2f} us + torch.cat {t_copy:6.2f} us")


if __name__ == "__main__":
    main()
