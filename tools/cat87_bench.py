import ctypes, os, sys
sys.path.insert(0, "tools")
from dense_bench import timeit
import torch
from exo_amd import _native as nat
L = nat.lib(); dev = torch.device("cuda")
for prec in (1, 2):
    for N in (320, 1024):
        M = 1024
        parts = [torch.randn(M, 80, device=dev), torch.randn(M, 7, device=dev)]
        w = torch.randn(2, N, 87, device=dev); b = torch.randn(2, N, device=dev); y = torch.empty(2, M, N, device=dev)
        P = (ctypes.c_void_p * 2)(*[p.data_ptr() for p in parts]); SG = (ctypes.c_long * 2)(0, 0)
        LD = (ctypes.c_long * 2)(80, 7); WD = (ctypes.c_int32 * 2)(80, 7)
        t = timeit(lambda: L.td7_dense_fwd_cat(2, P, SG, LD, WD, nat.ptr(w), nat.ptr(b), nat.ptr(y), M * N, N, 2, M, N, 0 | prec << 8, nat.stream_ptr(dev)))
        full = torch.cat(parts, 1)
        t2 = timeit(lambda: L.td7_dense_fwd(nat.ptr(full), 0, 87, nat.ptr(w), nat.ptr(b), nat.ptr(y), M * N, N, 2, M, N, 87, 0 | prec << 8, nat.stream_ptr(dev)))
        print(f"prec {prec} N {N}: cat {t:.2f} us, plain {t2:.2f} us")
