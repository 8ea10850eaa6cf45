"""Diagnostic: per-phase cycles of the fused TD7 kernels from in-kernel
s_memtime stamps (libexo_amd_stamps.so: make -C csrc stamps).  Each fused layer
stamps [gemm start, gemm end (after the k-group reduction), epilogue end];
kernels stamp their start.  Prints the median (over workgroups) cycles between
consecutive stamps of one launch of each pass.  Never the measured number --
read the shares."""
import ctypes
import os
import sys

os.environ["EXO_AMD_LIB"] = "libexo_amd_stamps.so"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exo_amd import _native as nat  # noqa: E402
from exo_amd.td7 import Hyperparameters, TD7Learner  # noqa: E402

torch.manual_seed(0)
L = TD7Learner(80, 7, Hyperparameters(), device="cuda", precision=sys.argv[1] if len(sys.argv) > 1 else "bf16")
fz = L.fused
B = 1024
s = torch.randn(B, 80, device="cuda")
a = torch.rand(B, 7, device="cuda") * 2 - 1
obs = torch.randn(4096, 80, device="cuda")
lib = nat.lib()
lib.td7f_debug_set_stamps.argtypes = [ctypes.c_void_p]
buf = torch.zeros(512 * 64, dtype=torch.int64, device="cuda")
for name, fn, nblk in (("fixed", lambda: fz.fixed(s, a), 64), ("select", lambda: fz.select(obs), 256),
                       ("target_b (last of 2)", lambda: fz.target_heads(s), 128)):
    for k in range(5):
        fn()
    torch.cuda.synchronize()
    buf.zero_()
    assert lib.td7f_debug_set_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    fn()
    torch.cuda.synchronize()
    assert lib.td7f_debug_set_stamps(ctypes.c_void_p(0)) == 0
    st = buf.view(512, 64)[:nblk].cpu().numpy().astype(np.int64)
    n = int((st[0] != 0).sum())
    d = np.diff(st[:, :n], axis=1)
    med = np.median(d, axis=0)
    tot = np.median(st[:, n - 1] - st[:, 0])
    print(f"{name}: {n} stamps, median total {tot:.0f} cycles")
    print("  " + " ".join(f"{x:.0f}" for x in med))
