"""Diagnostic: per-phase cycles (s_memtime stamps, libexo_amd_stamps.so) of the
fused TD7 gradient passes: one bench-shape update (8 x 128 rows, bf16) with an
actor update, stamps of workgroup 0..n of each launch.  Layers stamp [gemm
start, gemm end, epilogue end]; see the kernels for the extra stamps.  Never
the measured number -- read the shares."""
import ctypes
import os
import sys

STAMPS = os.environ.get("EXO_FUSED_NOSTAMPS", "0") != "1"  # 1: product library, timing by rocprof
if STAMPS:
    os.environ["EXO_AMD_LIB"] = "libexo_amd_stamps.so"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exo_amd import _native as nat  # noqa: E402
from exo_amd.td7 import Hyperparameters, TD7Learner  # noqa: E402

torch.manual_seed(0)
L = TD7Learner(80, 7, Hyperparameters(), device="cuda", precision="bf16")
B = 1024
g = torch.Generator(device="cuda").manual_seed(1)
s, ns = torch.randn(B, 80, device="cuda", generator=g), torch.randn(B, 80, device="cuda", generator=g)
a = torch.rand(B, 7, device="cuda", generator=g) * 2 - 1
r, nd = torch.rand(B, 1, device="cuda", generator=g), torch.ones(B, 1, device="cuda")
lib = nat.lib()
if STAMPS:
    lib.td7f_train_debug_set_stamps.argtypes = [ctypes.c_void_p]
buf = torch.zeros(256 * 64, dtype=torch.int64, device="cuda")
tr = L.fused.train(B)
for _ in range(3):
    L.phase_grads(s, a, ns, r, nd)
    L.phase_steps()
    L.phase_actor_grads(s, a)
    L.phase_actor_step()
torch.cuda.synchronize()
zs, zsa = L.fused.fixed(s, a)
qt = L.fused.target_heads(ns)
passes = (("encoder", lambda: tr.encoder(s, a, ns), 64), ("critic", lambda: tr.critic(s, a, zs, zsa, qt, r, nd), 128),
          ("actor_a", lambda: tr.actor(0, s, zs), 64), ("actor_b", lambda: tr.actor(1, s, zs), 128),
          ("actor_c", lambda: tr.actor(2, s, zs), 64))
for name, fn, nblk in passes:
    fn()
    torch.cuda.synchronize()
    if not STAMPS:
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        continue
    buf.zero_()
    assert lib.td7f_train_debug_set_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    fn()
    torch.cuda.synchronize()
    assert lib.td7f_train_debug_set_stamps(ctypes.c_void_p(0)) == 0
    st = buf.view(256, 64)[:nblk].cpu().numpy().astype(np.int64)
    n = int((st[0] != 0).sum())
    d = np.diff(st[:, :n], axis=1)
    print(f"{name}: {n} stamps, median total {np.median(st[:, n - 1] - st[:, 0]):.0f} cycles")
    print("  " + " ".join(f"{x:.0f}" for x in np.median(d, axis=0)))
