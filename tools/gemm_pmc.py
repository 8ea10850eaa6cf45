"""Target for rocprofv3 --pmc passes: td7_dense_fwd (bf16 MFMA operands) on the
critic's largest layer, both Q heads ([2, 1024, 320, 920] + ELU), 50 launches."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402
from exo_amd import _native as nat  # noqa: E402

m, n, k, G = 1024, 320, 920, 2
L = nat.lib()
x = torch.randn(G, m, k, device="cuda")
w = torch.randn(G, n, k, device="cuda")
b = torch.randn(G, n, device="cuda")
y = torch.empty(G, m, n, device="cuda")
P = nat.ptr
for _ in range(50):
    L.td7_dense_fwd(P(x), m * k, k, P(w), P(b), P(y), m * n, n, G, m, n, k, 2 | 1 << 8, nat.stream_ptr(x.device))
torch.cuda.synchronize()
print("ok")
