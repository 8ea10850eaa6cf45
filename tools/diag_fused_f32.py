"""fp32 fused path diagnostics (EXO_FUSED_F32): (1) the packed operand layout
read back against the fp32 master weight; (2) the fixed-embedding pass with
zs2 / zs3 set to identity (zero bias), so the output is AvgL1Norm(elu(elu(zs1(s))))
against plain torch; (3) the full pass against the per-layer kernels."""
import sys
import torch
import torch.nn.functional as F

sys.path.insert(0, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd")
from exo_amd import fused, ops  # noqa: E402
from exo_amd.td7 import Hyperparameters, TD7Learner  # noqa: E402

fused.FUSED_F32 = True
torch.manual_seed(3)
L = TD7Learner(80, 7, Hyperparameters(), device="cuda", precision="fp32")
assert L.fused is not None
net = L.fused.nets["fixed_encoder"]
torch.cuda.synchronize()
for li, pl in enumerate(net.layers):
    W = pl.weight.detach().float().cpu()
    wf = pl.wf.view(torch.float32).cpu().view(-1, 64, 4)
    bad = 0
    for t in range(pl.ntf):
        for s in range(pl.ksf):
            blk = wf[t * pl.ksf + s]
            for l in (0, 5, 17, 33, 63):
                for j in range(4):
                    n, k = 16 * t + l % 16, 16 * s + 4 * (l // 16) + j
                    want = float(W[n, k]) if n < pl.N and k < pl.K else 0.0
                    if float(blk[l, j]) != want:
                        bad += 1
    wbad = 0
    if pl.wb is not None:
        wb = pl.wb.view(torch.float32).cpu().view(-1, 64, 4)
        for t in range(pl.ntb):
            for s in range(pl.ksb):
                blk = wb[t * pl.ksb + s]
                for l in (0, 5, 17, 33, 63):
                    for j in range(4):
                        c, n = 16 * t + l % 16, 16 * s + 4 * (l // 16) + j
                        want = float(W[n, c]) if n < pl.N and c < pl.K else 0.0
                        if float(blk[l, j]) != want:
                            wbad += 1
    print(f"layer {li}: N {pl.N} K {pl.K} ksf {pl.ksf} ntf {pl.ntf}: fwd mismatches {bad}, dX mismatches {wbad}")

g = torch.Generator(device="cuda").manual_seed(0)
s = torch.randn(1024, 80, device="cuda", generator=g)
a = torch.rand(1024, 7, device="cuda", generator=g) * 2 - 1
enc = L.fixed_encoder
with torch.no_grad():
    enc.zs2.weight.copy_(torch.eye(300)); enc.zs2.bias.zero_()
    enc.zs3.weight.copy_(torch.eye(300)); enc.zs3.bias.zero_()
L.fused.pack_all()
zs, zsa = L.fused.fixed(s, a)
with torch.no_grad():
    h = F.elu(F.elu(F.linear(s, enc.zs1.weight, enc.zs1.bias)))
    ref = h / h.abs().mean(-1, keepdim=True).clamp_min(1e-8)
torch.cuda.synchronize()
print("identity zs2/zs3: rel", float((zs - ref).norm() / ref.norm()))
print("row 0 fused", zs[0, :6].tolist())
print("row 0 ref  ", ref[0, :6].tolist())
print("row 1 fused", zs[1, :6].tolist())
print("row 1 ref  ", ref[1, :6].tolist())
print("col corr: fused[:, c] vs ref[:, c'] best c' for c=0..5:",
      [int(((ref - zs[:, c:c + 1]).abs().mean(0)).argmin()) for c in range(6)])
print("row corr: fused[r] vs ref[r'] best r' for r=0..5:",
      [int(((ref - zs[r:r + 1]).abs().mean(1)).argmin()) for r in range(6)])
