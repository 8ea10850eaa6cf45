"""Per-pass timing of the row-tile-fused TD7 launches (csrc/td7_fused.hip)
against the per-layer kernels of the same passes, at the bench's shapes
(bf16; select over 4,096 envs, the update's passes over 8 x 128 rows).  Each
pass is captured 20x in a HIP graph and timed with HIP events over 10 replays.

usage: python tools/fused_bench.py [--precision bf16|fp16] [--width W]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import torch  # noqa: E402

from exo_amd import ops  # noqa: E402
from exo_amd.td7 import Hyperparameters, TD7Learner  # noqa: E402


def timed(fn, reps=20, replays=10):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * replays) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--width", type=int, default=None)
    a = ap.parse_args()
    hp = Hyperparameters() if a.width is None else Hyperparameters(zs_dim=a.width, enc_hdim=a.width,
                                                                   critic_hdim=a.width, actor_hdim=a.width)
    torch.manual_seed(0)
    L = TD7Learner(80, 7, hp, device="cuda", precision=a.precision)
    fz = L.fused
    B, N = 1024, 4096
    obs = torch.randn(N, 80, device="cuda")
    s = torch.randn(B, 80, device="cuda")
    ns = torch.randn(B, 80, device="cuda")
    act = torch.rand(B, 7, device="cuda") * 2 - 1
    r = torch.rand(B, 1, device="cuda")
    nd = torch.ones(B, 1, device="cuda")

    def sel_ref():
        with torch.no_grad(), ops.matrix_precision(a.precision):
            ops.noisy_action(L.act(obs), None, L.exploration_noise_t, 0.0, rng=L._explore_rng)

    def tgt_ref():
        with torch.no_grad():
            L._target_chain(ns, r, nd, None, L.fixed_encoder_target.zs(ns), None)

    def fix_ref():
        with torch.no_grad(), ops.matrix_precision(a.precision):
            zs = L.fixed_encoder.zs(s)
            L.fixed_encoder.zsa(zs, act)

    rows = [("select_action 4096 envs", lambda: fz.select(obs), sel_ref),
            ("target chain 1024 rows (2 launches)", lambda: fz.target_heads(ns), tgt_ref),
            ("fixed zs/zsa 1024 rows", lambda: fz.fixed(s, act), fix_ref),
            ("pack critic_target", lambda: fz.pack("critic_target"), None),
            ("pack actor", lambda: fz.pack("actor"), None)]
    print(f"precision {a.precision}, widths {hp.zs_dim}/{hp.enc_hdim}/{hp.critic_hdim}/{hp.actor_hdim}")
    print(f"{'pass':40s} {'fused us':>10s} {'per-layer us':>13s}")
    for name, f, ref in rows:
        tf = timed(f)
        tr = timed(ref) if ref is not None else float("nan")
        print(f"{name:40s} {tf:10.2f} {tr:13.2f}")


if __name__ == "__main__":
    main()
