#!/usr/bin/env python3
"""exo_step_rp alone at the roofline shape (4,096 envs, all active, U(-1, 1)
actions): per-launch time with HIP events around n back-to-back launches (as
bench.py's roofline measurement), for the library EXO_AMD_LIB names, plus a
fixed 60-step trajectory's outputs digested for a bit-for-bit comparison
between libraries (tools/step_ab.py --compare A_traj.json B_traj.json).

usage: EXO_AMD_LIB=libexo_amd_base.so python tools/step_ab.py OUT_PREFIX [--rounds 5] [--n 100]
       python tools/step_ab.py --compare A_traj.json B_traj.json
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))


def compare(a, b):
    A, B = json.load(open(a)), json.load(open(b))
    bad = [k for k in A if A[k] != B[k]]
    print(json.dumps({"compared": sorted(A), "differ": bad}))
    return 1 if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--variant", default="rows", help="rows (the roofline shape) or rows_shared (the loop's)")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        sys.exit(compare(*args.compare))
    import torch
    from exo_amd import VecExoskeletonEnv

    N = args.envs
    env = VecExoskeletonEnv(N, seed=3)
    env.set_step_variant(args.variant)
    out = env.new_outputs(True)
    g = torch.Generator(device="cuda")
    # trajectory for the bit-for-bit check
    g.manual_seed(7)
    env.reset()
    obs, rew, done, info = [], [], [], []
    for _ in range(60):
        a = torch.rand((N, 7), device="cuda", generator=g) * 2 - 1
        o, r, d, i = env.step(a, out=out)
        obs.append(o.cpu().numpy().copy())
        rew.append(r.cpu().numpy().copy())
        done.append(d.cpu().numpy().copy())
        info.append(i.cpu().numpy().copy())
    # digests of every output of every step (the arrays would exceed gpurun's copy-back)
    dig = {k: hashlib.sha256(np.ascontiguousarray(np.stack(v)).tobytes()).hexdigest()
           for k, v in (("obs", obs), ("rew", rew), ("done", done), ("info", info))}
    with open(args.out + "_traj.json", "w") as f:
        json.dump(dig, f)
    # timing: reset, then n launches between one pair of events, per round
    times = []
    for k in range(args.rounds + 1):
        g.manual_seed(100 + k)
        env.reset()
        acts = torch.rand((args.n, N, 7), device="cuda", generator=g) * 2 - 1
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(args.n):
            env.step(acts[i], out=out)
        e1.record()
        torch.cuda.synchronize()
        if k:  # the first round warms up
            times.append(e0.elapsed_time(e1) / args.n * 1000.0)
    # the bulk reset (exo_reset_kernel over every env), n back-to-back calls per round
    rtimes = []
    for k in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            env.reset()
        e1.record()
        torch.cuda.synchronize()
        if k:
            rtimes.append(e0.elapsed_time(e1) / 10 * 1000.0)
    res = {"lib": os.environ.get("EXO_AMD_LIB", "libexo_amd.so"), "envs": N, "variant": args.variant, "us_per_launch": times,
           "best_us": min(times), "median_us": float(np.median(times)), "reset_us": rtimes}
    print(json.dumps(res))
    with open(args.out + ".json", "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
