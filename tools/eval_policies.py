"""Evaluate the 15 shipped policies (Simulation/AGENT_NNS, exported to
policies/*.safetensors by tools/export_policies.py) in the vectorised env, as
Simulation/Evaluate_control_performance.py does: 100 episodes x 8 envs (env
e follows motion e % 8; episode e // 8), checkpoint actor + checkpoint encoder,
no exploration (:126, TD7_multi_agent_Pink_noise.py:212-214), the evaluation
script's env arguments (:28-44: harmonics [3.75, 6.25] / [7.5, 12.5],
amplitude range [0.95, 1.05], DR 0.025 / 0.04 / 0.125, max forces 40 / 20) and
tremor sequence = the configuration + [0, 0, 0].  The statistics come from
the device kernel exo_eval_metrics (VecExoskeletonEnv.eval_metrics); the three
EVALUATION METRICS of :432-441 are then per-episode ratios averaged over the
100 episodes:
  occurrence  = sum(total < 0 steps) / sum(steps) * 100          (:421)
  total       = sum(negative totals) / count(negative totals)    (:423)
  torque_any  = sum(any-axis-suppressed steps) / sum(L - 3) * 100 (:425)
  torque_all  = sum(all-axes-suppressed steps) / sum(L - 3) * 100 (:426)

usage: python tools/eval_policies.py [--episodes 100] [--physics ideal|multibody] [--out FILE.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from safetensors.torch import load_file  # noqa: E402

from exo_amd import VecExoskeletonEnv  # noqa: E402
from exo_amd.td7 import Actor, Encoder, Hyperparameters  # noqa: E402

# Evaluation_logs/<cfg> EVALUATION METRICS blocks:
# (total amplitude suppression %, amplitude-suppression occurrence %, torque suppression any axis %)
ANCHORS = {
    "[0,0,0,1]": (-80.14, 65.41, 99.49), "[0,0,1,0]": (-34.63, 9.58, 83.27), "[0,0,1,1]": (-50.46, 49.05, 99.45),
    "[0,1,0,0]": (-31.70, 19.49, 57.00), "[0,1,0,1]": (-58.51, 88.06, 99.36), "[0,1,1,0]": (-30.22, 1.66, 87.18),
    "[0,1,1,1]": (-62.44, 65.65, 99.20), "[1,0,0,0]": (-32.76, 11.46, 79.09), "[1,0,0,1]": (-57.37, 58.45, 99.61),
    "[1,0,1,0]": (-36.76, 15.76, 82.99), "[1,0,1,1]": (-46.28, 51.43, 99.39), "[1,1,0,0]": (-40.75, 40.87, 84.00),
    "[1,1,0,1]": (-55.25, 87.83, 99.40), "[1,1,1,0]": (-38.13, 16.48, 82.67), "[1,1,1,1]": (-47.50, 59.38, 98.82)}
EVAL_ENV = dict(tremor_amplitude_range=(0.95, 1.05), first_harmonics_interval=(3.75, 6.25),
                second_harmonics_interval=(7.5, 12.5), max_force_shoulder=40.0, max_force_elbow=20.0,
                dr_actuator_end_pos_shift=0.025, dr_actuator_range=0.04, matrix_noise_fraction=0.125)


def policy(path, device):
    hp = Hyperparameters(actor_hdim=300)  # TD7_multi_agent_Pink_noise.py:54
    actor = Actor(80, 7, hp.zs_dim, hp.actor_hdim, hp.actor_activ).to(device)
    enc = Encoder(80, 7, hp.zs_dim, hp.enc_hdim, hp.enc_activ).to(device)
    t = load_file(path, device=str(device))
    actor.load_state_dict({k[6:]: v for k, v in t.items() if k.startswith("actor.")})
    enc.load_state_dict({k[8:]: v for k, v in t.items() if k.startswith("encoder.")}, strict=False)
    return actor.eval(), enc.eval()


@torch.no_grad()
def evaluate(cfg, path, episodes, physics, seed, device):
    seq = [int(c) for c in cfg.strip("[]").split(",")] + [0, 0, 0]
    n = 8 * episodes
    env = VecExoskeletonEnv(n, seed=seed, device=device, physics=physics, tremor_sequence=seq, **EVAL_ENV)
    actor, enc = policy(path, device)
    obs = env.reset()
    out = env.new_outputs(True)
    counters = torch.zeros((n, 5), dtype=torch.float32, device=device)
    done = out[2]
    steps = torch.zeros(n, dtype=torch.float32, device=device)
    for _ in range(env.max_len):
        active = done == 0
        a = actor(obs, enc.zs(obs)).clamp(-1, 1)
        obs, _, _, info = env.step(a, active=active, out=out)
        counters = env.eval_metrics(info, stepped=active, counters=counters)
        steps += active.float()
    assert bool(done.bool().all()), "episodes did not finish within max_len steps"
    c = counters.double().view(episodes, 8, 5).sum(1).cpu().numpy()
    denom = float((env.lengths_host[:8] - 3).sum())  # total_steps_for_ep (:95-96)
    occ = c[:, 2] / (c[:, 2] + c[:, 3]) * 100
    tot = c[:, 4] / np.maximum(c[:, 2], 1)
    any_ = c[:, 1] / denom * 100
    all_ = c[:, 0] / denom * 100
    r = dict(cfg=cfg, episodes=episodes, envs=n, physics=physics,
             total=[float(tot.mean()), float(tot.std())], occurrence=[float(occ.mean()), float(occ.std())],
             torque_any=[float(any_.mean()), float(any_.std())], torque_all=[float(all_.mean()), float(all_.std())],
             env_steps=int(steps.sum().item()))
    r["anchor"] = dict(zip(("total", "occurrence", "torque_any"), ANCHORS[cfg]))
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--physics", default="ideal")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dir", default=os.path.join(REPO, "policies"))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    res = []
    print(f"{'cfg':10s} {'total %':>16s} {'anchor':>8s} {'occur %':>15s} {'anchor':>8s} {'torque any %':>15s} {'anchor':>8s}  s")
    for f in sorted(os.listdir(a.dir)):
        if not f.endswith(".safetensors"):
            continue
        cfg = f[:-len(".safetensors")]
        t0 = time.time()
        r = evaluate(cfg, os.path.join(a.dir, f), a.episodes, a.physics, a.seed, dev)
        r["seconds"] = time.time() - t0
        res.append(r)
        an = r["anchor"]
        print(f"{cfg:10s} {r['total'][0]:8.2f}+-{r['total'][1]:5.2f} {an['total']:8.2f} "
              f"{r['occurrence'][0]:7.2f}+-{r['occurrence'][1]:5.2f} {an['occurrence']:8.2f} "
              f"{r['torque_any'][0]:7.2f}+-{r['torque_any'][1]:5.2f} {an['torque_any']:8.2f}  {r['seconds']:.1f}",
              flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
