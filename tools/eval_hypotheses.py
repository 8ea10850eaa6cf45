"""Which code revision produced the authors' Evaluation_logs?  

The logs' per-env blocks print the episode's max tremor torque per axis as
exactly {10, 5, 2.5, 5} on axes 0-3 in all 12,000 blocks (tools/parse_eval_logs.py),
while the shipped generator draws a magnitude in [0.95, 1.05] and scales
joint_max_values = {2.5, 5, 10, 5, ...} (Utilities/generate_parkinson_tremor.py:59,
Environment/Exoskeleton_env.py:198-199) and flips the sign of every sample (:70),
so its max would vary around {2.5, 5, 10, 5} x magnitude.  This evaluates the 15
shipped policies (tools/eval_policies.py: 100 episodes x 8 envs, checkpoint
nets, no exploration, the evaluation script's env arguments) under tremor
models that differ in exactly those three places (exo_set_tremor_model) and
compares every per-motion statistic of the logs' blocks
(tests/golden/eval_log_stats.json) and the three EVALUATION METRICS.

usage: python tools/eval_hypotheses.py [--models shipped,swap,...] [--episodes 100] [--out FILE.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from eval_policies import ANCHORS, EVAL_ENV, policy  # noqa: E402
from exo_amd import VecExoskeletonEnv  # noqa: E402
from exo_amd.vec_env import INFO_SLICES  # noqa: E402

SHIPPED = [2.5, 5, 10, 5, 5, 0.5, 0.5]
DOCSTRING = [10, 5, 2.5, 5, 5, 0.5, 0.5]  # generate_parkinson_tremor.py:44 "shoulder z 10, y 5, x 2.5, elbow 5"
# name: (joint maxima, magnitude range, sign mode)
MODELS = {
    "shipped": (SHIPPED, (0.95, 1.05), "per_sample"),
    "swap": (DOCSTRING, (0.95, 1.05), "per_sample"),
    "swap_mag1": (DOCSTRING, (1.0, 1.0), "per_sample"),
    "swap_mag1_axis": (DOCSTRING, (1.0, 1.0), "per_axis"),
    "swap_mag1_none": (DOCSTRING, (1.0, 1.0), "none"),
    "mag1_axis": (SHIPPED, (1.0, 1.0), "per_axis"),
}
METRICS = ("score", "pct_to_max", "torque_all", "torque_any", "ampl_occurrence", "ampl_total")


@torch.no_grad()
def evaluate(cfg, path, model, episodes, seed, device):
    jmax, amp, sign = MODELS[model]
    seq = [int(c) for c in cfg.strip("[]").split(",")] + [0, 0, 0]
    n = 8 * episodes
    kw = dict(EVAL_ENV, tremor_amplitude_range=amp)
    env = VecExoskeletonEnv(n, seed=seed, device=device, tremor_sequence=seq, **kw)
    env.set_tremor_model(jmax, sign)
    actor, enc = policy(path, device)
    obs = env.reset()
    out = env.new_outputs(True)
    counters = torch.zeros((n, 5), dtype=torch.float32, device=device)
    done = out[2]
    score = torch.full((n,), 2.0, dtype=torch.float64, device=device)
    ampl_axis = torch.zeros((n, 7), dtype=torch.float64, device=device)
    act_sum = torch.zeros((n, 7), dtype=torch.float64, device=device)   # mean action per actuator
    tau_abs = torch.zeros((n, 7), dtype=torch.float64, device=device)   # mean |exo torque| per joint axis
    max_nm = torch.as_tensor(np.stack([env.tremor(i).max(axis=1) for i in range(min(n, 64))]))
    sa, sta = INFO_SLICES["ampl_val"], INFO_SLICES["tremor_ampl_val"]
    for _ in range(env.max_len):
        active = done == 0
        a = actor(obs, enc.zs(obs)).clamp(-1, 1)
        obs, rew, _, info = env.step(a, active=active, out=out)
        counters = env.eval_metrics(info, stepped=active, counters=counters)
        score += torch.where(active, rew.double(), 0.0)
        am, tam = info[:, sa].double(), info[:, sta].double()
        red = (am.abs() - tam.abs()) / (tam + 1e-10).abs() * 100  # :192
        red = torch.nan_to_num(red, nan=0.0, posinf=0.0, neginf=0.0).clamp(max=0.0)  # :193, :244
        ampl_axis += torch.where(active[:, None], red, 0.0)
        act_sum += torch.where(active[:, None], a.double(), 0.0)
        tau_abs += torch.where(active[:, None], info[:, INFO_SLICES["actuator_torques"]].double().abs(), 0.0)
    assert bool(done.bool().all())
    L = torch.as_tensor(env.lengths_host, device=device, dtype=torch.float64)
    entries = torch.clamp(L, max=float(env.lengths_host.max() - 3))  # rows of the [:L] slices (:329, :336)
    c = counters.double()
    per_env = {
        "score": score, "pct_to_max": (score - 2) / (L - 2) * 100,
        "torque_all": c[:, 0] / (L - 3) * 100, "torque_any": c[:, 1] / (L - 3) * 100,
        "ampl_occurrence": c[:, 2] / L * 100, "ampl_total": c[:, 4] / entries,
    }
    r = {"cfg": cfg, "model": model, "motions": {}}
    for m in range(8):
        r["motions"][str(m)] = {k: [float(v.view(episodes, 8)[:, m].mean()), float(v.view(episodes, 8)[:, m].std())]
                                for k, v in per_env.items()}
        ax = (ampl_axis / entries[:, None]).view(episodes, 8, 7)[:, m]
        r["motions"][str(m)]["ampl_axis"] = ax.mean(0).tolist()
        r["motions"][str(m)]["mean_action"] = (act_sum / (L - 3)[:, None]).view(episodes, 8, 7)[:, m].mean(0).tolist()
        r["motions"][str(m)]["mean_abs_exo_torque"] = (tau_abs / (L - 3)[:, None]).view(episodes, 8, 7)[:, m].mean(0).tolist()
    # the three EVALUATION METRICS (per-episode ratios over the 8 envs, averaged)
    cc = c.view(episodes, 8, 5).sum(1).cpu().numpy()
    denom = float((env.lengths_host[:8] - 3).sum())
    r["total"] = float((cc[:, 4] / np.maximum(cc[:, 2], 1)).mean())
    r["occurrence"] = float((cc[:, 2] / (cc[:, 2] + cc[:, 3]) * 100).mean())
    r["torque_any"] = float((cc[:, 1] / denom * 100).mean())
    r["max_nm_first_envs"] = max_nm.max(0).values.tolist()
    env.close()
    return r


def compare(r, logs):
    """Per-metric mean |build - log| over the 8 motions, in units of the log's
    per-motion standard error (std / sqrt(100)) as well as absolute."""
    out = {}
    for k in METRICS:
        d, z = [], []
        for m in range(8):
            ours, lg = r["motions"][str(m)][k], logs[str(m)][k]
            d.append(ours[0] - lg["mean"])
            se = np.hypot(lg["std"], ours[1]) / 10.0
            z.append(abs(ours[0] - lg["mean"]) / max(se, 1e-9))
        out[k] = {"mean_abs_diff": float(np.mean(np.abs(d))), "mean_z": float(np.mean(z))}
    ax = np.array([r["motions"][str(m)]["ampl_axis"] for m in range(8)])
    lax = np.array([logs[str(m)]["ampl_axis"]["mean"] for m in range(8)])
    out["ampl_axis"] = {"mean_abs_diff": float(np.abs(ax - lax).mean())}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default=",".join(MODELS))
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dir", default=os.path.join(REPO, "policies"))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    logs = json.load(open(os.path.join(REPO, "tests", "golden", "eval_log_stats.json")))
    dev = torch.device("cuda:0")
    res = []
    cfgs = sorted(f[:-len(".safetensors")] for f in os.listdir(a.dir) if f.endswith(".safetensors"))
    for model in a.models.split(","):
        t0 = time.time()
        agg = {k: [] for k in METRICS + ("ampl_axis",)}
        hits = {"total": 0, "occurrence": 0, "torque_any": 0}
        for cfg in cfgs:
            r = evaluate(cfg, os.path.join(a.dir, cfg + ".safetensors"), model, a.episodes, a.seed, dev)
            r["vs_log"] = compare(r, logs[cfg])
            r["anchor"] = dict(zip(("total", "occurrence", "torque_any"), ANCHORS[cfg]))
            for k in hits:
                hits[k] += abs(r[k] - r["anchor"][k]) <= 10.0
            for k in agg:
                agg[k].append(r["vs_log"][k]["mean_abs_diff"])
            res.append(r)
            print(f"  {model:15s} {cfg}: total {r['total']:7.2f} ({r['anchor']['total']:7.2f}) "
                  f"occ {r['occurrence']:6.2f} ({r['anchor']['occurrence']:6.2f}) "
                  f"any {r['torque_any']:6.2f} ({r['anchor']['torque_any']:6.2f}) max_nm {r['max_nm_first_envs'][:4]}",
                  flush=True)
        print(f"{model:15s} within 10 points: total {hits['total']}/15, occurrence {hits['occurrence']}/15, "
              f"torque_any {hits['torque_any']}/15 | mean |build - log| per motion: "
              + ", ".join(f"{k} {np.mean(v):.2f}" for k, v in agg.items()) + f"  ({time.time() - t0:.0f} s)", flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=0)


if __name__ == "__main__":
    main()
