"""RK45 step attempts per env per step launch inside the training loop
(configs[3]'s slowest-env explanation).

Runs bench.py's training loop (VecTrainer, bf16 TD7, idealised physics) for a
workload -- `dr_sweep` (configs[3]: 16,384 envs, per-env matrix noise
U(0.05, 0.25), actuator DR U(0, 0.1), shift U(0, 0.04), tremor magnitude
[0.1, 1.0]) or `configs1` (4,096 envs, the defaults) -- with the diagnostic
library (libexo_amd_stamps.so: the row-parallel step kernel writes every
env's two step-attempt counts, accepted + rejected, of scipy's RK45 control),
and histograms them over `--launches` consecutive in-loop launches.  A launch
lasts as long as its slowest wavefront (4 envs x 2 solves at one wave per
SIMD), so the per-launch max and the per-wave max are reported next to the
per-env distribution.  Prints one JSON object.

usage: python tools/rk45_hist.py [--workload dr_sweep|configs1] [--launches 40]
"""
import argparse
import ctypes
import json
import os
import sys

os.environ["EXO_AMD_LIB"] = "libexo_amd_stamps.so"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from exo_amd import VecExoskeletonEnv  # noqa: E402
from exo_amd import _native as nat  # noqa: E402
from exo_amd.rollout import VecTrainer  # noqa: E402
from exo_amd.td7 import Agent  # noqa: E402


def make(workload):
    rank = 0
    if workload == "dr_sweep":  # bench.py main(): configs[3]
        N = 16384
        rng = np.random.default_rng(1000 + rank)
        kw = dict(matrix_noise_fraction=rng.uniform(0.05, 0.25, N), dr_actuator_range=rng.uniform(0.0, 0.1, N),
                  dr_actuator_end_pos_shift=rng.uniform(0.0, 0.04, N), tremor_amplitude_range=(0.1, 1.0))
    else:
        N, kw = 4096, {}
    env = VecExoskeletonEnv(N, seed=1000 + rank, **kw)
    torch.manual_seed(0)
    ag = Agent(80, 7, 1, env_num=8, precision="bf16", n_envs=N, graph_safe=True)
    return env, ag, kw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="dr_sweep", choices=["dr_sweep", "configs1"])
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--eager-launches", type=int, default=0)
    ap.add_argument("--budget", type=int, default=0,
                    help="exo_set_step_budget: a solve's attempts are then recorded in the launch that finishes it")
    a = ap.parse_args()
    env, ag, kw = make(a.workload)
    if a.budget:
        env.set_step_budget(a.budget)
    tr = VecTrainer(env, ag)
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    N = env.n
    buf = torch.full((2, N), -1, dtype=torch.int32, device="cuda")
    lib = nat.lib()
    lib.exo_debug_set_rksteps.argtypes = [ctypes.c_void_p]
    assert lib.exo_debug_set_rksteps(ctypes.c_void_p(buf.data_ptr())) == 0
    per_env, launch_max, launch_mean, wave_max, ks, graph_act = [], [], [], [], [], []
    env_sum, env_cnt = np.zeros(N), np.zeros(N)
    for _ in range(a.launches):
        buf.fill_(-1)
        k = tr.k if tr.k < tr.round_len else 0
        tr.step()
        torch.cuda.synchronize()
        c = buf.cpu().numpy()
        stepped = c[0] >= 0
        if not stepped.any():
            continue
        m = np.maximum(c[0], c[1])[stepped]           # the env's slower solve
        env_sum[stepped] += m
        env_cnt[stepped] += 1
        per_env.append(np.stack([c[0][stepped], c[1][stepped]], 1))
        launch_max.append(int(m.max()))
        launch_mean.append(float(m.mean()))
        w = np.where(stepped, np.maximum(c[0], c[1]), 0).reshape(-1, 4).max(1)  # 4 envs per wavefront
        wave_max.append(w[w > 0])
        ks.append(k)
        graph_act.append(float(tr.last_actions.abs().mean()))
    # the same loop's rollout launched eagerly (bench.py loop_kernel_timing):
    # HIP events around the env step and its attempt counts, launch by launch
    eager = []
    for _ in range(a.eager_launches):
        if tr.k == tr.round_len:
            env.reset(obs_out=tr.obs)
            tr._round_start()
        buf.fill_(-1)
        act = ag.select_action_batch(tr.obs, dec_count=tr.active_count)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        nobs, rew, done, _ = env.step(act, active=tr.active, out=tr._outs[tr._cur])
        e1.record()
        ag.replay_buffer.add_batch(tr.obs, act, nobs, rew, done, tr.strata, tr.active)
        tr._advance()
        torch.cuda.synchronize()
        c = buf.cpu().numpy()
        stepped = c[0] >= 0
        m = np.maximum(c[0], c[1])[stepped]
        eager.append({"k": tr.k, "ms": e0.elapsed_time(e1), "active": int(stepped.sum()),
                      "max_attempts": int(m.max()) if m.size else 0, "mean_attempts": float(m.mean()) if m.size else 0.0,
                      "act_abs_mean": float(act.abs().mean())})
        tr.k += 1
        tr._cur ^= 1
    assert lib.exo_debug_set_rksteps(ctypes.c_void_p(0)) == 0
    pe = np.concatenate(per_env)
    both = pe.max(1)
    wm = np.concatenate(wave_max)
    hist, edges = np.histogram(both, bins=[1, 2, 3, 4, 5, 6, 8, 10, 15, 20, 30, 50, 100, 200, 500, 5000])
    out = {
        "workload": a.workload, "envs": N, "launches": len(launch_max), "round_steps": ks, "step_budget": a.budget,
        "per_env_step_attempts": {"solves": "max of the actuated and the tremor-only solve",
                                  "mean": float(both.mean()), "median": float(np.median(both)),
                                  "p99": float(np.percentile(both, 99)), "p999": float(np.percentile(both, 99.9)),
                                  "max": int(both.max()),
                                  "histogram": {f"{int(edges[i])}-{int(edges[i + 1]) - 1}": int(hist[i])
                                                for i in range(len(hist))}},
        "actuated_vs_tremor_only_mean": [float(pe[:, 0].mean()), float(pe[:, 1].mean())],
        "per_launch_max": {"mean": float(np.mean(launch_max)), "min": int(np.min(launch_max)),
                           "max": int(np.max(launch_max))},
        "per_launch_mean": float(np.mean(launch_mean)),
        "per_wave_max": {"mean": float(wm.mean()), "median": float(np.median(wm)), "p99": float(np.percentile(wm, 99))},
        "slowest_over_mean": float(np.mean(launch_max) / np.mean(launch_mean)),
        "graph_act_abs_mean": graph_act,
    }
    if eager:
        out["eager_launches"] = eager
    if kw:  # which DR draw makes an env slow: mean attempts against its matrix noise fraction
        mf = np.asarray(kw["matrix_noise_fraction"])
        seen = env_cnt > 0
        mean_att = env_sum[seen] / env_cnt[seen]
        out["corr_attempts_vs_matrix_noise"] = float(np.corrcoef(mean_att, mf[seen])[0, 1])
        q = np.quantile(mf[seen], [0, 0.25, 0.5, 0.75, 1.0])
        out["mean_attempts_by_matrix_noise_quartile"] = [
            float(mean_att[(mf[seen] >= q[i]) & (mf[seen] <= q[i + 1])].mean()) for i in range(4)]
        # the slowest envs and their draws (the per-launch max is one env's solve)
        idx = np.flatnonzero(seen)[np.argsort(-mean_att)[:8]]
        obs = tr.obs.float().cpu().numpy()
        out["slowest_envs"] = [{"env": int(i), "mean_attempts": float(env_sum[i] / env_cnt[i]),
                                "launches_seen": int(env_cnt[i]), "motion": int(i % 8),
                                "obs_max_abs": float(np.abs(obs[i]).max()), "obs_finite": bool(np.isfinite(obs[i]).all()),
                                **{k: float(np.asarray(kw[k])[i]) for k in
                                   ("matrix_noise_fraction", "dr_actuator_range", "dr_actuator_end_pos_shift")}}
                               for i in idx]
        out["envs_over_100_attempts_mean"] = int((mean_att > 100).sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
