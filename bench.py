#!/usr/bin/env python3
"""Benchmark of the hot path named by BASELINE.json: the vectorised exoskeleton
env step (HIP) + the TD7 update with LAP replay, 4096 envs per MI355X
(BASELINE.json configs[1]).

One bench "step" (mode train, default) = one vectorised env step of all envs
(batched actor inference -> exo_step kernel -> LAP replay insert) followed by
one TD7 train() grad step at batch 8 strata x 128 = 1024 -- the reference's
ratio of one grad step per episode-round env step
(Simulation/Exoskeleton_agent_train.py:208 trains round(mean(ep_len)) steps
per round of max(ep_len) env steps).  Episodes (r04): async by default --
each env resets in place when its own episode ends, inside the timed
iterations, so every launch steps every env (`--episodes sync`: the
reference script's synchronous rounds, all envs reset together and done envs
idle until the longest motion, 344 steps, ends; reported beside the async
line as `sync_rounds`).  `value` counts ACTIVE env-steps only, over the timed
window's wall time.

mode env: the env alone (random actions), for the sim-kernel roofline.

Multi-GPU: one process per GPU (torchrun); envs shard with no exchange,
TD7 gradients are all-reduced over RCCL (weak scaling).  On RCCL the trainer
replays the iterations with the collectives captured in the graphs, the
target refresh included (`dp_layout` and `dist_settle_iterations` -- 0 by
default since r05 -- in the line).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd")
sys.path.insert(0, PKG)

# before the HIP runtime initialises (see exo_amd/__init__.py)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
# the reference schedule's burst steps sample the next batch at their end
# (RefScheduleTrainer.burst_prefetch; 74.5 vs 75.6 ms per burst): on here,
# where every finished phase's graphs are released with ballast streams (_release)
os.environ.setdefault("EXO_BURST_PREFETCH", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

# Algorithmic bytes of one active env-step of exo_step_kernel (DESIGN.md,
# "exo_step bytes"): every array the step logically reads or writes once.
STEP_READ_BYTES = {
    "action f32[7]": 28, "counts/L/motion/seq i32": 16, "max_output_shoulder/elbow f64[2]": 16,
    "joint positions f64[5]": 40, "cached reference CoMs f64[6]": 48, "dummy shift f64[42]": 336,
    "tremor rows f64[15] (7 at c, 4 at c-1, 4 at c+1)": 120, "prev/second-prev action f64[14]": 112,
    "position vectors f32[21]": 84, "config f64[4]": 32, "I^-1 blocks f64[16]": 128, "D, S sym nnz f64[28]": 224,
}
STEP_WRITE_BYTES = {
    "obs f32[80]": 320, "reward f32": 4, "done u8": 1, "info f32[40]": 160, "counts i32": 4,
    "joint positions f64[5]": 40, "reference CoMs f64[6]": 48, "position vectors f32[21]": 84,
    "prev/second-prev action f64[14]": 112,
}
BYTES_PER_ENV_STEP = sum(STEP_READ_BYTES.values()) + sum(STEP_WRITE_BYTES.values())


FP64_VALU_PEAK_TFS = 78.6   # MI355X fp64 vector peak (AMD spec)

# Useful fp64 flops of one env step: the step's arithmetic done once per env
# by a scalar (one-lane) implementation of the kernel's algorithm, as opposed
# to the PMC count of issued lane-flops (16 lanes per env, the FK on every
# lane, a pad row per 8-lane group).  Counted by hand from csrc/exo_step_rp.hip
# (a flop per add / mul / div, 2 per FMA, sqrt / exp / sincos polynomials as
# their flops):
#   RHS a = I^-1 (T - D v - K q): D and K 21 nonzeros (42 + 42), T - dq - kq 14,
#     I^-1 25 nonzeros (50)                                          -> 148
#   one RK45 step attempt: 6 RHS 888, stage sums 665 (7 rows x sum over
#     stages 1..5 of 4 st + 7), solution 182, error terms 224, norm 31,
#     step control 10                                                -> 2,000
#   per solve: scipy's initial step (2 RHS + norms)                  -> 385
#   FK 506, 7 actuators 567, torque sums 16, reward 180, observation 30,
#     joint targets 30                                               -> 1,329
# useful = 2 x 385 + attempts x 2,000 + 1,329, attempts = the env's actuated +
# tremor-only step attempts (accepted + rejected), measured in the loop by
# tools/rk45_hist.py (profiles/r03_dr_raw/rk45_hist_configs1.json).
USEFUL_FLOPS = {"rhs": 148, "attempt": 2000, "initial_step": 385, "non_ode": 1329}


def useful_fp64_flops_per_env_step():
    f = os.path.join(REPO, "profiles", "r03_dr_raw", "rk45_hist_configs1.json")
    att = sum(json.load(open(f))["actuated_vs_tremor_only_mean"])
    return (2 * USEFUL_FLOPS["initial_step"] + att * USEFUL_FLOPS["attempt"] + USEFUL_FLOPS["non_ode"],
            att, os.path.relpath(f, REPO))
FP32_MFMA_PEAK_TFS = 157.3  # v_mfma_f32_*_f32 dense peak (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFS = 2500.0  # bf16 / fp16 dense MFMA peak (MI355X_MICROARCH.md, no sparsity)
MFMA_PEAK_TFS = {"fp32": FP32_MFMA_PEAK_TFS, "bf16": BF16_MFMA_PEAK_TFS, "fp16": BF16_MFMA_PEAK_TFS}

# BASELINE.json configs: configs[1] is the bench line; configs[3] / configs[4]
# run with --workload (their own lines, not the driver's bench line)
WORKLOADS = {
    "configs1": "configs[1]: 4096 vectorised exo envs per MI355X",
    "dr_sweep": "configs[3]: domain-randomised tremor/DR sweep, per-env draws",
    "wide": "configs[4]: wide TD7 (1024-wide MLPs, reference layer count), fp16 MFMA",
}


def td7_flops(agent, n_envs):
    """Matrix flops of one training iteration: every Linear layer's 2*M*N*K,
    x3 where it is trained (forward, input grad, weight grad), per the
    reference's update (Agent/TD7_multi_agent.py:211-293) and select_action."""
    L = agent.learner
    hp = agent.hp
    B = hp.batch_size * agent.env_num
    def net(m, prefix=""):  # multiply-accumulates per row: sum of out*in over the weight matrices
        macs = 0
        for name, p in m.named_parameters():
            if name.startswith(prefix) and p.dim() >= 2:
                macs += p.numel()  # stacked critic heads [2, out, in] count both
        return macs

    enc_zs = net(L.encoder, "zs1") + net(L.encoder, "zs2") + net(L.encoder, "zs3")
    enc_zsa = net(L.encoder) - enc_zs
    actor, critic = net(L.actor), net(L.critic)
    macs = 0
    macs += 3 * (2 * B * enc_zs) + 3 * B * enc_zsa            # encoder: zs(s), zs(s') fwd (+bwd of zs(s)), zsa trained
    macs += B * (enc_zs + actor + enc_zsa + critic)            # target path (no grad)
    macs += B * (enc_zs + enc_zsa)                              # fixed embeddings
    macs += 3 * B * critic                                      # critic trained
    macs += 0.5 * B * (3 * actor + 2 * (enc_zsa + critic))     # actor update every policy_freq=2 steps
    macs += n_envs * (enc_zs + actor)                           # select_action for every env
    return 2.0 * macs


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (workload default: 4096 / 16384 / 65536)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="configs1")
    ap.add_argument("--mode", choices=["train", "env"], default="train")
    ap.add_argument("--physics", choices=["ideal", "multibody"], default="ideal",
                    help="stepSimulation model: idealised motors (default, SURVEY.md A.2) or the multibody solve")
    ap.add_argument("--precision", choices=["bf16", "fp16", "fp32"], default=None,
                    help="TD7 MFMA operands (workload default: bf16 per configs[1], fp16 for wide)")
    ap.add_argument("--batch", type=int, default=None, help="TD7 rows per stratum (default 128)")
    ap.add_argument("--episodes", choices=["sync", "async"], default=None,
                    help="VecTrainer episodes: sync = the script's synchronous rounds, async = each env resets in "
                         "place when its episode ends (exo_episode_advance); default: EXO_EPISODES or sync")
    ap.add_argument("--step-budget", type=int, default=None,
                    help="RK45 attempts per solve and env-step launch (exo_set_step_budget; default: 0 = no limit, "
                         "dr_sweep 160)")
    ap.add_argument("--cpu-threads", type=int, default=None, help="threads of the multi-core CPU baseline")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP graph capture of the training iteration")
    ap.add_argument("--kernel-timing-steps", type=int, default=100,
                    help="env-only launches timed with HIP events for the roofline line")
    ap.add_argument("--no-td7-variants", action="store_true",
                    help="skip the fp32-TD7 and 256-wide-alias sub-lines (configs[1] train mode)")
    ap.add_argument("--step-clock", choices=["auto", "on", "off"], default="auto",
                    help="configs[3] / [4]: device wall-clock kernels around every step launch inside the timed "
                         "window (exo_set_step_clock; two extra launches on the rollout chain); auto = on with "
                         "synchronous rounds only -- with async episodes the roofline launch is timed after the "
                         "window on the loop's own state")
    ap.add_argument("--no-sync-rounds", action="store_true",
                    help="skip the synchronous-round comparison of the async-episode loop (configs[1])")
    ap.add_argument("--no-reference-schedule", action="store_true",
                    help="skip the reference-schedule sub-line (RefScheduleTrainer, train mode)")
    a = ap.parse_args()
    if a.envs is None:
        a.envs = {"configs1": 4096, "dr_sweep": 16384, "wide": 65536}[a.workload]
    if a.precision is None:
        a.precision = "fp16" if a.workload == "wide" else "bf16"
    if a.step_budget is None:
        # configs[3]: 8 attempts per launch (profiles/r04o_raw, async episodes: 32.0 M
        # env-steps/s at 8, 31.7 M at 16, 29.6 M at 32, 26.8 M at 64; r04d_raw: 25.3 M
        # at 96, 21.5 M at 160, 10.5 M unbudgeted)
        a.step_budget = 8 if a.workload == "dr_sweep" and a.mode == "train" else 0
    if a.episodes is None:
        # the vectorised trainer's own episodes: every env resets in place when its
        # episode ends (EXO_EPISODES=sync: the script's synchronous rounds)
        a.episodes = os.environ.get("EXO_EPISODES", "async")
    return a


def pmc_traffic(bytes_per_launch):
    """HBM bytes per exo_step launch from the newest committed PMC summary
    (profiles/r*_rocprof_summary.json, FETCH_SIZE x2 + WRITE_SIZE, see
    profiles/summarize.py) -- only if it was taken on this same workload."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_rocprof_summary.json")))
    for f in reversed(files):
        d = json.load(open(f)).get("pmc_exo_step")
        if d and d.get("algorithmic_bytes_per_launch") == bytes_per_launch:
            return d["traffic_bytes_per_launch"], os.path.relpath(f, REPO)
    return None, None


def pmc_valu_flops(envs_per_launch):
    """fp64 VALU flops per exo_step launch from the newest committed PMC pass
    (profiles/r*_valu_exo_step.json, tools/env_valu_pmc.sh) on this env count."""
    import glob
    for f in reversed(sorted(glob.glob(os.path.join(REPO, "profiles", "r*_valu_exo_step.json")))):
        d = json.load(open(f))
        if d.get("envs_per_launch") == envs_per_launch:
            return d["fp64_flops_per_launch"], os.path.relpath(f, REPO)
    return None, None


def cpu_td7_update_seconds(hp, batch_rows, threads, budget=6.0):
    """Seconds per TD7 update on the host cores: the build's TD7Learner (the
    reference's update math, Agent/TD7_multi_agent.py:211-293) on torch-CPU
    fp32 with `threads` intra-op threads, a bounded sample of updates on a
    synthetic batch of the bench's size."""
    from exo_amd.td7 import TD7Learner
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        L = TD7Learner(80, 7, hp, device="cpu", fused_adam=False)
        g = torch.Generator().manual_seed(0)
        s = torch.randn(batch_rows, 80, generator=g)
        a = torch.rand(batch_rows, 7, generator=g) * 2 - 1
        ns = torch.randn(batch_rows, 80, generator=g)
        r = torch.rand(batch_rows, 1, generator=g)
        nd = torch.ones(batch_rows, 1)
        L.update(s, a, ns, r, nd)  # warm
        n, t0 = 0, time.perf_counter()
        while n < 2 or (time.perf_counter() - t0 < budget and n < 50):
            L.update(s, a, ns, r, nd)
            n += 1
        return (time.perf_counter() - t0) / n, n
    finally:
        torch.set_num_threads(prev)


def cpu_baseline(seconds, threads=None, td7=None):
    """The oracle (plain C, fp64) stepping 8 envs each, one per motion, with
    random actions -- the 'port' CPU baseline: one core for ~1/3 of the
    budget, then one stepping loop per host core (ctypes drops the GIL) for
    the rest.  With td7=(hp, batch_rows, env_steps_per_iteration) the same
    training loop as the GPU bench is priced on the host: per iteration the
    env-steps at the all-core env rate plus one TD7 update on all cores, and
    `value` is that loop's env-steps/s; otherwise `value` is the env rate."""
    import threading
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from exo_amd import motions
    angles, lengths = motions.load()
    O.bench(8, angles, lengths, 2000)  # warm
    chunk = 20000

    def run(budget, seed0, out, i):
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget:
            steps += O.bench(8, angles, lengths, chunk, seed=seed0 + steps + 1)
        out[i] = (steps, time.perf_counter() - t0)

    one = [None]
    run(seconds / 3, 0, one, 0)
    s1, d1 = one[0]
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    res = [None] * threads
    ts = [threading.Thread(target=run, args=(seconds * 2 / 3, 10 ** 9 * (i + 1), res, i)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    steps = sum(r[0] for r in res)
    env_rate = steps / dt
    out = {"value": env_rate, "unit": "env-steps/s", "cores": threads, "kind": "port",
           "env_only_value": env_rate, "single_core_value": s1 / d1,
           "sample": f"oracle/exo_oracle.c env.step (fp64, the reference's algorithm incl. scipy-RK45 control), "
                     f"8 envs (one per motion) per thread, random actions, episode-synchronous resets: "
                     f"{steps} env-steps in {dt:.1f} s on {threads} threads; 1 core: {s1} in {d1:.1f} s"}
    if td7 is not None:
        hp, rows, per_it = td7
        upd, n = cpu_td7_update_seconds(hp, rows, threads)
        it_s = per_it / env_rate + upd
        out["value"] = per_it / it_s
        out["td7_update_ms"] = upd * 1e3
        out["sample"] += (f"; + TD7 update (build's TD7Learner, torch-CPU fp32, {threads} threads, batch {rows}): "
                          f"{upd * 1e3:.1f} ms per update over {n} updates; value = the bench loop priced on the "
                          f"host: {per_it:.0f} active env-steps + 1 update per iteration")
    return out


def critic_gemm_timing(agent, reps=20, replays=10):
    """The critic's largest GEMM (both Q heads of Linear(2 zs + h -> h) + ELU,
    Agent/TD7_multi_agent.py:121-126) alone: td7_dense_fwd launches captured in
    a HIP graph, HIP events around the replays.  Returns (us per launch, flop)."""
    from exo_amd import ops
    L = agent.learner
    c = L.critic
    B = agent.hp.batch_size * agent.env_num
    dev = c.w1.device
    x = torch.randn(2, B, c.w1.shape[2], device=dev)
    fn = lambda: ops.dense(x, c.w1, c.b1, ops.ACT_CODES["elu"])  # noqa: E731
    with torch.no_grad(), ops.matrix_precision(L.precision):
        fn()
        st = torch.cuda.Stream(device=dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        from exo_amd.graphs import capture, new_graph
        g = new_graph()
        with torch.cuda.stream(st):
            with capture(g, stream=st):
                for _ in range(reps):
                    fn()
        torch.cuda.current_stream(dev).wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / (reps * replays) * 1e3
    return us, 2.0 * 2 * B * c.w1.shape[1] * c.w1.shape[2]


# per-CU L2 weight-stream rate, warm (tools/stream_bench.hip, profiles/r02b_raw/stream_bench.txt:
# 4-16 waves x 12-25 16-byte loads in flight per wave, 64 workgroups: 112-125 GB/s)
L2_STREAM_PER_CU_GBS = 125.0


def fused_critic_timing(agent, reps=20, replays=10):
    """The fused critic update pass alone (td7f_critic, csrc/td7_fused_train.hip:
    both heads' forward, LAP-Huber loss and backward to the gradient operands,
    Agent/TD7_multi_agent.py:248-262), graph-captured, HIP events around the
    replays.  Returns dict(us, mfma flop, weight bytes per workgroup,
    workgroups) or None when the fused path is off."""
    from exo_amd.fused import _ks, _tiles
    L = agent.learner
    fz = L.fused
    if fz is None:
        return None
    hp = agent.hp
    B = hp.batch_size * agent.env_num
    dev = L.device
    tr = fz.train(B)
    S, A, Z, Hc = tr.S, tr.A, hp.zs_dim, hp.critic_hdim
    g = torch.Generator(device=dev).manual_seed(0)
    state = torch.randn(B, S, device=dev, generator=g)
    action = torch.rand(B, A, device=dev, generator=g) * 2 - 1
    zs, zsa = torch.randn(B, Z, device=dev, generator=g), torch.randn(B, Z, device=dev, generator=g)
    qt = torch.randn(B, 2, device=dev, generator=g)
    reward, nd = torch.rand(B, 1, device=dev, generator=g), torch.ones(B, 1, device=dev)
    fn = lambda: tr.critic(state, action, zs, zsa, qt, reward, nd)  # noqa: E731
    fn()
    st = torch.cuda.Stream(device=dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    from exo_amd.graphs import capture, new_graph
    gr = new_graph()
    with torch.cuda.stream(st):
        with capture(gr, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream(dev).wait_stream(st)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / (reps * replays) * 1e3
    # MFMA work of both heads (the N = 1 head on the VALU excluded): forward
    # q0, q1, q2; backward dX of q2 and of q1's q window (q0's dX is not needed)
    flop = 2 * (2.0 * B * (Hc * (S + A) + Hc * (Hc + 2 * Z) + Hc * Hc) + 2.0 * B * (Hc * Hc + Hc * Hc))
    # weight fragments one workgroup (16 rows, one head) streams: the forward
    # packs of q0, q1, q2 and the dX packs of q2 and of q1's first Hc inputs
    kib = 1024
    per_wg = kib * _tiles(Hc) * (_ks(S + A) + _ks(Hc + 2 * Z) + _ks(Hc)) + kib * _ks(Hc) * (_tiles(Hc) + Hc // 16)
    return {"us": us, "flop": flop, "bytes_per_wg": per_wg, "workgroups": 2 * (-(-B // 16))}


# the reference's update-to-data ratio: per episode round of its 8 envs
# (Σ(L-3) = 2,257 active env-steps) it trains round(mean(ep_len)) = 283 steps
# (Simulation/Exoskeleton_agent_train.py:115,145,208 -> TD7_multi_agent.py:315-325)
REFERENCE_ENV_STEPS_PER_UPDATE = 2257 / 283


def _release(tr):
    """Release a finished phase's graphs with the device idle
    (exo_amd.rollout.retire_graphs: execs and memory pools destroyed, then
    ballast streams created so the runtime streams they held are replaced on
    the least-loaded hardware queues -- destroying execs alone can make the
    ROCm 7.0 runtime's launch of a later graph read past its stream vector,
    DESIGN.md 4, "The graph-replay crash")."""
    from exo_amd.rollout import retire_graphs
    torch.cuda.synchronize()
    retire_graphs(tr)
    torch.cuda.synchronize()


def _collect():
    import gc
    gc.collect()
    torch.cuda.synchronize()


def sync_rounds(env, dev, args, hp, group=None, warm=40):
    """The same training loop with the script's synchronous episode rounds
    (VecTrainer episodes="sync": every env resets when the longest motion ends,
    envs whose motion ended idle until then), for comparison with the default
    async episodes: fresh agent on the bench's envs, `warm` untimed iterations,
    then one whole round (its reset included) timed end to end, barrier +
    synchronize on both sides, max over ranks; active env-steps summed."""
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent
    rank = dist.get_rank(group) if group is not None else 0
    torch.manual_seed(5 + rank)
    ag = Agent(80, 7, 1, env_num=8, hp=hp, device=dev, precision=args.precision, n_envs=env.n, graph_safe=True,
               process_group=group)
    tr = VecTrainer(env, ag, episodes="sync")
    tr.plan(warm)
    for _ in range(warm):
        tr.step()
    tr.plan(None)
    while not tr.next_step_resets():
        tr.step()

    def sync_all():
        torch.cuda.synchronize()
        if group is not None:
            dist.barrier(group)
        torch.cuda.synchronize()

    tr.plan(None if tr.budget else tr.round_len)  # the round's iterations (pair graphs inside)
    tr.prepare()
    sync_all()
    t = time.perf_counter()
    n, its = tr.step(), 1
    while not tr.next_step_resets():
        n += tr.step()
        its += 1
    sync_all()
    v = torch.tensor([time.perf_counter() - t, float(n)], device=dev, dtype=torch.float64)
    if group is not None:
        dt = v[:1].clone()
        dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(v, op=dist.ReduceOp.SUM, group=group)
        v[0] = dt[0]
    sec, total = float(v[0]), float(v[1])
    _release(tr)
    del tr, ag
    _collect()
    return {"value": total / sec, "seconds": sec, "iterations": its, "ms_per_iteration": sec / its * 1e3,
            "active_env_steps": total,
            "note": "VecTrainer(episodes='sync'): one whole round incl. its reset, timed end to end after "
                    f"{warm} warm-up iterations; envs whose motion ended idle until the round's longest ends"}


def reference_schedule(env, dev, args, hp, rounds=3, warm_rounds=3, group=None):
    """The reference training script's schedule on the same envs
    (exo_amd.rollout.RefScheduleTrainer, Simulation/Exoskeleton_agent_train.py:
    110-211): per episode round a synchronous rollout of every env (uniform
    actions until 25,000 env-steps, then select_action with exploration;
    transitions inserted with the reference's shared replay pointer), then
    maybe_train_and_checkpoint's burst of round(mean(ep_len)) = 283
    graph-replayed TD7 steps with the policy-checkpoint rule.  Fresh agent;
    `warm_rounds` untimed (the first is the random warm-up and captures the
    graphs, the third captures the policy round's rollout graph), then
    `rounds` timed with the rollout and the burst timed apart.  Data parallel
    (group): every rank runs its envs; the warm-up counts every rank's
    env-steps, the checkpoint rule sees the MIN of the ranks' returns, the
    bursts' gradients are all-reduced; times are the max over
    ranks and env-steps the sum."""
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent
    rank = dist.get_rank(group) if group is not None else 0
    torch.manual_seed(2 + rank)  # per-rank warm-up actions; the weights are rank 0's broadcast
    ag = Agent(80, 7, 1, env_num=8, hp=hp, device=dev, precision=args.precision, n_envs=env.n, graph_safe=True,
               process_group=group)
    tr = RefScheduleTrainer(env, ag, warmup=25_000)
    for _ in range(warm_rounds):
        tr.run_round()
    torch.cuda.synchronize()
    # the rollout and the burst of each round timed apart (host clock, synchronised)
    t_roll = t_burst = 0.0
    orig = ag.maybe_train_and_checkpoint

    def timed_burst(ep_timesteps, ep_return, train=None):
        nonlocal t_burst
        torch.cuda.synchronize()
        t = time.perf_counter()
        orig(ep_timesteps, ep_return, train=train)
        torch.cuda.synchronize()
        t_burst += time.perf_counter() - t
    ag.maybe_train_and_checkpoint = timed_burst
    env_steps = updates = 0
    t0 = time.perf_counter()
    for _ in range(rounds):
        n, b = tr.run_round()
        env_steps += n
        updates += b
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if group is not None:  # max of the ranks' times, sum of their env-steps
        t = torch.tensor([dt, t_burst, -float(env_steps)], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dt, t_burst = float(t[0]), float(t[1])
        env_steps = int(-float(t[2])) * dist.get_world_size(group)
    t_roll = dt - t_burst
    out = {"env_steps_per_sec": env_steps / dt, "grad_steps_per_sec": updates / dt,
           "burst_grad_steps_per_sec": updates / t_burst, "rollout_env_steps_per_sec": env_steps / t_roll,
           "ms_per_round": dt / rounds * 1e3, "rollout_ms_per_round": t_roll / rounds * 1e3,
           "burst_ms_per_round": t_burst / rounds * 1e3, "updates_per_round": updates / rounds,
           "env_steps_per_round": env_steps / rounds, "rounds_timed": rounds,
           "env_steps_per_grad_step": env_steps / max(updates, 1),
           "checkpoint_refreshes": ag.checkpoint_refreshes, "replay": "reference shared pointer (add_batch_ref)",
           "burst_prefetch": tr.burst_prefetch,
           "n_gpus": dist.get_world_size(group) if group is not None else 1,
           "dp_layout": dp_layout(tr) if group is not None else None,
           "note": "Exoskeleton_agent_train.py:110-211 on the device: warm-up 25,000 env-steps of uniform actions, "
                   "then select_action with Gaussian exploration; per round round(mean(ep_len)) = 283 "
                   "graph-replayed Agent.train steps and the policy-checkpoint rule (TD7_multi_agent.py:296-325)"}
    # the script's per-round agent.save (:290; RefScheduleTrainer(save_prefix=)):
    # its host cost per round, timed apart (3 saves of the 8 files into a
    # temporary directory, rank 0)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        tr.save_prefix = os.path.join(d, "test_agent")
        for _ in range(3):
            tr.save_round()
        tr.save_prefix = None
    if tr.saves:
        out["save_ms_per_round"] = tr.save_seconds / tr.saves * 1e3
    # the script's per-step tremor statistics (:149-205) and per-round outputs
    # (:213-317) on the device (RefScheduleTrainer(stats=True)): one round to
    # capture the rollout graphs with them, then rounds timed as above
    tr.stats = True
    tr.run_round()
    torch.cuda.synchronize()
    t_burst = 0.0
    t0 = time.perf_counter()
    for _ in range(2):
        tr.run_round()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if group is not None:
        t = torch.tensor([dt, t_burst], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        dt, t_burst = float(t[0]), float(t[1])
    st = {k: v for k, v in tr.round_stats[-1].items() if not k.endswith("_per_env")}
    out["tremor_statistics"] = {
        "rollout_ms_per_round_with": (dt - t_burst) / 2 * 1e3, "rollout_ms_per_round_without": t_roll / rounds * 1e3,
        "last_round": st,
        "note": "Exoskeleton_agent_train.py:149-205 per rollout step (exo_tremor_metrics + a row of the round's "
                "device record, 2 launches) and :213-317 per round (one host sync), RefScheduleTrainer(stats=True)"}
    # the timing wrapper removed (not re-assigned: an instance attribute holding
    # the bound method would tie the agent into a reference cycle), then the
    # trainer, its graphs and the agent freed HERE, not by a later garbage
    # collection that could land inside the next phase's graph capture
    del ag.maybe_train_and_checkpoint
    _release(tr)
    del tr, ag
    _collect()
    return out


def dp_layout(trainer):
    if not trainer.dp:
        return None
    return "one graph, collectives captured (RCCL)" if trainer.dp_inline else "three graphs, eager collectives"


def td7_variants(env, dev, args, iters=60, warmup=8):
    """Sub-lines next to the bf16 headline (configs[1]): the same training
    iteration with exact fp32 TD7 (the reference's precision) -- the
    row-tile-fused passes with fp32 operands (the default) and the per-layer
    kernels (EXO_FUSED_F32=0) -- and with the
    256-wide alias of BASELINE configs[1]'s "256-wide MLPs" wording, each on a
    fresh graph-replayed trainer over the same envs: ms per iteration."""
    from exo_amd import fused
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    out = {}
    f0 = fused.FUSED_F32
    for name, hp, prec, f32 in (("fp32_300_320", Hyperparameters(), "fp32", True),
                                ("fp32_per_layer_300_320", Hyperparameters(), "fp32", False),
                                ("bf16_alias256", Hyperparameters(zs_dim=256, enc_hdim=256, critic_hdim=256,
                                                                  actor_hdim=256), "bf16", False)):
        torch.manual_seed(1)
        fused.FUSED_F32 = f32
        try:
            ag = Agent(80, 7, 1, env_num=8, hp=hp, device=dev, precision=prec, n_envs=env.n, graph_safe=True)
        finally:
            fused.FUSED_F32 = f0
        tr = VecTrainer(env, ag, use_graphs=True)
        tr.plan(warmup)
        for _ in range(warmup):
            tr.step()
        tr.plan(iters)
        tr.prepare()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            tr.step()
        torch.cuda.synchronize()
        out[name] = {"ms_per_iteration": (time.perf_counter() - t0) / iters * 1e3, "precision": prec,
                     "fused": ag.learner.fused is not None,
                     "widths": [hp.zs_dim, hp.enc_hdim, hp.critic_hdim, hp.actor_hdim], "iterations": iters}
        _release(tr)
        del tr, ag
        _collect()
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # test hooks: EXO_BENCH_DEVICE pins every rank to one GPU, EXO_DIST_BACKEND=gloo
    # (tests/test_dp_gpu.py runs 2 ranks on a 1-GPU box); the driver uses RCCL.
    local = int(os.environ.get("EXO_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = os.environ.get("EXO_DIST_BACKEND", "nccl")
    # EXO_FORCE_DIST=1 (under torchrun, one rank): the data-parallel layout and
    # its collectives at world 1, so a one-GPU box runs the RCCL path too
    dist_on = world > 1 or os.environ.get("EXO_FORCE_DIST") == "1"
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from exo_amd import VecExoskeletonEnv

    N = args.envs
    env_kw = {}
    if args.workload == "dr_sweep":  # per-env DR draws
        rng = np.random.default_rng(1000 + rank)
        env_kw = dict(matrix_noise_fraction=rng.uniform(0.05, 0.25, N), dr_actuator_range=rng.uniform(0.0, 0.1, N),
                      dr_actuator_end_pos_shift=rng.uniform(0.0, 0.04, N), tremor_amplitude_range=(0.1, 1.0))
    env = VecExoskeletonEnv(N, seed=1000 + rank, device=dev, physics=args.physics, **env_kw)
    Ls = env.lengths_host
    round_len = int(Ls.max()) - 3
    active_per_k = np.array([(Ls - 3 > k).sum() for k in range(round_len)])
    agent = trainer = None
    if args.mode == "train":
        from exo_amd.rollout import VecTrainer
        from exo_amd.td7 import Agent, Hyperparameters
        hp = Hyperparameters()
        if args.workload == "wide":  # 1024-wide encoder / critic / actor
            hp = Hyperparameters(zs_dim=1024, enc_hdim=1024, critic_hdim=1024, actor_hdim=1024)
        if args.batch:
            hp.batch_size = args.batch
        agent = Agent(80, 7, 1, env_num=8, hp=hp, device=dev, precision=args.precision, n_envs=N,
                      process_group=dist.group.WORLD if dist_on else None, graph_safe=not args.eager)
        if args.step_budget:
            env.set_step_budget(args.step_budget)
        trainer = VecTrainer(env, agent, use_graphs=not args.eager, episodes=args.episodes)
        args.episodes = trainer.episodes
    # configs[3] / [4]: the env step inside the timed window itself -- device
    # wall-clock reads on the step's stream either side of every step launch,
    # captured into the trainer's graphs with it (exo_set_step_clock)
    use_clock = trainer is not None and args.workload != "configs1" and (
        args.step_clock == "on" or (args.step_clock == "auto" and args.episodes == "sync"))
    clock = env.set_step_clock() if use_clock else None
    out = env.new_outputs(True)
    state = {"k": 0, "obs": env.reset() if trainer is None else None}  # the trainer resets its envs itself
    ev = []

    def one_step(timed):
        if trainer is not None:
            return trainer.step()
        k = state["k"]
        if k == round_len:
            state["obs"] = env.reset()
            state["resets"] = state.get("resets", 0) + 1
            k = 0
        act = torch.rand((N, 7), device=dev) * 2 - 1
        e0 = e1 = None
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        state["obs"] = env.step(act, out=out)[0]
        if timed:
            e1.record()
            ev.append((e0, e1))
        state["k"] = k + 1
        return int(active_per_k[k])

    def multibody_timing(n=50):
        """exo_multibody_kernel alone (multibody physics): HIP events around
        exo_multibody_advance launches over all envs, on the launch stream."""
        tgt = torch.zeros((5, N), dtype=torch.float64, device=dev)
        env.multibody_advance(tgt)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            env.multibody_advance(tgt)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    def reset_timing(n=5):
        """One episode-round reset (exo_reset_kernel over all envs), HIP events
        on the launch stream; after the timed loop (the trainer is done)."""
        env.reset()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            env.reset()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    def kernel_timing(n, variant=None):
        """exo_step_kernel alone, HIP events on the launch stream, all envs active
        (variant: the env's kernel variant for this measurement, restored after)."""
        prev = env.step_variant
        if variant is not None:
            env.set_step_variant(variant)
        try:
            return _kernel_timing(n)
        finally:
            env.set_step_variant(prev)

    def _kernel_timing(n):
        # the n launches back to back between one pair of HIP events (actions
        # drawn beforehand): per-launch event pairs added the event packets'
        # own latency to every launch (28.1 vs 25.5 us rocprof at 4,096 envs)
        env.reset()
        acts = torch.rand((n, N, 7), device=dev) * 2 - 1
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            env.step(acts[i], out=out)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n, float(min(n, round_len) and N)

    def loop_kernel_timing(n):
        """The env step kernel on the training loop's own inputs (VERDICT r2 item
        6): one rollout at a time, eager, exactly as the trainer's rollout branch
        runs it -- the policy's exploring actions for the current observations,
        the current active mask, mid-round state, the loop's kernel variant --
        with HIP events around the step launch on its stream.  After the timed
        window (it advances the trainer like its own rollouts do, without the
        TD7 update).  Returns (ms per launch, mean active envs per launch)."""
        tr = trainer
        evs, act_n = [], []
        for _ in range(n):
            if tr.next_step_resets():
                env.reset(obs_out=tr.obs)
                tr._round_start()
            a = agent.select_action_batch(tr.obs, dec_count=tr.active_count)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            nobs, rew, done, _ = env.step(a, active=tr.active, out=tr._outs[tr._cur],
                                          obs_cur=tr.obs if tr.budget else None)
            e1.record()
            evs.append((e0, e1))
            act_n.append(int(tr.active_count) if (tr.budget or tr.episodes == "async") else int(tr.active_counts[tr.k]))
            agent.replay_buffer.add_batch(tr.obs, a, nobs, rew, done, tr.strata, tr.active)
            tr._advance()
            tr.k += 1
            tr._cur ^= 1
        torch.cuda.synchronize()
        return float(np.mean([x.elapsed_time(y) for x, y in evs])), float(np.mean(act_n))

    def measured_round_timing():
        """One whole episode round timed end to end (SURVEY
        8(d) config 2 "whole rounds"): after the window, iterate untimed to the
        round boundary, then time exactly round_len iterations -- the first
        runs the episode reset -- bracketed by barrier + synchronize, max over
        ranks.  Returns (seconds, active env-steps of this rank).  Async episodes:
        there is no round boundary (every env resets in place when its own
        episode ends), so exactly round_len (344) consecutive iterations, their
        in-place resets included, are timed the same way."""
        if trainer.episodes == "async":
            trainer.plan(round_len)
            trainer.prepare()
            torch.cuda.synchronize()
            if dist_on:
                dist.barrier()
            torch.cuda.synchronize()
            s0 = trainer.env_steps_total() if trainer.budget else None
            t = time.perf_counter()
            n = 0
            for _ in range(round_len):
                n += trainer.step()
            torch.cuda.synchronize()
            if dist_on:
                dist.barrier()
            torch.cuda.synchronize()
            dt = torch.tensor([time.perf_counter() - t], device=dev, dtype=torch.float64)
            if dist_on:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            if s0 is not None:  # step budget: step() returns 0, the device counts the env-steps
                n = trainer.env_steps_total() - s0
            return float(dt), n, round_len
        trainer.plan(None)
        while not trainer.next_step_resets():
            trainer.step()
        trainer.plan(None if trainer.budget else round_len)
        trainer.prepare()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        n = trainer.step()  # the episode reset and the round's first iteration
        its = 1
        while not trainer.next_step_resets():
            n += trainer.step()
            its += 1
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        dt = torch.tensor([time.perf_counter() - t], device=dev, dtype=torch.float64)
        if dist_on:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        if trainer.budget:  # every env finishes its episode within the round
            n = int(active_per_k.sum())
        return float(dt), n, its

    # RCCL settle (data parallel on RCCL only): untimed iterations of the same
    # trainer BEFORE the W warm-up steps.  r04 ran 3,000 of them to hide the
    # first RCCL process's slow mode; r05 found its cause -- the first eager
    # all-reduce after the captured ones (the target refresh at training step
    # 250) cost 96 ms of host time with the GPU idle, 31-35 ms in later
    # processes -- and replays the refresh from a graph captured with the
    # iteration graphs (VecTrainer._refresh_targets; DESIGN.md 7,
    # profiles/r05rccl_raw), so the default is now 0.  Reported as
    # dist_settle_iterations (EXO_DIST_SETTLE_ITERS sets it).
    settle = 0
    if dist_on and backend == "nccl" and trainer is not None:
        settle = int(os.environ.get("EXO_DIST_SETTLE_ITERS", "0"))
        for _ in range(settle):
            one_step(False)
    if trainer is not None:
        trainer.plan(args.warmup)
    for _ in range(args.warmup):
        one_step(False)
    prepared = 0
    if trainer is not None:
        # the graphs the window replays recorded (not run) before it starts: the
        # overlapped pair's capture landed inside a short window
        trainer.plan(args.steps)
        prepared = trainer.prepare()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    resets0 = trainer.resets if trainer is not None else state.get("resets", 0)
    steps0 = trainer.env_steps_total() if trainer is not None and trainer.budget else None
    async_eps = trainer is not None and trainer.episodes == "async"
    if clock is not None:
        clock.zero_()
        torch.cuda.synchronize()
    if trainer is not None:
        trainer.plan(args.steps)  # the window's iterations: pair graphs never run past it
    t0 = time.perf_counter()
    env_steps = 0
    for _ in range(args.steps):
        env_steps += one_step(True)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    resets_in_window = (trainer.resets if trainer is not None else state.get("resets", 0)) - resets0
    if steps0 is not None:  # step budget: the window's env-steps are counted on the device
        env_steps = trainer.env_steps_total() - steps0
    window_clock = None
    if clock is not None:
        window_clock = env.step_clock_ms()
        env.set_step_clock(False)
    # async episodes: no rounds (every env resets in place inside the timed
    # iterations), the window itself is the whole-job rate
    measured_round = measured_round_timing() if trainer is not None else None
    reset_ms = reset_timing()
    loop_kern_ms = None
    if ev:  # env mode: the timed launches themselves
        kern_ms, kern_active = float(np.mean([a.elapsed_time(b) for a, b in ev])), env_steps / args.steps
    else:   # train mode: the env kernel is inside graph replays; time it separately afterwards
        # the roofline kernel: the env step's default shape alone (the shape
        # profiles/*_env kernel stats time); a trainer that runs another shape
        # (EXO_TRAIN_STEP_SHARED=1: rows_shared) has it timed alone too, reported with it
        nk = max(1, min(args.kernel_timing_steps, int(Ls.min()) - 3))  # (>= 1 launch: a rate needs one)
        # configs[3] / [4]: one whole round of the loop's launches (every round
        # position once: the launch time varies ~5x with which stiff
        # domain-randomised envs are still running, profiles/r03_dr)
        loop_ms, loop_active = loop_kernel_timing(nk if args.workload == "configs1" else round_len)
        alone_ms, alone_active = kernel_timing(nk, "auto")
        loop_kern_ms = kernel_timing(nk)[0] if env.step_variant != "auto" else None
        if args.workload == "configs1":
            # the driver's line keeps the default shape alone, all envs active
            # (the launch the committed PMC traffic and the env-mode rocprof
            # summary describe); the loop's own workload is reported beside it
            kern_ms, kern_active = alone_ms, alone_active
        else:
            # configs[3] / [4]: the loop's own workload in the timed window (a
            # freshly reset env stepped with U(-1, 1) actions is not what these
            # loops run, and the slowest domain-randomised env of a round sets
            # every launch of that round: profiles/r03_dr)
            if window_clock is not None:
                kern_ms, kern_active = window_clock[0], env_steps / args.steps
            else:
                # async episodes: no round whose stiffest env sets every launch;
                # the loop's own launches timed right after the window
                kern_ms, kern_active = loop_ms, loop_active
    # Whole-round rate, independent of where the K-iteration window falls in
    # the 344-step episode round: one round = round_len iterations (active
    # env-steps A_round = sum over k of the envs still running) + one reset.
    # t_iter = the window's time per iteration with any resets it contained
    # taken out; value = A_round / (round_len * t_iter + t_reset), summed over
    # ranks (max of the ranks' times).
    t = torch.tensor([elapsed, float(env_steps), (elapsed - resets_in_window * reset_ms * 1e-3) / args.steps,
                      reset_ms * 1e-3], device=dev, dtype=torch.float64)
    if dist_on:
        tmax, tsum = t.clone(), t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, total_env_steps = float(tmax[0]), float(tsum[1])
        t_iter, t_reset = float(tmax[2]), float(tmax[3])
    else:
        total_env_steps = float(env_steps)
        t_iter, t_reset = float(t[2]), float(t[3])
    A_round = float(active_per_k.sum())
    round_value = world * A_round / (round_len * t_iter + t_reset)
    if async_eps:
        round_value = total_env_steps / elapsed
    elif measured_round is not None and trainer.budget:
        # a budgeted round lasts as many iterations as its stiffest env needs:
        # the whole measured round is the value
        round_value = world * measured_round[1] / measured_round[0]
    finite = None
    if agent is not None:
        finite = {n: bool(torch.isfinite(torch.cat([p.detach().reshape(-1) for p in m.parameters()])).all())
                  for n, m in (("actor", agent.learner.actor), ("critic", agent.learner.critic),
                               ("encoder", agent.learner.encoder))}
    dp_sync = dp_ck = dp_lay_ranks = None
    ref_sched = None
    if agent is not None and args.mode == "train" and not args.no_reference_schedule:
        # every rank (collectives inside); rank 0 reports
        ref_sched = reference_schedule(env, dev, args, agent.hp, group=dist.group.WORLD if dist_on else None)
    sync_cmp = None
    if (agent is not None and args.mode == "train" and async_eps and args.workload == "configs1"
            and not args.no_sync_rounds):
        sync_cmp = sync_rounds(env, dev, args, agent.hp, group=dist.group.WORLD if dist_on else None)
    if agent is not None and dist_on:
        # data-parallel replicas must hold bit-identical weights
        ck = torch.stack([torch.cat([p.detach().reshape(-1) for p in m.parameters()]).double().sum()
                          for m in (agent.learner.actor, agent.learner.critic, agent.learner.encoder)]
                         + [agent.replay_buffer._maxp.double().reshape(())])  # and the global max_priority
        allck = [torch.zeros_like(ck) for _ in range(world)]
        dist.all_gather(allck, ck)
        dp_sync = all(torch.equal(allck[0], x) for x in allck)
        dp_ck = [x.tolist() for x in allck]
        # every rank's layout: in-graph collectives, overlapped pairs
        lay = torch.tensor([float(trainer.dp_inline) if trainer is not None else -1.0,
                            float(any(isinstance(k, tuple) and k[-1] == "overlap" for k in trainer.graphs))
                            if trainer is not None else -1.0], device=dev)
        all_lay = [torch.zeros_like(lay) for _ in range(world)]
        dist.all_gather(all_lay, lay)
        dp_lay_ranks = [x.tolist() for x in all_lay]
    if rank == 0:
        active_avg = kern_active
        achieved = BYTES_PER_ENV_STEP * active_avg / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(float(BYTES_PER_ENV_STEP * active_avg))
        res = {
            "metric": "env steps/sec (batched exo sim) + TD7 grad-steps/sec at 1/2/4/8 MI355X",
            "value": round_value,
            "unit": "env-steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "dist_settle_iterations": settle,
            "graphs_prepared": prepared,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64" if agent is None else f"f64 sim + {args.precision} TD7",
            "data": "synthetic: reference motions 0-7 (env i -> motion i mod 8), Philox tremor/DR draws, "
                    + ("random actions" if agent is None else (f"random-init TD7 (widths {agent.hp.zs_dim}/{agent.hp.critic_hdim})")),
            "config": {"workload": WORKLOADS[args.workload]
                                   + (f", TD7 batch 8x{agent.hp.batch_size}" if agent else ", env only"),
                       "envs_per_gpu": N, "mode": args.mode, "physics": args.physics,
                       "step_budget": args.step_budget,
                       **({"episodes": args.episodes} if trainer is not None else {}),
                       "parallelism": f"env-shard x{world}"
                       + (" + TD7 DP all-reduce" if agent and dist_on else "")},
            "value_formula": ("async episodes: the timed window's env-steps (every launch steps every env without a "
                              "pending budgeted solve; episodes end and reset in place inside the window) / window "
                              "time, summed over ranks (max of the ranks' times)") if async_eps else
                             ("whole episode rounds: world * A_round / (round_len * t_iter + t_reset); A_round = "
                              f"{A_round:.0f} active env-steps per {round_len}-iteration round and rank, t_iter = "
                              f"{t_iter * 1e3:.4f} ms (window time minus {resets_in_window} reset(s), per iteration), "
                              f"t_reset = {t_reset * 1e3:.4f} ms (exo_reset_kernel, HIP events)")
                             if not (trainer is not None and trainer.budget) else
                             ("step budget: world * A_round / (one whole measured round incl. its reset); the round "
                              f"lasts as many iterations as its stiffest env needs (measured_round.iterations)"),
            "window_value": total_env_steps / elapsed,
            "measured_round_value": (world * measured_round[1] / measured_round[0]) if measured_round else None,
            "measured_round": ({"seconds": measured_round[0], "iterations": measured_round[2],
                                "active_env_steps_per_rank": measured_round[1],
                                "value_over_measured": round_value / (world * measured_round[1] / measured_round[0]),
                                "note": "one whole episode round timed end to end after the window, max over "
                                        "ranks: sync episodes the reset + round_len graph-replayed iterations, "
                                        "async episodes round_len consecutive iterations with their in-place "
                                        "resets"}
                               if measured_round else None),
            "env_kernel_env_steps_per_sec": active_avg / (kern_ms * 1e-3),
            "reset_kernel_ms": reset_ms,  # one reset of every env (exo_reset_kernel), HIP events
            "roofline": {"kernel": ("exo_step_rp_kernel" if N <= 16384 else "exo_step_kernel")
                                   + (" + exo_multibody_kernel" if args.physics == "multibody" else ""), "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_unit": "bytes per launch", "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": BYTES_PER_ENV_STEP * active_avg,
                         "bytes_per_env_step": BYTES_PER_ENV_STEP, "avg_kernel_ms": kern_ms,
                         "active_envs_per_launch": active_avg},
        }
        if ev == [] and agent is not None:
            res["roofline"]["measured_on"] = ("default shape alone, all envs active, U(-1, 1) actions"
                                              if args.workload == "configs1" else
                                              "the timed window's own step launches inside the graph-replayed "
                                              "training loop: device wall-clock reads either side of each launch "
                                              "on its stream (exo_set_step_clock), averaged over the window"
                                              if window_clock is not None else
                                              "the loop's own step launches right after the timed window (its "
                                              "policy, observations, masks and carried solves), eager, HIP events "
                                              "(loop_workload); --step-clock on times them inside the window")
            if window_clock is not None:
                res["roofline"]["window_step_clock"] = {"avg_ms": window_clock[0], "launches": window_clock[1],
                                                        "ms_per_iteration": elapsed / args.steps * 1e3}
            res["roofline"]["loop_workload"] = {
                "measured_on": "one whole round of rollout launches after the window, eager, HIP events "
                               "(the round after the window: other domain-randomisation draws)",
                "avg_kernel_ms": loop_ms, "active_envs_per_launch": loop_active, "variant": env.step_variant,
                "achieved_gbs": BYTES_PER_ENV_STEP * loop_active / (loop_ms * 1e-3) / 1e9,
                "frac": BYTES_PER_ENV_STEP * loop_active / (loop_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
            res["roofline"]["alone_default_shape"] = {"avg_kernel_ms": alone_ms, "active_envs_per_launch": alone_active}
        if loop_kern_ms is not None:
            res["roofline"]["training_loop_variant"] = {
                "variant": env.step_variant, "avg_kernel_ms_alone": loop_kern_ms,
                "note": "32 envs per 512-thread workgroup: half the CUs at 4,096 envs, so the fused TD7 "
                        "workgroups beside it keep whole CUs (DESIGN.md 4)"}
        vfl, vsrc = pmc_valu_flops(N) if args.physics == "ideal" and N <= 16384 else (None, None)
        if vfl and kern_active == N:
            # the env kernel is fp64-VALU/latency bound -- its
            # compute fraction next to the HBM one (flops: PMC, issued lanes)
            res["valu_roofline"] = {"kernel": res["roofline"]["kernel"], "bound": "valu",
                                    "achieved": vfl / (kern_ms * 1e-3) / 1e12, "peak": FP64_VALU_PEAK_TFS,
                                    "unit": "TFLOP/s (fp64)", "frac": vfl / (kern_ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFS,
                                    "flops_per_launch": vfl, "flops_source": vsrc,
                                    "flops_kind": "issued lane-flops (PMC, every lane of the wave)"}
            if args.workload == "configs1":
                uf, att, usrc = useful_fp64_flops_per_env_step()
                ua = uf * N / (kern_ms * 1e-3) / 1e12
                res["valu_roofline"]["useful"] = {
                    "flops_per_env_step": uf, "achieved": ua, "frac": ua / FP64_VALU_PEAK_TFS,
                    "issued_over_useful": vfl / (uf * N), "rk45_attempts_per_env_step": att, "attempts_source": usrc,
                    "model": "bench.py USEFUL_FLOPS: the step's arithmetic once per env (a scalar implementation "
                             "of the kernel's algorithm), counted by hand"}
        if args.physics == "multibody":
            # q, qd of 19 joints read + written (f64), 5 targets, 1 flag byte read + cleared
            mb_ms = multibody_timing()
            res["multibody_kernel"] = {"kernel": "exo_multibody_kernel", "avg_kernel_ms": mb_ms,
                                       "bytes_per_env_step": 19 * 8 * 4 + 5 * 8 + 2, "envs_per_launch": N,
                                       "note": "included in ms_per_step; the roofline object above is the step kernel"}
        if agent is not None:
            gs = args.steps / elapsed  # data-parallel ranks share one update: a grad step is per iteration
            res["grad_steps_per_sec"] = gs
            per_update = (total_env_steps / world / args.steps) if async_eps else A_round / round_len
            ref_ratio = REFERENCE_ENV_STEPS_PER_UPDATE
            res["update_to_data"] = {
                "env_steps_per_grad_step": world * per_update,
                "reference_env_steps_per_grad_step": ref_ratio,
                "env_steps_per_sec_at_reference_ratio": gs * ref_ratio,
                "note": "this loop trains one grad step per vectorised env step (the reference script's ratio per "
                        "vectorised step of its 8 envs, Exoskeleton_agent_train.py:208); at the reference's ratio "
                        f"per env-step ({ref_ratio:.2f} = 2,257 active env-steps / 283 updates per round) the loop "
                        "is update bound: grad_steps_per_sec x that ratio"}
            # TD7 on the MFMA roofline: the update's GEMM flops per
            # grad step over the whole iteration time.  The env step runs on a
            # concurrent graph branch, so subtracting a standalone env-kernel time
            # is not meaningful (at configs[3]'s stiff DR draws the standalone
            # launch outlasts the iteration): a lower bound on the TD7 fraction.
            fl = td7_flops(agent, N)
            td7_s = elapsed / args.steps
            peak = MFMA_PEAK_TFS[args.precision]
            res["td7_roofline"] = {"bound": "mfma", "achieved": fl / td7_s / 1e12, "peak": peak,
                                   "unit": "TFLOP/s", "frac": fl / td7_s / 1e12 / peak,
                                   "gflop_per_step": fl / 1e9, "mfma_operands": args.precision,
                                   "formula": "sum over Linear layers of 2*M*N*K: x3 (fwd, dX, dW) where trained, "
                                              "x1 no-grad; actor update x0.5 (policy_freq 2); + select_action "
                                              "over all envs (bench.td7_flops)",
                                   "note": "GEMM flops of one train() step (B=8x128) + batched actor inference "
                                           "over the envs, per whole iteration time (env step included: a lower bound)"}
            us, cfl = critic_gemm_timing(agent)
            res["critic_gemm_roofline"] = {
                "kernel": "td7_dense_fwd, critic Linear(2*zs+h -> h) + ELU, both Q heads", "bound": "mfma",
                "shape": [2, agent.hp.batch_size * agent.env_num, agent.learner.critic.w1.shape[1],
                          agent.learner.critic.w1.shape[2]],
                "achieved": cfl / (us * 1e-6) / 1e12, "peak": peak, "unit": "TFLOP/s",
                "frac": cfl / (us * 1e-6) / 1e12 / peak, "avg_kernel_us": us,
                "note": "the per-layer kernel of the fp32 and wide paths; the bf16 bench runs fused_critic_roofline"}
            fc = fused_critic_timing(agent)
            if fc is not None:
                gbs = fc["bytes_per_wg"] / (fc["us"] * 1e-6) / 1e9
                res["fused_critic_roofline"] = {
                    "kernel": "td7f critic_kernel: both Q heads' forward, LAP-Huber loss and backward in one launch "
                              "(16 rows x one head per workgroup)",
                    "bound": "l2_weight_stream_per_cu", "achieved": gbs, "peak": L2_STREAM_PER_CU_GBS,
                    "unit": "GB/s per workgroup (one workgroup per CU)", "frac": gbs / L2_STREAM_PER_CU_GBS,
                    "bytes_per_workgroup": fc["bytes_per_wg"], "workgroups": fc["workgroups"],
                    "avg_kernel_us": fc["us"],
                    "mfma": {"achieved": fc["flop"] / (fc["us"] * 1e-6) / 1e12, "peak": peak, "unit": "TFLOP/s",
                             "frac": fc["flop"] / (fc["us"] * 1e-6) / 1e12 / peak, "flop_per_launch": fc["flop"]},
                    "peak_source": "tools/stream_bench.hip (profiles/r02b_raw/stream_bench.txt)"}
        if agent is not None and args.workload == "configs1" and world == 1 and not args.no_td7_variants:
            res["td7_variants"] = td7_variants(env, dev, args)
        if dp_sync is not None:
            res["dp_layout"] = dp_layout(trainer)
            res["dp_layout_per_rank"] = [("one graph, collectives captured (RCCL)" if a == 1.0 else
                                          "three graphs, eager collectives") for a, _ in dp_lay_ranks]
            res["overlapped_pairs_per_rank"] = [b == 1.0 for _, b in dp_lay_ranks]
        if trainer is not None:
            # the graph-replayed loop's schedule ("The training
            # iteration's schedule"): an actor iteration and the next one per
            # graph, the second's update beside the first's actor passes
            res["overlapped_pairs"] = any(isinstance(k, tuple) and k[-1] == "overlap" for k in trainer.graphs)
        if ref_sched is not None:
            res["reference_schedule"] = ref_sched
        if sync_cmp is not None:
            res["sync_rounds"] = sync_cmp
        if finite is not None:
            res["weights_finite"] = all(finite.values()) or finite
        if dp_sync is not None:
            res["dp_weights_in_sync"] = dp_sync
            if not dp_sync:
                res["dp_weight_checksums"] = dp_ck
        if not args.no_cpu_baseline and world == 1:
            td7 = None
            if agent is not None:
                td7 = (agent.hp, agent.hp.batch_size * agent.env_num, total_env_steps / args.steps)
            res["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, args.cpu_threads, td7)
        print(json.dumps(res))
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a host-side crash prints its Python stack
    if os.environ.get("EXO_BENCH_STREAM") == "high":  # r05 experiment: every launch from a high-priority stream
        with torch.cuda.stream(torch.cuda.Stream(priority=-1)):
            main()
    else:
        main()
