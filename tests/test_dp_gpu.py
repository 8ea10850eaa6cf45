"""Data-parallel training on the GPU.

* gloo ranks pinned to cuda:0 (several ranks on a 1-GPU box) through bench.py's
  DP path and through tests/dp_worker.py at configs[2]'s per-rank shape (4,096
  envs per rank; 2 and 8 ranks): three graphs per iteration with the gradient
  all-reduces between them.  The replicas' weights must stay bit-identical and
  every rank's env trajectories must match the oracle.
* RCCL at world 1 (RCCL refuses two ranks on one device): the one-graph layout
  with the collectives captured inside it, bit-identical to the one-GPU graph.
* The reference schedule (RefScheduleTrainer) on 2 ranks: steps counted over
  ranks, MIN-reduced episode returns, one checkpoint decision sequence, a
  global max_priority."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from helpers import model_host, philox_draws

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    from _ports import free_port
    return free_port()


def test_two_rank_training_keeps_replicas_in_sync():
    env = dict(os.environ, EXO_BENCH_DEVICE="0", EXO_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "12", "--warmup", "6", "--envs", "256", "--no-cpu-baseline",
           "--kernel-timing-steps", "5"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-4000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2
    assert res["dp_weights_in_sync"] is True
    assert res["value"] > 0


def _failure_text(out, name="child"):
    """A failed child's story: the error lines of its stderr (a watchdog's
    stack trace otherwise buries the message), its stdout tail and the tail
    of stderr.  The whole stdout and stderr are kept in
    gpurun_out/<name>.log (the r05 watchdog abort's log
    was lost)."""
    try:
        d = os.path.join(REPO, "gpurun_out")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{name}.log"), "w") as f:
            f.write(f"returncode {out.returncode}\n--- stdout ---\n{out.stdout}\n--- stderr ---\n{out.stderr}")
    except OSError:
        pass
    err = out.stderr.splitlines()
    keys = ("Error", "error", "HIP", "NCCL", "RCCL", "Timeout", "timed out", "Traceback")
    lines = [l for l in err if any(k in l for k in keys) and "frame #" not in l]
    return ("\n".join(lines[:40]) + "\n--- stdout tail ---\n" + out.stdout[-1500:]
            + "\n--- stderr tail ---\n" + out.stderr[-1500:])


def test_rccl_data_parallel_layout_at_world_one():
    """The RCCL branch the multi-GPU runs take, on a one-GPU box: torchrun with
    one rank and EXO_FORCE_DIST=1 -- bench.py initialises the nccl (RCCL)
    process group, the agent's GradSync is active at world 1, so VecTrainer
    replays the three-graph data-parallel layout with the flat-bucket
    all-reduces, the max_priority MAX reduction and the replica checksum
    all_gather on RCCL between the graphs (RCCL refuses two ranks on one
    device, so world 1 is the most of that path one GPU can run)."""
    # NCCL_DEBUG=WARN: RCCL's own message for an asynchronous error reaches stderr
    env = dict(os.environ, EXO_FORCE_DIST="1", NCCL_DEBUG="WARN")
    env.pop("EXO_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--steps", "20", "--warmup", "8", "--envs", "512", "--no-cpu-baseline", "--no-td7-variants",
           "--no-reference-schedule", "--kernel-timing-steps", "5"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, _failure_text(out, "rccl_world1_bench_child")
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith('{"metric')][-1])
    assert res["n_gpus"] == 1
    assert "DP all-reduce" in res["config"]["parallelism"]
    assert res["dp_weights_in_sync"] is True
    assert res["dp_layout"] == "one graph, collectives captured (RCCL)"
    assert res["dp_layout_per_rank"] == ["one graph, collectives captured (RCCL)"]
    assert res["overlapped_pairs_per_rank"] == [True]
    assert res["weights_finite"] is True, res["weights_finite"]
    assert res["value"] > 0


def _run_workers(tmp_path, world, mode, extra, timeout=900):
    env = dict(os.environ, EXO_BENCH_DEVICE="0", EXO_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "dp_worker.py"),
           "--mode", mode, "--out", str(tmp_path)] + extra
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    assert out.returncode == 0, _failure_text(out)
    return [json.load(open(os.path.join(tmp_path, f"out_r{r}.json"))) for r in range(world)]


def _oracle_replay(tmp_path, rank, n_envs, iters):
    """The rank's sampled envs (seed 1000 + rank, motion e mod 8, defaults) on
    the oracle: the constructor's episode 0, the trainer's reset (episode 1),
    then the recorded actions; states, next states and rewards compared."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from exo_amd import motions
    from test_env_gpu import _close_obs, env_kwargs_default
    rows = np.load(os.path.join(tmp_path, f"rows_r{rank}.npz"))
    angles, lengths = motions.load()
    lib = model_host()
    cfg = env_kwargs_default()
    for e in rows["envs"]:
        e = int(e)
        m = e % 8
        L = int(lengths[m])
        oe = O.OracleEnv(angles[m][:, :L], cfg["seq"], cfg["amp"], cfg["h1"], cfg["h2"], 40.0, 20.0, 0.02, 0.03, 0.1)
        oe.reset(philox_draws(L, 1000 + rank, e, 0, lib))
        ob = oe.reset(philox_draws(L, 1000 + rank, e, 1, lib))
        st, ac, ns, rw = (rows[f"{k}_{e}"] for k in ("state", "action", "next_state", "reward"))
        assert st.shape == (iters, 80)
        _close_obs(st[0], ob)
        for k in range(iters):
            if k:
                np.testing.assert_array_equal(st[k], ns[k - 1])
            ob, r, dn, info, _ = oe.step(ac[k].astype(np.float64))
            _close_obs(ns[k], ob)
            np.testing.assert_allclose(rw[k], r, rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("world,iters", [(2, 16), (8, 8)])
def test_data_parallel_at_configs2_shape_per_rank(tmp_path, world, iters):
    """configs[2]'s per-rank shape: 4,096 envs per rank (2 ranks: 8,192 envs;
    8 ranks: 32,768 -- configs[2]'s whole job, every rank pinned to the one
    GPU over gloo).  Replicas bit-identical; each rank's envs (its own seed)
    replayed on the oracle from its replay rows."""
    outs = _run_workers(tmp_path, world, "vec", ["--envs", "4096", "--iters", str(iters)])
    assert [o["rank"] for o in outs] == list(range(world))
    assert all(o["dp_inline"] is False for o in outs)  # gloo: the eager-collective layout
    assert all(o["checksums"] == outs[0]["checksums"] for o in outs)
    assert all(o["training_steps"] == iters for o in outs)
    for r in (0, world - 1):
        _oracle_replay(tmp_path, r, 4096, iters)


def test_reference_schedule_on_two_ranks(tmp_path):
    """RefScheduleTrainer with 2 ranks (gloo on one GPU), 64 envs each, 3 rounds
    (a random warm-up round, then the policy): steps_count counts both ranks'
    env-steps (Exoskeleton_agent_train.py:146, 210-211), the episode return
    the checkpoint rule sees is the MIN over the ranks' round returns
    (TD7_multi_agent.py:296-312), every rank takes the same checkpoint
    decisions and training bursts, the replicas and the global max_priority
    (TD7_buffer_multi_agent.py:116, 120) agree, and the exploration noise fell
    by one decrement per env-step of EVERY rank."""
    outs = _run_workers(tmp_path, 2, "ref", ["--envs", "64", "--rounds", "3"])
    A = outs[0]["round_env_steps"]
    assert A == 8 * 2257
    for o in outs:
        assert o["steps_count"] == 3 * A * 2
        assert [t["steps_count"] for t in o["trace"]] == [A * 2, 2 * A * 2, 3 * A * 2]
        assert [t["random_actions"] for t in o["trace"]] == [True, False, False]
        assert o["training_steps"] == 3 * 283
    keys = ("training_steps", "eps_since_update", "best_min_return", "max_eps_before_update",
            "checkpoint_refreshed", "ep_timesteps")
    for a, b in zip(outs[0]["trace"], outs[1]["trace"]):
        assert {k: a[k] for k in keys} == {k: b[k] for k in keys}
    # round 1 always checkpoints (best_min_return = -1e8): best_min_return = the MIN-reduced return
    r1 = [o["trace"][0] for o in outs]
    assert r1[0]["checkpoint_refreshed"]
    assert r1[0]["ep_return"] != r1[1]["ep_return"]  # the ranks' envs differ (seed 1000 + rank)
    assert r1[0]["best_min_return"] == min(t["ep_return"] for t in r1)
    assert outs[0]["checksums"] == outs[1]["checksums"]  # weights and max_priority
    assert outs[0]["exploration_noise"] == outs[1]["exploration_noise"]
    from exo_amd.td7 import Hyperparameters
    hp = Hyperparameters()
    want = hp.exploration_noise - 2 * A * 2 * hp.exploration_noise / 100000  # 2 policy rounds, both ranks' envs
    assert abs(outs[0]["exploration_noise"] - want) < 2e-5


def test_rccl_inline_layout_is_bit_identical_to_the_one_gpu_graph():
    """RCCL world 1 (EXO_FORCE_DIST=1): VecTrainer captures each iteration as
    ONE graph with the AVG all-reduces of the encoder (on its branch), critic
    and actor buckets and the MAX of max_priority inside it.  At world 1 every
    collective is the identity, so the run must equal the one-GPU graph bit
    for bit -- weights, optimiser moments, replay trees -- with and without the
    overlapped pairs (r05), and so must the eager-collective three-graph
    layout (EXO_DP_CAPTURE=0).  Targets refresh every 5 steps: the in-graph
    layout replays the refresh (copies, repack, MAX-reduced bounds and
    max_priority) from its own captured graph.  Run in a process of its own
    (tests/rccl_inline_worker.py): destroying the process group releases
    RCCL's streams, after which the ROCm 7.0 runtime's graph-launch stream
    assignment can over-read in a later test's first replay (DESIGN.md 4,
    "The graph-replay crash")."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "tests", "rccl_inline_worker.py"), str(_port())],
                         capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, (out.stdout[-3000:], out.stderr[-3000:])
    assert "OK" in out.stdout


def _single_process_two_shards(iters, precision, envs=4096):
    """ONE process stepping both ranks' envs (2 x 4,096 = 8,192: env seeds 1000
    and 1001) and training on the concatenation of the two ranks' batches,
    in VecTrainer's order (iteration 0: rollout, then the batch; later ones:
    the batch sampled at the end of the previous iteration, then the rollout;
    the update; the priority update + next sample per shard; the global
    max_priority).  Each shard keeps its rank's replay (8 strata) and sampling
    stream (torch seed 7 + rank, folded with the rank, as tests/dp_worker.py
    and Agent do); exploration and target-policy noise are 0, so those
    streams draw nothing that matters.  Returns the learner, both replays and
    the per-iteration sampled indices."""
    from exo_amd import VecExoskeletonEnv
    from exo_amd.td7 import Agent, Hyperparameters
    hp = Hyperparameters(exploration_noise=0.0, target_policy_noise=0.0)
    shards = []
    for r in range(2):
        torch.manual_seed(7 + r)
        env = VecExoskeletonEnv(envs, seed=1000 + r)
        ag = Agent(80, 7, 1, env_num=8, hp=hp, precision=precision, n_envs=envs,
                   buffer_size=max(8192, iters * envs // 8))
        ag.replay_buffer._rng.fold(r)
        ag.learner._explore_rng.fold(r)
        strata = torch.as_tensor(env.motions % 8, dtype=torch.int32, device=env.device)
        shards.append((env, ag, strata, [env.reset()]))
    L = shards[0][1].learner  # rank 0's initial weights are the ones the data-parallel run broadcasts
    inds = []

    def rollout():
        for env, ag, strata, obs in shards:
            act = L_select(ag, obs[0])
            nobs, rew, done, _ = env.step(act)
            nobs = nobs.clone()
            ag.replay_buffer.add_batch(obs[0], act, nobs, rew, done, strata)
            obs[0] = nobs

    def L_select(ag, o):  # the shard's own agent object, the shared weights
        ag.learner = L
        return ag.select_action_batch(o)

    for it in range(iters):
        if it == 0:
            rollout()
            batches = [sh[1].replay_buffer.sample(0) for sh in shards]
            batches = [tuple(t.clone() for t in b) for b in batches]
            idx = [sh[1].replay_buffer.ind.clone() for sh in shards]
        else:
            rollout()
        cat = [torch.cat([b[k] for b in batches]) for k in range(5)]
        prio = L.update(*cat).reshape(2, -1)
        nxt = []
        for r, (env, ag, strata, obs) in enumerate(shards):
            rb = ag.replay_buffer
            b = rb.update_priority_and_sample(prio[r], idx[r], slot=1)
            nxt.append((tuple(t.clone() for t in b), rb.ind.clone()))
        m = torch.maximum(shards[0][1].replay_buffer._maxp, shards[1][1].replay_buffer._maxp)
        for sh in shards:
            sh[1].replay_buffer._maxp.copy_(m)
        batches = [n[0] for n in nxt]
        idx = [n[1] for n in nxt]
        inds.append([i.cpu() for i in idx])
    torch.cuda.synchronize()
    return L, [sh[1].replay_buffer for sh in shards], inds


def test_data_parallel_full_loop_matches_one_process(tmp_path):
    """the data-parallel training loop itself (VecTrainer on
    2 gloo ranks x 4,096 envs, fp32 TD7, graph-replayed, the gradient buckets
    averaged) against one process that steps both ranks' 8,192 envs and
    trains on the concatenated batches (_single_process_two_shards).  Every
    iteration's sampled indices must agree exactly (the LAP descent over the
    shard's priorities: a priority off by more than the rounding would move
    one), the final weights within tests/test_dp_bench_gpu.py's fp32 bounds
    and the two shards' priority trees within fp32 rounding."""
    iters = 12
    outs = _run_workers(tmp_path, 2, "vec", ["--envs", "4096", "--iters", str(iters), "--precision", "fp32",
                                             "--no-noise", "--dump"])
    assert outs[0]["checksums"] == outs[1]["checksums"]
    d = [torch.load(os.path.join(tmp_path, f"final_r{r}.pt"), weights_only=True) for r in range(2)]
    L, rbs, inds = _single_process_two_shards(iters, "fp32")
    for r in range(2):
        for it in range(iters):
            assert torch.equal(d[r]["ind"][it], inds[it][r]), f"rank {r} iteration {it}: sampled indices differ"
        torch.testing.assert_close(rbs[r]._tree.cpu(), d[r]["tree"], rtol=1e-5, atol=1e-6)
        assert float(rbs[r]._maxp) == float(d[r]["maxp"]) or abs(float(rbs[r]._maxp) - float(d[r]["maxp"])) < 1e-5
    rtol, atol = 2e-5, 2e-6
    outliers = total = 0
    for n in ("actor", "critic", "encoder"):
        for k, v in getattr(L, n).state_dict().items():
            a, b = d[0][f"{n}.{k}"].double().numpy(), v.detach().cpu().double().numpy()
            bad = np.abs(a - b) > atol + rtol * np.abs(b)
            total += a.size
            outliers += int(bad.sum())
            assert not bad.any() or np.abs(a - b)[bad].max() <= 2 * 3e-4 * iters, f"{n}.{k}"
    assert outliers <= 1e-3 * total, f"{outliers} of {total} entries outside rtol {rtol} / atol {atol}"
