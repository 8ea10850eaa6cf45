"""One rank of a data-parallel test run (launched by torch.distributed.run from
tests/test_dp_gpu.py; test infrastructure, not a test module).

--mode vec: bench.py's data-parallel training loop (VecTrainer, graph-replayed)
  with `--envs` envs per rank (env seed 1000 + rank, as bench.py).  Writes the
  replay rows of a sample of each rank's envs (state, action, next_state,
  reward of every step -- the env trajectories the oracle replays) and the
  weight / max_priority checksums.
--mode ref: the reference training schedule (RefScheduleTrainer,
  Simulation/Exoskeleton_agent_train.py:110-211) on every rank: per-round
  decision trace, local episode returns, the global max_priority, checksums.

Every rank pins cuda:<EXO_BENCH_DEVICE or LOCAL_RANK>; EXO_DIST_BACKEND picks
gloo (several ranks on one GPU) or nccl."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SAMPLE = (0, 1, 7, 8, 13, 63)  # env indices (taken modulo the env count) replayed on the oracle


def checksums(agent):
    L = agent.learner
    return [float(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).double().sum())
            for m in (L.actor, L.critic, L.encoder)] + [float(agent.replay_buffer._maxp)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["vec", "ref"], default="vec")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", required=True)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--no-noise", action="store_true",
                    help="exploration and target-policy noise 0 (the full-loop comparison with one process)")
    ap.add_argument("--dump", action="store_true",
                    help="vec: save the sampled indices of every iteration and the final nets / trees")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("EXO_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = os.environ.get("EXO_DIST_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer, VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(7 + rank)  # per-rank random streams; the weights come from rank 0's broadcast
    env = VecExoskeletonEnv(a.envs, seed=1000 + rank, device=dev)
    out = {"rank": rank, "world": world}
    if a.mode == "vec":
        hp = Hyperparameters(exploration_noise=0.0, target_policy_noise=0.0) if a.no_noise else Hyperparameters()
        agent = Agent(80, 7, 1, env_num=8, hp=hp, device=dev, precision=a.precision, n_envs=a.envs,
                      process_group=dist.group.WORLD, graph_safe=True,
                      buffer_size=max(8192, a.iters * a.envs // 8))
        tr = VecTrainer(env, agent)
        out["dp_inline"] = tr.dp_inline
        inds = []
        for _ in range(a.iters):
            tr.step()
            if a.dump:  # the batch sampled for the next iteration: its slot is the new observation parity
                inds.append(agent.replay_buffer._slot(tr._cur)[1].cpu().clone())
        torch.cuda.synchronize()
        if a.dump:
            L = agent.learner
            torch.save({"ind": torch.stack(inds), "tree": agent.replay_buffer._tree.cpu(),
                        "maxp": agent.replay_buffer._maxp.cpu(),
                        **{f"{n}.{k}": v.detach().cpu() for n in ("actor", "critic", "encoder")
                           for k, v in getattr(L, n).state_dict().items()}},
                       os.path.join(a.out, f"final_r{rank}.pt"))
        rb = agent.replay_buffer
        per = a.envs // 8
        envs = sorted({e % a.envs for e in SAMPLE})
        rows = {}
        for e in envs:
            slots = [k * per + e // 8 for k in range(a.iters)]  # per-stratum ring, env order within a step
            s = e % 8
            rows[f"state_{e}"] = rb.state[s, slots].cpu().numpy()
            rows[f"action_{e}"] = rb.action[s, slots].cpu().numpy()
            rows[f"next_state_{e}"] = rb.next_state[s, slots].cpu().numpy()
            rows[f"reward_{e}"] = rb.reward[s, slots, 0].cpu().numpy()
        np.savez(os.path.join(a.out, f"rows_r{rank}.npz"), envs=np.array(envs), **rows)
        out["checksums"] = checksums(agent)
        out["training_steps"] = agent.learner.training_steps
    else:
        hp = Hyperparameters(batch_size=32)
        agent = Agent(80, 7, 1, learning_steps=100000, env_num=8, hp=hp, device=dev, precision="bf16",
                      n_envs=a.envs, process_group=dist.group.WORLD, graph_safe=True, buffer_size=4096)
        tr = RefScheduleTrainer(env, agent, warmup=1)
        out["dp_inline"] = tr.dp_inline
        for _ in range(a.rounds):
            tr.run_round()
        torch.cuda.synchronize()
        out["trace"] = tr.trace
        out["round_env_steps"] = tr.round_env_steps
        out["steps_count"] = tr.steps_count
        out["checksums"] = checksums(agent)
        out["training_steps"] = agent.learner.training_steps
        out["exploration_noise"] = float(agent.learner.exploration_noise_t)
        out["graphs"] = sorted(str(k) for k in tr.graphs)
    with open(os.path.join(a.out, f"out_r{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
