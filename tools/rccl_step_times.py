"""Host time of every VecTrainer.step() on RCCL at world 1 (EXO_FORCE_DIST=1,
the in-graph collective layout, 4,096 envs): where the first RCCL process's
slow windows come from (r05).  Prints the slowest steps and what they did
(a target refresh every 250 steps runs eager collectives).  Run without a
launcher: RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=... python tools/rccl_step_times.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
os.environ.setdefault("EXO_FORCE_DIST", "1")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 800
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent
    torch.manual_seed(0)
    env = VecExoskeletonEnv(4096, seed=1000, device=dev)
    ag = Agent(80, 7, 1, env_num=8, precision="bf16", n_envs=4096, process_group=dist.group.WORLD, graph_safe=True)
    tr = VecTrainer(env, ag, episodes="async")
    print("dp_inline", tr.dp_inline, flush=True)
    times = []
    t_all = time.perf_counter()
    for i in range(steps):
        t = time.perf_counter()
        tr.step()
        times.append((time.perf_counter() - t, i, ag.learner.training_steps))
    torch.cuda.synchronize()
    total = time.perf_counter() - t_all
    print(f"{steps} steps in {total:.3f} s: {total / steps * 1e3:.4f} ms per step", flush=True)
    for dt, i, ts in sorted(times, reverse=True)[:12]:
        print(f"  step {i:5d} (training_steps {ts}): {dt * 1e3:9.3f} ms host", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
