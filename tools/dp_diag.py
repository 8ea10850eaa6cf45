"""Data-parallel / split-graph diagnostic: after every VecTrainer iteration
print, per rank, whether the encoder/critic/actor weights and gradients are
finite and their checksums.  torchrun --nproc-per-node N tools/dp_diag.py
(EXO_BENCH_DEVICE pins ranks to one GPU; gloo).  DIAG_SPLIT=1 forces the
3-graph data-parallel capture layout even at world size 1."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dev = torch.device("cuda", int(os.environ.get("EXO_BENCH_DEVICE", os.environ["LOCAL_RANK"])))
    torch.cuda.set_device(dev)
    dist.init_process_group(os.environ.get("EXO_DIST_BACKEND", "gloo"))
    torch.manual_seed(int(os.environ.get("DIAG_TORCH_SEED", 0)))
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent
    env = VecExoskeletonEnv(256, seed=int(os.environ.get("DIAG_SEED", 1000)) + rank, device=dev)
    agent = Agent(80, 7, 1, env_num=8, device=dev, n_envs=256,
                  process_group=dist.group.WORLD if world > 1 else None, graph_safe=True)
    tr = VecTrainer(env, agent, use_graphs=os.environ.get("DIAG_EAGER") is None)
    if os.environ.get("DIAG_SPLIT"):
        tr.dp = True
    L = agent.learner
    n_it = int(os.environ.get("DIAG_STEPS", "10"))
    for it in range(n_it):
        tr.step()
        if (it + 1) % int(os.environ.get("DIAG_CHECK_EVERY", 1)) and it != n_it - 1:
            continue
        torch.cuda.synchronize()
        row = []
        for name, m in (("actor", L.actor), ("critic", L.critic), ("enc", L.encoder)):
            w = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
            gs = [p.grad.reshape(-1) for p in m.parameters() if p.grad is not None]
            g = torch.cat(gs) if gs else torch.zeros(1, device=dev)
            row.append(f"{name}: w {'ok' if torch.isfinite(w).all() else 'NaN'} {float(w.double().sum()):.9e} "
                       f"g {'ok' if torch.isfinite(g).all() else 'NaN'}")
        if not os.environ.get("DIAG_QUIET") or "NaN" in " ".join(row) or it == n_it - 1:
            print(f"rank {rank} iter {it} graphs={sorted(tr.graphs)} " + " | ".join(row), flush=True)
            if "NaN" in " ".join(row):
                break
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
