"""Minimal copy of bench.py's training path at 256 envs, for bisecting."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(int(os.environ.get("REPRO_SEED", 7)))
    n = int(os.environ.get("REPRO_N", 256))
    env = VecExoskeletonEnv(n, seed=1000, device=dev)
    agent = Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="fp32", n_envs=n,
                  process_group=None, graph_safe=True)
    tr = VecTrainer(env, agent, use_graphs=True)
    iters = int(os.environ.get("REPRO_ITERS", 7))
    for it in range(iters):
        tr.step()
        if os.environ.get("REPRO_SYNC") == "1":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    L = agent.learner
    fin = {n: all(bool(torch.isfinite(p).all()) for p in m.parameters())
           for n, m in (("actor", L.actor), ("critic", L.critic), ("encoder", L.encoder))}
    print("REPRO", iters, fin, flush=True)


if __name__ == "__main__":
    main()
