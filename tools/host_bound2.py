"""Host issue time vs wall time per training iteration of the bench's default
loop (VecTrainer, async episodes, bf16): K steps with no synchronisation, then
until the GPU drains.  Equal numbers mean the GPU waits on graph submission."""
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402


def main(K=400):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    dev = torch.device("cuda", 0)
    env = VecExoskeletonEnv(4096, seed=1000, device=dev)
    agent = Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="bf16", n_envs=4096,
                  graph_safe=True)
    tr = VecTrainer(env, agent, episodes="async")
    for _ in range(60):
        tr.step()
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(K):
            tr.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"trainer.step: host issue {1e3 * (t1 - t0) / K:.4f} ms/iter, wall {1e3 * (t2 - t0) / K:.4f} ms/iter")
    keys = sorted(tr.graphs, key=str)
    print("graphs:", keys)
    for k in keys:
        g = tr.graphs[k]
        g = g[0] if isinstance(g, tuple) else g
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"replay {k}: host {1e3 * (t1 - t0) / K:.4f} ms, wall {1e3 * (t2 - t0) / K:.4f} ms")


if __name__ == "__main__":
    main()
