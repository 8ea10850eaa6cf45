"""Is the training iteration bound by the host? Time K trainer steps with no
synchronisation (host issue time) and until the GPU drains (wall): equal
numbers mean the GPU waits on graph submission."""
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402


def main(K=200):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import VecTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    dev = torch.device("cuda", 0)
    env = VecExoskeletonEnv(4096, seed=1000, device=dev)
    agent = Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="bf16", n_envs=4096,
                  graph_safe=True)
    tr = VecTrainer(env, agent)
    for _ in range(40):
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        tr.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e3 * (t1 - t0) / K:.3f} ms/iter, wall {1e3 * (t2 - t0) / K:.3f} ms/iter")
    # the two parities' graphs alternately, nothing else
    gs = [tr.graphs[k][0] for k in sorted(tr.graphs)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        gs[i & 1].replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"alternating replays: host {1e3 * (t1 - t0) / K:.3f} ms, wall {1e3 * (t2 - t0) / K:.3f} ms")
    # per-step host pieces
    L = agent.learner
    t0 = time.perf_counter()
    for i in range(K):
        tr.active.copy_(tr.active_table[i % 10])
    t1 = time.perf_counter()
    for i in range(K):
        L.maybe_update_targets()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"active copy {1e3 * (t1 - t0) / K:.3f} ms, maybe_update_targets {1e3 * (t2 - t1) / K:.3f} ms")
    # replay alone (no per-step host work besides the launch)
    g = next(v for k, v in tr.graphs.items() if not k[0])[0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay() if hasattr(g, "replay") else None
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph replay only: host {1e3 * (t1 - t0) / K:.3f} ms, wall {1e3 * (t2 - t0) / K:.3f} ms", type(g))


if __name__ == "__main__":
    main()
