"""Host issue vs wall time of the reference schedule's burst train steps
(RefScheduleTrainer.train_step, graph-replayed), 4,096 envs, bf16."""
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402


def main(K=283):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    dev = torch.device("cuda", 0)
    env = VecExoskeletonEnv(4096, seed=1000, device=dev)
    ag = Agent(80, 7, 1, env_num=8, hp=Hyperparameters(), device=dev, precision="bf16", n_envs=4096, graph_safe=True)
    tr = RefScheduleTrainer(env, ag, warmup=25_000)
    for _ in range(3):
        tr.run_round()
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(K):
            tr.train_step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"burst train_step: host issue {1e3 * (t1 - t0) / K:.4f} ms/step, wall {1e3 * (t2 - t0) / K:.4f} ms/step")


if __name__ == "__main__":
    main()
