"""Reference-schedule rollout under the kernel tracer: 4,096 envs, bf16 TD7,
warm-up 25,000 env-steps, 5 rounds (the last two: policy rounds replayed from
the round graph, or per-step graphs with EXO_REF_ROUND_GRAPH=0).  Run under
rocprofv3 --kernel-trace; tools/iter_timeline-style analysis by hand."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402

from exo_amd import VecExoskeletonEnv  # noqa: E402
from exo_amd.rollout import RefScheduleTrainer  # noqa: E402
from exo_amd.td7 import Agent  # noqa: E402

torch.manual_seed(2)
env = VecExoskeletonEnv(4096, seed=1000)
ag = Agent(80, 7, 1, env_num=8, precision="bf16", n_envs=4096, graph_safe=True)
tr = RefScheduleTrainer(env, ag, warmup=25_000)
for _ in range(5):
    tr.run_round()
torch.cuda.synchronize()
print("done", tr.rounds)
