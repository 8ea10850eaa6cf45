"""Diagnostic: graph capture of the fused-path VecTrainer at small shapes
(r04f: a segfault in capture_end at batch 8 x 32, 64 envs).  usage:
python tools/seg_bisect.py BATCH ENVS PREFETCH(0/1)"""
import faulthandler
import os
import sys

faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import torch  # noqa: E402

from exo_amd import VecExoskeletonEnv  # noqa: E402
from exo_amd.rollout import VecTrainer  # noqa: E402
from exo_amd.td7 import Agent, Hyperparameters  # noqa: E402

batch, envs, pf = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1"
VecTrainer.prefetch_targets = pf
torch.manual_seed(11)
hp = Hyperparameters(batch_size=batch, target_update_rate=5)
env = VecExoskeletonEnv(envs, seed=11)
ag = Agent(80, 7, 1, hp=hp, env_num=8, precision="bf16", n_envs=envs, buffer_size=8192, graph_safe=True)
tr = VecTrainer(env, ag)
for i in range(8):
    print("iter", i, flush=True)
    tr.step()
torch.cuda.synchronize()
print("ok", batch, envs, pf, sorted(map(str, tr.graphs)), flush=True)
