"""Drop-in module path of the reference's Agent/TD7_multi_agent.py: the TD7
agent runs on PyTorch-ROCm with HIP LAP replay (see exo_amd.td7)."""
from exo_amd.td7 import (LAP_huber, Actor, Agent, AvgL1Norm, Critic, Encoder,  # noqa: F401
                         Hyperparameters)
