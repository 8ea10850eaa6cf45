"""Drop-in module path of Agent/TD7_multi_agent_Pink_noise.py: same Agent;
select_action(state, timestep, first_step, ...) uses per-episode coloured
noise (exo_amd.pink) when a timestep is given.  Actor width 300 as in the
reference's Pink-noise hyperparameters (:54)."""
from dataclasses import dataclass

from exo_amd.td7 import (LAP_huber, Actor, Agent, AvgL1Norm, Critic, Encoder,  # noqa: F401
                         Hyperparameters as _HP)


@dataclass
class Hyperparameters(_HP):
    actor_hdim: int = 300
