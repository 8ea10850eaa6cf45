"""exo_amd -- MI355X-native vectorised exoskeleton environment and TD7/LAP trainer.

Hot path (BASELINE.json north_star): the exoskeleton env step/reset as HIP
kernels for gfx950 (csrc/exo_env.hip) and the TD7 update with a HIP LAP sum
tree (csrc/lap.hip, td7.py).  See DESIGN.md.
"""
import os as _os

# ROCm 7.x CLR "graph packet capture" replays captured hipMemsetAsync nodes out of
# order with the kernels around them: every multi-block torch reduction (its
# semaphores are memset inside the graph) returns wrong sums from the second
# replay on -- NaN bias gradients in the TD7 update.  Off it goes; it must be set
# before the HIP runtime initialises (rollout.VecTrainer checks that it took).
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from .vec_env import VecExoskeletonEnv, DEFAULTS, draws_per_episode  # noqa: F401
