"""exo_amd -- MI355X-native vectorised exoskeleton environment and TD7/LAP trainer.

Hot path (BASELINE.json north_star): the exoskeleton env step/reset as HIP
kernels for gfx950 (csrc/exo_env.hip) and the TD7 update with a HIP LAP sum
tree (csrc/lap.hip, td7.py).  See DESIGN.md.
"""
from .vec_env import VecExoskeletonEnv, DEFAULTS, draws_per_episode  # noqa: F401
