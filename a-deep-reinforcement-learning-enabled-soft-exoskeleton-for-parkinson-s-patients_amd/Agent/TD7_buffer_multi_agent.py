"""Drop-in module path of Agent/TD7_buffer_multi_agent.py (HIP sum-tree LAP)."""
from exo_amd.replay import LAP  # noqa: F401
