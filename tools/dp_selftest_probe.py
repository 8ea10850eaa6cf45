"""RCCL world 1: GradSync._capture_selftest with the capture's exception
printed (diagnostic).  usage: python tools/dp_selftest_probe.py PORT"""
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
os.environ["EXO_FORCE_DIST"] = "1"
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import exo_amd  # noqa: E402,F401
from exo_amd import td7  # noqa: E402

dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{sys.argv[1]}", rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
sync = td7.GradSync(dist.group.WORLD)
orig = td7.capture


def traced(g, **kw):
    cm = orig(g, **kw)

    class W:
        def __enter__(self):
            return cm.__enter__()

        def __exit__(self, *exc):
            if exc[0] is not None:
                print("exception inside the capture:", flush=True)
                traceback.print_exception(*exc)
            try:
                return cm.__exit__(*exc)
            except Exception:
                print("exception at capture exit:", flush=True)
                traceback.print_exc()
                raise
    return W()


td7.capture = traced
try:
    print("selftest ->", sync._capture_selftest(torch.device("cuda", 0)), flush=True)
except Exception:
    traceback.print_exc()
dist.destroy_process_group()
