#!/usr/bin/env python3
"""Diagnostic: per-wave phase shares of the row-parallel exo_step kernel from
in-kernel s_memtime stamps (libexo_amd_stamps.so, `make -C csrc stamps`).
Never the measured number -- stamps serialise the phases; read the SHARES."""
import ctypes
import json
import os
import sys

os.environ.setdefault("EXO_AMD_LIB", "libexo_amd_stamps.so")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from exo_amd import VecExoskeletonEnv  # noqa: E402
from exo_amd import _native as nat  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
env = VecExoskeletonEnv(N, seed=1)
env.set_step_variant("rows")
env.reset()
blocks = (N + 3) // 4
buf = torch.zeros(blocks * 16, dtype=torch.int64, device="cuda")
lib = nat.lib()
lib.exo_debug_set_stamps.argtypes = [ctypes.c_void_p]
out = env.new_outputs(True)
phases = ["fk", "actuator", "torques+reward+obs+state", "ode", "targets+motor"]
res = {}
for k in range(60):
    if k == 50:
        assert lib.exo_debug_set_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    env.step(torch.rand((N, 7), device="cuda") * 2 - 1, out=out)
    torch.cuda.synchronize()
    if k >= 50:
        st = buf.view(blocks, 16)[:, :6].cpu().numpy().astype(np.int64)
        d = np.diff(st, axis=1)
        tot = st[:, 5] - st[:, 0]
        for i, p in enumerate(phases):
            res.setdefault(p, []).append(float(np.median(d[:, i])))
        res.setdefault("total_median", []).append(float(np.median(tot)))
        res.setdefault("total_max", []).append(float(np.max(tot)))
        w = int(np.argmax(tot))  # the slowest wave's phases
        for i, p in enumerate(phases):
            res.setdefault("slowest:" + p, []).append(float(d[w, i]))
        res.setdefault("ode_p90", []).append(float(np.percentile(d[:, 3], 90)))
        res.setdefault("ode_max", []).append(float(np.max(d[:, 3])))
        full = buf.view(blocks, 16).cpu().numpy().astype(np.int64)
        if (full[:, 8] > 0).all():  # EXO_STAMPS_MEMWAIT build: all kernel-start loads returned
            res.setdefault("memwait_median", []).append(float(np.median(full[:, 8] - full[:, 0])))
            res.setdefault("memwait_max", []).append(float(np.max(full[:, 8] - full[:, 0])))
        if (full[:, 6] > 0).all() and (full[:, 7] > 0).all():  # sub-phases of torques+reward+obs+state
            res.setdefault("sub:torque_table", []).append(float(np.median(full[:, 6] - full[:, 2])))
            res.setdefault("sub:sync+reward", []).append(float(np.median(full[:, 7] - full[:, 6])))
            res.setdefault("sub:obs+state", []).append(float(np.median(full[:, 3] - full[:, 7])))
summary = {k: float(np.median(v)) for k, v in res.items()}
summary["shares"] = {p: summary[p] / summary["total_median"] for p in phases}
print(json.dumps(summary, indent=1))
