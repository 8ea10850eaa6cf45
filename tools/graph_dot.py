"""Dump the topology of the forked test graphs (tests/test_graph_lifetime_gpu.py)
as hipGraphDebugDotPrint DOT files plus per-node dependent counts, to check
exo_graph_branch_bound.  usage: python tools/graph_dot.py OUTDIR"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402

from exo_amd.graphs import branch_bound  # noqa: E402
from test_graph_lifetime_gpu import _forked_graph  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
hip = ctypes.CDLL("libamdhip64.so.7")
side = [torch.cuda.Stream() for _ in range(5)]
ctr = torch.zeros(8, dtype=torch.int64, device="cuda")
for b in (2, 3, 5):
    g = _forked_graph(side, b, ctr)
    raw = ctypes.c_void_p(g.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    hip.hipGraphGetNodes(raw, None, ctypes.byref(n))
    nodes = (ctypes.c_void_p * n.value)()
    hip.hipGraphGetNodes(raw, nodes, ctypes.byref(n))
    deps = []
    for v in nodes:
        d = ctypes.c_size_t(0)
        rc = hip.hipGraphNodeGetDependentNodes(ctypes.c_void_p(v), None, ctypes.byref(d))
        dd = ctypes.c_size_t(0)
        rc2 = hip.hipGraphNodeGetDependencies(ctypes.c_void_p(v), None, ctypes.byref(dd))
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(v), ctypes.byref(t))
        deps.append((t.value, d.value, rc, dd.value, rc2))
    path = os.path.join(out, f"forked_{b}.dot").encode()
    rc = hip.hipGraphDebugDotPrint(raw, path, 0)
    print(f"branches {b}: {n.value} nodes, (type, dependents, rc, dependencies, rc) {deps}, "
          f"branch_bound {branch_bound(g)}, dot rc {rc}", flush=True)
