"""HIP graphs: creation, and release without the ROCm 7.0 graph-launch fault.

Every graph exec owns runtime streams (one per parallel branch, created at
instantiate) spread over the GPU_MAX_HW_QUEUES = 4 hardware queues.  The ROCm
7.0 runtime assigns them at each launch, skipping a stream that sits on the
launch stream's queue, with no bound on the stream index: once destroyed
execs have left the launch queue least loaded by two, a new exec puts two of
its streams there and its launch reads past its stream vector (libamdhip64
+0xaee41).  tools/graph_stream_pool_repro.hip, torch-free, faults exactly
there when it destroys execs and runs clean when it keeps them or replaces
the released streams ("The graph-replay crash").

So a graph is never destroyed by garbage collection: new_graph() keeps a
reference until release_graphs() destroys it (its exec and memory pool) and
then creates ballast streams (exo_stream_ballast) -- new streams go to the
least-loaded queue, so at least as many as were released bring the queue
loads back within one of each other.  How many an exec released is bounded
from its captured graph (exo_graph_branch_bound: the graph's roots plus its
extra dependents), so graphs keep their hipGraph_t (keep_graph=True) and are
instantiated by capture() right after the capture, as torch does without it."""
import contextlib

import torch

_KEEP = []

# ballast streams per released graph when its captured graph is not available
FALLBACK_BALLAST = 64


def new_graph():
    """torch.cuda.CUDAGraph(keep_graph=True) kept alive until release_graphs()
    (or process exit); capture into it with capture()."""
    g = torch.cuda.CUDAGraph(keep_graph=True)
    _KEEP.append(g)
    return g


@contextlib.contextmanager
def capture(g, **kw):
    """torch.cuda.graph(g, **kw), then the exec instantiated at once (with
    keep_graph=True torch would instantiate at the first replay)."""
    with torch.cuda.graph(g, **kw):
        yield g
    g.instantiate()


def branch_bound(g):
    """An upper bound on the streams g's exec owns (None: no captured graph)."""
    from . import _native as nat
    import ctypes
    try:
        raw = g.raw_cuda_graph()
    except RuntimeError:
        return None
    if not raw:
        return None
    out = ctypes.c_int32(0)
    if nat.lib().exo_graph_branch_bound(ctypes.c_void_p(raw), ctypes.byref(out)) != 0:
        return None
    return int(out.value)


def _graphs_in(obj, out):
    if isinstance(obj, torch.cuda.CUDAGraph):
        out.append(obj)
    elif isinstance(obj, dict):
        for v in obj.values():
            _graphs_in(v, out)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _graphs_in(v, out)
    return out


def release_graphs(*objs):
    """Destroy the graphs found in objs (graphs, or dicts / lists / tuples of
    them): the device is synchronised first, each exec, captured graph and
    memory pool freed (CUDAGraph.reset), then ballast streams replace the
    streams the execs held (their branch bound + 1 each).  Returns the number
    of graphs released."""
    gs = []
    for o in objs:
        _graphs_in(o, gs)
    seen, uniq = set(), []
    for g in gs:
        if id(g) not in seen:
            seen.add(id(g))
            uniq.append(g)
    if not uniq:
        return 0
    from . import _native as nat
    torch.cuda.synchronize()
    ballast = 0
    for g in uniq:
        b = branch_bound(g)
        ballast += FALLBACK_BALLAST if b is None else b + 1
        for i, k in enumerate(_KEEP):
            if k is g:
                del _KEEP[i]
                break
        g.reset()
    rc = nat.lib().exo_stream_ballast(ballast)
    if rc < 0:
        raise RuntimeError(f"exo_stream_ballast failed ({rc})")
    return len(uniq)


def kept_graphs():
    """The graphs alive through new_graph() (not yet released)."""
    return len(_KEEP)
