"""HIP graphs that live as long as the process.

Every graph exec owns up to 4 runtime streams spread over the
GPU_MAX_HW_QUEUES = 4 hardware queues.  Destroying execs frees those streams
unevenly; the ROCm 7.0 runtime's first-launch stream assignment of a later
exec can then put two of its streams on the launch stream's queue, skip both
and read past its stream array -- the round-4 segfault in hipGraphLaunch
("The graph-replay crash").  With streams only ever added, new
streams keep going to the least-loaded queue, the loads stay within one of
each other and no exec gets two streams on its launch queue.  So every graph
this package (and its tests and bench) captures comes from new_graph() and is
never destroyed; a graph's memory pool lives as long (a few MB per trainer
graph at the bench's shape)."""
import torch

_KEEP = []


def new_graph():
    """torch.cuda.CUDAGraph() kept alive until the process exits."""
    g = torch.cuda.CUDAGraph()
    _KEEP.append(g)
    return g
