"""Do the trainers' HIP graphs replay correctly with ROCm CLR's graph packet
capture ON (DEBUG_CLR_GRAPH_PACKET_CAPTURE=1, the runtime's default)?

exo_amd sets the variable to 0 on import because packet capture replays
captured hipMemsetAsync nodes -- the semaphores of PyTorch's multi-block
reductions -- out of order (tools/graph_reduce_check.py).  This checks, in a
process started with the variable at 1 and EXO_GRAPH_CHECK=0 (the trainer's
reduction self-check captures a torch reduction on purpose):

  1. every graph the two trainers capture holds no memset node
     (hipGraphGetNodes / hipGraphNodeGetType on the kept graphs) -- nothing
     packet capture mis-orders;
  2. the graph-replayed VecTrainer matches eager execution (tools/graph_vs_eager.py,
     single and data-parallel 3-graph layouts);
  3. the graph-replayed RefScheduleTrainer matches its eager execution bit for bit.

Prints one JSON line; exit status 1 on any failure.
usage: DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 EXO_GRAPH_CHECK=0 python tools/packet_capture_check.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "a-deep-reinforcement-learning-enabled-soft-exoskeleton-for-parkinson-s-patients_amd"))

import torch  # noqa: E402


def _ref_schedule(use_graphs, seed=4):
    from exo_amd import VecExoskeletonEnv
    from exo_amd.rollout import RefScheduleTrainer
    from exo_amd.td7 import Agent, Hyperparameters
    torch.manual_seed(seed)
    hp = Hyperparameters(zs_dim=32, enc_hdim=32, critic_hdim=32, actor_hdim=32, batch_size=16, target_update_rate=50)
    env = VecExoskeletonEnv(16, seed=seed)
    ag = Agent(80, 7, 1, hp=hp, env_num=8, buffer_size=2048, graph_safe=use_graphs)
    tr = RefScheduleTrainer(env, ag, warmup=1, use_graphs=use_graphs)
    return tr, ag


def _node_types(graphs):
    """Node-type histogram of the captured hipGraphs (hipGraphGetNodes /
    hipGraphNodeGetType on CUDAGraph.raw_cuda_graph(); every graph is
    created with keep_graph=True here): 0 kernel, 1 memcpy, 2 memset, ..."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hist = {}
    for g in graphs:
        h = ctypes.c_void_p(g.raw_cuda_graph())
        n = ctypes.c_size_t(0)
        assert hip.hipGraphGetNodes(h, None, ctypes.byref(n)) == 0
        nodes = (ctypes.c_void_p * max(n.value, 1))()
        assert hip.hipGraphGetNodes(h, nodes, ctypes.byref(n)) == 0
        for k in range(n.value):
            t = ctypes.c_int(-1)
            assert hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[k]), ctypes.byref(t)) == 0
            hist[t.value] = hist.get(t.value, 0) + 1
    return hist


def main():
    assert os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "1", "run with DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"
    out = {"packet_capture": os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"]}
    import graph_vs_eager
    base = torch.cuda.CUDAGraph

    class KeepGraph(base):  # keep every captured hipGraph_t for the node audit
        def __new__(cls, keep_graph=True):
            return super().__new__(cls, keep_graph)

        def __init__(self, keep_graph=True):  # pybind11 constructs in __init__
            super().__init__(keep_graph)
    torch.cuda.CUDAGraph = KeepGraph
    out["vectrainer_single_max_diff"] = graph_vs_eager.run("single", iters=10, quiet=True)
    out["vectrainer_split_max_diff"] = graph_vs_eager.run("split", iters=10, quiet=True)
    # reference schedule: two rounds (random, then the policy) eager vs graphs
    res = {}
    for use_graphs in (False, True):
        tr, ag = _ref_schedule(use_graphs)
        for _ in range(2):
            tr.run_round()
        torch.cuda.synchronize()
        res[use_graphs] = (tr, [p.detach().clone() for m in (ag.learner.actor, ag.learner.critic, ag.learner.encoder)
                                for p in m.parameters()])
    out["ref_schedule_max_diff"] = max(float((a - b).abs().max()) for a, b in zip(res[False][1], res[True][1]))
    # memset audit of every graph captured above (the VecTrainer's are gone with
    # their trainer: capture a fresh one of each layout)
    from test_rollout_gpu import _make
    tg, _, _ = _make(True, seed=1)
    for _ in range(6):
        tg.step()
    tgs, _, _ = _make(True, seed=1)
    tgs.dp = True
    for _ in range(6):
        tgs.step()
    graphs = [g for tr in (tg, tgs, res[True][0]) for parts in tr.graphs.values()
              for g in (parts if isinstance(parts, list) else [parts]) if isinstance(g, base)]
    out["graphs_audited"] = len(graphs)
    try:
        hist = _node_types(graphs)
        out["node_types"] = {str(k): v for k, v in sorted(hist.items())}
        out["memset_nodes"] = hist.get(2, 0)
    except Exception as e:  # the node query unavailable: say so, do not guess
        out["memset_audit_error"] = repr(e)
    ok = (out["vectrainer_single_max_diff"] <= 1e-5 and out["vectrainer_split_max_diff"] <= 1e-5
          and out["ref_schedule_max_diff"] == 0.0 and out.get("memset_nodes", 1) == 0)
    out["ok"] = ok
    print(json.dumps(out))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
