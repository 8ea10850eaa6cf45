// Ballast streams for releasing HIP graph execs (r06).
//
// The ROCm 7.0 runtime (torch's bundled libamdhip64) assigns a graph exec's
// own streams to its parallel branches at launch, skipping a stream on the
// launch stream's hardware queue, with no bound on its stream index: once
// destroyed execs have left the launch queue least loaded by two, the next
// exec gets two streams there and its launch reads past its stream vector
// (+0xaee41; tools/graph_stream_pool_repro.hip faults this way without torch,
// DESIGN.md 4 "The graph-replay crash").  New streams go to the least-loaded
// of the GPU_MAX_HW_QUEUES queues, so creating at least as many streams as
// the destroyed execs released brings the queue loads back within one of
// each other (the repro's "ballast" arm ran clean where "destroy" faulted).
// The streams are kept for the life of the process.
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "exo_amd.h"

namespace {
std::mutex g_mu;
std::vector<hipStream_t> g_ballast;
}  // namespace

extern "C" int exo_stream_ballast(int32_t n) {
    if (n < 0) return EXO_EINVAL;
    std::lock_guard<std::mutex> lock(g_mu);
    for (int32_t i = 0; i < n; ++i) {
        hipStream_t s;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return EXO_EDEVICE;
        g_ballast.push_back(s);
    }
    return (int)g_ballast.size();
}

// An upper bound on the parallel branches of a captured graph (the streams
// its exec can own): 1 + the sum over nodes of (dependents - 1).  Diagnostic
// for BALLAST_PER_GRAPH (exo_amd/graphs.py; tests/test_graph_lifetime_gpu.py).
extern "C" int exo_graph_branch_bound(void *graph, int32_t *out) {
    if (!graph || !out) return EXO_EINVAL;
    hipGraph_t g = (hipGraph_t)graph;
    size_t n = 0;
    if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return EXO_EDEVICE;
    std::vector<hipGraphNode_t> nodes(n);
    if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return EXO_EDEVICE;
    long long bound = 1;
    for (hipGraphNode_t v : nodes) {
        size_t d = 0;
        if (hipGraphNodeGetDependentNodes(v, nullptr, &d) != hipSuccess) return EXO_EDEVICE;
        if (d > 1) bound += (long long)d - 1;
    }
    *out = (int32_t)bound;
    return EXO_OK;
}
