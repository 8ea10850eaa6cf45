// Torch-free repro for the graph-launch fault of r04/r05.
//
// Claim under test ("The graph-replay crash"): a graph exec owns
// one HIP stream per parallel branch beyond the first (created at
// instantiate); its launch assigns them to the branches, skipping a stream
// that maps to the launch stream's hardware queue, with no bound on the pool
// index.  New streams go to the least-loaded of the GPU_MAX_HW_QUEUES queues,
// so once destroyed execs have left the launch stream's queue least loaded by
// two, a new exec puts two of its streams there and its launch reads past its
// stream vector.
//
// What this program does: one launch stream and the same fork/join graph
// shapes a trainer captures (a root on the launch stream, B - 1 forked
// branches of one small kernel each, joined back), instantiated into a pool of
// live execs.  Every trial instantiates 1-3 new execs (2-5 branches), destroys
// a random subset of the live ones ("destroy" arm) or none ("keep" arm, the
// r05 mitigation: no exec destroyed), or destroys them and creates 4 ballast
// streams per destroyed exec ("ballast" arm: new streams go to the least-loaded
// queues, so at least as many new streams as were released bring the queue
// loads back within one of each other), then launches every live exec on the
// launch stream and checks the counters every branch increments.  A fault is
// printed with per-library offsets (the tools/segv_trace.c handler, linked in)
// so it can be matched against libamdhip64.so's disassembly.
//
// Build: hipcc --offload-arch=gfx950 -O1 -g -o tools/graph_stream_pool_repro tools/graph_stream_pool_repro.hip
// Run:   tools/graph_stream_pool_repro keep|ballast|destroy [trials] [seed]
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <random>
#include <vector>

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            exit(2);                                                                                 \
        }                                                                                            \
    } while (0)

static void on_segv(int sig, siginfo_t *si, void *) {
    char line[512];
    int n = snprintf(line, sizeof line, "segv: signal %d, fault address %p\n", sig, si->si_addr);
    write(2, line, n);
    void *frames[64];
    int k = backtrace(frames, 64);
    for (int i = 0; i < k; ++i) {
        Dl_info d;
        memset(&d, 0, sizeof d);
        if (dladdr(frames[i], &d) && d.dli_fname) {
            unsigned long off = (unsigned long)frames[i] - (unsigned long)d.dli_fbase;
            n = snprintf(line, sizeof line, "  #%02d %s+0x%lx (%s)\n", i, d.dli_fname, off,
                         d.dli_sname ? d.dli_sname : "?");
        } else {
            n = snprintf(line, sizeof line, "  #%02d %p ?\n", i, frames[i]);
        }
        write(2, line, n);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

// one vector atomic per branch (global memory through the vector path)
__global__ void bump(unsigned *ctr, int slot) {
    if (threadIdx.x == 0) atomicAdd(ctr + slot, 1u);
}

struct Shape {
    hipGraph_t graph;
    int branches;
};

// root on the capture stream, branches - 1 forked streams each running one
// kernel, joined back, then a tail kernel: the graph executor's parallel
// lists are the branches
static Shape capture_shape(hipStream_t cap, std::vector<hipStream_t> &side, int branches, unsigned *ctr) {
    Shape s{nullptr, branches};
    hipEvent_t fork, join[8];
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    for (int b = 0; b < branches; ++b) CK(hipEventCreateWithFlags(&join[b], hipEventDisableTiming));
    CK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, cap, ctr, 0);
    CK(hipEventRecord(fork, cap));
    for (int b = 1; b < branches; ++b) {
        CK(hipStreamWaitEvent(side[b - 1], fork, 0));
        hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, side[b - 1], ctr, b);
        CK(hipEventRecord(join[b], side[b - 1]));
    }
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, cap, ctr, 0);
    for (int b = 1; b < branches; ++b) CK(hipStreamWaitEvent(cap, join[b], 0));
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, cap, ctr, 7);
    CK(hipStreamEndCapture(cap, &s.graph));
    CK(hipEventDestroy(fork));
    for (int b = 0; b < branches; ++b) CK(hipEventDestroy(join[b]));
    return s;
}

int main(int argc, char **argv) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
    setvbuf(stdout, nullptr, _IOLBF, 0);

    const bool ballast = argc > 1 && !strcmp(argv[1], "ballast");
    const bool destroy = ballast || (argc > 1 && !strcmp(argv[1], "destroy"));
    const int trials = argc > 2 ? atoi(argv[2]) : 200;
    const unsigned seed = argc > 3 ? (unsigned)atoi(argv[3]) : 1u;
    const char *q = getenv("GPU_MAX_HW_QUEUES");
    printf("arm=%s trials=%d seed=%u GPU_MAX_HW_QUEUES=%s\n", ballast ? "ballast" : destroy ? "destroy" : "keep",
           trials, seed,
           q ? q : "(default)");

    CK(hipSetDevice(0));
    unsigned *ctr;
    CK(hipMalloc(&ctr, 8 * sizeof(unsigned)));
    CK(hipMemset(ctr, 0, 8 * sizeof(unsigned)));
    hipStream_t launch, cap;
    CK(hipStreamCreateWithFlags(&launch, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
    std::vector<hipStream_t> side(4);
    for (auto &s : side) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<Shape> shapes;
    for (int b = 2; b <= 5; ++b) shapes.push_back(capture_shape(cap, side, b, ctr));

    std::mt19937 rng(seed);
    struct Live {
        hipGraphExec_t exec;
        int branches;
    };
    std::vector<Live> live;
    std::vector<hipStream_t> ballast_streams;
    unsigned long long want[8] = {0};
    long launches = 0, created = 0, destroyed = 0;
    for (int t = 0; t < trials; ++t) {
        const int add = 1 + (int)(rng() % 3);
        for (int i = 0; i < add; ++i) {
            const Shape &s = shapes[rng() % shapes.size()];
            Live l{nullptr, s.branches};
            CK(hipGraphInstantiate(&l.exec, s.graph, nullptr, nullptr, 0));
            live.push_back(l);
            ++created;
        }
        if (destroy) {
            for (size_t i = 0; i < live.size();) {
                if (rng() % 2 == 0 && live.size() > 1) {
                    CK(hipGraphExecDestroy(live[i].exec));
                    for (int k = 0; ballast && k < 4; ++k) {
                        hipStream_t b;
                        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
                        ballast_streams.push_back(b);
                    }
                    live[i] = live.back();
                    live.pop_back();
                    ++destroyed;
                } else {
                    ++i;
                }
            }
        }
        printf("trial %d: live %zu execs (created %ld, destroyed %ld, ballast streams %zu), launching\n", t,
               live.size(), created, destroyed, ballast_streams.size());
        for (const Live &l : live) {
            CK(hipGraphLaunch(l.exec, launch));
            ++launches;
            want[0] += 2;
            for (int b = 1; b < l.branches; ++b) want[b] += 1;
            want[7] += 1;
        }
        CK(hipStreamSynchronize(launch));
    }
    unsigned got[8];
    CK(hipMemcpy(got, ctr, sizeof got, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 8; ++i) bad |= (unsigned long long)got[i] != want[i];
    printf("done: %ld launches, %ld execs created, %ld destroyed, counters %s\n", launches, created, destroyed,
           bad ? "WRONG" : "ok");
    for (const Live &l : live) CK(hipGraphExecDestroy(l.exec));
    for (auto &s : shapes) CK(hipGraphDestroy(s.graph));
    for (auto &b : ballast_streams) CK(hipStreamDestroy(b));
    return bad ? 1 : 0;
}
