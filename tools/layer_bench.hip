// Per-layer cost of the fused TD7 layer chain (csrc/td7_fused.h) in isolation:
// G workgroups each run NL forward layers of 320 x 320 (bf16, ks 10, 20 tiles,
// TH 5) with distinct packed weights, 16 rows in LDS, like one network pass.
// MODE 0: layer_fwd (gemm + exchange + ELU epilogue + barrier); MODE 1: gemm
// (incl. exchange) + barrier, no epilogue; MODE 2: ring streaming only (the
// same loads, no MFMA / exchange / barrier).  Prints us per launch and the
// per-workgroup weight-stream rate.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../<pkg>/csrc -o layer_bench layer_bench.hip
#include "td7_fused.h"

#include <cstdio>
#include <vector>

using namespace td7f;

constexpr int NL = 8, K = 320, N = 320, KS = 10, NT = 20, THH = 5;

struct Args {
    Lin L[NL];
    R16 A, B;
    int lds;
};

template <int MODE>
__global__ __launch_bounds__(NTH) void chain_kernel(Args a, float *sink) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    int si = 0;
    zero_lds(lds, a.lds);
    __syncthreads();
    u32x4 R[PD][THH];
    ring_fill(R, GDesc{a.L[0].wf, a.L[0].ksf, 0});
    if constexpr (MODE == 2) {
        u32x4 x = {0u, 0u, 0u, 0u};
        const int wv = threadIdx.x >> 6, w = wv % NW, kg = wv / NW, lane = threadIdx.x & 63;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            int kb, ke;
            kgroup_range(KS, kg, kb, ke);
#pragma unroll
            for (int p = 0; p < PD; ++p)
#pragma unroll
                for (int i = 0; i < THH; ++i) {
                    x ^= R[p][i];
                    if (l + 1 < NL)
                        R[p][i] = ldg(a.L[l + 1].wf + ((size_t)(w + NW * i) * KS + kb + p) * 64 + lane);
                    __builtin_amdgcn_sched_barrier(0);
                }
        }
        if (x.x == 0x12345u) sink[threadIdx.x] = 1.f;
        return;
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        const R16 in = (l & 1) ? a.B : a.A, out = (l & 1) ? a.A : a.B;
        const GDesc nx = l + 1 < NL ? GDesc{a.L[l + 1].wf, a.L[l + 1].ksf, 0} : GDesc{nullptr, 0, 0};
        if constexpr (MODE == 0) {
            layer_fwd<PREC_BF16, 1, THH>(lds, R, in, a.L[l], l + 1 < NL ? &nx : nullptr, ACT_ELU, out, 0, NO32,
                                        nullptr, 0, 0, 16, si);
        } else {
            floatx4 acc[1][THH], bias[1][THH];
            gemm<PREC_BF16, 1, THH>(lds, in.off, in.ld, GDesc{a.L[l].wf, a.L[l].ksf, 0}, R, acc,
                                    l + 1 < NL ? &nx : nullptr, EpiSrc{a.L[l].b, 0, 0, 0, 0, N}, bias);
            __syncthreads();
            if (acc[0][0][0] == 12345.f) sink[threadIdx.x] = acc[0][1][1] + bias[0][0][0];
        }
    }
}

template <typename F>
float timeit(F launch) {
    launch();
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 50; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / 50;
}

int main() {
    const size_t wbytes = (size_t)KS * NT * 1024;  // one layer's forward pack
    u32x4 *w;
    float *b, *sink;
    hipMalloc(&w, wbytes * NL);
    hipMalloc(&b, N * sizeof(float));
    hipMalloc(&sink, 4096 * sizeof(float));
    std::vector<uint16_t> h(wbytes * NL / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0x3c00 + (uint16_t)(i * 2654435761u >> 28);  // small bf16 values
    hipMemcpy(w, h.data(), wbytes * NL, hipMemcpyHostToDevice);
    hipMemset(b, 0, N * sizeof(float));
    Args a{};
    for (int l = 0; l < NL; ++l) a.L[l] = Lin{w + l * wbytes / 16, nullptr, b, N, K, KS, KS, nullptr, 0};
    const int ld = ((KS + PD - 1) / PD * PD) * 32 + 16;
    a.A = R16{red_bytes(1, THH), ld};
    a.B = R16{red_bytes(1, THH) + 16 * ld * 2, ld};
    a.lds = red_bytes(1, THH) + 2 * 16 * ld * 2;
    const char *names[3] = {"layer_fwd (gemm+exchange+epilogue)", "gemm+exchange, no epilogue", "ring stream only"};
    printf("%-38s %5s %9s %10s %14s\n", "mode", "WGs", "us", "us/layer", "GB/s per WG");
    for (int mode = 0; mode < 3; ++mode)
        for (int G : {64, 256}) {
            auto launch = [&] {
                if (mode == 0) {
                    hipFuncSetAttribute((const void *)chain_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, a.lds);
                    hipLaunchKernelGGL(chain_kernel<0>, dim3(G), dim3(NTH), a.lds, 0, a, sink);
                } else if (mode == 1) {
                    hipFuncSetAttribute((const void *)chain_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, a.lds);
                    hipLaunchKernelGGL(chain_kernel<1>, dim3(G), dim3(NTH), a.lds, 0, a, sink);
                } else {
                    hipFuncSetAttribute((const void *)chain_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, a.lds);
                    hipLaunchKernelGGL(chain_kernel<2>, dim3(G), dim3(NTH), a.lds, 0, a, sink);
                }
            };
            const float us = timeit(launch);
            printf("%-38s %5d %9.2f %10.2f %14.1f\n", names[mode], G, us, us / NL, wbytes * NL / (us * 1e-6) / 1e9);
        }
    return 0;
}
