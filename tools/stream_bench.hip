// Per-CU weight-stream rate microbenchmark for the fused TD7 kernels
// (csrc/td7_fused.h gemm): G workgroups each read the same S-byte packed
// buffer once (1 KiB per wave instruction, tiles of 16 B per lane), the way a
// fused layer streams its weights from L2.  Variants: waves per workgroup,
// loads in flight per wave, cache policy of the load (plain / sc1 / nt), and
// LDS-DMA (global_load_lds_dwordx4) into an LDS ring.  Timing: HIP events
// over 50 launches.  Build: hipcc --offload-arch=gfx950 -O3 -o stream_bench stream_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, 0x7fffffff, 0x00020000);
}

// each wave reads blocks b = wave, wave + NWAVE, ... of 1 KiB (64 lanes x 16 B),
// keeping DEPTH blocks in flight; consumes them with an xor into acc
template <int NWAVE, int DEPTH, int AUX>
__global__ __launch_bounds__(64 * NWAVE) void stream_kernel(const u32x4 *buf, long nblocks, u32x4 *sink) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const auto rs = rsrc(buf);
    u32x4 acc = {0u, 0u, 0u, 0u};
    u32x4 ring[DEPTH];
    long b = w;
#pragma unroll
    for (int p = 0; p < DEPTH; ++p) {
        ring[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((b + (long)p * NWAVE) * 64 + lane) * 16), 0, AUX));
        __builtin_amdgcn_sched_barrier(0);
    }
    for (; b + (long)DEPTH * NWAVE < nblocks; b += (long)DEPTH * NWAVE) {
#pragma unroll
        for (int p = 0; p < DEPTH; ++p) {
            acc ^= ring[p];
            const long nb = b + (long)(p + DEPTH) * NWAVE;
            ring[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((nb * 64 + lane) * 16), 0, AUX));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int p = 0; p < DEPTH; ++p) acc ^= ring[p];
    if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}

// LDS-DMA: each wave streams its blocks into a private LDS ring of DEPTH KiB
template <int NWAVE, int DEPTH, int AUX>
__global__ __launch_bounds__(64 * NWAVE) void dma_kernel(const u32x4 *buf, long nblocks, u32x4 *sink) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    char *ring = lds + w * DEPTH * 1024;
    u32x4 acc = {0u, 0u, 0u, 0u};
    long b = w;
#pragma unroll
    for (int p = 0; p < DEPTH; ++p) {
        __builtin_amdgcn_global_load_lds((const void *)(buf + (b + (long)p * NWAVE) * 64 + lane),
                                         (__attribute__((address_space(3))) void *)(ring + p * 1024), 16, 0, AUX);
    }
    for (; b + (long)DEPTH * NWAVE < nblocks; b += (long)DEPTH * NWAVE) {
#pragma unroll
        for (int p = 0; p < DEPTH; ++p) {
            __builtin_amdgcn_s_waitcnt(0x0f70 | ((DEPTH - 1) & 0xf) | (((DEPTH - 1) >> 4) << 14));  // vmcnt(DEPTH-1)
            acc ^= *(const u32x4 *)(ring + p * 1024 + lane * 16);
            const long nb = b + (long)(p + DEPTH) * NWAVE;
            __builtin_amdgcn_global_load_lds((const void *)(buf + nb * 64 + lane),
                                             (__attribute__((address_space(3))) void *)(ring + p * 1024), 16, 0, AUX);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);
#pragma unroll
    for (int p = 0; p < DEPTH; ++p) acc ^= *(const u32x4 *)(ring + p * 1024 + lane * 16);
    if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}

// cold: launch i reads buffer i % NCOLD of a 64 MiB pool (> the 32 MiB of L2,
// < the Infinity Cache): the weights a fused pass streams come from MALL, not L2
static int g_cold = 0;
static const u32x4 *g_pool = nullptr;
constexpr int NCOLD = 64;
template <typename K>
float timeit(K k, int grid, int threads, int lds, const u32x4 *buf, long nblocks, u32x4 *sink) {
    if (lds) hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k, dim3(grid), dim3(threads), lds, 0, buf, nblocks, sink);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    const int reps = 50;
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k, dim3(grid), dim3(threads), lds, 0, g_cold ? g_pool + (long)(i % NCOLD) * nblocks * 64 : buf,
                           nblocks, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e3f / reps;
}

int main() {
    const long S = 1 << 20;  // 1 MiB per workgroup (a fused pass's weights)
    const long nblocks = S / 1024;
    u32x4 *buf, *sink;
    hipMalloc(&buf, S);
    hipMalloc(&sink, 1 << 16);
    hipMemset(buf, 1, S);
    u32x4 *pool;
    hipMalloc(&pool, S * NCOLD);
    hipMemset(pool, 1, S * NCOLD);
    g_pool = pool;
    printf("%-34s %6s %5s %9s %12s\n", "variant", "WGs", "cold", "us", "GB/s per WG");
    for (int cold : {0, 1})
    for (int grid : {64, 256}) {
        g_cold = cold;
#define RUN(NAME, K, TH, LDS)                                                                 \
    {                                                                                         \
        const float us = timeit(K, grid, TH, LDS, buf, nblocks, sink);                        \
        printf("%-34s %6d %5d %9.2f %12.1f\n", NAME, grid, cold, us, S / (us * 1e-6) / 1e9);  \
    }
        RUN("plain   4 waves x 25", (stream_kernel<4, 25, 0>), 256, 0);
        RUN("plain   8 waves x 25", (stream_kernel<8, 25, 0>), 512, 0);
        RUN("plain  16 waves x 12", (stream_kernel<16, 12, 0>), 1024, 0);
        RUN("plain  16 waves x 25", (stream_kernel<16, 25, 0>), 1024, 0);
        RUN("sc1     8 waves x 25", (stream_kernel<8, 25, 16>), 512, 0);
        RUN("sc1    16 waves x 25", (stream_kernel<16, 25, 16>), 1024, 0);
        RUN("nt      8 waves x 25", (stream_kernel<8, 25, 2>), 512, 0);
        RUN("sc0     8 waves x 25", (stream_kernel<8, 25, 1>), 512, 0);
        RUN("dma     8 waves x 16 KiB", (dma_kernel<8, 16, 0>), 512, 8 * 16 * 1024);
        RUN("dma    16 waves x 8 KiB", (dma_kernel<16, 8, 0>), 1024, 16 * 8 * 1024);
        RUN("dma     4 waves x 32 KiB", (dma_kernel<4, 32, 0>), 256, 4 * 32 * 1024);
        RUN("dma sc1 8 waves x 16 KiB", (dma_kernel<8, 16, 16>), 512, 8 * 16 * 1024);
    }
    hipFree(buf);
    hipFree(sink);
    return 0;
}
