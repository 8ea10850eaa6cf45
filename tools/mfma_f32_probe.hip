// Probe of v_mfma_f32_16x16x4_f32's operand / result layout on gfx950 and of
// the fused path's 4-sub-step fp32 k-step (td7_fused.h Ty<PREC_F32>::mfma):
// lane l holds W[l & 15][4 (l >> 4) + j] and X[l & 15][4 (l >> 4) + j], j < 4,
// the 16-deep product C[n][row] = sum_k W[n][k] X[row][k] is expected at lane
// l, register e: n = 4 (l >> 4) + e, row = l & 15.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// (element-wise bit_cast(float, a[j]) of the u32x4 compiled to a[0] for every j
// on this toolchain: the vector is cast whole, then indexed)
__device__ __forceinline__ floatx4 sub(u32x4 a, u32x4 b, floatx4 c, int j) {
    const floatx4 af = __builtin_bit_cast(floatx4, a), bf = __builtin_bit_cast(floatx4, b);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(af[j], bf[j], c, 0, 0, 0);
}
__device__ float W(int n, int k) { return 0.01f * (n + 1) + 0.37f * k - 0.05f * n * k; }
__device__ float X(int r, int k) { return 0.5f - 0.11f * r + 0.03f * k * k; }
__global__ void probe(float *out) {
    const int l = threadIdx.x;
    float wa[4], xb[4];
    for (int j = 0; j < 4; ++j) {
        wa[j] = W(l & 15, 4 * (l >> 4) + j);
        xb[j] = X(l & 15, 4 * (l >> 4) + j);
    }
    const u32x4 a = __builtin_bit_cast(u32x4, floatx4{wa[0], wa[1], wa[2], wa[3]});
    const u32x4 b = __builtin_bit_cast(u32x4, floatx4{xb[0], xb[1], xb[2], xb[3]});
    floatx4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) c = sub(a, b, c, j);
    for (int e = 0; e < 4; ++e) out[l * 4 + e] = c[e];
}
static float Wh(int n, int k) { return 0.01f * (n + 1) + 0.37f * k - 0.05f * n * k; }
static float Xh(int r, int k) { return 0.5f - 0.11f * r + 0.03f * k * k; }
int main() {
    float *d, h[256];
    if (hipMalloc(&d, 1024) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 4; ++e) {
            const int n = 4 * (l >> 4) + e, r = l & 15;
            double want = 0;
            for (int k = 0; k < 16; ++k) want += (double)Wh(n, k) * Xh(r, k);
            if (fabs(h[l * 4 + e] - want) > 1e-4 * (1 + fabs(want))) {
                if (bad < 8) printf("lane %d e %d: got %g want %g\n", l, e, h[l * 4 + e], want);
                ++bad;
            }
        }
    printf("mismatches: %d of 256\n", bad);
    return 0;
}
