// adam_math.h -- the per-element Adam update shared by every optimiser kernel
// (td7_ops.hip: FlatAdam steps; td7_fused.hip: the step fused with the weight
// packing), so all of them compute bit-identical parameters and moments.
//
// torch.optim.Adam semantics (Agent/TD7_multi_agent.py:165-170, weight_decay):
//   g += wd * p;  m = lerp(m, g, 1 - b1);  v = b2 v + (1 - b2) g^2;
//   p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
// step_size = lr / bc1 and bc2s = sqrt(bc2) are computed once per launch.
#pragma once

#include <hip/hip_runtime.h>

__device__ __forceinline__ void adam_one(float &p, float g, float &m, float &v, float step_size, float bc2s,
                                         float b1, float b2, float eps, float wd, float gscale) {
    // no FMA contraction: every kernel rounds every operation alike, whatever
    // the surrounding code lets the backend fuse
#pragma clang fp contract(off)
    g *= gscale;
    if (wd != 0.0f) g += wd * p;
    m += (1.0f - b1) * (g - m); // lerp_(grad, 1 - beta1)
    v = v * b2 + (1.0f - b2) * g * g;
    p -= step_size * (m / (sqrtf(v) / bc2s + eps));
}
