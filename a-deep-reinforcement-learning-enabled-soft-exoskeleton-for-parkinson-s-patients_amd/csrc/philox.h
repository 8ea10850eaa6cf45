// philox.h -- Philox4x32-10 counter-based random numbers (Salmon et al., SC'11),
// shared by the env reset draws (exo_model.h) and the in-kernel noise / replay
// uniforms of the TD7 update (td7_loss.hip, lap.hip).
#pragma once
#ifndef EXO_HOST_ONLY
#include <hip/hip_runtime.h>
#endif

#include <cstdint>

__host__ __device__ inline void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

#ifndef EXO_HOST_ONLY
// Draw block j of call `call` of a device stream (seed, tag): 4 x 32 random bits.
__device__ inline void philox_block(uint64_t seed, uint32_t tag, uint64_t call, uint32_t j, uint32_t out[4]) {
    out[0] = j;
    out[1] = (uint32_t)call;
    out[2] = (uint32_t)(call >> 32);
    out[3] = tag;
    philox4x32(out, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// [0, 1) and (0, 1] floats from 24 random bits
__device__ inline float u01_open_hi(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-8f; }
__device__ inline float u01_open_lo(uint32_t x) { return (float)((x >> 8) + 1u) * 5.9604644775390625e-8f; }

// two standard normals (Box-Muller) from one Philox block
__device__ inline void box_muller(const uint32_t r[4], float &z0, float &z1) {
    const float rad = sqrtf(-2.0f * logf(u01_open_lo(r[0])));
    float s, c;
    sincosf(6.283185307179586f * u01_open_hi(r[1]), &s, &c);
    z0 = rad * c;
    z1 = rad * s;
}
#endif
