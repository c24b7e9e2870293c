// bf_common.h — shared helpers for the gfx950 kernels of libboxfusion_hip.so
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/boxfusion_hip.h"

#define BF_API extern "C" __attribute__((visibility("default")))

static inline hipStream_t bf_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int bf_check_launch() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? BF_OK : BF_ERR_LAUNCH;
}

static inline unsigned bf_cdiv(unsigned a, unsigned b) { return (a + b - 1) / b; }

// wave64 helpers ---------------------------------------------------------------------------
__device__ __forceinline__ int bf_lane() { return threadIdx.x & 63; }

__device__ __forceinline__ int bf_wave_sum_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ long long bf_wave_sum_i64(long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// number of set lanes below this lane in a 64-bit ballot mask
__device__ __forceinline__ int bf_lanes_below(unsigned long long mask) {
    unsigned long long below = (bf_lane() == 0) ? 0ull : (mask & ((1ull << bf_lane()) - 1ull));
    return __popcll(below);
}

// 4x4 inverse by cofactors in f64, rounded to f32 (rigid poses: exact to ~1 ulp)
__device__ __forceinline__ void bf_inv4(const float* m32, float* out) {
    double m[16], inv[16];
    for (int i = 0; i < 16; ++i) m[i] = m32[i];
    inv[0] = m[5]*m[10]*m[15] - m[5]*m[11]*m[14] - m[9]*m[6]*m[15] + m[9]*m[7]*m[14] + m[13]*m[6]*m[11] - m[13]*m[7]*m[10];
    inv[4] = -m[4]*m[10]*m[15] + m[4]*m[11]*m[14] + m[8]*m[6]*m[15] - m[8]*m[7]*m[14] - m[12]*m[6]*m[11] + m[12]*m[7]*m[10];
    inv[8] = m[4]*m[9]*m[15] - m[4]*m[11]*m[13] - m[8]*m[5]*m[15] + m[8]*m[7]*m[13] + m[12]*m[5]*m[11] - m[12]*m[7]*m[9];
    inv[12] = -m[4]*m[9]*m[14] + m[4]*m[10]*m[13] + m[8]*m[5]*m[14] - m[8]*m[6]*m[13] - m[12]*m[5]*m[10] + m[12]*m[6]*m[9];
    inv[1] = -m[1]*m[10]*m[15] + m[1]*m[11]*m[14] + m[9]*m[2]*m[15] - m[9]*m[3]*m[14] - m[13]*m[2]*m[11] + m[13]*m[3]*m[10];
    inv[5] = m[0]*m[10]*m[15] - m[0]*m[11]*m[14] - m[8]*m[2]*m[15] + m[8]*m[3]*m[14] + m[12]*m[2]*m[11] - m[12]*m[3]*m[10];
    inv[9] = -m[0]*m[9]*m[15] + m[0]*m[11]*m[13] + m[8]*m[1]*m[15] - m[8]*m[3]*m[13] - m[12]*m[1]*m[11] + m[12]*m[3]*m[9];
    inv[13] = m[0]*m[9]*m[14] - m[0]*m[10]*m[13] - m[8]*m[1]*m[14] + m[8]*m[2]*m[13] + m[12]*m[1]*m[10] - m[12]*m[2]*m[9];
    inv[2] = m[1]*m[6]*m[15] - m[1]*m[7]*m[14] - m[5]*m[2]*m[15] + m[5]*m[3]*m[14] + m[13]*m[2]*m[7] - m[13]*m[3]*m[6];
    inv[6] = -m[0]*m[6]*m[15] + m[0]*m[7]*m[14] + m[4]*m[2]*m[15] - m[4]*m[3]*m[14] - m[12]*m[2]*m[7] + m[12]*m[3]*m[6];
    inv[10] = m[0]*m[5]*m[15] - m[0]*m[7]*m[13] - m[4]*m[1]*m[15] + m[4]*m[3]*m[13] + m[12]*m[1]*m[7] - m[12]*m[3]*m[5];
    inv[14] = -m[0]*m[5]*m[14] + m[0]*m[6]*m[13] + m[4]*m[1]*m[14] - m[4]*m[2]*m[13] - m[12]*m[1]*m[6] + m[12]*m[2]*m[5];
    inv[3] = -m[1]*m[6]*m[11] + m[1]*m[7]*m[10] + m[5]*m[2]*m[11] - m[5]*m[3]*m[10] - m[9]*m[2]*m[7] + m[9]*m[3]*m[6];
    inv[7] = m[0]*m[6]*m[11] - m[0]*m[7]*m[10] - m[4]*m[2]*m[11] + m[4]*m[3]*m[10] + m[8]*m[2]*m[7] - m[8]*m[3]*m[6];
    inv[11] = -m[0]*m[5]*m[11] + m[0]*m[7]*m[9] + m[4]*m[1]*m[11] - m[4]*m[3]*m[9] - m[8]*m[1]*m[7] + m[8]*m[3]*m[5];
    inv[15] = m[0]*m[5]*m[10] - m[0]*m[6]*m[9] - m[4]*m[1]*m[10] + m[4]*m[2]*m[9] + m[8]*m[1]*m[6] - m[8]*m[2]*m[5];
    double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    for (int i = 0; i < 16; ++i) out[i] = (float)(inv[i] / det);
}

// corner sign table of GeneralInstance3DBoxes.corners (boxes.py:757-766)
__device__ __forceinline__ float bf_vsign_x(int c) { return (c == 1 || c == 2 || c == 5 || c == 6) ? 1.f : -1.f; }
__device__ __forceinline__ float bf_vsign_y(int c) { return (c == 2 || c == 3 || c == 6 || c == 7) ? 1.f : -1.f; }
__device__ __forceinline__ float bf_vsign_z(int c) { return (c >= 4) ? 1.f : -1.f; }

// pose disparity of box_manager.py:168-215 in float32
__device__ __forceinline__ void bf_pose_disparity(const float* P1, const float* P2, float* baseline,
                                                  float* angle) {
    float dx = P2[3] - P1[3], dy = P2[7] - P1[7], dz = P2[11] - P1[11];
    *baseline = sqrtf((dx * dx + dy * dy) + dz * dz);
    float tr = 0.f;
    for (int i = 0; i < 3; ++i) {
        float s = P2[4 * i + 0] * P1[4 * i + 0];
        s = s + P2[4 * i + 1] * P1[4 * i + 1];
        s = s + P2[4 * i + 2] * P1[4 * i + 2];
        tr = tr + s;
    }
    float t = (tr - 1.0f) / 2.0f;
    t = t < -1.0f ? -1.0f : (t > 1.0f ? 1.0f : t);
    *angle = acosf(t) * 180.0f / 3.14159265358979323846f;
}
