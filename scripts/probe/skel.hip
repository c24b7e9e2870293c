// Probe: the MFMA + barrier skeleton of the persistent GEMM (8 waves, 2 per SIMD, waves 4-7 one
// barrier behind), operands in registers, no memory traffic -- sections of SEC v_mfma_f32_16x16x32_bf16
// between barrier pairs (SEC = 16: k_gemm256q's four phases per K-tile; 32: two phases; 64: one).
// W32: the same 128 x 64 wave tile and FLOPs per section on v_mfma_f32_32x32x16_bf16 (SEC / 2
// instructions, half the operand elements per FLOP).  Thread 0 of each workgroup stamps
// s_memtime / s_memrealtime around the loop (clock = d(memtime) / d(realtime) x 100 MHz).
#include <hip/hip_runtime.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int SEC, bool BAR, bool W32>
__global__ void __launch_bounds__(512, 1) k_skel(float* out, unsigned long long* stamps, int iters, float seed) {
    const int t = threadIdx.x, wave = t >> 6;
    bf16x8 a[8], b[4];
    // seed > 0: smooth low-entropy operands; seed < 0: hashed pseudo-random values in [-1, 1)
    auto val = [&](unsigned k) -> float {
        if (seed > 0.f) return seed * (float)(k & 1023);
        unsigned h = k * 2654435761u + (unsigned)blockIdx.x * 40503u;
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        return (float)(h & 0xFFFF) / 32768.f - 1.f;
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) for (int e = 0; e < 8; ++e) a[i][e] = (__bf16)val(t * 64 + i * 8 + e);
#pragma unroll
    for (int i = 0; i < 4; ++i) for (int e = 0; e < 8; ++e) b[i][e] = (__bf16)val(100000 + t * 32 + i * 8 + e);
    f32x4 acc[32];
    f32x16 acc2[8];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i)
        for (int e = 0; e < 16; ++e) acc2[i][e] = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (BAR && wave >= 4) __builtin_amdgcn_s_barrier();
    for (int it = 0; it < iters; ++it) {
        // one K-tile = 64 MFMAs per wave (32 on 32x32x16), in 64 / SEC sections
#pragma unroll
        for (int s = 0; s < 64 / SEC; ++s) {
            if (BAR) __builtin_amdgcn_s_barrier();
            if constexpr (W32) {
#pragma unroll
                for (int m = 0; m < SEC / 2; ++m) {
                    const int q = (s * SEC / 2 + m) & 7;
                    acc2[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m & 7], b[(m >> 1) & 3], acc2[q], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int m = 0; m < SEC; ++m) {
                    const int q = (s * SEC + m) & 31;
                    acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[m & 3], a[(m >> 2) & 7], acc[q], 0, 0, 0);
                }
            }
            if (BAR) __builtin_amdgcn_s_barrier();
        }
    }
    if (BAR && wave < 4) __builtin_amdgcn_s_barrier();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    if constexpr (W32) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            for (int e = 0; e < 16; ++e) s += acc2[i][e];
    } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    }
    out[blockIdx.x * 512 + t] = s;
    if (t == 0) {
        volatile unsigned long long* d = stamps + (size_t)blockIdx.x * 2;
        d[0] = t1 - t0;
        d[1] = r1 - r0;
    }
}

extern "C" int skel_launch(int variant, float* out, unsigned long long* stamps, int grid, int iters, float seed,
                           void* stream) {
    hipStream_t st = (hipStream_t)stream;
    switch (variant) {
    case 8: hipLaunchKernelGGL((k_skel<8, true, false>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    case 16: hipLaunchKernelGGL((k_skel<16, true, false>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    case 32: hipLaunchKernelGGL((k_skel<32, true, false>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    case 64: hipLaunchKernelGGL((k_skel<64, true, false>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    case 0: hipLaunchKernelGGL((k_skel<64, false, false>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    case 116: hipLaunchKernelGGL((k_skel<16, true, true>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    case 164: hipLaunchKernelGGL((k_skel<64, true, true>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    case 100: hipLaunchKernelGGL((k_skel<64, false, true>), dim3(grid), dim3(512), 0, st, out, stamps, iters, seed); break;
    default: return -1;
    }
    return (int)hipGetLastError();
}
