// bf_gemm.hip — bf16 MFMA GEMM with fused epilogues for the ViT / CLIP towers (gfx950).
//
//   C[orow(r), n] = (resid ? resid[rrow(r), n] : 0) + act(sum_k A[r,k] * W[n,k] + bias[n])
//     A: bf16 [M,K] (row stride lda), W: bf16 [N,K] (nn.Linear layout, row stride ldw)
//     orow(r) = row_map ? row_map[r] : r   (row_map[r] < 0 drops the row: window un-partition)
//     rrow(r) = resid_mod > 0 ? r % resid_mod : orow(r)   (broadcast tables, e.g. pos-embed)
//     act: 0 none, 1 GELU (erf, nn.GELU default), 2 ReLU;  C is f32 or bf16.
//
// Tiling: 128x128 output tile per 256-thread workgroup (2x2 waves, 64x64 per wave as 2x2
// v_mfma_f32_32x32x16_bf16 tiles), BK = 64, two LDS stages (64 KiB) fed by register staging:
// the next K-tile's global loads are issued before the current tile's MFMAs and written to the
// other LDS stage after them.  LDS rows are 128 B with a 16-B-chunk XOR swizzle (chunk ^ row&7)
// so the 32-row fragment reads (ds_read_b128) spread over the banks.  XCD-aware block order:
// consecutive output tiles of one A row-panel land on the same XCD (shared L2).
#include "bf_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

#define GB_M 128
#define GB_N 128
#define GB_K 64
#define G_THREADS 256

struct alignas(16) U128 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ u16 f2bf(float f) {
    // round-to-nearest-even (NaN stays NaN via the plain cast path)
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<u16*>(&b);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// byte offset of 16-B chunk `c` (0..7) of row `r` in a [rows][64 bf16] swizzled tile
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

template <bool OUT_BF16, int ACT>
__global__ void __launch_bounds__(G_THREADS, 2) k_gemm(const u16* __restrict__ A, int lda,
                                                        const u16* __restrict__ W, int ldw,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ resid, int ldr,
                                                        int resid_mod, void* __restrict__ Cv,
                                                        int ldc, const int32_t* __restrict__ row_map,
                                                        int M, int N, int K, int tiles_n,
                                                        int tiles_m) {
    extern __shared__ __attribute__((aligned(16))) unsigned char g_smem[];
    // stage s: A at s*32K, W at s*32K + 16K
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    // XCD-aware remap of the linear block id (bijective), then row-panel-major tile order
    const int nwg = tiles_m * tiles_n;
    int bid = blockIdx.x;
    {
        const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    }
    const int tm = bid / tiles_n, tn = bid % tiles_n;
    const int m0 = tm * GB_M, n0 = tn * GB_N;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

    // global load assignment: 1024 16-B chunks per operand tile, 4 per thread
    U128 ra0, ra1, ra2, ra3, rw0, rw1, rw2, rw3;
#define G_LOAD1(i, RA, RW, k0)                                                                   \
    {                                                                                            \
        const int ch = t + (i) * G_THREADS, r = ch >> 3, c = ch & 7;                             \
        const int gm = m0 + r, gn = n0 + r, gk = (k0) + c * 8;                                   \
        RA = *reinterpret_cast<const U128*>(A + (size_t)min(gm, M - 1) * lda + gk);              \
        RW = *reinterpret_cast<const U128*>(W + (size_t)min(gn, N - 1) * ldw + gk);              \
        if (gm >= M) RA.x = RA.y = RA.z = RA.w = 0u;                                             \
        if (gn >= N) RW.x = RW.y = RW.z = RW.w = 0u;                                             \
    }
#define G_LOAD(k0)                                                                               \
    G_LOAD1(0, ra0, rw0, k0) G_LOAD1(1, ra1, rw1, k0) G_LOAD1(2, ra2, rw2, k0)                    \
        G_LOAD1(3, ra3, rw3, k0)
#define G_STORE1(i, RA, RW, stage)                                                               \
    {                                                                                            \
        const int ch = t + (i) * G_THREADS, r = ch >> 3, c = ch & 7;                             \
        unsigned char* sa_ = g_smem + (stage) * 32768;                                           \
        *reinterpret_cast<U128*>(sa_ + swz(r, c)) = RA;                                          \
        *reinterpret_cast<U128*>(sa_ + 16384 + swz(r, c)) = RW;                                  \
    }
#define G_STORE(stage)                                                                           \
    G_STORE1(0, ra0, rw0, stage) G_STORE1(1, ra1, rw1, stage) G_STORE1(2, ra2, rw2, stage)        \
        G_STORE1(3, ra3, rw3, stage)

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int nk = K / GB_K;
    G_LOAD(0);
    G_STORE(0);
    __syncthreads();
    const int fr = lane & 31, fh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int st = kt & 1;
        // the prefetch address stays inside the operands on the last step as well (the compiler
        // may issue these loads unconditionally; an offset of K would read past the last row)
        G_LOAD((kt + 1 < nk ? kt + 1 : kt) * GB_K);
        const unsigned char* sa = g_smem + st * 32768;
        const unsigned char* sw = sa + 16384;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {  // 4 x k16 per BK=64
            bf16x8 af[2], bfr[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                int r = wm + i * 32 + fr;
                af[i] = *reinterpret_cast<const bf16x8*>(sa + swz(r, ks * 2 + fh));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                int r = wn + j * 32 + fr;
                bfr[j] = *reinterpret_cast<const bf16x8*>(sw + swz(r, ks * 2 + fh));
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) G_STORE(st ^ 1);
        __syncthreads();
    }

    // epilogue: C/D layout col = lane&31, row = (e&3) + 8*(e>>2) + 4*(lane>>5)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn + j * 32 + fr;
        if (n >= N) continue;
        const float bv = bias ? bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + wm + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
                if (m >= M) continue;
                const int orow = row_map ? row_map[m] : m;
                if (orow < 0) continue;
                float v = acc[i][j][e] + bv;
                if (ACT == 1) v = gelu_erf(v);
                else if (ACT == 2) v = fmaxf(v, 0.f);
                if (resid) {
                    const int rrow = resid_mod > 0 ? (m % resid_mod) : orow;
                    v += resid[(size_t)rrow * ldr + n];
                }
                if (OUT_BF16) reinterpret_cast<u16*>(Cv)[(size_t)orow * ldc + n] = f2bf(v);
                else reinterpret_cast<float*>(Cv)[(size_t)orow * ldc + n] = v;
            }
        }
    }
}

BF_API int bf_gemm_bf16(const void* A, int lda, const void* W, int ldw, const float* bias,
                        const float* resid, int ldr, int resid_mod, void* C, int ldc, int c_bf16,
                        const int32_t* row_map, int M, int N, int K, int act, void* stream) {
    if (!A || !W || !C || M < 0 || N <= 0 || K <= 0) return BF_ERR_ARG;
    if (K % GB_K != 0 || lda % 8 != 0 || ldw % 8 != 0) return BF_ERR_UNSUPPORTED;
    if (M == 0) return BF_OK;
    const int tiles_m = (M + GB_M - 1) / GB_M, tiles_n = (N + GB_N - 1) / GB_N;
    const int nwg = tiles_m * tiles_n;
    const size_t lds = 2 * 32768;
    if (act < 0 || act > 2) return BF_ERR_ARG;
#define GEMM_LAUNCH(OB, AC)                                                                       \
    hipLaunchKernelGGL((k_gemm<OB, AC>), dim3(nwg), dim3(G_THREADS), lds, bf_stream(stream),       \
                       (const u16*)A, lda, (const u16*)W, ldw, bias, resid, ldr, resid_mod, C, ldc, \
                       row_map, M, N, K, tiles_n, tiles_m)
    if (c_bf16) {
        if (act == 0) GEMM_LAUNCH(true, 0);
        else if (act == 1) GEMM_LAUNCH(true, 1);
        else GEMM_LAUNCH(true, 2);
    } else {
        if (act == 0) GEMM_LAUNCH(false, 0);
        else if (act == 1) GEMM_LAUNCH(false, 1);
        else GEMM_LAUNCH(false, 2);
    }
#undef GEMM_LAUNCH
    return bf_check_launch();
}
