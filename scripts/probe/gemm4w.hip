#include "/root/repo/boxfusion_amd/csrc/bf_common.h"
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
#define W4_STAGE 32768
#define W4_LDS (4 * W4_STAGE)
#ifndef W4_PIPE
#define W4_PIPE 1
#endif
#ifndef W4_NA
#define W4_NA 32
#endif
#ifndef NBJ
#define NBJ 8
#endif
__device__ __forceinline__ void w4_glds(const void* base, int nbytes, void* lds, int vo, int so) {
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nbytes, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, vo, so, 0, 0);
}
__device__ __forceinline__ uint32_t w4_pk(float a, float b) {
    typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2v));
}
__device__ __forceinline__ void mfma_a(f32x4& acc, const bf16x8& b, const bf16x8& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
template <bool OUT_BF16>
__global__ void __launch_bounds__(256, 1) k_gemm4w(const u16* __restrict__ A, int lda, const u16* __restrict__ W,
                                                   int ldw, const float* __restrict__ bias, void* __restrict__ Cv,
                                                   int ldc, int M, int N, int K, int tiles_m, int tiles_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int wm = wave >> 1, wn = wave & 1;
    const int lr = lane & 15, lq = lane >> 4;
    const int nwg = tiles_m * tiles_n;
    int bid = blockIdx.x;
    { const int xcd = bid % 8, q = nwg / 8, r = nwg % 8; bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8; }
    int tm, tn;
    { const int gm = 8, per = gm * tiles_n, grp = bid / per, in = bid - grp * per; const int rows = min(gm, tiles_m - grp * gm); tm = grp * gm + in % rows; tn = in / rows; }
    const int m0 = tm * 256, n0 = tn * (32 * NBJ);
    const int srow = lane >> 2, sq = (lane >> 4) & 3;
    const int schunk = (lane & 3) ^ (sq == 0 ? 0 : sq == 1 ? 2 : sq == 2 ? 3 : 1);
    int voa[4], vow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 64 * wave + 16 * i + srow;
        voa[i] = min(m0 + r, M - 1) * lda * 2 + schunk * 16;
        vow[i] = (r < 32 * NBJ) ? min(n0 + r, N - 1) * ldw * 2 + schunk * 16 : (int)0x80000000;
    }
    const int bytesA = (int)(((size_t)(M - 1) * lda + K) * 2);
    const int bytesW = (int)(((size_t)(N - 1) * ldw + K) * 2);
    const int nk = K / 32;
    auto stage = [&](int kt) {
        unsigned char* s = smem + (kt & 3) * W4_STAGE + wave_u * 4096;
        const int so = kt < nk ? kt * 64 : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            w4_glds(A, bytesA, s + i * 1024, kt < nk ? voa[i] : (int)0x80000000, so);
            w4_glds(W, bytesW, s + 16384 + i * 1024, kt < nk ? vow[i] : (int)0x80000000, so);
        }
    };
    const int rslot = lq ^ ((lr >> 2) == 0 ? 0 : (lr >> 2) == 1 ? 2 : (lr >> 2) == 2 ? 3 : 1);
    bf16x8 fa[2][8], fb[2][NBJ];
#define W4_READ(SET, KT) { const unsigned char* s_ = smem + ((KT) & 3) * W4_STAGE; \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) fa[SET][i] = *reinterpret_cast<const bf16x8*>(s_ + (128 * wm + 16 * i + lr) * 64 + rslot * 16); \
        _Pragma("unroll") for (int j = 0; j < NBJ; ++j) fb[SET][j] = *reinterpret_cast<const bf16x8*>(s_ + 16384 + ((16 * NBJ) * wn + 16 * j + lr) * 64 + rslot * 16); }
    f32x4 acc[8][NBJ];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NBJ; ++j) { acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f}; asm volatile("" : "+a"(acc[i][j])); }
#define W4_MFMA(SET) { _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int j = 0; j < NBJ; ++j) mfma_a(acc[i][j], fb[SET][j], fa[SET][i]); }
#if W4_PIPE != 2
    stage(0); stage(1); stage(2); stage(3);
    asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    __syncthreads();
    W4_READ(0, 0);
#endif
#if W4_PIPE == 2
    // register staging: global_load_dwordx4 into VGPRs one K-tile ahead, ds_write_b128 into a 2-slot
    // ring (the LDS image of the DMA form); part B MFMAs straddle the barrier as in W4_PIPE 1
    typedef unsigned u32x4r __attribute__((ext_vector_type(4)));
    u32x4r stg[8];
    auto gload = [&](int kt) {
        if (kt < nk) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                stg[i] = *reinterpret_cast<const u32x4r*>(reinterpret_cast<const unsigned char*>(A) + voa[i] + kt * 64);
                stg[4 + i] = *reinterpret_cast<const u32x4r*>(reinterpret_cast<const unsigned char*>(W) + vow[i] + kt * 64);
            }
        }
    };
    auto swrite = [&](int kt) {
        unsigned char* s_ = smem + (kt & 1) * W4_STAGE + wave_u * 4096 + lane * 16;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            *reinterpret_cast<u32x4r*>(s_ + i * 1024) = stg[i];
            *reinterpret_cast<u32x4r*>(s_ + 16384 + i * 1024) = stg[4 + i];
        }
    };
    auto mf = [&](int set, int idx) { mfma_a(acc[idx / NBJ][idx % NBJ], fb[set][idx % NBJ], fa[set][idx / NBJ]); };
    gload(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    swrite(0);
    gload(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    W4_READ(0, 0);
    for (int g = 0; g < nk; g += 2) {
#define W4_RITER(CUR, G) { \
            _Pragma("unroll") for (int x = 0; x < W4_NA; ++x) mf(CUR, x); \
            if ((G) + 1 < nk) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); swrite((G) + 1); } \
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); \
            gload((G) + 2); \
            { const unsigned char* r_ = smem + (((G) + 1) & 1) * W4_STAGE; \
              _Pragma("unroll") for (int x = 0; x < 8 * NBJ - W4_NA; ++x) { \
                  if (x < 8) fa[(CUR) ^ 1][x] = *reinterpret_cast<const bf16x8*>(r_ + (128 * wm + 16 * x + lr) * 64 + rslot * 16); \
                  else if (x < 8 + NBJ) fb[(CUR) ^ 1][x - 8] = *reinterpret_cast<const bf16x8*>(r_ + 16384 + ((16 * NBJ) * wn + 16 * (x - 8) + lr) * 64 + rslot * 16); \
                  mf(CUR, W4_NA + x); asm volatile("" ::: "memory"); } } }
        W4_RITER(0, g);
        W4_RITER(1, g + 1);
#undef W4_RITER
    }
#elif W4_PIPE
    // part A: MFMAs 0 .. NA-1 of the current set; barrier; then the next K-tile's DMA and fragment
    // reads interleaved one for one with MFMAs NA .. 8*NBJ-1 of the current set
    auto mf = [&](int set, int idx) { mfma_a(acc[idx / NBJ][idx % NBJ], fb[set][idx % NBJ], fa[set][idx / NBJ]); };
    for (int g = 0; g < nk; g += 2) {
#define W4_PITER(CUR, G) { \
            _Pragma("unroll") for (int x = 0; x < W4_NA; ++x) mf(CUR, x); \
            asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); \
            { unsigned char* s_ = smem + (((G) + 4) & 3) * W4_STAGE + wave_u * 4096; const int kt_ = (G) + 4; const int so_ = kt_ < nk ? kt_ * 64 : 0; \
              const unsigned char* r_ = smem + (((G) + 1) & 3) * W4_STAGE; \
              _Pragma("unroll") for (int x = 0; x < 8 * NBJ - W4_NA; ++x) { \
                  if (x < 8 && (x & 1) == 0) w4_glds(A, bytesA, s_ + (x >> 1) * 1024, kt_ < nk ? voa[x >> 1] : (int)0x80000000, so_); \
                  if (x < 8 && (x & 1) == 1) w4_glds(W, bytesW, s_ + 16384 + (x >> 1) * 1024, kt_ < nk ? vow[x >> 1] : (int)0x80000000, so_); \
                  if (x < 8) fa[(CUR) ^ 1][x] = *reinterpret_cast<const bf16x8*>(r_ + (128 * wm + 16 * x + lr) * 64 + rslot * 16); \
                  else if (x < 8 + NBJ) fb[(CUR) ^ 1][x - 8] = *reinterpret_cast<const bf16x8*>(r_ + 16384 + ((16 * NBJ) * wn + 16 * (x - 8) + lr) * 64 + rslot * 16); \
                  mf(CUR, W4_NA + x); asm volatile("" ::: "memory"); } } }
        W4_PITER(0, g);
        W4_PITER(1, g + 1);
#undef W4_PITER
    }
#else
    for (int g = 0; g < nk; g += 2) {
#define W4_ITER(CUR, G) { asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); \
            stage((G) + 4); W4_READ((CUR) ^ 1, (G) + 1); W4_MFMA(CUR); }
        W4_ITER(0, g);
        W4_ITER(1, g + 1);
#undef W4_ITER
    }
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = m0 + 128 * wm + 16 * i + lr;
#pragma unroll
        for (int j = 0; j < NBJ; ++j) {
            const int c = n0 + (16 * NBJ) * wn + 16 * j + 4 * lq;
            f32x4 x = acc[i][j];
            if (r >= M || c >= N) continue;
            if (bias) { x.x += bias[c]; x.y += bias[c + 1]; x.z += bias[c + 2]; x.w += bias[c + 3]; }
            if (OUT_BF16) *reinterpret_cast<u32x2v*>(reinterpret_cast<u16*>(Cv) + (size_t)r * ldc + c) = (u32x2v){w4_pk(x.x, x.y), w4_pk(x.z, x.w)};
            else *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cv) + (size_t)r * ldc + c) = x;
        }
    }
}


extern "C" int gemm4w_launch(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                             void* stream) {
    if (K % 64 || N % (32 * NBJ)) return -1;
    const int tm = (M + 255) / 256, tn = N / (32 * NBJ);
    static bool init = false;
    if (!init) {
        hipFuncSetAttribute((const void*)k_gemm4w<true>, hipFuncAttributeMaxDynamicSharedMemorySize, W4_LDS);
        init = true;
    }
    hipLaunchKernelGGL(k_gemm4w<true>, dim3(tm * tn), dim3(256), W4_LDS, (hipStream_t)stream, (const u16*)A, lda,
                       (const u16*)W, ldw, (const float*)nullptr, C, ldc, M, N, K, tm, tn);
    return (int)hipGetLastError();
}
