// bf_gemm.hip — bf16 MFMA GEMM with fused epilogues for the ViT / CLIP towers (gfx950).
//
//   C[orow(r), n] = (resid ? resid[rrow(r), n] : 0) + act(sum_k A[r,k] * W[n,k] + bias[n])
//     A: bf16 [M,K] (row stride lda), W: bf16 [N,K] (nn.Linear layout, row stride ldw)
//     orow(r) = row_map ? row_map[r] : r   (row_map[r] < 0 drops the row: window un-partition)
//     rrow(r) = resid_mod > 0 ? r % resid_mod : orow(r)   (broadcast tables, e.g. pos-embed)
//     act: 0 none, 1 GELU (erf, nn.GELU default), 2 ReLU;  C is f32 or bf16.
//
// Tiling: 128x128 output tile per 256-thread workgroup (2x2 waves, 64x64 per wave as 2x2
// v_mfma_f32_32x32x16_bf16 tiles), BK = 64, two LDS stages (64 KiB) filled by direct-to-LDS
// loads (global_load_lds_dwordx4): the next K-tile is issued before the current tile's MFMAs,
// one vmcnt(0) + barrier per K-tile.  LDS rows are 128 B with a 16-B-chunk XOR swizzle
// (chunk ^ row&7, applied on the source address) so the 32-row fragment reads (ds_read_b128)
// spread over the banks.  XCD-aware block order: consecutive output tiles of one A row-panel
// land on the same XCD (shared L2).
#include "bf_common.h"

#include <mutex>
#include <set>
#include <string>

// wave priority in the K loop: 0 = raise to 1 around every MFMA quadrant (default), 1 = waves 4-7
// at priority 1 for the whole walk (MI355X_MICROARCH "static priority for the younger half"),
// 2 = never raised
#ifndef GEMM_PRIO_MODE
#define GEMM_PRIO_MODE 0
#endif

// gemm_tile_mb1's cost model: a tile of BM rows takes (GEMM_TILE_FIXED + (1 - GEMM_TILE_FIXED) BM / 256)
// of a 256-row tile's time.  The K loop has a per-K-tile cost that does not shrink with the MFMA
// count (staging, fragment reads, barriers: scripts/gemm_tile_sweep.py, CuTR 12800 x 768 x 3072 in
// one round: 160 rows 78.7 us vs 256 rows 82.6; scripts/gemm_l2_probe.py: L2-resident operands
// take 5-21 % off), so a smaller tile pays only where it saves a round.
#ifndef GEMM_TILE_FIXED
#define GEMM_TILE_FIXED 0.7
#endif

// k_gemm256p accumulator layout: 0 (default) = D[m][n] blocks; 1 = transposed (C^T = W A^T on the
// MFMA: 16-B residual loads, one ds_write_b128 per block in the epilogue, bias + activation after
// the LDS transpose).  Both pass the same tests; measured on one box the transposed form was no
// faster (CLIP proj 167.6 vs 165.0 us, bench 130.1 vs 131.2 frames/s): the residual's cost is the
// lock-step burst at tile boundaries, not the load instruction count.  Kept as a variant.
#ifndef GEMM_TACC
#define GEMM_TACC 0
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
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

// nn.GELU (erf form).  erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16
// output rounding): one v_rcp, one v_exp and a handful of FMAs instead of the library erff.
// With z = x/sqrt(2) and erf(|z|) = 1 - P(t) e^{-z^2}:
//   GELU(x) = relu(x) - 0.5 |x| P(t) e^{-x^2/2},   t = 1 / (1 + p |x| / sqrt(2))
// (constants folded; no 1 - (1 - small) cancellation for negative x).
__device__ __forceinline__ float gelu_erf(float x) {
    const float a = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, a, 1.0f));
    float p = fmaf(0.5f * 1.061405429f, t, 0.5f * -1.453152027f);
    p = fmaf(p, t, 0.5f * 1.421413741f);
    p = fmaf(p, t, 0.5f * -0.284496736f);
    p = fmaf(p, t, 0.5f * 0.254829592f);
    const float e = __builtin_amdgcn_exp2f(a * -0.72134752044448170f * a);
    return fmaxf(x, 0.f) - a * (p * t) * e;
}

// the same GELU on two values with packed f32 VALU ops (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32
// on gfx950), rearranged: with z = x/sqrt(2) and erf(|z|) = 1 - P(t) e^{-z^2} (A&S 7.1.26),
//   GELU(x) = 0.5 x (1 + erf(z)) = relu(x) - 0.5 |x| P(t) e^{-x^2/2},   t = 1 / (1 + p |x| / sqrt(2))
// (the 1/sqrt(2), the 0.5 and log2(e) folded into the constants).  18 VALU + 4 transcendental
// instructions per pair instead of 22 + 4, and no 1 - (1 - small) cancellation for negative x.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
    const f32x2 ax = __builtin_elementwise_abs(x);
    const f32x2 d = (0.3275911f * 0.70710678118654752f) * ax + 1.0f;
    f32x2 tt;
    tt.x = __builtin_amdgcn_rcpf(d.x);
    tt.y = __builtin_amdgcn_rcpf(d.y);
    f32x2 p = (0.5f * 1.061405429f) * tt + (0.5f * -1.453152027f);     // 0.5 P(t) / t
    p = p * tt + (0.5f * 1.421413741f);
    p = p * tt + (0.5f * -0.284496736f);
    p = p * tt + (0.5f * 0.254829592f);
    const f32x2 q = (ax * -0.72134752044448170f) * ax;                 // -x^2/2 * log2(e)
    f32x2 ex;
    ex.x = __builtin_amdgcn_exp2f(q.x);
    ex.y = __builtin_amdgcn_exp2f(q.y);
    const f32x2 m = ax * (p * tt) * ex;
    f32x2 r;
    r.x = fmaxf(x.x, 0.f);
    r.y = fmaxf(x.y, 0.f);
    return r - m;
}

// two packed pairs at once: the four v_rcp and the four v_exp issue back to back, so their
// results are not consumed right behind them (fewer trans-use hazard wait states)
__device__ __forceinline__ void gelu_erf2x2(f32x2& x0, f32x2& x1) {
    const f32x2 a0 = __builtin_elementwise_abs(x0), a1 = __builtin_elementwise_abs(x1);
    const f32x2 d0 = (0.3275911f * 0.70710678118654752f) * a0 + 1.0f;
    const f32x2 d1 = (0.3275911f * 0.70710678118654752f) * a1 + 1.0f;
    const f32x2 q0 = (a0 * -0.72134752044448170f) * a0;
    const f32x2 q1 = (a1 * -0.72134752044448170f) * a1;
    f32x2 t0, t1, e0, e1;
    t0.x = __builtin_amdgcn_rcpf(d0.x); t0.y = __builtin_amdgcn_rcpf(d0.y);
    t1.x = __builtin_amdgcn_rcpf(d1.x); t1.y = __builtin_amdgcn_rcpf(d1.y);
    e0.x = __builtin_amdgcn_exp2f(q0.x); e0.y = __builtin_amdgcn_exp2f(q0.y);
    e1.x = __builtin_amdgcn_exp2f(q1.x); e1.y = __builtin_amdgcn_exp2f(q1.y);
    f32x2 p0 = (0.5f * 1.061405429f) * t0 + (0.5f * -1.453152027f);
    f32x2 p1 = (0.5f * 1.061405429f) * t1 + (0.5f * -1.453152027f);
    p0 = p0 * t0 + (0.5f * 1.421413741f);      p1 = p1 * t1 + (0.5f * 1.421413741f);
    p0 = p0 * t0 + (0.5f * -0.284496736f);     p1 = p1 * t1 + (0.5f * -0.284496736f);
    p0 = p0 * t0 + (0.5f * 0.254829592f);      p1 = p1 * t1 + (0.5f * 0.254829592f);
    const f32x2 m0 = a0 * (p0 * t0) * e0, m1 = a1 * (p1 * t1) * e1;
    f32x2 r0, r1;
    r0.x = fmaxf(x0.x, 0.f); r0.y = fmaxf(x0.y, 0.f);
    r1.x = fmaxf(x1.x, 0.f); r1.y = fmaxf(x1.y, 0.f);
    x0 = r0 - m0;
    x1 = r1 - m1;
}

// byte offset of 16-B chunk `c` (0..7) of row `r` in a [rows][64 bf16] swizzled tile
// Two 128-B tile rows share one 256-B LDS bank row, so the XOR key is (r >> 1) & 7: the 16 rows
// of every ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) then hit 16
// distinct 16-B slots (conflict-free; the key r & 7 left them 2-way).
__device__ __forceinline__ int swz_key(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ swz_key(r)) << 4); }

template <bool OUT_BF16, int ACT>
__global__ void __launch_bounds__(G_THREADS, 2) k_gemm(const u16* __restrict__ A, int lda,
                                                        const u16* __restrict__ W, int ldw,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ resid, int ldr,
                                                        int resid_mod, void* __restrict__ Cv,
                                                        int ldc, const int32_t* __restrict__ row_map,
                                                        int M, int N, int K, int tiles_n,
                                                        int tiles_m, int vec_epi) {
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

    // Direct-to-LDS staging (global_load_lds_dwordx4): one wave-instruction fills 1 KiB = 8 tile
    // rows of 128 B at a wave-uniform LDS base, lane l at +16*l.  The XOR swizzle therefore moves
    // to the per-lane SOURCE address: lane l of the instruction covering rows 8q..8q+7 writes
    // physical chunk p = l&7 of row r = 8q + (l>>3), which must hold logical chunk p ^ key(r).
    // Each wave issues 4 instructions per operand per K-tile (16 KiB per operand per stage).
    // Rows past M / N are clamped to the last row (valid addresses; those outputs are not stored).
    const u16* ga[4];
    const u16* gw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (wave * 4 + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swz_key(r);
        ga[i] = A + (size_t)min(m0 + r, M - 1) * lda + c * 8;
        gw[i] = W + (size_t)min(n0 + r, N - 1) * ldw + c * 8;
    }
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
#define G_STAGE(stage, k0)                                                                       \
    {                                                                                            \
        unsigned char* sa_ = g_smem + (stage) * 32768 + wave * 4096;                             \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                          \
            __builtin_amdgcn_global_load_lds((const void*)(ga[i] + (k0)),                        \
                                             (lds_ptr_t)(sa_ + i * 1024), 16, 0, 0);             \
            __builtin_amdgcn_global_load_lds((const void*)(gw[i] + (k0)),                        \
                                             (lds_ptr_t)(sa_ + 16384 + i * 1024), 16, 0, 0);     \
        }                                                                                        \
    }

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int nk = K / GB_K;
    G_STAGE(0, 0);
    __builtin_amdgcn_s_waitcnt(0);     // vmcnt(0): the first tile has landed in LDS
    __syncthreads();
    const int fr = lane & 31, fh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int st = kt & 1;
        // prefetch the next K-tile into the other stage (its last readers passed the barrier
        // that ended the previous iteration)
        if (kt + 1 < nk) G_STAGE(st ^ 1, (kt + 1) * GB_K);
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
        // the LDS-DMA of the next tile is a pending VM op: retire it, then one barrier makes it
        // visible to every wave and ends all reads of this stage
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
#undef G_STAGE

    // ---- epilogue ----------------------------------------------------------------------------
    // C/D layout: col = lane&31, row = (e&3) + 8*(e>>2) + 4*(lane>>5).  Every lane holds columns,
    // so the tile is transposed through LDS (free after the K loop) and written row-wise in 16-B
    // chunks: coalesced stores and coalesced residual reads.  bias + activation are applied
    // before the transpose, the residual after it.
    if (vec_epi) {
        float* T = reinterpret_cast<float*>(g_smem);   // [128][128] f32, column XOR-swizzled
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int nl = wn + j * 32 + fr;
            const float bv = (bias && n0 + nl < N) ? bias[min(n0 + nl, N - 1)] : 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int ml = wm + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
                    float v = acc[i][j][e] + bv;
                    if (ACT == 1) v = gelu_erf(v);
                    else if (ACT == 2) v = fmaxf(v, 0.f);
                    T[ml * 128 + (nl ^ (((ml >> 2) & 1) << 5))] = v;   // rows r, r+4: other banks
                }
        }
        __syncthreads();
        constexpr int CW = OUT_BF16 ? 8 : 4;            // output elements per 16-B chunk
        constexpr int CPR = 128 / CW;                   // chunks per tile row
#pragma unroll 4
        for (int id = t; id < 128 * CPR; id += G_THREADS) {
            const int ml = id / CPR, cl = (id % CPR) * CW;
            const int m = m0 + ml, n = n0 + cl;
            if (m >= M || n >= N) continue;
            const int orow = row_map ? row_map[m] : m;
            if (orow < 0) continue;
            const int sw = ((ml >> 2) & 1) << 5;
            float v[CW];
#pragma unroll
            for (int q = 0; q < CW; q += 4) {
                const float4 x = *reinterpret_cast<const float4*>(T + ml * 128 + ((cl + q) ^ sw));
                v[q] = x.x; v[q + 1] = x.y; v[q + 2] = x.z; v[q + 3] = x.w;
            }
            if (resid) {
                const int rrow = resid_mod > 0 ? (m % resid_mod) : orow;
                const float* rp = resid + (size_t)rrow * ldr + n;
#pragma unroll
                for (int q = 0; q < CW; q += 4) {
                    const float4 x = *reinterpret_cast<const float4*>(rp + q);
                    v[q] += x.x; v[q + 1] += x.y; v[q + 2] += x.z; v[q + 3] += x.w;
                }
            }
            if (OUT_BF16) {
                U128 o;
                o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
                o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
                o.z = (uint32_t)f2bf(v[4 % CW]) | ((uint32_t)f2bf(v[5 % CW]) << 16);
                o.w = (uint32_t)f2bf(v[6 % CW]) | ((uint32_t)f2bf(v[7 % CW]) << 16);
                *reinterpret_cast<U128*>(reinterpret_cast<u16*>(Cv) + (size_t)orow * ldc + n) = o;
            } else {
                *reinterpret_cast<float4*>(reinterpret_cast<float*>(Cv) + (size_t)orow * ldc + n) =
                    make_float4(v[0], v[1], v[2], v[3]);
            }
        }
        return;
    }
    // scalar fallback (unaligned / ragged N): one element per register
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn + j * 32 + fr;
        if (n >= N) continue;
        const float bv = bias ? bias[min(n, N - 1)] : 0.f;
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

// ------------------------------------------------------------------------------------------
// Persistent 256x256 kernel: one 512-thread workgroup per CU walks its tiles (round r gives block
// b the tile r*grid + xcd_slot(b), so 32 consecutive tiles -- one A row panel -- share an XCD's
// L2).  Per tile: 8 waves (2 M x 4 N), 128x64 per wave = 4x2 v_mfma_f32_32x32x16_bf16 tiles,
// BK = 64.  The K-tile ring runs ACROSS tiles: two 64-KiB LDS stages filled by global_load_lds,
// K-tile g+2 (possibly of the next tile) issued into stage g&1 once every wave has read it;
// fragments software-pipelined one k-step ahead (register sets FA/FB); one raw s_barrier per
// K-tile.  The epilogue is wave-private (each wave transposes its 128x64 sub-tile 16 rows at a
// time through its own 4-KiB slice of the remaining 32 KiB of LDS, no block barrier) and runs
// while the next tile's first two K-tiles are in flight; its global stores drain under the next
// tile's MFMAs.
// ------------------------------------------------------------------------------------------
#define G2_THREADS 512
#define G2_STAGES_BYTES (2 * 65536)
#define G2_LDS (G2_STAGES_BYTES + 8 * 4096)
#define CBAR() asm volatile("" ::: "memory")
#define RAW_BARRIER() do { CBAR(); __builtin_amdgcn_s_barrier(); CBAR(); } while (0)

// 16-B LDS-DMA through a buffer descriptor: byte offset `vo` (per lane) + `so` (wave-uniform)
// from `base` (`nbytes` readable), written at the wave-uniform LDS address `lds` + 16*lane.
__device__ __forceinline__ void glds_buf16(const void* base, int nbytes, void* lds, int vo, int so) {
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nbytes, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, vo, so, 0, 0);
}

// Grouped tile order of the persistent kernels: the linear tile index walks column-major inside
// groups of `gm` row panels, so the 32 tiles an XCD runs concurrently (consecutive indices) form a
// gm x (32/gm) patch -- gm A panels and 32/gm W panels per K-step in that XCD's L2 instead of
// ~1.6 A panels and every W panel of the problem.  gm <= 1: plain row-major order.
__device__ __forceinline__ void tile_coords(int tile, int tiles_m, int tiles_n, int gm, int& m0, int& n0,
                                            int bm = 256) {
    if (gm <= 1) { m0 = (tile / tiles_n) * bm; n0 = (tile % tiles_n) * 256; return; }
    const int per = gm * tiles_n;
    const int grp = tile / per, in = tile - grp * per;
    const int rows = min(gm, tiles_m - grp * gm);
    m0 = (grp * gm + in % rows) * bm;
    n0 = (in / rows) * 256;
}

// ------------------------------------------------------------------------------------------
// Persistent 256x256 kernel, staggered 4-phase schedule (k_gemm256p).
//
// 256x256 tiles, 8 waves (2 M x 4 N, 128x64 per wave, v_mfma_f32_16x16x32_bf16), a persistent
// K-tile walk (the first form, one MFMA block per K-tile, is in the git history); every K-tile (BK = 64) runs as 4 phases, one output quadrant (64x32) of
// the wave each:  P1 (0,0)  P2 (0,1)  P3 (1,1)  P4 (1,0).  A phase = memory section (fragment
// reads + one half-tile of LDS-DMA staging) | s_barrier | 16 MFMAs | s_barrier.  Waves 4-7 run one
// barrier behind waves 0-3, so on every SIMD one wave's memory section overlaps its partner's
// MFMAs.
//
// LDS stage (64 KiB) = four 16-KiB half-tiles: A-half h holds the rows {wr*128 + h*64 + [0,64)},
// B-half h the columns {wc*64 + h*32 + [0,32)} of all waves, so quadrant (mi, ni) reads exactly
// A-half mi and B-half ni.  Reads:  P1 B0 then A0 (the 4 B0 reads retired before the barrier),
// P2 B1 (retired before the barrier), P3 A1, P4 none (A1 and B0 still in registers).  Each half is
// restaged (for K-tile g+2, same stage) one phase after its reads were retired, two after
// otherwise:  P2 B0, P3 A0, P4 B1, next P1 A1.  One counted wait per K-tile, vmcnt(6) in P4 before
// its first barrier, retires K-tile g+1 with three half-tiles (6 LDS-DMA) still in flight; the
// staggered half's readers are covered because every read sits one phase after that wait.
// ------------------------------------------------------------------------------------------
#define SB0() __builtin_amdgcn_sched_barrier(0)
#define PHASE_BARRIER() do { SB0(); CBAR(); __builtin_amdgcn_s_barrier(); CBAR(); SB0(); } while (0)

// k_gemm256p output stores and residual loads, optionally nontemporal (streamed past L2 so the
// bursts at tile boundaries do not evict the operand panels).  GEMM_NT bits: 1 = bf16 output
// stores, 2 = f32 output stores, 4 = residual loads.  Default 3 (measured on one box, same run:
// CLIP fc1 546.8 -> 524.2 us, qkv 295.4 -> 286.5, proj 164.9 -> 151.3, fc2 439.7 -> 429.4, CuTR
// fc1 164.8 -> 155.3; bench 132.4-132.6 -> 133.6-133.8 frames/s).  Nontemporal residual loads
// (bit 4) were slower on the residual GEMMs (CuTR global proj 39.5 -> 47.9 us).
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
#ifndef GEMM_NT
#define GEMM_NT 3
#endif
#if GEMM_NT & 4
#define GEMM_LD_F(p) __builtin_nontemporal_load(p)
#define GEMM_LD_F4(p) __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(p))
#else
#define GEMM_LD_F(p) (*(p))
#define GEMM_LD_F4(p) (*reinterpret_cast<const f32x4v*>(p))
#endif
#if GEMM_NT & 2
#define GEMM_ST_F4(p, a, b, c, d) __builtin_nontemporal_store((f32x4v){a, b, c, d}, reinterpret_cast<f32x4v*>(p))
#else
#define GEMM_ST_F4(p, a, b, c, d) (*reinterpret_cast<f32x4v*>(p) = (f32x4v){a, b, c, d})
#endif
#if GEMM_NT & 1
#define GEMM_ST_U4(p, o) __builtin_nontemporal_store((u32x4v){(o).x, (o).y, (o).z, (o).w}, reinterpret_cast<u32x4v*>(p))
#else
#define GEMM_ST_U4(p, o) (*reinterpret_cast<U128*>(p) = (o))
#endif
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
#if GEMM_NT & 1
#define GEMM_ST_U2(p, a, b) __builtin_nontemporal_store((u32x2v){(unsigned)(a), (unsigned)(b)}, reinterpret_cast<u32x2v*>(p))
#else
#define GEMM_ST_U2(p, a, b) (*reinterpret_cast<u32x2v*>(p) = (u32x2v){(unsigned)(a), (unsigned)(b)})
#endif
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
// one 32-B fp8 MFMA fragment from two 16-B LDS reads
__device__ __forceinline__ i32x8 frag32(bf16x8 a, bf16x8 b) {
    return __builtin_shufflevector(__builtin_bit_cast(i32x4, a), __builtin_bit_cast(i32x4, b), 0, 1, 2, 3, 4, 5, 6, 7);
}

// F8 (bit 0): A and W are fp8 e4m3 (OCP) with BK = 128 elements per K-tile (the same 128-B LDS rows),
// on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales (E8M0 127): twice
// the bf16 MFMA rate.  The epilogue then computes acc * csc + bias[n] (csc = activation scale x
// weight scale, both per tensor: a scalar, no extra VGPRs beside the 246-255 the kernel already
// holds); an in-place residual initialises the accumulators with resid / csc.  F8 bit 1: fp8 output, v * oqs clamped to +-448 (OUT_BF16 must be set: 8
// columns per lane, one 8-B store).  The fp8 lane fragment is the bf16 kernel's two k-step
// fragments (16-B chunks lq and 4+lq of the 128-B row): the MFMA's k order inside a fragment only
// has to agree between A and B, and the bf16 chunk pattern keeps the LDS reads conflict-free.
template <bool OUT_BF16, int ACT, int F8 = 0>
__global__ void __launch_bounds__(G2_THREADS, 1) k_gemm256p(const u16* __restrict__ A, int lda,
                                                            const u16* __restrict__ W, int ldw,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ resid, int ldr,
                                                            int resid_mod, void* __restrict__ Cv,
                                                            int ldc, const int32_t* __restrict__ row_map,
                                                            int M, int N, int K, int tiles_n,
                                                            int tiles_m, int stagger, int gm, int ablate,
                                                            float csc = 1.f, float oqs = 1.f) {
    extern __shared__ __attribute__((aligned(16))) unsigned char g_smem[];
#if GEMM_TACC
    static_assert(F8 == 0, "fp8 operands use the default accumulator layout");
#endif
    static_assert(!(F8 & 2) || OUT_BF16, "fp8 output takes the 8-column store path");
    constexpr int ESZ = (F8 & 1) ? 1 : 2;           // operand bytes
    constexpr int KTE = GB_K * 2 / ESZ;             // K elements per 128-B K-tile row
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int lr = lane & 15, lq = lane >> 4;
    const int ntiles = tiles_m * tiles_n;
    const int G = gridDim.x;
    const int slot = (G % 8 == 0) ? ((int)blockIdx.x % 8) * (G / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int my_tiles = ntiles > slot ? (ntiles - slot + G - 1) / G : 0;
    const int nk = K / KTE;
    const int total = my_tiles * nk;
    if (total == 0) return;

    // half-tile staging: wave w, instruction i fills local rows (2w+i)*8 + lane/8 of a half.
    // Buffer loads (LDS-DMA form): per-lane 32-bit byte offsets of the rows, computed once per
    // output tile; the K position is the scalar soffset.
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    int a_row[2][2], b_row[2][2], scol[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int L = (wave * 2 + i) * 8 + (lane >> 3);
        scol[i] = ((lane & 7) ^ swz_key(L)) * 16;                 // bytes
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            a_row[h][i] = (L >> 6) * 128 + h * 64 + (L & 63);     // tile row of A-half h
            b_row[h][i] = (L >> 5) * 64 + h * 32 + (L & 31);      // tile column of B-half h
        }
    }
    const int bytesA = (int)(((size_t)(M - 1) * lda + K) * ESZ);  // < 2^31 (checked on the host)
    const int bytesW = (int)(((size_t)(N - 1) * ldw + K) * ESZ);
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    // K-tile coordinates of the walk, advanced incrementally (a division only at tile boundaries);
    // past the end of the walk the last K-tile is repeated (same bytes into the same stage)
    struct KT { int idx, m0, n0, k0, buf; };
    auto kt_at_tile = [&](int tile_k, int idx) {
        const int tile = slot + tile_k * G;
        KT r;
        r.idx = idx; tile_coords(tile, tiles_m, tiles_n, gm, r.m0, r.n0); r.k0 = 0; r.buf = idx & 1;
        return r;
    };
    int tile_ord = 0;       // tile ordinal (within this block's walk) of the newest KT built
    auto kt_next = [&](KT c) {
        if (c.idx >= total - 1) return c;
        if (c.k0 + KTE < K) { c.k0 += KTE; c.idx += 1; c.buf ^= 1; return c; }
        ++tile_ord;
        return kt_at_tile(tile_ord, c.idx + 1);
    };
    // per-lane row byte offsets of a K-tile's tile ([0..1] A-half h row i, [2..3] B-half)
    struct VO { int a[2][2], b[2][2]; };
    auto vo_of = [&](const KT& c) {
        VO v;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                v.a[h][i] = min(c.m0 + a_row[h][i], M - 1) * lda * ESZ + scol[i];
                v.b[h][i] = min(c.n0 + b_row[h][i], N - 1) * ldw * ESZ + scol[i];
            }
        return v;
    };
    // issue half `which` (0 A0, 1 A1, 2 B0, 3 B1) of K-tile c into its stage
#define STAGE_HALF(c, v, which)                                                                    \
    {                                                                                              \
        unsigned char* dst_ = g_smem + (c).buf * 65536 + (which) * 16384 + wave_u * 2048;          \
        _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                         \
            if ((which) < 2)                                                                       \
                glds_buf16(A, bytesA, dst_ + i_ * 1024, (v).a[(which) & 1][i_], (c).k0 * ESZ);     \
            else                                                                                   \
                glds_buf16(W, bytesW, dst_ + i_ * 1024, (v).b[(which) & 1][i_], (c).k0 * ESZ);     \
        }                                                                                          \
    }

    f32x4 acc[8][4];
    // In-place style residual (C = resid + A W^T + bias, no row map / broadcast): the accumulators
    // start from the residual tile (loaded with 64-B row segments per 16 lanes), so the epilogue
    // has no loads queued behind its own stores.
    const bool acc_init = resid != nullptr && row_map == nullptr && resid_mod <= 0;
#if GEMM_TACC
    // transposed accumulators: lane (lr, lq) of block (i, j) holds row m = i*16 + lr, columns
    // n = j*16 + 4*lq + [0,4) -- one 16-B load per block (N % 4 == 0 for residual GEMMs)
#define ACC_INIT(m0_, n0_)                                                                         \
    {                                                                                              \
        if (acc_init) {                                                                            \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                       \
                const float* rp_ = resid + (size_t)min((m0_) + wr * 128 + i * 16 + lr, M - 1) * ldr; \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                    \
                    const f32x4v x_ = GEMM_LD_F4(rp_ + min((n0_) + wc * 64 + j * 16 + 4 * lq, N - 4)); \
                    acc[i][j][0] = x_.x; acc[i][j][1] = x_.y; acc[i][j][2] = x_.z; acc[i][j][3] = x_.w; \
                }                                                                                  \
            }                                                                                      \
        } else {                                                                                   \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int j = 0; j < 4; ++j) \
                _Pragma("unroll") for (int e = 0; e < 4; ++e) acc[i][j][e] = 0.f;                  \
        }                                                                                          \
    }
#else
#define ACC_INIT(m0_, n0_)                                                                         \
    {                                                                                              \
        if (acc_init) {                                                                            \
            const float rc_ = (F8 & 1) ? 1.f / csc : 1.f;                                         \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int e = 0; e < 4; ++e) { \
                const float* rp_ = resid + (size_t)min((m0_) + wr * 128 + i * 16 + 4 * lq + e, M - 1) * ldr; \
                _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                    \
                    acc[i][j][e] = GEMM_LD_F(rp_ + min((n0_) + wc * 64 + j * 16 + lr, N - 1));      \
                    if (F8 & 1) acc[i][j][e] *= rc_;                                               \
                }                                                                                  \
            }                                                                                      \
        } else {                                                                                   \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int j = 0; j < 4; ++j) \
                _Pragma("unroll") for (int e = 0; e < 4; ++e) acc[i][j][e] = 0.f;                  \
        }                                                                                          \
    }
#endif

    bf16x8 fa[8], fb0[4], fb1[4];     // fa: A-half fragments [i*2 + ks]; fb*: [j*2 + ks]
    i32x8 ga[4], gb0[2], gb1[2];      // fp8: the two 16-B chunks of a lane as one 32-B fragment
#define LDS16(off) (*reinterpret_cast<const bf16x8*>(g_smem + (off)))
#define RD_A(stage, mi)                                                                            \
    if constexpr ((F8 & 1) != 0) {                                                                 \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                            \
            const int b_ = (stage) * 65536 + (mi) * 16384;                                         \
            ga[i] = frag32(LDS16(b_ + swz(wr * 64 + i * 16 + lr, lq)),                             \
                           LDS16(b_ + swz(wr * 64 + i * 16 + lr, 4 + lq)));                        \
        }                                                                                          \
    } else {                                                                                       \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) \
            fa[i * 2 + ks] = LDS16((stage) * 65536 + (mi) * 16384 + swz(wr * 64 + i * 16 + lr, ks * 4 + lq)); \
    }
#define RD_B(FB, GB, stage, ni)                                                                    \
    if constexpr ((F8 & 1) != 0) {                                                                 \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                            \
            const int b_ = (stage) * 65536 + 32768 + (ni) * 16384;                                 \
            GB[j] = frag32(LDS16(b_ + swz(wc * 32 + j * 16 + lr, lq)),                             \
                           LDS16(b_ + swz(wc * 32 + j * 16 + lr, 4 + lq)));                        \
        }                                                                                          \
    } else {                                                                                       \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) \
            FB[j * 2 + ks] = LDS16((stage) * 65536 + 32768 + (ni) * 16384 + swz(wc * 32 + j * 16 + lr, ks * 4 + lq)); \
    }
#if GEMM_TACC
#define MFMA_OP(FA, FB, C) __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB, FA, C, 0, 0, 0)   // C^T += W A^T
#else
#define MFMA_OP(FA, FB, C) __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA, FB, C, 0, 0, 0)
#endif
#define MFMA_Q(mi, ni, FB, GB)                                                                     \
    {                                                                                              \
        if (GEMM_PRIO_MODE == 0) __builtin_amdgcn_s_setprio(1);                                    \
        if constexpr ((F8 & 1) != 0) {                                                             \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
                acc[(mi) * 4 + i][(ni) * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4( \
                    ga[i], GB[j], acc[(mi) * 4 + i][(ni) * 2 + j], 0, 0, 0, 127, 0, 127);          \
            /* the scaled MFMA builtin is not convergent: pin the results to this phase, or IR     \
               sinking moves all four quadrants' MFMAs behind the last barrier */                  \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
                asm volatile("" : "+v"(acc[(mi) * 4 + i][(ni) * 2 + j]));                          \
        } else {                                                                                   \
            _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int i = 0; i < 4; ++i) \
                _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[(mi) * 4 + i][(ni) * 2 + j] =    \
                    MFMA_OP(fa[i * 2 + ks], FB[j * 2 + ks], acc[(mi) * 4 + i][(ni) * 2 + j]);       \
        }                                                                                          \
        if (GEMM_PRIO_MODE == 0) __builtin_amdgcn_s_setprio(0);                                    \
    }

    // prologue: K-tile 0 complete, K-tile 1 in flight
    KT kc = kt_at_tile(0, 0);
    KT k1 = kt_next(kc);
    KT k2 = kt_next(k1);
    VO v2 = vo_of(k2);
    ACC_INIT(kc.m0, kc.n0);
    {
        const VO v0 = vo_of(kc);
        STAGE_HALF(kc, v0, 2); STAGE_HALF(kc, v0, 0); STAGE_HALF(kc, v0, 3); STAGE_HALF(kc, v0, 1);
    }
    {
        const VO v1 = vo_of(k1);
        STAGE_HALF(k1, v1, 2); STAGE_HALF(k1, v1, 0); STAGE_HALF(k1, v1, 3); STAGE_HALF(k1, v1, 1);
    }
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    PHASE_BARRIER();
    if (stagger && wr == 1) PHASE_BARRIER();      // stagger: waves 4-7 run one barrier behind
    if (GEMM_PRIO_MODE == 1 && wr == 1) __builtin_amdgcn_s_setprio(1);   // static: waves 4-7 win arbitration

    float* scratch = reinterpret_cast<float*>(g_smem + G2_STAGES_BYTES + wave * 4096);  // [16][64]
    constexpr int CW = OUT_BF16 ? 8 : 4;
    constexpr int NIT = 16 * (64 / CW) / 64;      // 16-B stores per lane per 16-row pass
    int stores_pending = 0;   // stores of a full-tile epilogue issued after K-tile g+1's halves
#if GEMM_TACC
    // the epilogue adds the bias after the LDS transpose: a lane's CW output columns are fixed
    const int cl_lane = (lane % (64 / CW)) * CW;
    float bv[CW];
#else
    float bv[4];
#endif
    for (int g = 0; g < total; ++g) {
        const int st = g & 1;
        if (kc.k0 == 0) {     // first K-tile of a tile: its bias columns (loaded well before use)
#if GEMM_TACC
#pragma unroll
            for (int q = 0; q < CW; ++q) {
                const int n = kc.n0 + wc * 64 + cl_lane + q;
                bv[q] = bias ? bias[min(n, N - 1)] : 0.f;
            }
#else
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = kc.n0 + wc * 64 + j * 16 + lr;
                bv[j] = bias ? bias[min(n, N - 1)] : 0.f;
            }
#endif
        }
        // ---- P1: quadrant (0,0); reads B0 (retired before the barrier) then A0
        RD_B(fb0, gb0, st, 0);
        SB0();
        RD_A(st, 0);
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        PHASE_BARRIER();
        MFMA_Q(0, 0, fb0, gb0);
        PHASE_BARRIER();
        // ---- P2: quadrant (0,1); reads B1 (retired before the barrier); stage B0 of g+2
        RD_B(fb1, gb1, st, 1);
        STAGE_HALF(k2, v2, 2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PHASE_BARRIER();
        MFMA_Q(0, 1, fb1, gb1);
        PHASE_BARRIER();
        // ---- P3: quadrant (1,1); reads A1 (retired before the barrier); stage A0 of g+2
        RD_A(st, 1);
        STAGE_HALF(k2, v2, 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PHASE_BARRIER();
        MFMA_Q(1, 1, fb1, gb1);
        PHASE_BARRIER();
        // ---- P4: quadrant (1,0) from registers; stage B1 and A1 of g+2; retire K-tile g+1 (the
        // stores of an epilogue issued since K-tile g+1 was staged may stay in flight)
        STAGE_HALF(k2, v2, 3);
        STAGE_HALF(k2, v2, 1);
        if (stores_pending) {
            if (OUT_BF16) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");   // 8 + 8*NIT
            else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
            stores_pending = 0;
        } else {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        PHASE_BARRIER();
        MFMA_Q(1, 0, fb0, gb0);
        PHASE_BARRIER();
        const KT kd = kc;
        kc = k1; k1 = k2;
        {
            const KT kn = kt_next(k2);
            if (kn.k0 == 0 && kn.idx != k2.idx) v2 = vo_of(kn);   // entered a new tile
            k2 = kn;
        }
        if (kd.k0 != K - KTE) continue;
        if (ablate == 1) {          // diagnostic: no epilogue at all (keeps acc live)
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
            ACC_INIT(kc.m0, kc.n0);
            continue;
        }

        // ---- epilogue of this tile (wave-private, 16 rows = one row block per pass) ----------
        // Full in-bounds sub-tiles without a row map or residual loads take the fast path: no
        // bounds tests, exactly 8*NIT stores, which the next K-tile's counted wait leaves in flight.
        const int m0 = kd.m0 + wr * 128, n0 = kd.n0 + wc * 64;
        const bool fast = row_map == nullptr && (resid == nullptr || acc_init) && m0 + 128 <= M &&
                          n0 + 64 <= N && ablate == 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#if GEMM_TACC
            // row lr of the pass, 16-B slot (4j + lq) ^ lr: the 16 lanes of a write group and
            // the lanes of a read group hit 16 distinct slots of the 256-B bank row
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<float4*>(scratch + lr * 64 + (((4 * j + lq) ^ lr) << 2)) =
                    make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
#else
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                f32x2 v01, v23;
                if constexpr ((F8 & 1) != 0) {
                    v01 = {fmaf(acc[i][j][0], csc, bv[j]), fmaf(acc[i][j][1], csc, bv[j])};
                    v23 = {fmaf(acc[i][j][2], csc, bv[j]), fmaf(acc[i][j][3], csc, bv[j])};
                } else {
                    v01 = {acc[i][j][0] + bv[j], acc[i][j][1] + bv[j]};
                    v23 = {acc[i][j][2] + bv[j], acc[i][j][3] + bv[j]};
                }
                if (ACT == 1) gelu_erf2x2(v01, v23);
                else if (ACT == 2) {
                    v01.x = fmaxf(v01.x, 0.f); v01.y = fmaxf(v01.y, 0.f);
                    v23.x = fmaxf(v23.x, 0.f); v23.y = fmaxf(v23.y, 0.f);
                }
                const int rl = 4 * lq;
                const int col = (j * 16 + lr) ^ (lq << 4);
                scratch[(rl + 0) * 64 + col] = v01.x;
                scratch[(rl + 1) * 64 + col] = v01.y;
                scratch[(rl + 2) * 64 + col] = v23.x;
                scratch[(rl + 3) * 64 + col] = v23.y;
            }
#endif
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int id = it * 64 + lane;
                const int rl = id / (64 / CW), cl = (id % (64 / CW)) * CW;
                const int m = m0 + i * 16 + rl, n = n0 + cl;
                float v[CW];
#if GEMM_TACC
#pragma unroll
                for (int q = 0; q < CW; q += 4) {
                    const float4 x = *reinterpret_cast<const float4*>(
                        scratch + rl * 64 + ((((cl + q) >> 2) ^ rl) << 2));
                    v[q] = x.x; v[q + 1] = x.y; v[q + 2] = x.z; v[q + 3] = x.w;
                }
#pragma unroll
                for (int q = 0; q < CW; q += 2) {
                    f32x2 p = {v[q] + bv[q], v[q + 1] + bv[q + 1]};
                    if (ACT == 1) p = gelu_erf2(p);
                    else if (ACT == 2) { p.x = fmaxf(p.x, 0.f); p.y = fmaxf(p.y, 0.f); }
                    v[q] = p.x; v[q + 1] = p.y;
                }
#else
                const int sw = ((rl >> 2) & 3) << 4;
#pragma unroll
                for (int q = 0; q < CW; q += 4) {
                    const float4 x = *reinterpret_cast<const float4*>(scratch + rl * 64 + ((cl + q) ^ sw));
                    v[q] = x.x; v[q + 1] = x.y; v[q + 2] = x.z; v[q + 3] = x.w;
                }
#endif
                int orow = m;
                bool keep = true;
                if (ablate == 2) {   // diagnostic: no global stores
#pragma unroll
                    for (int q = 0; q < CW; ++q) asm volatile("" :: "v"(v[q]));
                    keep = false;
                } else if (!fast) {
                    keep = m < M && n < N;
                    if (keep && row_map) orow = row_map[m];
                    keep = keep && orow >= 0;
                    if (keep && resid && !acc_init) {
                        const int rrow = resid_mod > 0 ? (m % resid_mod) : orow;
                        const float* rp = resid + (size_t)rrow * ldr + n;
#pragma unroll
                        for (int q = 0; q < CW; q += 4) {
                            const float4 x = *reinterpret_cast<const float4*>(rp + q);
                            v[q] += x.x; v[q + 1] += x.y; v[q + 2] += x.z; v[q + 3] += x.w;
                        }
                    }
                }
                if (keep) {
                    if constexpr ((F8 & 2) != 0) {
                        int lo = 0, hi = 0;
#pragma unroll
                        for (int q = 0; q < 8; ++q) v[q] = fminf(fmaxf(v[q] * oqs, -448.f), 448.f);
                        lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], lo, false);
                        lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
                        hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], hi, false);
                        hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
                        GEMM_ST_U2(reinterpret_cast<unsigned char*>(Cv) + (size_t)orow * ldc + n, lo, hi);
                    } else if (OUT_BF16) {
                        U128 o;
                        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
                        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
                        o.z = (uint32_t)f2bf(v[4 % CW]) | ((uint32_t)f2bf(v[5 % CW]) << 16);
                        o.w = (uint32_t)f2bf(v[6 % CW]) | ((uint32_t)f2bf(v[7 % CW]) << 16);
                        GEMM_ST_U4(reinterpret_cast<u16*>(Cv) + (size_t)orow * ldc + n, o);
                    } else {
                        GEMM_ST_F4(reinterpret_cast<float*>(Cv) + (size_t)orow * ldc + n, v[0], v[1], v[2], v[3]);
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // scratch reads done before reuse
        }
        // the next tile's accumulator init loads would be ordered behind these stores
        stores_pending = (fast && !acc_init) ? 1 : 0;
        ACC_INIT(kc.m0, kc.n0);    // the next tile (kc is its first K-tile; a repeat past the end)
    }
    if (stagger && wr == 0) PHASE_BARRIER();      // both halves leave with the same barrier count
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outstanding at exit
#undef RD_A
#undef RD_B
#undef LDS16
#undef MFMA_Q
#undef MFMA_OP
#undef STAGE_HALF
#undef ACC_INIT
}

// ------------------------------------------------------------------------------------------
// k_gemm256q: k_gemm256p's K loop with the epilogue spread over the phases around the tile
// boundary instead of run as one block after the last K-tile.
//
// The accumulators are transposed (C^T = W A^T on the MFMA): lane (lr, lq) of block (i, j) holds
// row 16i + lr, columns 16j + 4lq + [0,4) -- four consecutive columns, so a lane adds its bias /
// residual and stores straight from registers (f32: one 16-B store per block; bf16: two blocks'
// packed halves exchanged between lane rows by v_permlane16_swap, one 16-B store per block pair).
// No LDS round trip, so nothing in the epilogue touches LDS but the bias row (staged once per
// walk by LDS-DMA into the 32 KiB beside the stages).
//
// A wave's 128x64 sub-tile is four 64x32 quadrants Q(mi, ni); phase P1..P4 of every K-tile runs the
// MFMAs of Q00, Q01, Q11, Q10.  On the last K-tile of a tile, quadrant Q is final after its phase;
// its epilogue (+ bias, activation, store) and its re-initialisation for the next tile (zero, or
// the next tile's residual for an in-place residual GEMM) run in the memory section of the next
// phase -- Q00 in P2, Q01 in P3, Q11 in P4, Q10 in P1 of the next tile's first K-tile -- where the
// staggered partner wave on the same SIMD is in its MFMA section.  So the store burst is spread
// over four phases and the epilogue VALU work runs beside MFMAs instead of on an idle chip.
//
// Counted waits (per wave, S stores and R residual loads per quadrant epilogue, VMEM ops are
// counted in issue order): the last K-tile's P4 retires K-tile g+1 with its own 8 LDS-DMA and the
// three epilogues' 3(S+R) younger ops in flight; the first K-tile's P4 with 8 + S + R (the Q10
// epilogue of P1).  Stores go through a buffer descriptor with out-of-range offsets for rows >= M
// / columns >= N, so every store instruction is issued by every wave and the counts hold.
// Needs nk >= 3 K-tiles, N <= 8192 (bias row in LDS), no row map / broadcast residual; the host
// falls back to k_gemm256p otherwise.
//
// Measured (scripts/gemm_bench.py, interleaved in one process): bf16 outputs gain 6-16 % (CLIP
// fc1+GELU 444.6 -> 397.2 us, qkv 278.2 -> 253.2, CuTR fc1 145.7 -> 123.0); the f32 residual
// GEMMs do not (CLIP fc2 400.1 vs 406.5, proj 139.5 vs 141.9), so those keep k_gemm256p by
// default.  Their cost is the residual read at the tile boundaries (proj: 139.5 us with it, 106.2
// without).  Tried for it and not kept: touching the next tile's residual rows in the middle of
// the current tile (LDS-DMA into a dummy slot, plain or streaming: 3-9 % slower -- the lines evict
// the operand panels), and skewing the tile boundaries per XCD (the first tile split into a
// leading and a trailing segment, the trailing one re-initialised from C: proj 151.9 -> 189.9 us;
// with offsets of only 1, 2 or 4 K-tiles per XCD index still 148.7 -> 187.8-190.0 us, CuTR fc2
// 173.8 -> 191.6-192.2 -- the XCDs' lock-step walk over the same A / W panels is what keeps them
// in the Infinity Cache).
// ------------------------------------------------------------------------------------------
#define G2Q_BIAS_MAX 8192
#ifndef GEMM_STAMP        // diagnostic builds only: per-workgroup s_memtime / s_memrealtime stamps of k_gemm256q
#define GEMM_STAMP 0
#endif
#if GEMM_STAMP
__device__ unsigned long long g_gemm_stamps[4096 * 4];
BF_API int bf_gemm_read_stamps(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_stamps), (size_t)n * 4 * sizeof(unsigned long long));
}
#endif
#ifndef GEMM_ABL          // diagnostic builds only (wrong results): 1 no K-loop LDS-DMA, 2 no fragment reads,
                          // 4 k_gemm256q epilogue stores dropped (out-of-range offsets: same vmcnt counts)
#define GEMM_ABL 0
#endif
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2v));
}

// F8 (as in k_gemm256p): bit 0 fp8 e4m3 operands (128-element K-tiles, block-scaled MFMA with unit
// scales, epilogue acc * csc + bias), bit 1 fp8 output (v * oqs saturated to +-448; 8 bytes per lane
// after the permlane exchange).  Not combined with RES.
//
// MB1 (1..4): 16-row blocks in the second M-half of a wave, so the tile is BM = 2 (64 + 16 MB1)
// rows (160 / 192 / 224 / 256) x 256 columns.  The tile height sets the round quantisation of the
// persistent walk: CLIP's 32896-row GEMMs with N = 1280 run 645 tiles of 256 rows (2.52 rounds of
// 256 CUs, 0.84 of the chip busy) but 735 of 224 rows (2.87 rounds, 0.96); CuTR's 12800 x 768 runs
// 150 tiles of 256 rows (one round on 150 CUs) but 240 of 160.  The second A-half then holds 16 MB1
// valid rows per wave row; its other staging lanes take an out-of-range buffer offset (the LDS-DMA
// fetches nothing), so every wave still issues the same number of VMEM operations and the counted
// waits below only change through the per-quadrant store / load counts.  Each output keeps the
// same K-order MFMA chain, so the tile height never changes a value.
template <bool OUT_BF16, int ACT, bool RES, int F8 = 0, int MB1 = 4>
__global__ void __launch_bounds__(G2_THREADS, 1) k_gemm256q(const u16* __restrict__ A, int lda,
                                                            const u16* __restrict__ W, int ldw,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ resid, int ldr,
                                                            void* __restrict__ Cv, int ldc, int M,
                                                            int N, int K, int tiles_n, int tiles_m,
                                                            int stagger, int gm, float csc = 1.f,
                                                            float oqs = 1.f) {
    extern __shared__ __attribute__((aligned(16))) unsigned char g_smem[];
    static_assert(!(RES && F8), "fp8 residual GEMMs keep k_gemm256p");
    static_assert(!(F8 & 2) || OUT_BF16, "fp8 output takes the narrow store path");
    constexpr int ESZ = (F8 & 1) ? 1 : 2;           // operand bytes
    constexpr int KTE = GB_K * 2 / ESZ;             // K elements per 128-B K-tile row
    static_assert(MB1 >= 1 && MB1 <= 4, "second M-half of 1..4 row blocks");
    constexpr int BMH = 64 + 16 * MB1;              // tile rows per wave row (BM = 2 BMH)
    // per-lane stores of a quadrant epilogue / residual loads of a quadrant re-init, for the
    // quadrants of the first (4 row blocks) and the second (MB1 row blocks) M-half
    constexpr int S0 = OUT_BF16 ? 4 : 8, S1 = S0 / 4 * MB1;
    constexpr int R0 = RES ? 8 : 0, R1 = RES ? 2 * MB1 : 0;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wr = wave >> 2, wc = wave & 3;
    const int lr = lane & 15, lq = lane >> 4;
    const int ntiles = tiles_m * tiles_n;
    const int G = gridDim.x;
    const int slot = (G % 8 == 0) ? ((int)blockIdx.x % 8) * (G / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int my_tiles = ntiles > slot ? (ntiles - slot + G - 1) / G : 0;
    const int nk = K / KTE;
    const int total = my_tiles * nk;
    if (total == 0) return;
#if GEMM_STAMP
    unsigned long long st_t0 = 0, st_r0 = 0;
    if (t == 0) { st_t0 = __builtin_amdgcn_s_memtime(); st_r0 = __builtin_amdgcn_s_memrealtime(); }
#endif
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);

    // bias row -> LDS (retired with K-tile 0 by the prologue's counted wait)
    const float* bias_lds = reinterpret_cast<const float*>(g_smem + G2_STAGES_BYTES);
    if (bias) {
        for (int c = wave_u; c * 256 < N; c += 8)
            glds_buf16(bias, N * 4, g_smem + G2_STAGES_BYTES + c * 1024, lane * 16, c * 1024);
    } else {
        for (int n = t; n < N; n += G2_THREADS) reinterpret_cast<float*>(g_smem + G2_STAGES_BYTES)[n] = 0.f;
    }

    int a_row[2][2], b_row[2][2], scol[2];
    bool a1_ok[2];        // this lane's A-half-1 staging row lies inside the tile (MB1 < 4)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int L = (wave * 2 + i) * 8 + (lane >> 3);
        scol[i] = ((lane & 7) ^ swz_key(L)) * 16;
        a1_ok[i] = (L & 63) < 16 * MB1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            a_row[h][i] = (L >> 6) * BMH + h * 64 + (L & 63);
            b_row[h][i] = (L >> 5) * 64 + h * 32 + (L & 31);
        }
    }
    const int bytesA = (int)(((size_t)(M - 1) * lda + K) * ESZ);
    const int bytesW = (int)(((size_t)(N - 1) * ldw + K) * ESZ);
    struct KT { int idx, m0, n0, k0, buf; };
    auto kt_at_tile = [&](int tile_k, int idx) {
        const int tile = slot + tile_k * G;
        KT r;
        r.idx = idx; tile_coords(tile, tiles_m, tiles_n, gm, r.m0, r.n0, 2 * BMH); r.k0 = 0; r.buf = idx & 1;
        return r;
    };
    int tile_ord = 0;
    auto kt_next = [&](KT c) {
        if (c.idx >= total - 1) return c;
        if (c.k0 + KTE < K) { c.k0 += KTE; c.idx += 1; c.buf ^= 1; return c; }
        ++tile_ord;
        return kt_at_tile(tile_ord, c.idx + 1);
    };
    struct VO { int a[2][2], b[2][2]; };
    auto vo_of = [&](const KT& c) {
        VO v;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                v.a[h][i] = (h == 1 && !a1_ok[i]) ? (int)0x80000000
                                                  : min(c.m0 + a_row[h][i], M - 1) * lda * ESZ + scol[i];
                v.b[h][i] = min(c.n0 + b_row[h][i], N - 1) * ldw * ESZ + scol[i];
            }
        return v;
    };
#define STAGE_HALF(c, v, which)                                                                    \
    if (!(GEMM_ABL & 1) || !in_loop_)                                                              \
    {                                                                                              \
        unsigned char* dst_ = g_smem + (c).buf * 65536 + (which) * 16384 + wave_u * 2048;          \
        _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                         \
            if ((which) < 2)                                                                       \
                glds_buf16(A, bytesA, dst_ + i_ * 1024, (v).a[(which) & 1][i_], (c).k0 * ESZ);     \
            else                                                                                   \
                glds_buf16(W, bytesW, dst_ + i_ * 1024, (v).b[(which) & 1][i_], (c).k0 * ESZ);     \
        }                                                                                          \
    }

    f32x4 acc[4 + MB1][4];
    // row blocks of M-half MI
#define NBLK(MI) ((MI) ? MB1 : 4)
    // quadrant (MI, NI) <- zero or the residual of the tile at (m0_, n0_) (clamped rows / columns:
    // every load is issued, out-of-range values are never stored)
#define QINIT(MI, NI, m0_, n0_)                                                                    \
    {                                                                                              \
        if constexpr (RES) {                                                                       \
            _Pragma("unroll") for (int i = 0; i < NBLK(MI); ++i) {                                \
                const float* rp_ = resid + (size_t)min((m0_) + wr * BMH + (MI) * 64 + i * 16 + lr, M - 1) * ldr; \
                _Pragma("unroll") for (int j = 0; j < 2; ++j)                                      \
                    acc[(MI) * 4 + i][(NI) * 2 + j] = *reinterpret_cast<const f32x4*>(            \
                        rp_ + min((n0_) + wc * 64 + (NI) * 32 + j * 16 + 4 * lq, N - 4));          \
            }                                                                                      \
        } else {                                                                                   \
            _Pragma("unroll") for (int i = 0; i < NBLK(MI); ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
                acc[(MI) * 4 + i][(NI) * 2 + j] = (f32x4){0.f, 0.f, 0.f, 0.f};                     \
        }                                                                                          \
    }
    // the same inside the K loop: the residual arrives by loads hidden from the compiler's waitcnt
    // pass (which would otherwise wait for nearly every outstanding operation before the next
    // MFMA on the quadrant), retired by the counted waits of the following phases
#define QINIT_ASYNC(MI, NI, T_)                                                                    \
    {                                                                                              \
        if constexpr (RES) {                                                                       \
            _Pragma("unroll") for (int i = 0; i < NBLK(MI); ++i) {                                \
                const float* rp_ = resid + (size_t)min((T_).m0 + wr * BMH + (MI) * 64 + i * 16 + lr, M - 1) * ldr; \
                _Pragma("unroll") for (int j = 0; j < 2; ++j)                                      \
                    asm volatile("global_load_dwordx4 %0, %1, off"                                 \
                                 : "=v"(acc[(MI) * 4 + i][(NI) * 2 + j])                           \
                                 : "v"(rp_ + min((T_).n0 + wc * 64 + (NI) * 32 + j * 16 + 4 * lq, N - 4)) \
                                 : "memory");                                                      \
            }                                                                                      \
        } else {                                                                                   \
            QINIT(MI, NI, (T_).m0, (T_).n0);                                                       \
        }                                                                                          \
    }
    // output buffer descriptor: byte offsets of rows < M only (the rest are dropped)
    const int esz = (F8 & 2) ? 1 : OUT_BF16 ? 2 : 4;
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        Cv, 0, (int)(((size_t)(M - 1) * ldc + N) * esz), 0x00020000);
    // epilogue of quadrant (MI, NI) of the tile at (em0_, en0_)
#define QEPI(MI, NI, em0_, en0_)                                                                   \
    {                                                                                              \
        const int cb_ = (en0_) + wc * 64 + (NI) * 32 + 4 * lq;                                     \
        const f32x4 b0_ = *reinterpret_cast<const f32x4*>(bias_lds + min(cb_, N - 4));            \
        const f32x4 b1_ = *reinterpret_cast<const f32x4*>(bias_lds + min(cb_ + 16, N - 4));       \
        _Pragma("unroll") for (int i = 0; i < NBLK(MI); ++i) {                                    \
            const int r_ = (em0_) + wr * BMH + (MI) * 64 + i * 16 + lr;                            \
            if constexpr ((F8 & 2) != 0) {                                                         \
                /* fp8 row segments, one block at a time (fewer live registers): 4 bytes per      \
                   block, exchanged between lane rows -> 8 consecutive bytes */                     \
                int XY_[2];                                                                        \
                _Pragma("unroll") for (int jj = 0; jj < 2; ++jj) {                                 \
                    f32x4 x_ = acc[(MI) * 4 + i][(NI) * 2 + jj] * csc + (jj ? b1_ : b0_);          \
                    if constexpr (ACT == 1) {                                                      \
                        f32x2 p0 = {x_.x, x_.y}, p1 = {x_.z, x_.w};                                \
                        gelu_erf2x2(p0, p1);                                                       \
                        x_ = (f32x4){p0.x, p0.y, p1.x, p1.y};                                      \
                    }                                                                              \
                    x_ = __builtin_elementwise_min(__builtin_elementwise_max(x_ * oqs,             \
                             (f32x4){-448.f, -448.f, -448.f, -448.f}), (f32x4){448.f, 448.f, 448.f, 448.f}); \
                    int q_ = __builtin_amdgcn_cvt_pk_fp8_f32(x_.x, x_.y, 0, false);                \
                    XY_[jj] = __builtin_amdgcn_cvt_pk_fp8_f32(x_.z, x_.w, q_, true);               \
                }                                                                                  \
                const auto s_ = __builtin_amdgcn_permlane16_swap((uint32_t)XY_[0], (uint32_t)XY_[1], false, false); \
                const int c_ = (en0_) + wc * 64 + (NI) * 32 + 16 * (lq & 1) + 8 * (lq >> 1);        \
                const int off_ = (r_ < M && c_ < N && !(GEMM_ABL & 4)) ? (r_ * ldc + c_) : (int)0x80000000; \
                __builtin_amdgcn_raw_buffer_store_b64((u32x2v){s_[0], s_[1]}, crs, off_, 0, 2);   \
                continue;                                                                          \
            }                                                                                      \
            f32x4 x0, x1;                                                                          \
            if constexpr ((F8 & 1) != 0) {                                                         \
                x0 = acc[(MI) * 4 + i][(NI) * 2] * csc + b0_;                                      \
                x1 = acc[(MI) * 4 + i][(NI) * 2 + 1] * csc + b1_;                                  \
            } else {                                                                               \
                x0 = acc[(MI) * 4 + i][(NI) * 2] + b0_;                                            \
                x1 = acc[(MI) * 4 + i][(NI) * 2 + 1] + b1_;                                        \
            }                                                                                      \
            if constexpr (ACT == 1) {                                                              \
                f32x2 p0 = {x0.x, x0.y}, p1 = {x0.z, x0.w}, p2 = {x1.x, x1.y}, p3 = {x1.z, x1.w}; \
                gelu_erf2x2(p0, p1); gelu_erf2x2(p2, p3);                                          \
                x0 = (f32x4){p0.x, p0.y, p1.x, p1.y}; x1 = (f32x4){p2.x, p2.y, p3.x, p3.y};         \
            } else if constexpr (ACT == 2) {                                                       \
                x0 = __builtin_elementwise_max(x0, (f32x4){0.f, 0.f, 0.f, 0.f});                   \
                x1 = __builtin_elementwise_max(x1, (f32x4){0.f, 0.f, 0.f, 0.f});                   \
            }                                                                                      \
            if constexpr (false) {                                                                 \
            } else if constexpr (OUT_BF16) {                                                       \
                uint32_t X0 = pk_bf16(x0.x, x0.y), X1 = pk_bf16(x0.z, x0.w);                       \
                uint32_t Y0 = pk_bf16(x1.x, x1.y), Y1 = pk_bf16(x1.z, x1.w);                       \
                const auto s0_ = __builtin_amdgcn_permlane16_swap(X0, Y0, false, false);           \
                const auto s1_ = __builtin_amdgcn_permlane16_swap(X1, Y1, false, false);           \
                const int c_ = (en0_) + wc * 64 + (NI) * 32 + 16 * (lq & 1) + 8 * (lq >> 1);        \
                const int off_ = (r_ < M && c_ < N && !(GEMM_ABL & 4)) ? (r_ * ldc + c_) * 2 : (int)0x80000000; \
                __builtin_amdgcn_raw_buffer_store_b128((u32x4v){s0_[0], s1_[0], s0_[1], s1_[1]},   \
                                                       crs, off_, 0, 2);                           \
            } else {                                                                               \
                const int o0_ = (r_ < M && cb_ < N && !(GEMM_ABL & 4)) ? (r_ * ldc + cb_) * 4 : (int)0x80000000; \
                const int o1_ = (r_ < M && cb_ + 16 < N && !(GEMM_ABL & 4)) ? (r_ * ldc + cb_ + 16) * 4 : (int)0x80000000; \
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, x0), crs, o0_, 0, 2); \
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, x1), crs, o1_, 0, 2); \
            }                                                                                      \
        }                                                                                          \
    }

    bf16x8 fa[8], fb0[4], fb1[4];
    i32x8 ga[4], gb0[2], gb1[2];      // fp8: a lane's two 16-B chunks as one 32-B fragment
#define LDS16(off) (*reinterpret_cast<const bf16x8*>(g_smem + (off)))
#define RD_A(stage, mi)                                                                            \
    if ((GEMM_ABL & 2) && in_loop_) {} else if constexpr ((F8 & 1) != 0) {                                                                 \
        _Pragma("unroll") for (int i = 0; i < NBLK(mi); ++i) {                                     \
            const int b_ = (stage) * 65536 + (mi) * 16384;                                         \
            ga[i] = frag32(LDS16(b_ + swz(wr * 64 + i * 16 + lr, lq)),                             \
                           LDS16(b_ + swz(wr * 64 + i * 16 + lr, 4 + lq)));                        \
        }                                                                                          \
    } else {                                                                                       \
        _Pragma("unroll") for (int i = 0; i < NBLK(mi); ++i) _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) \
            fa[i * 2 + ks] = LDS16((stage) * 65536 + (mi) * 16384 + swz(wr * 64 + i * 16 + lr, ks * 4 + lq)); \
    }
#define RD_B(FB, GB, stage, ni)                                                                    \
    if ((GEMM_ABL & 2) && in_loop_) {} else if constexpr ((F8 & 1) != 0) {                                                                 \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                            \
            const int b_ = (stage) * 65536 + 32768 + (ni) * 16384;                                 \
            GB[j] = frag32(LDS16(b_ + swz(wc * 32 + j * 16 + lr, lq)),                             \
                           LDS16(b_ + swz(wc * 32 + j * 16 + lr, 4 + lq)));                        \
        }                                                                                          \
    } else {                                                                                       \
        _Pragma("unroll") for (int j = 0; j < 2; ++j) _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) \
            FB[j * 2 + ks] = LDS16((stage) * 65536 + 32768 + (ni) * 16384 + swz(wc * 32 + j * 16 + lr, ks * 4 + lq)); \
    }
#define MFMA_Q(mi, ni, FB, GB)                                                                     \
    {                                                                                              \
        if (GEMM_PRIO_MODE == 0) __builtin_amdgcn_s_setprio(1);                                    \
        if constexpr ((F8 & 1) != 0) {                                                             \
            _Pragma("unroll") for (int i = 0; i < NBLK(mi); ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
                acc[(mi) * 4 + i][(ni) * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4( \
                    GB[j], ga[i], acc[(mi) * 4 + i][(ni) * 2 + j], 0, 0, 0, 127, 0, 127);          \
            /* not convergent: pin the results to this phase (see k_gemm256p) */                   \
            _Pragma("unroll") for (int i = 0; i < NBLK(mi); ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
                asm volatile("" : "+v"(acc[(mi) * 4 + i][(ni) * 2 + j]));                          \
        } else {                                                                                   \
            _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) _Pragma("unroll") for (int i = 0; i < NBLK(mi); ++i) \
                _Pragma("unroll") for (int j = 0; j < 2; ++j) acc[(mi) * 4 + i][(ni) * 2 + j] =    \
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j * 2 + ks], fa[i * 2 + ks],        \
                                                            acc[(mi) * 4 + i][(ni) * 2 + j], 0, 0, 0); \
        }                                                                                          \
        if (GEMM_PRIO_MODE == 0) __builtin_amdgcn_s_setprio(0);                                    \
    }

    bool in_loop_ = false;    // GEMM_ABL diagnostics act inside the K loop only
    KT kc = kt_at_tile(0, 0);
    KT k1 = kt_next(kc);
    KT k2 = kt_next(k1);
    VO v2 = vo_of(k2);
    QINIT(0, 0, kc.m0, kc.n0); QINIT(0, 1, kc.m0, kc.n0); QINIT(1, 1, kc.m0, kc.n0); QINIT(1, 0, kc.m0, kc.n0);
    {
        const VO v0 = vo_of(kc);
        STAGE_HALF(kc, v0, 2); STAGE_HALF(kc, v0, 0); STAGE_HALF(kc, v0, 3); STAGE_HALF(kc, v0, 1);
    }
    {
        const VO v1 = vo_of(k1);
        STAGE_HALF(k1, v1, 2); STAGE_HALF(k1, v1, 0); STAGE_HALF(k1, v1, 3); STAGE_HALF(k1, v1, 1);
    }
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    PHASE_BARRIER();
    if (stagger && wr == 1) PHASE_BARRIER();
    if (GEMM_PRIO_MODE == 1 && wr == 1) __builtin_amdgcn_s_setprio(1);

    int em0 = 0, en0 = 0;     // the tile whose quadrant Q10 is still pending
    if (GEMM_ABL & 2) { RD_B(fb0, gb0, 0, 0); RD_B(fb1, gb1, 0, 1); RD_A(0, 0); }
    in_loop_ = true;
    for (int g = 0; g < total; ++g) {
        const int st = g & 1;
        const bool isL = kc.k0 == K - KTE;
        const bool isF = kc.k0 == 0 && g > 0;
        // ---- P1: Q00; reads B0 then A0; [first K-tile: the previous tile's Q10]
        RD_B(fb0, gb0, st, 0);
        SB0();
        RD_A(st, 0);
        if (isF) {
            QEPI(1, 0, em0, en0); QINIT_ASYNC(1, 0, kc);
            CBAR();
            if constexpr (RES) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + S0 + R0 + 2 * (S1 + R1)) : "memory");  // Q00's residual (L.P2)
        }
        CBAR();
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        PHASE_BARRIER();
        MFMA_Q(0, 0, fb0, gb0);
        PHASE_BARRIER();
        // ---- P2: Q01; reads B1; stage B0 of g+2; [last K-tile: Q00]
        RD_B(fb1, gb1, st, 1);
        STAGE_HALF(k2, v2, 2);
        if (isL) { QEPI(0, 0, kc.m0, kc.n0); QINIT_ASYNC(0, 0, k1); }
        if (isF) {
            if constexpr (RES) { CBAR(); asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + 2 * (S1 + R1)) : "memory"); }  // Q01 (L.P3)
        }
        CBAR();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PHASE_BARRIER();
        MFMA_Q(0, 1, fb1, gb1);
        PHASE_BARRIER();
        // ---- P3: Q11; reads A1; stage A0 of g+2; [last K-tile: Q01]
        RD_A(st, 1);
        STAGE_HALF(k2, v2, 0);
        if (isL) { QEPI(0, 1, kc.m0, kc.n0); QINIT_ASYNC(0, 1, k1); }
        if (isF) {
            if constexpr (RES) { CBAR(); asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 + S1 + R1) : "memory"); }    // Q11 (L.P4)
        }
        CBAR();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PHASE_BARRIER();
        MFMA_Q(1, 1, fb1, gb1);
        PHASE_BARRIER();
        // ---- P4: Q10 from registers; stage B1 and A1 of g+2; [last K-tile: Q11]; retire g+1
        STAGE_HALF(k2, v2, 3);
        STAGE_HALF(k2, v2, 1);
        if (isL) {
            QEPI(1, 1, kc.m0, kc.n0); QINIT_ASYNC(1, 1, k1);
            CBAR();
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(8 + 2 * (S0 + R0) + S1 + R1) : "memory");
            em0 = kc.m0; en0 = kc.n0;
        } else if (isF) {
            // K-tile g+1, and (RES) Q10's residual from P1: 8 younger LDS-DMA
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(RES ? 8 : 8 + S1) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        PHASE_BARRIER();
        MFMA_Q(1, 0, fb0, gb0);
        PHASE_BARRIER();
        kc = k1; k1 = k2;
        {
            const KT kn = kt_next(k2);
            if (kn.k0 == 0 && kn.idx != k2.idx) v2 = vo_of(kn);
            k2 = kn;
        }
    }
    QEPI(1, 0, em0, en0);          // the last tile's Q10
    if (stagger && wr == 0) PHASE_BARRIER();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if GEMM_STAMP
    if (t == 0 && blockIdx.x < 4096) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        volatile unsigned long long* d = g_gemm_stamps + blockIdx.x * 4;
        d[0] = st_t0; d[1] = t1; d[2] = st_r0; d[3] = r1;
    }
#endif
#undef RD_A
#undef RD_B
#undef LDS16
#undef MFMA_Q
#undef STAGE_HALF
#undef QINIT
#undef QINIT_ASYNC
#undef QEPI
#undef NBLK
}

// Per-call configuration (bf_gemm_plan of the C-ABI; NULL = the defaults): the library keeps no
// process-wide GEMM state, so concurrent calls on different streams with different plans are
// independent.  Variant: 1 k_gemm256p (staggered 4-phase schedule), 2 k_gemm256p unstaggered, 3 / 4
// k_gemm256p timing ablations (no epilogue / no global stores: wrong results), 5 (default)
// k_gemm256q for bf16 outputs, k_gemm256p otherwise, 6 k_gemm256q wherever it applies.
struct GemmCfg {
    int n_cu_dev;    // CUs of the device: every kernel CHOICE is made against this (value-invariant
                     // across ranks whatever their budgets)
    int n_cu;        // CUs the persistent grid and the tile-height model assume (the budget)
    int tile_rows;   // 0 = the per-shape model
    int kernel;      // 0 = the shape rule, 1 = 128x128 tiles, -1 = the persistent kernels
    int variant;     // 1..6 (above)
    int group_m;     // row panels per tile group (tile_coords); 1 = row-major
    int balanced;    // 0 one workgroup per CU, 1 balanced when the last round is >= 1/4 full, 2 always
};

static int gemm_device_cus() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    // per device, cached (read once; never changes)
    static int cache[64] = {0};
    if (dev < 0 || dev >= 64) dev = 0;
    if (cache[dev] == 0) {
        hipDeviceProp_t prop;
        cache[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    }
    return cache[dev];
}

static GemmCfg gemm_cfg(const bf_gemm_plan* p) {
    GemmCfg c;
    c.n_cu_dev = gemm_device_cus();
    c.n_cu = (p && p->cu_budget > 0 && p->cu_budget < c.n_cu_dev) ? p->cu_budget : c.n_cu_dev;
    c.tile_rows = (p && p->tile_rows >= 160 && p->tile_rows <= 256 && p->tile_rows % 32 == 0) ? p->tile_rows : 0;
    c.kernel = p ? (p->kernel > 0 ? 1 : p->kernel < 0 ? -1 : 0) : 0;
    c.variant = (p && p->variant >= 1 && p->variant <= 6) ? p->variant : 5;
    c.group_m = (p && p->group_m > 0) ? p->group_m : 8;
    c.balanced = !p || p->balanced == 0 ? 1 : p->balanced == 2 ? 2 : 0;
    return c;
}

template <bool OB, int AC>
static void launch_gemm256(const GemmCfg& cfg, int grid, hipStream_t st, const void* A, int lda, const void* W,
                           int ldw, const float* bias, const float* resid, int ldr, int resid_mod, void* C,
                           int ldc, const int32_t* row_map, int M, int N, int K, int tiles_n,
                           int tiles_m) {
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_gemm256p<OB, AC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            G2_LDS);
        attr = true;
    }
    hipLaunchKernelGGL((k_gemm256p<OB, AC>), dim3(grid), dim3(G2_THREADS), G2_LDS, st, (const u16*)A,
                       lda, (const u16*)W, ldw, bias, resid, ldr, resid_mod, C, ldc, row_map, M, N,
                       K, tiles_n, tiles_m, cfg.variant == 2 ? 0 : 1, cfg.group_m,
                       (cfg.variant == 3 || cfg.variant == 4) ? cfg.variant - 2 : 0);
}

// Large problems (N >= 512, at least half a round of 256x256 tiles on the DEVICE's CUs) run the
// persistent kernels: per tile they are 3-4x the 128x128 kernel's rate (CLIP patch embed 32768 x
// 1280 x 640 with its row map: 240 us on 128x128 tiles, profiles/r05_bench_kernel_stats.csv), which
// no round quantisation of the 128x128 grid makes up for.  The rule reads the device's CU count,
// not a plan's budget, so ranks with different budgets run the same kernels (same bits).
static bool gemm_large_tiles(int M, int N, int K, int n_cu_dev) {
    const long long t2 = (long long)((M + 255) / 256) * ((N + 255) / 256);
    (void)K;
    return N >= 512 && t2 >= n_cu_dev / 2;
}

// which kernel bf_gemm_bf16 runs for an aligned problem of this shape (1 = 256x256 persistent)
static bool gemm_use_large(int M, int N, int K, const GemmCfg& cfg) {
    return cfg.kernel < 0 ? true : cfg.kernel > 0 ? false : gemm_large_tiles(M, N, K, cfg.n_cu_dev);
}

BF_API int bf_gemm_large_tiles(int M, int N, int K) { return gemm_large_tiles(M, N, K, gemm_device_cus()) ? 1 : 0; }

// Persistent grid size for `tiles` tiles: one workgroup per CU, or, when the last round of tiles
// is at least a quarter full, as many workgroups as the round count needs (every block walks the
// same number of tiles, +-1): the CUs a partial last round would leave idle at the end are free
// for the other streams' kernels from the start instead.  A nearly empty last round costs little,
// and a full-width grid runs the same tiles ~5 % faster alone (measured on CLIP fc1, 2580 tiles).
static int gemm_grid(long long tiles, const GemmCfg& cfg) {
    const int n_cu = cfg.n_cu;
    int grid = (int)(tiles < n_cu ? tiles : n_cu);
    if (cfg.balanced && tiles > n_cu && (cfg.balanced == 2 || tiles % n_cu >= n_cu / 4)) {
        const long long rounds = (tiles + n_cu - 1) / n_cu;
        const int g = (int)(((tiles + rounds - 1) / rounds + 7) & ~7LL);
        grid = g < n_cu ? g : n_cu;
    }
    return grid;
}

// Tile height of k_gemm256q for an M x N x K problem, from the shape (and the grid's CU count):
// the height with the lowest rounds(BM) x t(BM), rounds = ceil(tiles / CUs), t(BM) the per-tile
// time model above.  Against the sweep of every path shape (profiles/r05_gemm_tile_sweep.log) it
// picks the fastest height or one within 1 %: 224 rows for CLIP proj / fc2 (N = 1280) and CuTR's
// window qkv, 160 for CuTR's N = 768 residual GEMMs, 256 elsewhere.  Every height gives the same
// K-order MFMA chain per output, so this choice never changes a value.
static int gemm_tile_mb1(int M, int N, int K, const GemmCfg& cfg) {
    if (cfg.tile_rows) return (cfg.tile_rows / 2 - 64) / 16;
    const int n_cu = cfg.n_cu;
    const long long tn = (N + 255) / 256;
    int best = 4;
    double best_cost = 0.0;
    for (int mb1 = 4; mb1 >= 1; --mb1) {
        const int bm = 2 * (64 + 16 * mb1);
        const long long tiles = ((M + bm - 1) / bm) * tn;
        const long long rounds = (tiles + n_cu - 1) / n_cu;
        const double cost = (double)rounds * (GEMM_TILE_FIXED + (1.0 - GEMM_TILE_FIXED) * bm / 256.0);
        if (mb1 == 4 || cost < best_cost) { best = mb1; best_cost = cost; }
    }
    (void)K;
    return best;
}

template <bool OB, int AC, bool RS, int F8, int MB1>
static void gemm256q_attr() {
    static bool done = false;
    if (!done) {
        hipFuncSetAttribute((const void*)k_gemm256q<OB, AC, RS, F8, MB1>, hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
        done = true;
    }
}

template <bool OB, int AC, bool RS, int F8>
static int launch_gemm256q(int mb1, int gm, int grid, void* stream, const void* A, int lda, const void* W, int ldw,
                           const float* bias, const float* resid, int ldr, void* C, int ldc, int M, int N, int K,
                           int tiles_n, int tiles_m, float csc, float oqs) {
#define GQ(MB)                                                                                              \
    {                                                                                                       \
        gemm256q_attr<OB, AC, RS, F8, MB>();                                                                \
        hipLaunchKernelGGL((k_gemm256q<OB, AC, RS, F8, MB>), dim3(grid), dim3(G2_THREADS), G2_LDS,           \
                           bf_stream(stream), (const u16*)A, lda, (const u16*)W, ldw, bias, resid, ldr, C,   \
                           ldc, M, N, K, tiles_n, tiles_m, 1, gm, csc, oqs);                                 \
    }
    switch (mb1) {
        case 1: GQ(1); break;
        case 2: GQ(2); break;
        case 3: GQ(3); break;
        default: GQ(4); break;
    }
#undef GQ
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// k_gemm_skinny: few-row GEMMs (CLIP's output projection over the 128 class tokens, 128 x 1024 x
// 1280; the cls-only last block's proj / fc1 / fc2, 128 x {1280, 5120} x {1280, 5120}).  The tiled
// kernels give those 8-40 workgroups; here a 512-thread workgroup owns a 128-row x 32-column
// output tile and its 8 waves split K (wave w takes the 32-wide k-steps w, w + 8, ...), so a
// 128-row problem runs N / 32 workgroups, each reading its 32 weight rows once.  Operands go
// straight from global memory into MFMA fragments (C^T = W A^T on v_mfma_f32_16x16x32_bf16: lane
// (lr, lq) of block (i, j) holds row 16i + lr, columns 16j + 4lq + [0, 4)) through a 3-deep
// register ring, so three k-steps of loads are in flight per wave.  The 8 partial tiles meet in
// LDS and are summed in wave order (deterministic), then bias / activation / residual / row map
// as in bf_gemm_bf16.  Needs N % 32 == 0 and K % 256 == 0 (every wave the same k-step count).
// ------------------------------------------------------------------------------------------
#define SK_THREADS 512
#define SK_LDS (8 * 128 * 32 * 4)
template <bool OUT_BF16, int ACT>
__global__ void __launch_bounds__(SK_THREADS, 1) k_gemm_skinny(const u16* __restrict__ A, int lda,
                                                               const u16* __restrict__ W, int ldw,
                                                               const float* __restrict__ bias,
                                                               const float* __restrict__ resid, int ldr,
                                                               int resid_mod, void* __restrict__ Cv, int ldc,
                                                               const int32_t* __restrict__ row_map, int M,
                                                               int N, int K) {
    extern __shared__ __attribute__((aligned(16))) unsigned char g_smem[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int lr = lane & 15, lq = lane >> 4;
    const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 128;
    const int cnt = K / 256;                     // k-steps per wave
    const u16* ap[8];
    const u16* wp[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) ap[i] = A + (size_t)min(m0 + 16 * i + lr, M - 1) * lda + 8 * lq + 32 * wave;
#pragma unroll
    for (int j = 0; j < 2; ++j) wp[j] = W + (size_t)(n0 + 16 * j + lr) * ldw + 8 * lq + 32 * wave;
    f32x4 acc[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    bf16x8 ra[3][8], rw[3][2];
    // k-step s of this wave (clamped: a load past the end re-reads the last step, never used)
#define SK_LOAD(slot, s)                                                                           \
    {                                                                                              \
        const int o_ = 256 * min((s), cnt - 1);                                                    \
        _Pragma("unroll") for (int i = 0; i < 8; ++i)                                              \
            ra[slot][i] = *reinterpret_cast<const bf16x8*>(ap[i] + o_);                            \
        _Pragma("unroll") for (int j = 0; j < 2; ++j)                                              \
            rw[slot][j] = *reinterpret_cast<const bf16x8*>(wp[j] + o_);                            \
    }
#define SK_MFMA(slot)                                                                              \
    {                                                                                              \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rw[slot][j], ra[slot][i], acc[i][j], 0, 0, 0); \
    }
    SK_LOAD(0, 0);
    SK_LOAD(1, 1);
    SK_LOAD(2, 2);
    int s = 0;
    for (; s + 3 <= cnt; s += 3) {
        SK_MFMA(0); SK_LOAD(0, s + 3);
        SK_MFMA(1); SK_LOAD(1, s + 4);
        SK_MFMA(2); SK_LOAD(2, s + 5);
    }
    if (s < cnt) SK_MFMA(0);
    if (s + 1 < cnt) SK_MFMA(1);
#undef SK_LOAD
#undef SK_MFMA
    // partial tiles -> LDS [wave][128][32] f32; rows XOR-swizzled by 16-B slot against the bank rows
    float* red = reinterpret_cast<float*>(g_smem);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = 16 * i + lr, c4 = (4 * j + lq) ^ (r & 7);
            *reinterpret_cast<f32x4*>(red + wave * 4096 + r * 32 + 4 * c4) = acc[i][j];
        }
    __syncthreads();
    // thread t: row t / 4, columns 8 (t % 4) + [0, 8)
    const int rl = t >> 2, cq = t & 3;
    const int m = m0 + rl;
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c4 = (2 * cq + h) ^ (rl & 7);
            const f32x4 x = *reinterpret_cast<const f32x4*>(red + w * 4096 + rl * 32 + 4 * c4);
            v[4 * h] += x.x; v[4 * h + 1] += x.y; v[4 * h + 2] += x.z; v[4 * h + 3] += x.w;
        }
    if (m >= M) return;
    const int orow = row_map ? row_map[m] : m;
    if (orow < 0) return;
    const int n = n0 + 8 * cq;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        float x = v[q] + (bias ? bias[n + q] : 0.f);
        if (ACT == 1) x = gelu_erf(x);
        else if (ACT == 2) x = fmaxf(x, 0.f);
        v[q] = x;
    }
    if (resid) {
        const float* rp = resid + (size_t)(resid_mod > 0 ? m % resid_mod : orow) * ldr + n;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] += rp[q];
    }
    if (OUT_BF16) {
        U128 o;
        o.x = pk_bf16(v[0], v[1]); o.y = pk_bf16(v[2], v[3]);
        o.z = pk_bf16(v[4], v[5]); o.w = pk_bf16(v[6], v[7]);
        *reinterpret_cast<U128*>(reinterpret_cast<u16*>(Cv) + (size_t)orow * ldc + n) = o;
    } else {
        float* cp = reinterpret_cast<float*>(Cv) + (size_t)orow * ldc + n;
        *reinterpret_cast<f32x4*>(cp) = (f32x4){v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(cp + 4) = (f32x4){v[4], v[5], v[6], v[7]};
    }
}

// few-row problems: the 128 x 128 kernel would give fewer than half the CUs a workgroup
// (the device's CU count, as gemm_large_tiles: a rank's budget never changes the kernel)
static bool gemm_use_skinny(int M, int N, int K, int vec_epi, const GemmCfg& cfg) {
    if (cfg.kernel != 0 || !vec_epi || N % 32 != 0 || K % 256 != 0) return false;
    const long long t1 = (long long)((M + GB_M - 1) / GB_M) * ((N + GB_N - 1) / GB_N);
    return t1 < cfg.n_cu_dev / 2;
}

template <bool OB, int AC>
static int launch_gemm_skinny(void* stream, const void* A, int lda, const void* W, int ldw, const float* bias,
                              const float* resid, int ldr, int resid_mod, void* C, int ldc,
                              const int32_t* row_map, int M, int N, int K) {
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_gemm_skinny<OB, AC>, hipFuncAttributeMaxDynamicSharedMemorySize, SK_LDS);
        attr = true;
    }
    hipLaunchKernelGGL((k_gemm_skinny<OB, AC>), dim3(N / 32, (M + 127) / 128), dim3(SK_THREADS), SK_LDS,
                       bf_stream(stream), (const u16*)A, lda, (const u16*)W, ldw, bias, resid, ldr, resid_mod, C,
                       ldc, row_map, M, N, K);
    return bf_check_launch();
}

// BF_GEMM_LOG=1: each distinct (shape, epilogue, kernel) choice of bf_gemm_bf16 once on stderr
static void gemm_log(int M, int N, int K, int act, int resid, int resid_mod, int row_map, int c_bf16,
                     const char* kern, int bm) {
    static const bool on = [] { const char* e = getenv("BF_GEMM_LOG"); return e && e[0] == '1'; }();
    if (!on) return;
    // never destroyed: no static destructor runs at process exit (exit order)
    static std::mutex& mu = *new std::mutex;
    static std::set<std::string>& seen = *new std::set<std::string>;
    char buf[256];
    snprintf(buf, sizeof buf, "bf_gemm M=%d N=%d K=%d act=%d resid=%d resid_mod=%d row_map=%d out=%s -> %s rows=%d",
             M, N, K, act, resid, resid_mod, row_map, c_bf16 ? "bf16" : "f32", kern, bm);
    std::lock_guard<std::mutex> g(mu);
    if (seen.insert(buf).second) fprintf(stderr, "%s\n", buf);
}

// The product entry point: hand-written kernels only, chosen from the shape alone; the plan (NULL =
// defaults) sizes the persistent grid and carries the measurement hooks, per call.
BF_API int bf_gemm_bf16_plan(const void* A, int lda, const void* W, int ldw, const float* bias,
                             const float* resid, int ldr, int resid_mod, void* C, int ldc, int c_bf16,
                             const int32_t* row_map, int M, int N, int K, int act, const bf_gemm_plan* plan,
                             void* stream) {
    const GemmCfg cfg = gemm_cfg(plan);
    if (!A || !W || !C || M < 0 || N <= 0 || K <= 0) return BF_ERR_ARG;
    if (K % GB_K != 0 || lda % 8 != 0 || ldw % 8 != 0) return BF_ERR_UNSUPPORTED;
    if (M == 0) return BF_OK;
    // the operand buffer descriptors (num_records) and per-lane row offsets are 32-bit: operands
    // whose byte extent reaches 2^31 would wrap (split M on the host instead)
    if ((long long)(M - 1) * lda * 2 + (long long)K * 2 >= (1LL << 31) ||
        (long long)(N - 1) * ldw * 2 + (long long)K * 2 >= (1LL << 31))
        return BF_ERR_CAPACITY;
    const int tiles_m = (M + GB_M - 1) / GB_M, tiles_n = (N + GB_N - 1) / GB_N;
    const int nwg = tiles_m * tiles_n;
    const size_t lds = 2 * 32768;
    if (act < 0 || act > 2) return BF_ERR_ARG;
    // 16-B row chunks need N % 8 (bf16) / N % 4 (f32) and 16-B aligned rows of C and resid
    const int cw = c_bf16 ? 8 : 4;
    const int vec_epi = (N % cw == 0) && ((uintptr_t)C % 16 == 0) && ((size_t)ldc * (c_bf16 ? 2 : 4) % 16 == 0) &&
                        (!resid || (((uintptr_t)resid % 16 == 0) && (ldr % 4 == 0)));
    const int t2m = (M + 255) / 256, t2n = (N + 255) / 256;
    const long long t2 = (long long)t2m * t2n;
    // 16-B row chunks of C / resid also carry the skinny kernel's epilogue (8 columns per thread)
    if (gemm_use_skinny(M, N, K, vec_epi && (c_bf16 || N % 8 == 0), cfg)) {
        gemm_log(M, N, K, act, resid != nullptr, resid_mod, row_map != nullptr, c_bf16, "k_gemm_skinny", 128);
#define GSK(OB, AC) return launch_gemm_skinny<OB, AC>(stream, A, lda, W, ldw, bias, resid, ldr, resid_mod, C, ldc, \
                                                      row_map, M, N, K)
        if (c_bf16) {
            if (act == 0) GSK(true, 0);
            if (act == 1) GSK(true, 1);
            GSK(true, 2);
        }
        if (act == 0) GSK(false, 0);
        if (act == 1) GSK(false, 1);
        GSK(false, 2);
#undef GSK
    }
    if (vec_epi && gemm_use_large(M, N, K, cfg)) {
        const int grid2 = gemm_grid(t2, cfg);
        // the overlapped-epilogue kernel: plain / in-place residual outputs, >= 3 K-tiles, the bias
        // row fits its LDS slot, 32-bit byte offsets into C and the residual.  Variant 5 (default):
        // bf16 outputs, and the f32 residual GEMMs whose tile height (gemm_tile_rows) is below 256;
        // at 256 rows those measured 1-4 % slower on it than on k_gemm256p.  Variant 6: every
        // eligible shape.
        const int mb1 = gemm_tile_mb1(M, N, K, cfg);
        const bool q_fit = row_map == nullptr && resid_mod <= 0 && K / 64 >= 3 && N <= G2Q_BIAS_MAX && act <= 1 &&
                           !(resid && act) && !(resid && c_bf16) && !(act && !c_bf16) &&
                           (long long)(M - 1) * ldc * (c_bf16 ? 2 : 4) + (long long)N * 4 < (1LL << 31) &&
                           (!resid || (long long)(M - 1) * ldr * 4 + (long long)N * 4 < (1LL << 31));
        const bool q_ok = q_fit && (cfg.variant == 6 || (cfg.variant == 5 && (c_bf16 || mb1 < 4)));
        if (q_ok) {
            const int bm = 2 * (64 + 16 * mb1);
            const int tqm = (M + bm - 1) / bm;
            const int gq = gemm_grid((long long)tqm * t2n, cfg);
            gemm_log(M, N, K, act, resid != nullptr, resid_mod, row_map != nullptr, c_bf16, "k_gemm256q", bm);
            int rc = 0;
            if (resid) rc = launch_gemm256q<false, 0, true, 0>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, resid, ldr, C, ldc, M, N, K, t2n, tqm, 1.f, 1.f);
            else if (!c_bf16) rc = launch_gemm256q<false, 0, false, 0>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, resid, ldr, C, ldc, M, N, K, t2n, tqm, 1.f, 1.f);
            else if (act == 0) rc = launch_gemm256q<true, 0, false, 0>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, resid, ldr, C, ldc, M, N, K, t2n, tqm, 1.f, 1.f);
            else rc = launch_gemm256q<true, 1, false, 0>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, resid, ldr, C, ldc, M, N, K, t2n, tqm, 1.f, 1.f);
            return rc;
        }
        gemm_log(M, N, K, act, resid != nullptr, resid_mod, row_map != nullptr, c_bf16, "k_gemm256p", 256);
#define GEMM2(OB, AC) launch_gemm256<OB, AC>(cfg, grid2, bf_stream(stream), A, lda, W, ldw, bias, \
                                            resid, ldr, resid_mod, C, ldc, row_map, M, N, K, t2n, t2m)
        if (c_bf16) {
            if (act == 0) GEMM2(true, 0);
            else if (act == 1) GEMM2(true, 1);
            else GEMM2(true, 2);
        } else {
            if (act == 0) GEMM2(false, 0);
            else if (act == 1) GEMM2(false, 1);
            else GEMM2(false, 2);
        }
#undef GEMM2
        return bf_check_launch();
    }
    gemm_log(M, N, K, act, resid != nullptr, resid_mod, row_map != nullptr, c_bf16, "k_gemm", 128);
#define GEMM_LAUNCH(OB, AC)                                                                       \
    hipLaunchKernelGGL((k_gemm<OB, AC>), dim3(nwg), dim3(G_THREADS), lds, bf_stream(stream),       \
                       (const u16*)A, lda, (const u16*)W, ldw, bias, resid, ldr, resid_mod, C, ldc, \
                       row_map, M, N, K, tiles_n, tiles_m, vec_epi)
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

// ------------------------------------------------------------------------------------------
// fp8 e4m3 GEMM (CLIP ViT-H fp8 path, BASELINE configs[4]): C = act(A W^T * scale + bias[n])
// (+ resid), A [M,K] and W [N,K] fp8 (row strides in elements = bytes), scale = activation scale x
// weight scale (per-tensor both).  out_kind 0: f32 C (optionally + resid, in place allowed),
// 1: bf16 C, 2: fp8 C = sat448(value * out_qscale).  The persistent 256x256 kernel only.
// ------------------------------------------------------------------------------------------
template <bool OB, int AC, int F8>
static void launch_gemm256_f8(int gm, int grid, hipStream_t st, const void* A, int lda, const void* W, int ldw,
                              float csc, const float* bias, const float* resid, int ldr, void* C,
                              int ldc, float oqs, int M, int N, int K, int tiles_n, int tiles_m) {
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_gemm256p<OB, AC, F8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            G2_LDS);
        attr = true;
    }
    hipLaunchKernelGGL((k_gemm256p<OB, AC, F8>), dim3(grid), dim3(G2_THREADS), G2_LDS, st, (const u16*)A,
                       lda, (const u16*)W, ldw, bias, resid, ldr, 0, C, ldc, (const int32_t*)nullptr, M, N,
                       K, tiles_n, tiles_m, 1, gm, 0, csc, oqs);
}

BF_API int bf_gemm_fp8_plan(const void* A, int lda, const void* W, int ldw, float scale,
                            const float* bias, const float* resid, int ldr, void* C, int ldc, int out_kind,
                            float out_qscale, int M, int N, int K, int act, const bf_gemm_plan* plan,
                            void* stream) {
    const GemmCfg cfg = gemm_cfg(plan);
    if (!A || !W || !C || !(scale > 0.f) || M < 0 || N <= 0 || K <= 0 || act < 0 || act > 1 ||
        out_kind < 0 || out_kind > 2)
        return BF_ERR_ARG;
    if (K % 128 != 0 || lda % 16 != 0 || ldw % 16 != 0) return BF_ERR_UNSUPPORTED;
    if (resid && (out_kind != 0 || (uintptr_t)resid % 16 != 0 || ldr % 4 != 0)) return BF_ERR_UNSUPPORTED;
    if (out_kind == 0 && (N % 4 || ldc % 4 || (uintptr_t)C % 16)) return BF_ERR_UNSUPPORTED;
    if (out_kind == 1 && (N % 8 || ldc % 8 || (uintptr_t)C % 16)) return BF_ERR_UNSUPPORTED;
    if (out_kind == 2 && (N % 8 || ldc % 8 || (uintptr_t)C % 8)) return BF_ERR_UNSUPPORTED;
    if (M == 0) return BF_OK;
    if ((long long)(M - 1) * lda + K >= (1LL << 31) || (long long)(N - 1) * ldw + K >= (1LL << 31))
        return BF_ERR_CAPACITY;
    const int t2m = (M + 255) / 256, t2n = (N + 255) / 256;
    const long long t2 = (long long)t2m * t2n;
    const int grid = gemm_grid(t2, cfg);
    // the overlapped-epilogue kernel for the fp8 GEMMs with bf16 outputs (CLIP qkv: 203.0 -> 161.4
    // us); fp8 outputs only under variant 6 (CLIP fc1 + GELU -> fp8 measured 286.7 -> 303.7 us on it:
    // at the fp8 MFMA rate the K loop is short beside that epilogue's VALU work)
    if ((cfg.variant == 6 || (cfg.variant == 5 && out_kind == 1)) && !resid && out_kind != 0 && K / 128 >= 3 &&
        N <= G2Q_BIAS_MAX && (long long)(M - 1) * ldc * (out_kind == 1 ? 2 : 1) + (long long)N * 2 < (1LL << 31)) {
        const int mb1 = gemm_tile_mb1(M, N, K, cfg);
        const int bm = 2 * (64 + 16 * mb1);
        const int tqm = (M + bm - 1) / bm;
        const int gq = gemm_grid((long long)tqm * t2n, cfg);
        if (out_kind == 1) {
            if (act == 0) return launch_gemm256q<true, 0, false, 1>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, nullptr, 0, C, ldc, M, N, K, t2n, tqm, scale, out_qscale);
            return launch_gemm256q<true, 1, false, 1>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, nullptr, 0, C, ldc, M, N, K, t2n, tqm, scale, out_qscale);
        }
        if (act == 0) return launch_gemm256q<true, 0, false, 3>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, nullptr, 0, C, ldc, M, N, K, t2n, tqm, scale, out_qscale);
        return launch_gemm256q<true, 1, false, 3>(mb1, cfg.group_m, gq, stream, A, lda, W, ldw, bias, nullptr, 0, C, ldc, M, N, K, t2n, tqm, scale, out_qscale);
    }
#define GEMM8(OB, AC, F8) launch_gemm256_f8<OB, AC, F8>(cfg.group_m, grid, bf_stream(stream), A, lda, W, ldw, scale, bias, \
                                                         resid, ldr, C, ldc, out_qscale, M, N, K, t2n, t2m)
    if (out_kind == 0) {
        if (act != 0) return BF_ERR_UNSUPPORTED;   // (f32 GELU output: not on the path)
        GEMM8(false, 0, 1);
    } else if (out_kind == 1) {
        if (act == 0) GEMM8(true, 0, 1);
        else GEMM8(true, 1, 1);
    } else {
        if (act == 0) GEMM8(true, 0, 3);
        else GEMM8(true, 1, 3);
    }
#undef GEMM8
    return bf_check_launch();
}

BF_API int bf_gemm_bf16(const void* A, int lda, const void* W, int ldw, const float* bias,
                        const float* resid, int ldr, int resid_mod, void* C, int ldc, int c_bf16,
                        const int32_t* row_map, int M, int N, int K, int act, void* stream) {
    return bf_gemm_bf16_plan(A, lda, W, ldw, bias, resid, ldr, resid_mod, C, ldc, c_bf16, row_map, M, N, K, act,
                             nullptr, stream);
}

BF_API int bf_gemm_fp8(const void* A, int lda, const void* W, int ldw, float scale,
                       const float* bias, const float* resid, int ldr, void* C, int ldc, int out_kind,
                       float out_qscale, int M, int N, int K, int act, void* stream) {
    return bf_gemm_fp8_plan(A, lda, W, ldw, scale, bias, resid, ldr, C, ldc, out_kind, out_qscale, M, N, K, act,
                            nullptr, stream);
}
