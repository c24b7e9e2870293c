// bf_attn.hip — fused multi-head attention (flash-style online softmax) on gfx950 MFMA.
//
// Used for CuTR's joint RGB+depth window attention (vit.py:170-203: 512 keys per window, the
// row softmax spans all concatenated keys, so it is exact joint attention), its global blocks
// (1600 tokens), and CLIP ViT-H/14 (257 tokens, head_dim 80).
//
// Element (b, h, s, d) of X in {Q, K, V, O} lives at X + b*x_bs + s*x_rs + h*D + d (token-major,
// straight out of / into the QKV and proj GEMMs; no transposes in HBM).
//
// Structure (per 256-thread workgroup = 4 wave64, 128 queries, one (batch, head)):
//   * each wave owns 32 queries; Q^T fragments stay in registers for the whole key loop;
//   * key tiles of 64: K tile [64][D] and V^T tile [D][64] staged in LDS (V transposed once at
//     staging so the P.V operand is read as two 8-byte runs per lane);
//   * S^T = K Q^T via v_mfma_f32_32x32x16_bf16 -> the query sits on the lane, keys in the 16
//     accumulator registers (+ the lane half), so the row max/sum is an in-lane reduction plus one
//     cross-half exchange, and the rescale of O^T is a per-lane scalar;
//   * the S^T accumulator, converted to bf16, is directly the B operand of O^T = V^T P^T (the
//     k-order permutation of the 32x32x16 accumulator is mirrored in the V^T reads);
//   * softmax in f32 with exp2 (scale*log2e folded), O normalised once at the end.
#include "bf_common.h"

#include <type_traits>
#include <climits>
#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

#define AT_THREADS 256
#define AT_QT 128
#define AT_KT 64

struct alignas(16) V128 {
    uint32_t x, y, z, w;
};
struct alignas(8) V64 {
    uint32_t x, y;
};

__device__ __forceinline__ u16 at_f2bf(float f) {
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<u16*>(&b);
}

// element offset of output row (batch b, query q): b*o_bs + q*o_rs, or through o_map (row
// o_map[b*sq + q] of O, < 0 = not stored): the window attention writes its rows straight back in
// token order, pad queries dropped, so the proj GEMM runs on the real rows only
__device__ __forceinline__ long long attn_out_offset(const int32_t* __restrict__ o_map, int b, int q,
                                                     int sq, long long o_bs, int o_rs) {
    if (!o_map) return b * o_bs + (long long)q * o_rs;
    if (q >= sq) return -1;
    const int r = o_map[(long long)b * sq + q];
    return r < 0 ? -1 : (long long)r * o_rs;
}

// NW waves of 32 queries per workgroup; NT key tiles resident in LDS at once: NT == 1 streams
// the keys tile by tile, NT > 1 (short sequences, sk <= 64*NT) stages every key and V^T column
// of the (batch, head) once and runs the whole key loop without barriers.
template <int D, int NW, int NT>
__global__ void __launch_bounds__(NW * 64) k_attn(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                     const u16* __restrict__ V, u16* __restrict__ O,
                                                     int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                     int o_rs, long long q_bs, long long k_bs,
                                                     long long v_bs, long long o_bs, float scale_log2,
                                                     const int32_t* __restrict__ o_map) {
    constexpr int KS = D / 16;            // k16 steps over the head dim
    constexpr int DB = (D + 31) / 32;     // 32-row blocks of O^T
    constexpr int DP = DB * 32;           // padded head dim (V^T rows)
    constexpr int KROW = D + 8;           // K tile row stride (elements), 16-B aligned, de-banked
    constexpr int VROW = NT * AT_KT + 8;  // V^T row stride (elements)
    __shared__ __attribute__((aligned(16))) u16 sK[NT * AT_KT * KROW];
    __shared__ __attribute__((aligned(16))) u16 sV[DP * VROW];

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int h = blockIdx.y, b = blockIdx.z;
    const int fr = lane & 31, fh = lane >> 5;
    const int q = blockIdx.x * (NW * 32) + wave * 32 + fr;  // this lane's query
    const u16* Qb = Q + b * q_bs + h * D;
    const u16* Kb = K + b * k_bs + h * D;
    const u16* Vb = V + b * v_bs + h * D;

    // Q^T fragments (B operand): element j of k-step ks = Q[q][16ks + 8fh + j]
    bf16x8 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        qf[ks] = *reinterpret_cast<const bf16x8*>(Qb + (size_t)min(q, sq - 1) * q_rs + 16 * ks + 8 * fh);
    }
    // zero the padded V^T rows once (only matter for D % 32 != 0)
    for (int i = t; i < (DP - D) * VROW; i += NW * 64) sV[D * VROW + i] = 0;

    f32x16 o[DB];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    for (int k0 = 0; k0 < sk; k0 += AT_KT) {
      // LDS key offset of this tile: 0 when streaming, k0 when every tile is resident
      const int kl = (NT == 1) ? 0 : k0;
      if (NT == 1 || k0 == 0) {
        const int k0s = (NT == 1) ? k0 : 0;
        __syncthreads();
        // ---- stage K tile(s) (row-major) ---------------------------------------------------
        constexpr int KCH = NT * AT_KT * D / 8;  // 16-B chunks
        for (int c = t; c < KCH; c += NW * 64) {
            int r = c / (D / 8), cc = c % (D / 8);
            V128 v = *reinterpret_cast<const V128*>(Kb + (size_t)min(k0s + r, sk - 1) * k_rs + cc * 8);
            if (k0s + r >= sk) v.x = v.y = v.z = v.w = 0u;
            *reinterpret_cast<V128*>(sK + r * KROW + cc * 8) = v;
        }
        // ---- stage V^T tile: thread handles 4 keys x 8 dims, writes 8 x (4 keys) ------------
        constexpr int VTASK = (NT * AT_KT / 4) * (D / 8);
        for (int c = t; c < VTASK; c += NW * 64) {
            int kq = c / (D / 8), dq = c % (D / 8);
            V128 rv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int key = k0s + kq * 4 + i;
                V128 v = *reinterpret_cast<const V128*>(Vb + (size_t)min(key, sk - 1) * v_rs + dq * 8);
                if (key >= sk) v.x = v.y = v.z = v.w = 0u;
                rv[i] = v;
            }
#define VT_WORD(i, j) ((((j) >> 1) == 0 ? rv[i].x : ((j) >> 1) == 1 ? rv[i].y : ((j) >> 1) == 2 ? rv[i].z : rv[i].w) >> (16 * ((j) & 1)) & 0xffffu)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                V64 w;
                w.x = VT_WORD(0, j) | (VT_WORD(1, j) << 16);
                w.y = VT_WORD(2, j) | (VT_WORD(3, j) << 16);
                *reinterpret_cast<V64*>(sV + (dq * 8 + j) * VROW + kq * 4) = w;
            }
#undef VT_WORD
        }
        __syncthreads();
      }

        // ---- S^T = K Q^T for two 32-key sub-tiles ------------------------------------------
        f32x16 s[2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
            for (int e = 0; e < 16; ++e) s[sub][e] = 0.f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                bf16x8 kf = *reinterpret_cast<const bf16x8*>(sK + (kl + sub * 32 + fr) * KROW + 16 * ks + 8 * fh);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[sub], 0, 0, 0);
            }
        }
        // ---- online softmax (query = lane column, keys = registers + lane half) -------------
        float mt = -INFINITY;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                int key = k0 + sub * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
                float v = (key < sk) ? s[sub][e] * scale_log2 : -INFINITY;
                s[sub][e] = v;
                mt = fmaxf(mt, v);
            }
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float m_new = fmaxf(m_run, mt);
        const float alpha = exp2f(m_run - m_new);  // m_run = -inf -> 0
        float ls = 0.f;
        bf16x8 pf[2][2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                float p = exp2f(s[sub][e] - m_new);
                ls += p;
                pf[sub][e >> 3][e & 7] = (__bf16)p;
            }
        ls += __shfl_xor(ls, 32, 64);
        l_run = l_run * alpha + ls;
        m_run = m_new;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[db][e] *= alpha;
        // ---- O^T += V^T P^T ------------------------------------------------------------------
        // A element j (lane row r = d, half fh) = V^T[d][key = 32sub + 16s + 8(j>>2) + 4fh + (j&3)]
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const u16* vrow = sV + (db * 32 + fr) * VROW;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const int kb = kl + 32 * sub + 16 * ss + 4 * fh;
                    V64 lo = *reinterpret_cast<const V64*>(vrow + kb);
                    V64 hi = *reinterpret_cast<const V64*>(vrow + kb + 8);
                    bf16x8 vf;
                    V128 pk = {lo.x, lo.y, hi.x, hi.y};
                    vf = *reinterpret_cast<bf16x8*>(&pk);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[sub][ss], o[db], 0, 0, 0);
                }
        }
    }
    // ---- normalise and store O[q][h*D + d] (4 consecutive d per register group) -------------
    const long long o_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
    if (q < sq && o_off >= 0) {
        const float inv = 1.0f / l_run;
        u16* orow = O + o_off + h * D;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d0 = db * 32 + 8 * g + 4 * fh;
                if (d0 >= D) continue;
                V64 w;
                w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                *reinterpret_cast<V64*>(orow + d0) = w;
            }
    }
}

// ------------------------------------------------------------------------------------------
// Streaming variant (k_attn_s): K/V pass through a double-buffered LDS ring of 64-key tiles.
// The global loads of tile t+1 are issued into registers before tile t's MFMAs and written to
// the other buffer after them (one barrier per tile), so HBM latency overlaps the compute.
// V stays row-major ([key][VROW], VROW*2 = 64 or 192 mod 256 bytes so the 4 rows of one
// transposed read land in disjoint banks) and the A operand of O^T = V^T P^T is read with
// ds_read_b64_tr_b16: per 16-lane group a 4-key x 16-column block arrives column-major, two such
// reads (keys base..base+3 and base+8..base+11) form the 32x32x16 fragment in the k order of the
// S^T accumulator.  K rows are padded to D+8 elements (conflict-free ds_read_b128 fragments).
// ------------------------------------------------------------------------------------------
typedef short s16x4 __attribute__((ext_vector_type(4)));

// Online-softmax step over one 64-key tile held as S^T (raw scores, query on the lane, keys in
// the accumulator registers + lane half): returns the bf16 P^T fragments and rescales O^T.
//  * the score scale (scale * log2 e) is folded into the exponent: p = 2^(s*c - m), m = max(s)*c,
//    one FMA per element; the raw v_exp_f32 is enough (arguments <= 0; results below 2^-126 do
//    not change an f32 row sum of terms >= 1)
//  * keys past sk are masked only on the tile that has them
template <int DB>
__device__ __forceinline__ void attn_softmax_tile(f32x16 (&s)[2], int k0, int sk, int fh, float c,
                                                  float& m_run, float& l_run, f32x16 (&o)[DB],
                                                  bf16x8 (&pf)[2][2]) {
    if (k0 + AT_KT > sk) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int key = k0 + sub * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
                s[sub][e] = (key < sk) ? s[sub][e] : -INFINITY;
            }
    }
    float mt = s[0][0];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int e = 0; e < 16; ++e) mt = fmaxf(mt, s[sub][e]);
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float m_new = fmaxf(m_run, mt * c);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);   // m_run = -inf -> 0
    float ls = 0.f;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[sub][e], c, -m_new));
            ls += p;
            pf[sub][e >> 3][e & 7] = (__bf16)p;
        }
    ls += __shfl_xor(ls, 32, 64);
    l_run = l_run * alpha + ls;
    m_run = m_new;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] *= alpha;
}

// XCD-aware block order: consecutive workgroup ids land on different XCDs (id % 8 names the
// XCD group), so the blocks of one XCD are given a contiguous range of (query block, head, batch)
// -- the query blocks of one head (same K / V) and the neighbouring heads of one token row (the
// same 128-B lines when 2*D is not a multiple of 128, e.g. CLIP's D = 80) then meet in that XCD's
// L2 instead of being fetched once per XCD.  Bijective for any grid size.
struct AttnBlk {
    int qb, h, b;
};
__device__ __forceinline__ AttnBlk attn_block(int remap) {
    const unsigned nx = gridDim.x, ny = gridDim.y, nz = gridDim.z;
    if (!remap) return AttnBlk{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const unsigned n = nx * ny * nz;
    const unsigned id = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    const unsigned xcd = id % 8u, k = id / 8u, q = n / 8u, r = n % 8u;
    const unsigned lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
    return AttnBlk{(int)(lin % nx), (int)((lin / nx) % ny), (int)(lin / (nx * ny))};
}

__host__ __device__ constexpr int attn_vrow_bytes(int d) {
    int sb = 2 * d;
    while (sb % 256 != 64 && sb % 256 != 192) sb += 32;
    return sb;
}

template <int D, int NW>
__global__ void __launch_bounds__(NW * 64) k_attn_s(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                       const u16* __restrict__ V, u16* __restrict__ O,
                                                       int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                       int o_rs, long long q_bs, long long k_bs,
                                                       long long v_bs, long long o_bs, float scale_log2,
                                                     const int32_t* __restrict__ o_map, int remap) {
    constexpr int KS = D / 16;
    constexpr int DB = (D + 31) / 32;
    constexpr int KROW = D + 8;
    constexpr int VROW = attn_vrow_bytes(D) / 2;
    constexpr int KTILE = AT_KT * KROW;
    constexpr int VTILE = AT_KT * VROW;
    constexpr int CPR = D / 8;                       // 16-B chunks per row
    constexpr int CH = AT_KT * CPR;                  // chunks per operand tile
    constexpr int NT = NW * 64;
    __shared__ __attribute__((aligned(16))) u16 sK[2 * KTILE];
    __shared__ __attribute__((aligned(16))) u16 sV[2 * VTILE];

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const AttnBlk blk = attn_block(remap);
    const int h = blk.h, b = blk.b;
    const int fr = lane & 31, fh = lane >> 5;
    const int q = blk.qb * (NW * 32) + wave * 32 + fr;
    const u16* Qb = Q + b * q_bs + h * D;
    const u16* Kb = K + b * k_bs + h * D;
    const u16* Vb = V + b * v_bs + h * D;

    bf16x8 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
        qf[ks] = *reinterpret_cast<const bf16x8*>(Qb + (size_t)min(q, sq - 1) * q_rs + 16 * ks + 8 * fh);
    // padded V columns (read by the last 32-row block of O^T when D % 32 != 0): zero once
    if (VROW > D)
        for (int i = t; i < 2 * AT_KT * (VROW - D); i += NT) {
            const int r = i / (VROW - D), c = i % (VROW - D);
            sV[r * VROW + D + c] = 0;
        }

    // staging: thread t moves chunk c = t + i*NT (key row c / CPR, 16-B column c % CPR) of both
    // the K and the V tile; row / column computed once, per tile only the key clamp and two
    // addresses.  CH and NT are multiples of 64, so the i-guard is wave-uniform.
    static_assert(CH % 64 == 0 && NT % 64 == 0, "wave-uniform staging guard");
    constexpr int NSO = (CH + NT - 1) / NT;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 stk[NSO], stv[NSO];
    int srow[NSO], scol[NSO];
#pragma unroll
    for (int i = 0; i < NSO; ++i) {
        const int c = min(t + i * NT, CH - 1);
        srow[i] = c / CPR;
        scol[i] = (c % CPR) * 8;
    }
#define ATS_LOAD(k0_)                                                                             \
    _Pragma("unroll") for (int i = 0; i < NSO; ++i) {                                            \
        const int key = min((k0_) + srow[i], sk - 1);                                             \
        stk[i] = *reinterpret_cast<const u32x4*>(Kb + (size_t)key * k_rs + scol[i]);              \
        stv[i] = *reinterpret_cast<const u32x4*>(Vb + (size_t)key * v_rs + scol[i]);              \
    }
#define ATS_STORE(buf_)                                                                           \
    _Pragma("unroll") for (int i = 0; i < NSO; ++i) {                                            \
        if (t + i * NT < CH) {                                                                    \
            *reinterpret_cast<u32x4*>(sK + (buf_) * KTILE + srow[i] * KROW + scol[i]) = stk[i];   \
            *reinterpret_cast<u32x4*>(sV + (buf_) * VTILE + srow[i] * VROW + scol[i]) = stv[i];   \
        }                                                                                         \
    }

    f32x16 o[DB];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;

    // transposed-read lane roles: 16-lane group (d half g16), row q4 / column quad p4 of the block
    const int g16 = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int ntiles = (sk + AT_KT - 1) / AT_KT;
    ATS_LOAD(0);
    ATS_STORE(0);
    __syncthreads();
    for (int tile = 0; tile < ntiles; ++tile) {
        const int k0 = tile * AT_KT, buf = tile & 1;
        const bool more = tile + 1 < ntiles;
        if (more) { ATS_LOAD(k0 + AT_KT); }              // in flight during this tile
        const u16* kt = sK + buf * KTILE;
        const u16* vt = sV + buf * VTILE;
        // a last tile whose keys all fall in the first 32 (CLIP: 257 = 4*64 + 1) skips the second
        // sub-tile's MFMAs: its scores would be masked to -inf, its probabilities exactly 0
        const bool sub1 = k0 + 32 < sk;
        // ---- S^T = K Q^T for two 32-key sub-tiles ------------------------------------------
        f32x16 s[2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            if (sub == 1 && !sub1) {
#pragma unroll
                for (int e = 0; e < 16; ++e) s[1][e] = -INFINITY;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (sub * 32 + fr) * KROW + 16 * ks + 8 * fh);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], ks == 0 ? f32x16{} : s[sub], 0, 0, 0);
            }
        }
        // ---- online softmax ----------------------------------------------------------------
        bf16x8 pf[2][2];
        attn_softmax_tile<DB>(s, k0, sk, fh, scale_log2, m_run, l_run, o, pf);
        // ---- O^T += V^T P^T, V^T fragments by transposed reads -------------------------------
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const int d0 = db * 32 + g16 * 16 + 4 * p4;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    if (sub == 1 && !sub1) continue;
                    const int kb = 32 * sub + 16 * ss + 4 * fh + q4;
                    typedef __attribute__((address_space(3))) s16x4* lds_s4;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s4)(vt + kb * VROW + d0));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s4)(vt + (kb + 8) * VROW + d0));
                    typedef short s16x8 __attribute__((ext_vector_type(8)));
                    const s16x8 lohi = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    const bf16x8 vf = __builtin_bit_cast(bf16x8, lohi);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[sub][ss], o[db], 0, 0, 0);
                }
        }
        if (more) { ATS_STORE(buf ^ 1); }
        __syncthreads();
    }
    const long long o_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
    if (q < sq && o_off >= 0) {
        const float inv = 1.0f / l_run;
        u16* orow = O + o_off + h * D;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d0 = db * 32 + 8 * g + 4 * fh;
                if (d0 >= D) continue;
                V64 w;
                w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                *reinterpret_cast<V64*>(orow + d0) = w;
            }
    }
}

#undef ATS_LOAD
#undef ATS_STORE

// ------------------------------------------------------------------------------------------
// k_attn2: the streaming structure of k_attn_s, restructured for the VALU budget of short heads
//   * full 64-key tiles run a branch-free body (no masks, both 32-key sub-tiles); only the tail
//     tile (sk % 64 keys, CLIP: 1 key of 257) runs the masked body, with its empty sub-tile off
//   * deferred max (RESCALE_THRESHOLD, cdna_hip_programming.md T13): O^T and l are rescaled only
//     when a row's max grows by more than 2^8 in the exp2 domain (wave-uniform decision, taken
//     before the tile's P is formed, so everything at the old max is scaled exactly once);
//     P <= 2^8 then, which bf16 P and f32 O hold with no loss
//   * D % 32 != 0 (CLIP D = 80): the zero padding rows of V^T become a ones row at d = D, so the
//     P.V MFMA produces the row sum l in O^T's row D (the sum of the same bf16 P the numerator
//     uses) and the 32 per-tile adds disappear
//   * XCD-aware block order (attn_block)
// ------------------------------------------------------------------------------------------
#define AT2_THR 8.0f

template <int D, int DB, bool ONES>
__device__ __forceinline__ void attn2_softmax(f32x16 (&s)[2], bool sub1, bool mask, int k0, int sk,
                                              int fh, float c, float& m_run, float& l_run,
                                              f32x16 (&o)[DB], bf16x8 (&pf)[2][2], int kmax = INT_MAX) {
    // keys past sk (the tail tile) and, for causal attention, keys after the lane's query (kmax)
    if (mask) {
        const int klim = min(sk - 1, kmax);
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int key = k0 + sub * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
                s[sub][e] = (key <= klim) ? s[sub][e] : -INFINITY;
            }
    }
    float mt = s[0][0];
#pragma unroll
    for (int e = 1; e < 16; ++e) mt = fmaxf(mt, s[0][e]);
    if (sub1) {
#pragma unroll
        for (int e = 0; e < 16; ++e) mt = fmaxf(mt, s[1][e]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * c;
    // rescale only when some row's max grew by more than the threshold (wave-uniform)
    if (__any(mt > m_run + AT2_THR)) {
        const float m_new = fmaxf(m_run, mt);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);   // m_run = -inf -> 0
        m_run = m_new;
        l_run *= alpha;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[db][e] *= alpha;
    }
    float ls = 0.f;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
        if (sub == 1 && !sub1) {
#pragma unroll
            for (int e = 0; e < 16; ++e) pf[1][e >> 3][e & 7] = (__bf16)0.0f;
            continue;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[sub][e], c, -m_run));
            if (!ONES) ls += p;
            pf[sub][e >> 3][e & 7] = (__bf16)p;
        }
    }
    if (!ONES) l_run += ls;
}

// F8O: the output is fp8 e4m3 (OCP), saturate_448(o * oqs) -- the fp8 CLIP path's out_proj input
// CAUSAL: query q sees keys 0..q only (the CLIP text tower's attn_mask); every tile runs the masked
// body, tiles past the workgroup's last query are skipped (sq == sk)
// XQ (short heads with sq = 32 NW + 1, CLIP's 257 tokens): NW = 8 waves take queries 0..255 on
// MFMA (two waves per SIMD instead of a ninth wave holding one real query on one SIMD), and the
// last query runs beside them in f32 VALU while each K/V tile is in LDS: wave w scores keys
// 8w..8w+7 of the tile (lane group of 8 = one key, D/8 dims per lane), keeps its own online
// softmax (m, l, o[D]); the eight partial states merge through LDS after the loop.
// LW (light last wave, short heads with sq = 32 (NW - 1) + 1..16, CLIP's 257 tokens): waves 0..NW-2
// take queries 0..32 (NW - 1) - 1 on 32x32x16 MFMAs; the last wave takes only the next 16 queries on
// v_mfma_f32_16x16x32_bf16 (S^T = K Q^T in four 16-key blocks, O^T += V^T P^T in 16-row blocks with
// the same transposed V reads and the ones row), i.e. half the MFMA cycles of a full 32-query wave
// on the SIMD that holds three waves.  Its accumulators alias the registers of o / qf / s.
// (3- and 5-wave workgroups of short heads -- several per CU -- are held to 3 waves per SIMD, as
// the 9-wave workgroup is by its size: without it they compile to one wave per SIMD)
// PP (variant 12, measured slower: CLIP 153.1 vs 124.2 us; 168 VGPRs with 20 spilled, and five
// staging waves instead of nine).  Ping-pong for short non-causal heads: waves 4-7 run every tile's chain rotated by half a tile
// -- softmax and P.V of tile n-1, then S^T of tile n, whose scores they carry across the barrier --
// while the other waves run S^T, softmax, P.V of tile n.  Waves w and w + 4 share a SIMD, so one
// of them issues MFMAs while the other runs its softmax instead of both doing the same kind of
// work between two barriers.  K / V ring of three tiles (P.V of tile n-1 reads V n-1 while tile
// n + 1 is staged).  Arithmetic per query is unchanged (bit-identical to the default).
template <int D, int NW, bool F8O = false, bool CAUSAL = false, bool XQ = false, bool LW = false,
          bool PP = false, bool LSTQ = false>
__global__ void __launch_bounds__(NW * 64, (NW == 3 || NW == 5) ? 3 : 1) k_attn2(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                      const u16* __restrict__ V, u16* __restrict__ O,
                                                      int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                      int o_rs, long long q_bs, long long k_bs,
                                                      long long v_bs, long long o_bs, float scale_log2,
                                                      const int32_t* __restrict__ o_map, float oqs = 1.f) {
    constexpr int KS = D / 16;
    constexpr int DB = (D + 31) / 32;
    constexpr bool ONES = (D % 32) != 0;                 // a padding row of V^T carries the row sum
    constexpr int KROW = D + 8;
    constexpr int VROW = attn_vrow_bytes(D) / 2;
    constexpr int KTILE = AT_KT * KROW;
    constexpr int VTILE = AT_KT * VROW;
    constexpr int CPR = D / 8;
    constexpr int CH = AT_KT * CPR;
    constexpr int NT = NW * 64;
    constexpr int NBUF = PP ? 3 : 2;
    static_assert(!PP || (!CAUSAL && !XQ && !LW && NW > 4), "PP: short non-causal heads");
    __shared__ __attribute__((aligned(16))) u16 sK[NBUF * KTILE];
    __shared__ __attribute__((aligned(16))) u16 sV[NBUF * VTILE];
    // LST (the default for one-workgroup short heads): the bf16 output rows go through a per-wave
    // LDS region of their own and leave as whole 2D-byte head rows (16 B per lane along the row)
    // instead of 8-byte fragments of 32 rows per store instruction (CLIP: 122.8 -> 115.8 us)
    // (9-wave workgroups: an LDS region of their own, free at one workgroup per CU; 4-wave ones
    // reuse the K ring after a barrier, so their occupancy is unchanged)
    constexpr bool LST = LSTQ && !XQ && !LW && !CAUSAL && D % 16 == 0;
    constexpr int EB = F8O ? 1 : 2;                                 // output bytes per element
    constexpr int OROW = ((EB * D + 16) / 32) * 32 + 16;           // bytes per staged row (16-B aligned)
    constexpr bool OWN = NW == 9;
    static_assert(!LST || OWN || NW * 32 * OROW <= NBUF * KTILE * 2, "staged rows fit the K ring");
    __shared__ __attribute__((aligned(16))) unsigned char sO[LST && OWN ? NW * 32 * OROW : 16];

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const AttnBlk blk = attn_block(1);
    const int h = blk.h, b = blk.b;
    const int fr = lane & 31, fh = lane >> 5;
    static_assert(!LW || (ONES && !CAUSAL && !XQ && D % 16 == 0), "LW: short non-causal heads, D % 32 != 0");
    constexpr int QPB = LW ? (NW - 1) * 32 + 16 : NW * 32;      // queries per workgroup
    const bool light = LW && wave == NW - 1;                    // wave-uniform
    const int c16 = lane & 15, g4 = lane >> 4;
    const int q = blk.qb * QPB + (light ? (NW - 1) * 32 + c16 : wave * 32 + fr);
    const u16* Qb = Q + b * q_bs + h * D;
    const u16* Kb = K + b * k_bs + h * D;
    const u16* Vb = V + b * v_bs + h * D;

    // the light wave's 16x16x32 operands: Q^T columns = its 16 queries, k = dims 32 ks + 8 g4 .. + 8
    constexpr int KS16 = (D + 31) / 32;
    bf16x8 qf[KS];
    if (light) {
#pragma unroll
        for (int ks = 0; ks < KS16; ++ks) {
            const int d0 = 32 * ks + 8 * g4;
            qf[ks] = d0 < D ? *reinterpret_cast<const bf16x8*>(Qb + (size_t)min(q, sq - 1) * q_rs + d0) : bf16x8{};
        }
    } else {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            qf[ks] = *reinterpret_cast<const bf16x8*>(Qb + (size_t)min(q, sq - 1) * q_rs + 16 * ks + 8 * fh);
    }
    // V padding columns: a ones column at d = D (the row sum), zeros after it
    if (VROW > D)
        for (int i = t; i < NBUF * AT_KT * (VROW - D); i += NT) {
            const int r = i / (VROW - D), c = i % (VROW - D);
            sV[r * VROW + D + c] = (ONES && c == 0) ? (u16)0x3F80 : (u16)0;
        }

    static_assert(CH % 64 == 0 && NT % 64 == 0, "wave-uniform staging guard");
    // PP: only waves 0-3 and 8 stage K / V (the late waves carry their scores instead)
    constexpr int NTS = PP ? 5 * 64 : NT;
    const int ts = !PP ? t : (wave < 4 ? t : (wave == 8 ? 4 * 64 + lane : -1));
    constexpr int NSO = (CH + NTS - 1) / NTS;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 stk[NSO], stv[NSO];
    int srow[NSO], scol[NSO];
#pragma unroll
    for (int i = 0; i < NSO; ++i) {
        const int c = min(max(ts, 0) + i * NTS, CH - 1);
        srow[i] = c / CPR;
        scol[i] = (c % CPR) * 8;
    }
    auto stage_load = [&](int k0_) {
        if (PP && ts < 0) return;
#pragma unroll
        for (int i = 0; i < NSO; ++i) {
            const int key = min(k0_ + srow[i], sk - 1);
            stk[i] = *reinterpret_cast<const u32x4*>(Kb + (size_t)key * k_rs + scol[i]);
            stv[i] = *reinterpret_cast<const u32x4*>(Vb + (size_t)key * v_rs + scol[i]);
        }
    };
    auto stage_store = [&](int buf_) {
        if (PP && ts < 0) return;
#pragma unroll
        for (int i = 0; i < NSO; ++i) {
            if (ts + i * NTS < CH) {
                *reinterpret_cast<u32x4*>(sK + buf_ * KTILE + srow[i] * KROW + scol[i]) = stk[i];
                *reinterpret_cast<u32x4*>(sV + buf_ * VTILE + srow[i] * VROW + scol[i]) = stv[i];
            }
        }
    };

    f32x16 o[DB];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    const int g16 = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int ntiles = (sk + AT_KT - 1) / AT_KT;
    const int nfull = sk / AT_KT;

    // XQ: the last query's state (key group kg = lane / 8, dims dg * DPL .. + DPL)
    constexpr int DPL = D / 8;
    static_assert(!XQ || (D % 16 == 0 && NW == 8), "XQ: 8 waves, D a multiple of 16");
    const int kg = lane >> 3, dg = lane & 7;
    float xq[XQ ? DPL : 1], xo[XQ ? DPL : 1];
    float xm = -INFINITY, xl = 0.f;
    if constexpr (XQ) {
        const uint32_t* qr = reinterpret_cast<const uint32_t*>(Qb + (size_t)(sq - 1) * q_rs + dg * DPL);
#pragma unroll
        for (int j = 0; j < DPL / 2; ++j) {
            const uint32_t w2 = qr[j];
            xq[2 * j] = __uint_as_float(w2 << 16) * scale_log2;
            xq[2 * j + 1] = __uint_as_float(w2 & 0xFFFF0000u) * scale_log2;
        }
#pragma unroll
        for (int j = 0; j < DPL; ++j) xo[j] = 0.f;
    }
    auto extra_query = [&](const u16* kt, const u16* vt, int k0) {
        const int kk = wave * 8 + kg;
        const uint32_t* kr = reinterpret_cast<const uint32_t*>(kt + kk * KROW + dg * DPL);
        float sx = 0.f;
#pragma unroll
        for (int j = 0; j < DPL / 2; ++j) {
            const uint32_t w2 = kr[j];
            sx = fmaf(__uint_as_float(w2 << 16), xq[2 * j], sx);
            sx = fmaf(__uint_as_float(w2 & 0xFFFF0000u), xq[2 * j + 1], sx);
        }
        sx += __shfl_xor(sx, 1, 64);
        sx += __shfl_xor(sx, 2, 64);
        sx += __shfl_xor(sx, 4, 64);
        if (k0 + kk >= sk) sx = -INFINITY;
        float mt = fmaxf(sx, __shfl_xor(sx, 8, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        if (mt > xm) {                                   // wave-uniform
            const float alpha = __builtin_amdgcn_exp2f(xm - mt);
            xm = mt;
            xl *= alpha;
#pragma unroll
            for (int j = 0; j < DPL; ++j) xo[j] *= alpha;
        }
        const float pr = __builtin_amdgcn_exp2f(sx - xm);
        float ps = pr + __shfl_xor(pr, 8, 64);
        ps += __shfl_xor(ps, 16, 64);
        ps += __shfl_xor(ps, 32, 64);
        xl += ps;
        const uint32_t* vr = reinterpret_cast<const uint32_t*>(vt + kk * VROW + dg * DPL);
#pragma unroll
        for (int j = 0; j < DPL / 2; ++j) {
            const uint32_t w2 = vr[j];
            xo[2 * j] = fmaf(pr, __uint_as_float(w2 << 16), xo[2 * j]);
            xo[2 * j + 1] = fmaf(pr, __uint_as_float(w2 & 0xFFFF0000u), xo[2 * j + 1]);
        }
    };

    // one 64-key tile: S^T = K Q^T (qk), then softmax and O^T += V^T P^T (sm_pv; MASK: the tail tile)
    auto qk = [&](int tile, f32x16 (&s)[2], bool maybe_tail) {
        const int k0 = tile * AT_KT;
        const u16* kt = sK + (tile % NBUF) * KTILE;
        const bool sub1 = !maybe_tail || (k0 + 32 < sk);
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            if (sub == 1 && !sub1) {
#pragma unroll
                for (int e = 0; e < 16; ++e) s[1][e] = -INFINITY;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (sub * 32 + fr) * KROW + 16 * ks + 8 * fh);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], ks == 0 ? f32x16{} : s[sub], 0, 0, 0);
            }
        }
    };
    auto sm_pv = [&](int tile, f32x16 (&s)[2], auto mask_tag) {
        constexpr bool MASK = decltype(mask_tag)::value;
        const int k0 = tile * AT_KT;
        const u16* kt = sK + (tile % NBUF) * KTILE;
        const u16* vt = sV + (tile % NBUF) * VTILE;
        const bool sub1 = !MASK || (k0 + 32 < sk);
        bf16x8 pf[2][2];
        attn2_softmax<D, DB, ONES>(s, sub1, MASK, k0, sk, fh, scale_log2, m_run, l_run, o, pf,
                                   CAUSAL ? q : INT_MAX);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const int d0 = db * 32 + g16 * 16 + 4 * p4;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    if (MASK && sub == 1 && !sub1) continue;
                    const int kb = 32 * sub + 16 * ss + 4 * fh + q4;
                    typedef __attribute__((address_space(3))) s16x4* lds_s4;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + kb * VROW + d0));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + (kb + 8) * VROW + d0));
                    typedef short s16x8 __attribute__((ext_vector_type(8)));
                    const s16x8 lohi = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, lohi),
                                                                   pf[sub][ss], o[db], 0, 0, 0);
                }
        }
        if constexpr (XQ) extra_query(kt, vt, k0);
    };
    // LW: the light wave's tile.  S^T blocks: lane (c16, g4) holds query c16, keys 16 kb + 4 g4 + r;
    // O^T block i (rows d = 16 i .. + 16) lives in o[i / 4][4 (i % 4) + r], r < 4
    constexpr int NB16 = (D + 16) / 16;                          // D / 16 value blocks + the ones row
    static_assert(!LW || NB16 * 4 <= DB * 16, "LW: O^T blocks alias o");
    auto light_tile = [&](int tile, auto mask_tag) {
        constexpr bool MASK = decltype(mask_tag)::value;
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        const int k0 = tile * AT_KT;
        const u16* kt = sK + (tile % NBUF) * KTILE;
        const u16* vt = sV + (tile % NBUF) * VTILE;
        f32x4 sl[4];
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            sl[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS16; ++ks) {
                const int d0 = 32 * ks + 8 * g4;
                bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (kb * 16 + c16) * KROW + (d0 < D ? d0 : 0));
                if (d0 >= D) kf = bf16x8{};
                sl[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], sl[kb], 0, 0, 0);
            }
        }
        if (MASK) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (k0 + kb * 16 + 4 * g4 + r >= sk) sl[kb][r] = -INFINITY;
        }
        float mt = sl[0][0];
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
            for (int r = 0; r < 4; ++r) mt = fmaxf(mt, sl[kb][r]);
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * scale_log2;
        if (__any(mt > m_run + AT2_THR)) {
            const float m_new = fmaxf(m_run, mt);
            const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
            m_run = m_new;
#pragma unroll
            for (int i = 0; i < NB16; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) o[i >> 2][4 * (i & 3) + r] *= alpha;
        }
        // P^T as the B operand: k-slots 8 g4 + j = keys 32 ks + 4 g4 + j (j < 4), 32 ks + 16 + 4 g4 + j - 4
        bf16x8 pl[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                pl[ks][j] = (__bf16)__builtin_amdgcn_exp2f(fmaf(sl[2 * ks + (j >> 2)][j & 3], scale_log2, -m_run));
#pragma unroll
        for (int i = 0; i < NB16; ++i) {
            f32x4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = o[i >> 2][4 * (i & 3) + r];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                // per 16-lane group: rows 32 ks + 4 g4 + q4 (+ 16), columns 16 i + 4 p4 -> lane c16 gets
                // V^T row d = 16 i + c16 at those four keys
                typedef __attribute__((address_space(3))) s16x4* lds_s4;
                const u16* vb = vt + (32 * ks + 4 * g4 + q4) * VROW + 16 * i + 4 * p4;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)vb);
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vb + 16 * VROW));
                typedef short s16x8 __attribute__((ext_vector_type(8)));
                const s16x8 lohi = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, lohi), pl[ks], acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) o[i >> 2][4 * (i & 3) + r] = acc[r];
        }
    };
    auto tile_body = [&](int tile, auto mask_tag) {
        if constexpr (LW) {
            if (light) { light_tile(tile, mask_tag); return; }
        }
        f32x16 s[2];
        qk(tile, s, decltype(mask_tag)::value);
        sm_pv(tile, s, mask_tag);
    };

    stage_load(0);
    stage_store(0);
    __syncthreads();
    if constexpr (CAUSAL) {
        // keys beyond the workgroup's last query are masked for every row: stop there
        const int nt = min(ntiles, (min(blk.qb * (NW * 32) + NW * 32, sq) - 1) / AT_KT + 1);
        for (int tile = 0; tile < nt; ++tile) {
            const bool more = tile + 1 < nt;
            if (more) stage_load((tile + 1) * AT_KT);
            tile_body(tile, std::true_type{});
            if (more) stage_store((tile + 1) & 1);
            __syncthreads();
        }
    } else if constexpr (PP) {
        const bool late = wave >= 4 && wave < 8;                   // wave-uniform
        f32x16 sl[2];                                              // the late waves' pending scores
        for (int tile = 0; tile < nfull; ++tile) {
            const bool more = tile + 1 < ntiles;
            if (more) stage_load((tile + 1) * AT_KT);
            if (!late) {                 // (the same score registers as the late waves' carried ones)
                qk(tile, sl, false);
                sm_pv(tile, sl, std::false_type{});
            } else {
                if (tile > 0) sm_pv(tile - 1, sl, std::false_type{});
                qk(tile, sl, false);
            }
            if (more) stage_store((tile + 1) % NBUF);
            __syncthreads();
        }
        if (nfull < ntiles) {
            if (!late) {
                qk(nfull, sl, true);
                sm_pv(nfull, sl, std::true_type{});
            } else {
                if (nfull > 0) sm_pv(nfull - 1, sl, std::false_type{});
                qk(nfull, sl, true);
                sm_pv(nfull, sl, std::true_type{});
            }
        } else if (late && nfull > 0) {
            sm_pv(nfull - 1, sl, std::false_type{});
        }
    } else {
        for (int tile = 0; tile < nfull; ++tile) {
            const bool more = tile + 1 < ntiles;
            if (more) stage_load((tile + 1) * AT_KT);          // in flight during this tile
            tile_body(tile, std::false_type{});
            if (more) stage_store((tile + 1) % NBUF);
            __syncthreads();
        }
        if (nfull < ntiles) tile_body(nfull, std::true_type{});
    }
    if constexpr (XQ) {
        // merge the eight waves' partial states of the last query through LDS (sK is free now)
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
            xo[j] += __shfl_xor(xo[j], 8, 64);
            xo[j] += __shfl_xor(xo[j], 16, 64);
            xo[j] += __shfl_xor(xo[j], 32, 64);
        }
        __syncthreads();
        float* scr = reinterpret_cast<float*>(sK);
        constexpr int SW = D + 2;
        if (lane < 8) {
#pragma unroll
            for (int j = 0; j < DPL; ++j) scr[wave * SW + 2 + dg * DPL + j] = xo[j];
        }
        if (lane == 0) { scr[wave * SW] = xm; scr[wave * SW + 1] = xl; }
        __syncthreads();
        if (wave == 0) {
            float M = scr[0];
#pragma unroll
            for (int w = 1; w < NW; ++w) M = fmaxf(M, scr[w * SW]);
            float Ls = 0.f, wt[NW];
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                wt[w] = __builtin_amdgcn_exp2f(scr[w * SW] - M);
                Ls = fmaf(scr[w * SW + 1], wt[w], Ls);
            }
            const float inv = 1.0f / Ls;
            const long long xoff = attn_out_offset(o_map, b, sq - 1, sq, o_bs, o_rs);
            if (xoff >= 0) {
                for (int d = lane; d < D; d += 64) {
                    float acc = 0.f;
#pragma unroll
                    for (int w = 0; w < NW; ++w) acc = fmaf(scr[w * SW + 2 + d], wt[w], acc);
                    if constexpr (F8O) {
                        const float a = fminf(fmaxf(acc * inv * oqs, -448.f), 448.f);
                        const int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a, a, 0, false);
                        reinterpret_cast<unsigned char*>(O)[xoff + h * D + d] = (unsigned char)(pk & 0xFF);
                    } else {
                        O[xoff + h * D + d] = at_f2bf(acc * inv);
                    }
                }
            }
        }
    }

    if constexpr (LW) {
        if (light) {
            // row sum: O^T row D = block D / 16, row D % 16 -> lane group (D % 16) / 4, register D % 4
            constexpr int il = D / 16, rl = D % 16;
            const float ll = __shfl(o[il >> 2][4 * (il & 3) + (rl & 3)], (rl >> 2) * 16 + c16, 64);
            const long long lo_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
            if (q < sq && lo_off >= 0) {
                const float inv = 1.0f / ll;
#pragma unroll
                for (int i = 0; i < D / 16; ++i) {
                    const int d0 = 16 * i + 4 * g4;
                    float a[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) a[r] = o[i >> 2][4 * (i & 3) + r] * inv;
                    if constexpr (F8O) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) a[r] = fminf(fmaxf(a[r] * oqs, -448.f), 448.f);
                        int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[0], a[1], 0, false);
                        pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[2], a[3], pk, true);
                        *reinterpret_cast<int*>(reinterpret_cast<unsigned char*>(O) + lo_off + h * D + d0) = pk;
                    } else {
                        V64 w;
                        w.x = (uint32_t)at_f2bf(a[0]) | ((uint32_t)at_f2bf(a[1]) << 16);
                        w.y = (uint32_t)at_f2bf(a[2]) | ((uint32_t)at_f2bf(a[3]) << 16);
                        *reinterpret_cast<V64*>(O + lo_off + h * D + d0) = w;
                    }
                }
            }
            return;
        }
    }
    // row sum: the ones row D of O^T (lane half 0, register 8 of block D / 32) or the f32 sum
    float l;
    if (ONES) {
        constexpr int rr = D % 32;   // row within the last block: (e & 3) + 8 (e >> 2) + 4 fh
        constexpr int e_l = ((rr >> 3) << 2) | (rr & 3);
        constexpr int fh_l = (rr >> 2) & 1;
        const float mine = o[DB - 1][e_l];
        const float other = __shfl_xor(mine, 32, 64);
        l = (fh == fh_l) ? mine : other;
    } else {
        l = l_run + __shfl_xor(l_run, 32, 64);
    }
    if constexpr (LST) {
        const float inv = 1.0f / l;
        if constexpr (!OWN) __syncthreads();                 // every wave is done with the K ring
        unsigned char* wreg = (OWN ? sO : reinterpret_cast<unsigned char*>(sK)) + wave * 32 * OROW;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d0 = db * 32 + 8 * g + 4 * fh;
                if (d0 >= D) continue;
                if constexpr (F8O) {
                    const float sc = inv * oqs;
                    float a[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) a[i] = fminf(fmaxf(o[db][4 * g + i] * sc, -448.f), 448.f);
                    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[0], a[1], 0, false);
                    pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[2], a[3], pk, true);
                    *reinterpret_cast<int*>(wreg + fr * OROW + d0) = pk;
                } else {
                    V64 w;
                    w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                    w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                    *reinterpret_cast<V64*>(wreg + fr * OROW + 2 * d0) = w;
                }
            }
        constexpr int CPRO = EB * D / 16;                    // 16-B chunks per head row
        unsigned char* Ob = reinterpret_cast<unsigned char*>(O);
#pragma unroll
        for (int j = 0; j < (32 * CPRO + 63) / 64; ++j) {
            const int c = lane + 64 * j;
            if (c >= 32 * CPRO) break;
            const int r = c / CPRO, col = c % CPRO;
            const int qr = q - fr + r;                         // this wave's row r
            const V128 val = *reinterpret_cast<const V128*>(wreg + r * OROW + 16 * col);
            const long long off = attn_out_offset(o_map, b, qr, sq, o_bs, o_rs);
            if (qr < sq && off >= 0) *reinterpret_cast<V128*>(Ob + EB * (off + h * D) + 16 * col) = val;
        }
        return;
    }
    const long long o_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
    if (q < sq && o_off >= 0) {
        const float inv = 1.0f / l;
        if constexpr (F8O) {
            unsigned char* orow = reinterpret_cast<unsigned char*>(O) + o_off + h * D;
            const float sc = inv * oqs;
#pragma unroll
            for (int db = 0; db < DB; ++db)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int d0 = db * 32 + 8 * g + 4 * fh;
                    if (d0 >= D) continue;
                    float a[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) a[i] = fminf(fmaxf(o[db][4 * g + i] * sc, -448.f), 448.f);
                    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[0], a[1], 0, false);
                    pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[2], a[3], pk, true);
                    *reinterpret_cast<int*>(orow + d0) = pk;
                }
        } else {
            u16* orow = O + o_off + h * D;
#pragma unroll
            for (int db = 0; db < DB; ++db)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int d0 = db * 32 + 8 * g + 4 * fh;
                    if (d0 >= D) continue;
                    V64 w;
                    w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                    w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                    *reinterpret_cast<V64*>(orow + d0) = w;
                }
        }
    }
}

__device__ __forceinline__ void attn_wait_vm(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
        case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
        case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
        case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
        case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
        case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
        case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
        case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
        case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
        case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
        case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
        case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
        case 27: asm volatile("s_waitcnt vmcnt(27)" ::: "memory"); break;
        case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
        case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
        case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
    }
}

__device__ const uint16_t g_attn_vpad5[16] = {0x3F80, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

// ------------------------------------------------------------------------------------------
// k_attn4: short heads (CLIP ViT-H/14: 257 queries, D = 80), one wave per SIMD.  One 4-wave
// workgroup per (batch, head); wave w owns TWO 32-query blocks, A = queries 64w .. 64w + 31 and
// B = 64w + 32 .. 64w + 63, each with the k_attn2 arithmetic (S^T = K Q^T on 32x32x16, deferred
// max, the ones row of V^T giving the row sum).  The chains of the two blocks run half a tile
// apart, so that one block's softmax (VALU, transcendental) issues beside the other block's MFMAs:
//   prologue:        S_A(0), softmax A(0), S_B(0)
//   tile t (alpha):  softmax B(t)   beside  O_A += V(t) P_A(t), S_A(t + 1) = K(t + 1) Q_A^T
//          (beta):   softmax A(t+1) beside  O_B += V(t) P_B(t), S_B(t + 1)
// The 16 queries past 256 (block C; CLIP's 257th token) are split over the waves by key: wave w
// takes keys 16w .. 16w + 15 of every tile (16x16x32 for S^T, 16x16x16 for O^T with the lane's
// own four P values as the B operand), keeps its own running max and O^T, and the four partial
// states merge through LDS after the loop -- every wave does the same work per tile.
// K / V: a 3-slot ring of 64-key tiles staged through registers (tile t + 2 loads during tile t,
// written after it); one barrier per staged tile, none in the last two tiles.
// Per query, blocks A and B compute exactly what k_attn2 computes (bit-identical rows 0..255).
// ------------------------------------------------------------------------------------------
template <int D>
__global__ void __launch_bounds__(256, 1) k_attn4(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                  const u16* __restrict__ V, u16* __restrict__ O,
                                                  int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                  int o_rs, long long q_bs, long long k_bs,
                                                  long long v_bs, long long o_bs, float scale_log2,
                                                  const int32_t* __restrict__ o_map) {
    constexpr int KS = D / 16;
    constexpr int DB = (D + 31) / 32;
    static_assert(D % 32 != 0 && D % 16 == 0, "k_attn4: a padding row of V^T carries the row sum");
    constexpr int KROW = D + 8;
    constexpr int VROW = attn_vrow_bytes(D) / 2;
    constexpr int KTILE = AT_KT * KROW;
    constexpr int VTILE = AT_KT * VROW;
    constexpr int CPR = D / 8;
    constexpr int CH = AT_KT * CPR;
    constexpr int NT = 256;
    constexpr int NBUF = 3;
    constexpr int NSO = (CH + NT - 1) / NT;
    constexpr int KS16 = (D + 31) / 32;            // block C: 32-dim k-steps of S^T
    constexpr int NB16 = (D + 16) / 16;            // block C: 16-row O^T blocks incl. the ones row
    constexpr int NQ = 272;                        // 256 queries of blocks A / B + the 16 of block C
    __shared__ __attribute__((aligned(16))) u16 sK[NBUF * KTILE];
    __shared__ __attribute__((aligned(16))) u16 sV[NBUF * VTILE];
    __shared__ __attribute__((aligned(16))) u16 sQ[NQ * KROW];
    static_assert(4 * (NB16 * 16 + 1) * 16 * 4 <= (int)sizeof(sK), "block C merge scratch fits in sK");
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) s16x4* lds_s4;
    typedef short s16x8 __attribute__((ext_vector_type(8)));

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const AttnBlk blk = attn_block(1);
    const int h = blk.h, b = blk.b;
    const int fr = lane & 31, fh = lane >> 5;
    const int c16 = lane & 15, g4 = lane >> 4;
    const int g16 = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int qa = wave * 64 + fr, qb = qa + 32, qc = 256 + c16;
    const bool hasC = sq > 256;                                  // uniform
    const u16* Qb = Q + b * q_bs + h * D;
    const u16* Kb = K + b * k_bs + h * D;
    const u16* Vb = V + b * v_bs + h * D;

    // the Q image (rows past sq: copies of the last query), read as MFMA operands at every use so
    // that the arch VGPRs hold only the scores, P and addresses (the O^T accumulators sit in AGPRs)
    typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
    {
        constexpr int QCH = NQ * CPR, NQO = (QCH + NT - 1) / NT;
        u32x4_ qv[NQO];
#pragma unroll
        for (int i = 0; i < NQO; ++i) {
            const int c = min(t + i * NT, QCH - 1);
            qv[i] = *reinterpret_cast<const u32x4_*>(Qb + (size_t)min(c / CPR, sq - 1) * q_rs + (c % CPR) * 8);
        }
#pragma unroll
        for (int i = 0; i < NQO; ++i) {
            const int c = t + i * NT;
            if (c < QCH) *reinterpret_cast<u32x4_*>(sQ + (c / CPR) * KROW + (c % CPR) * 8) = qv[i];
        }
    }
    auto qfrag = [&](int row, int ks) {
        return *reinterpret_cast<const bf16x8*>(sQ + row * KROW + 16 * ks + 8 * fh);
    };
    // K / V ring: 64-key tiles by LDS-DMA (1-KiB pieces, per-lane source rows; the V padding
    // chunks -- the ones column at d = D, zeros after it -- from a 32-B constant); wave w issues
    // pieces j = w, w + 4, ... of each tile, whose per-lane rows / columns are the same in every tile
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    constexpr int KP = KTILE * 2 / 1024, VP = VTILE * 2 / 1024, PT = KP + VP;
    static_assert(KP * 1024 == KTILE * 2 && VP * 1024 == VTILE * 2, "tiles of whole pieces");
    constexpr int MJ = (PT + 3) / 4;
    int prow[MJ], pcol[MJ];
#pragma unroll
    for (int m = 0; m < MJ; ++m) {
        const int j = wave + 4 * m;
        const bool isv = j >= KP;
        const int u = (isv ? j - KP : j) * 64 + lane;
        const int cpr = isv ? VROW / 8 : KROW / 8;
        prow[m] = u / cpr;
        const int c = u % cpr;
        pcol[m] = c < CPR ? 8 * c : (c == CPR ? -1 : -2);   // -1: the ones chunk, -2: zeros
    }
    auto issue = [&](int tile) {
        const int slot = tile % NBUF;
#pragma unroll
        for (int m = 0; m < MJ; ++m) {
            const int j = wave + 4 * m;
            if (j >= PT) continue;                              // uniform
            const bool isv = j >= KP;
            const int key = min(tile * AT_KT + prow[m], sk - 1);
            const u16* src = !isv ? Kb + (size_t)key * k_rs + max(pcol[m], 0)
                                  : (pcol[m] < 0 ? g_attn_vpad5 + (pcol[m] == -1 ? 0 : 8)
                                                 : Vb + (size_t)key * v_rs + pcol[m]);
            u16* dst = isv ? sV + slot * VTILE + (j - KP) * 512 : sK + slot * KTILE + j * 512;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)dst, 16, 0, 0);
        }
    };
    auto raw_barrier = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    auto qk = [&](int tile, int qrow, f32x16 (&s)[2], bool sub1) {
        const u16* kt = sK + (tile % NBUF) * KTILE;
        asm volatile("" ::: "memory");     // K fragments re-read per block, not held across blocks
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            if (sub == 1 && !sub1) {
#pragma unroll
                for (int e = 0; e < 16; ++e) s[1][e] = -INFINITY;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (sub * 32 + fr) * KROW + 16 * ks + 8 * fh);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qfrag(qrow, ks), ks == 0 ? f32x16{} : s[sub], 0, 0, 0);
            }
        }
    };
    auto pv = [&](int tile, const bf16x8 (&pf)[2][2], f32x16 (&o)[DB], bool sub1) {
        const u16* vt = sV + (tile % NBUF) * VTILE;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const int d0 = db * 32 + g16 * 16 + 4 * p4;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    if (sub == 1 && !sub1) continue;
                    const int kb = 32 * sub + 16 * ss + 4 * fh + q4;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + kb * VROW + d0));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + (kb + 8) * VROW + d0));
                    const s16x8 lohi = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, lohi), pf[sub][ss], o[db], 0, 0, 0);
                }
        }
    };

    // block C: this wave's 16 keys of the tile
    f32x4 oc[NB16];
#pragma unroll
    for (int i = 0; i < NB16; ++i) oc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float mc = -INFINITY;
    auto c_tile = [&](int tile) {
        const int kr = 16 * wave;                            // first key of the slice in the tile
        const int k0 = tile * AT_KT + kr;
        if (k0 >= sk) return;                                // uniform: the slice is past the last key
        const u16* kt = sK + (tile % NBUF) * KTILE;
        const u16* vt = sV + (tile % NBUF) * VTILE;
        f32x4 sc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS16; ++ks) {
            const int d0 = 32 * ks + 8 * g4;
            bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (kr + c16) * KROW + (d0 < D ? d0 : 0));
            bf16x8 qf = *reinterpret_cast<const bf16x8*>(sQ + qc * KROW + (d0 < D ? d0 : 0));
            if (d0 >= D) { kf = bf16x8{}; qf = bf16x8{}; }
            sc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, sc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (k0 + 4 * g4 + r >= sk) sc[r] = -INFINITY;
        float mt = fmaxf(fmaxf(sc[0], sc[1]), fmaxf(sc[2], sc[3]));
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * scale_log2;
        const float mn = fmaxf(mc, mt);                      // finite: key k0 < sk is in the slice
        const float alpha = __builtin_amdgcn_exp2f(mc - mn);
        mc = mn;
#pragma unroll
        for (int i = 0; i < NB16; ++i) oc[i] *= alpha;
        s16x4 pc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const __bf16 pb = (__bf16)__builtin_amdgcn_exp2f(fmaf(sc[r], scale_log2, -mc));
            pc[r] = __builtin_bit_cast(short, pb);
        }
#pragma unroll
        for (int i = 0; i < NB16; ++i) {
            // rows keys kr + 4 g4 + q4, columns 16 i + 4 p4: lane c16 of group g4 gets V^T row 16 i + c16
            const s16x4 vf = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + (kr + 4 * g4 + q4) * VROW + 16 * i + 4 * p4));
            oc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf, pc, oc[i], 0, 0, 0);
        }
    };

    const int nt = (sk + AT_KT - 1) / AT_KT;                 // 3 .. 5
    issue(0);
    issue(1);
    attn_wait_vm(0);
    raw_barrier();

    f32x16 oa[DB], ob[DB], sa[2], sb[2];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) { oa[db][e] = 0.f; ob[db][e] = 0.f; }
    float ma = -INFINITY, mb = -INFINITY, lz = 0.f;
    bf16x8 pa[2][2], pb[2][2];

    qk(0, qa, sa, true);
    attn2_softmax<D, DB, true>(sa, true, false, 0, sk, fh, scale_log2, ma, lz, oa, pa);
    qk(0, qb, sb, true);
    // tile t; NEXT_TAIL: tile t + 1 is the last one (masked), LAST: t is the last one
    auto body = [&](int tile, auto next_tail_tag, auto last_tag) {
        constexpr bool NEXT_TAIL = decltype(next_tail_tag)::value;
        constexpr bool LAST = decltype(last_tag)::value;
        const int k0 = tile * AT_KT, k1 = k0 + AT_KT;
        const bool sub1_t = !LAST || (k0 + 32 < sk);
        const bool sub1_n = !NEXT_TAIL || (k1 + 32 < sk);
        const bool stage = !LAST && !NEXT_TAIL;              // tile + 2 exists
        if (stage) issue(tile + 2);
        attn2_softmax<D, DB, true>(sb, sub1_t, LAST, k0, sk, fh, scale_log2, mb, lz, ob, pb);
        pv(tile, pa, oa, sub1_t);
        if (!LAST) {
            qk(tile + 1, qa, sa, sub1_n);
            attn2_softmax<D, DB, true>(sa, sub1_n, NEXT_TAIL, k1, sk, fh, scale_log2, ma, lz, oa, pa);
        }
        pv(tile, pb, ob, sub1_t);
        if (!LAST) qk(tile + 1, qb, sb, sub1_n);
        if (hasC) c_tile(tile);
        if (stage) {                                         // tile + 2 landed, slot tile - 1 free
            attn_wait_vm(0);
            raw_barrier();
        }
    };
    for (int tile = 0; tile < nt - 2; ++tile) body(tile, std::false_type{}, std::false_type{});
    body(nt - 2, std::true_type{}, std::false_type{});
    body(nt - 1, std::false_type{}, std::true_type{});

    // blocks A and B: the row sum is O^T row D (the ones row)
    constexpr int rr = D % 32;
    constexpr int e_l = ((rr >> 3) << 2) | (rr & 3);
    constexpr int fh_l = (rr >> 2) & 1;
    auto store_block = [&](const f32x16 (&o)[DB], int q) {
        const float mine = o[DB - 1][e_l];
        const float other = __shfl_xor(mine, 32, 64);
        const float l = (fh == fh_l) ? mine : other;
        const long long o_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
        if (q < sq && o_off >= 0) {
            const float inv = 1.0f / l;
            u16* orow = O + o_off + h * D;
#pragma unroll
            for (int db = 0; db < DB; ++db)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int d0 = db * 32 + 8 * g + 4 * fh;
                    if (d0 >= D) continue;
                    V64 w;
                    w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                    w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                    *reinterpret_cast<V64*>(orow + d0) = w;
                }
        }
    };
    store_block(oa, qa);
    store_block(ob, qb);

    if (hasC) {
        // merge the four key slices of block C: scr[w][row d][query], mscr[w][query] (sK is free)
        __syncthreads();
        float* scr = reinterpret_cast<float*>(sK);
        float* mscr = scr + 4 * NB16 * 16 * 16;
#pragma unroll
        for (int i = 0; i < NB16; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) scr[(wave * NB16 * 16 + 16 * i + 4 * g4 + r) * 16 + c16] = oc[i][r];
        if (g4 == 0) mscr[wave * 16 + c16] = mc;
        __syncthreads();
        for (int j = t; j < 16 * D; j += NT) {
            const int qq = j / D, d = j % D;
            if (256 + qq >= sq) continue;
            float M = mscr[qq];
#pragma unroll
            for (int w = 1; w < 4; ++w) M = fmaxf(M, mscr[w * 16 + qq]);
            float acc = 0.f, L = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const float wt = __builtin_amdgcn_exp2f(mscr[w * 16 + qq] - M);
                acc = fmaf(scr[(w * NB16 * 16 + d) * 16 + qq], wt, acc);
                L = fmaf(scr[(w * NB16 * 16 + D) * 16 + qq], wt, L);
            }
            const long long o_off = attn_out_offset(o_map, b, 256 + qq, sq, o_bs, o_rs);
            if (o_off >= 0) O[o_off + h * D + d] = at_f2bf(acc / L);
        }
    }
}

// ------------------------------------------------------------------------------------------
// k_attn6: persistent short-head attention (<= 9 query blocks, CLIP's 257 tokens).  One 9-wave
// workgroup per CU walks (batch, head) pairs in k_attn2's XCD-aware order; per pair k_attn2's
// default schedule (64-key tiles through a double-buffered register-staged ring, one barrier per
// tile, the same arithmetic: bit-identical output).  The output rows go through LDS and leave as
// whole head rows (16-B chunks, consecutive lanes along a row), and the next pair's Q fragments
// and first K / V tile are loaded BEFORE those stores: the stores are the youngest memory
// operations, so the next pair's first wait leaves them in flight and the write burst of one
// pair overlaps the next pair's first tile instead of idling the CU at every workgroup boundary.
// Output rows b*o_bs + q*o_rs (no o_map).
// ------------------------------------------------------------------------------------------
template <int D, int NW, bool F8O = false>
__global__ void __launch_bounds__(NW * 64, 1) k_attn6(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                     const u16* __restrict__ V, u16* __restrict__ O,
                                                     int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                     int o_rs, long long q_bs, long long k_bs,
                                                     long long v_bs, long long o_bs, float scale_log2,
                                                     int heads, int npairs, float oqs = 1.f) {
    constexpr int KS = D / 16;
    constexpr int DB = (D + 31) / 32;
    constexpr bool ONES = (D % 32) != 0;
    constexpr int KROW = D + 8;
    constexpr int VROW = attn_vrow_bytes(D) / 2;
    constexpr int KTILE = AT_KT * KROW;
    constexpr int VTILE = AT_KT * VROW;
    constexpr int CPR = D / 8;
    constexpr int CH = AT_KT * CPR;
    constexpr int NT = NW * 64;
    constexpr int EB = F8O ? 1 : 2;                        // output bytes per element
    constexpr int OROW = ((EB * D + 16) / 32) * 32 + 16;  // bytes per staged output row (16-B aligned)
    constexpr int OCH = EB * D / 16;                       // 16-B chunks per output row
    __shared__ __attribute__((aligned(16))) u16 sK[2 * KTILE];
    __shared__ __attribute__((aligned(16))) u16 sV[2 * VTILE];
    __shared__ __attribute__((aligned(16))) unsigned char sO[NW * 32 * OROW];
    typedef __attribute__((address_space(3))) s16x4* lds_s4;
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int fr = lane & 31, fh = lane >> 5;
    const int g16 = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int q = wave * 32 + fr;
    const int ntiles = (sk + AT_KT - 1) / AT_KT;
    const int nfull = sk / AT_KT;

    // pair p -> (head, batch): k_attn2's XCD-aware order over the virtual block id p (the grid is a
    // multiple of 8, so p % 8 is the block's own XCD group)
    auto pair_hb = [&](int p, int& h_, int& b_) {
        const unsigned n = (unsigned)npairs, id = (unsigned)p;
        const unsigned xcd = id % 8u, k = id / 8u, qq = n / 8u, r = n % 8u;
        const unsigned lin = (xcd < r ? xcd * (qq + 1) : r * (qq + 1) + (xcd - r) * qq) + k;
        h_ = (int)(lin % (unsigned)heads);
        b_ = (int)(lin / (unsigned)heads);
    };

    if (VROW > D)
        for (int i = t; i < 2 * AT_KT * (VROW - D); i += NT) {
            const int r = i / (VROW - D), c = i % (VROW - D);
            sV[r * VROW + D + c] = (ONES && c == 0) ? (u16)0x3F80 : (u16)0;
        }
    constexpr int NSO = (CH + NT - 1) / NT;
    u32x4 stk[NSO], stv[NSO];
    const u16 *Qb, *Kb, *Vb;
    int h, b;
    auto bc_off = [&](int b_) { return (long long)b_ * o_bs; };
    auto set_pair = [&](int p) {
        pair_hb(p, h, b);
        Qb = Q + b * q_bs + h * D;
        Kb = K + b * k_bs + h * D;
        Vb = V + b * v_bs + h * D;
    };
    // buffer loads / stores with 32-bit per-lane offsets from the pair's (uniform) bases: no
    // 64-bit per-lane addresses held across the walk (the register file is full at 3 waves / SIMD)
    // (num_records ends at the last row of the pair: rows past sk / sq read as zeros -- their
    // scores are masked, their outputs dropped -- so no per-lane clamping is held in registers)
    auto rsrc = [](const void* base, int nbytes) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, nbytes, 0x00020000);
    };
    auto stage_load = [&](int k0_) {
        const __amdgpu_buffer_rsrc_t rk = rsrc(Kb, 2 * ((sk - 1) * k_rs + D));
        const __amdgpu_buffer_rsrc_t rv = rsrc(Vb, 2 * ((sk - 1) * v_rs + D));
#pragma unroll
        for (int i = 0; i < NSO; ++i) {
            const int c = min(t + i * NT, CH - 1);
            const int row = k0_ + c / CPR, col = (c % CPR) * 8;
            stk[i] = __builtin_amdgcn_raw_buffer_load_b128(rk, 2 * (row * k_rs + col), 0, 0);
            stv[i] = __builtin_amdgcn_raw_buffer_load_b128(rv, 2 * (row * v_rs + col), 0, 0);
        }
    };
    auto stage_store = [&](int buf_) {
#pragma unroll
        for (int i = 0; i < NSO; ++i) {
            const int c = t + i * NT;
            if (c < CH) {
                const int row = c / CPR, col = (c % CPR) * 8;
                *reinterpret_cast<u32x4*>(sK + buf_ * KTILE + row * KROW + col) = stk[i];
                *reinterpret_cast<u32x4*>(sV + buf_ * VTILE + row * VROW + col) = stv[i];
            }
        }
    };
    bf16x8 qf[KS];
    auto load_q = [&]() {
        const __amdgpu_buffer_rsrc_t rq = rsrc(Qb, 2 * ((sq - 1) * q_rs + D));
        const int qo = 2 * (q * q_rs + 8 * fh);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            qf[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, qo + 32 * ks, 0, 0));
    };

    f32x16 o[DB];
    float m_run, l_run;
    auto tile_body = [&](int buf, int k0, bool mask) {
        const u16* kt = sK + buf * KTILE;
        const u16* vt = sV + buf * VTILE;
        const bool sub1 = !mask || (k0 + 32 < sk);
        f32x16 s[2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            if (sub == 1 && !sub1) {
#pragma unroll
                for (int e = 0; e < 16; ++e) s[1][e] = -INFINITY;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (sub * 32 + fr) * KROW + 16 * ks + 8 * fh);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], ks == 0 ? f32x16{} : s[sub], 0, 0, 0);
            }
        }
        bf16x8 pf[2][2];
        attn2_softmax<D, DB, ONES>(s, sub1, mask, k0, sk, fh, scale_log2, m_run, l_run, o, pf);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const int d0 = db * 32 + g16 * 16 + 4 * p4;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    if (sub == 1 && !sub1) continue;
                    const int kb = 32 * sub + 16 * ss + 4 * fh + q4;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + kb * VROW + d0));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + (kb + 8) * VROW + d0));
                    const s16x8 lohi = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, lohi), pf[sub][ss], o[db], 0, 0, 0);
                }
        }
    };

    int p = blockIdx.x;
    if (p >= npairs) return;                                   // uniform
    set_pair(p);
    load_q();
    stage_load(0);
    stage_store(0);
    __syncthreads();
    int boff = 0;                                              // the buffer of the pair's tile 0
    for (;;) {
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
        m_run = -INFINITY;
        l_run = 0.f;
        for (int tile = 0; tile < nfull; ++tile) {
            const bool more = tile + 1 < ntiles;
            if (more) stage_load((tile + 1) * AT_KT);
            tile_body((tile + boff) & 1, tile * AT_KT, false);
            if (more) stage_store((tile + 1 + boff) & 1);
            __syncthreads();
        }
        if (nfull < ntiles) tile_body((nfull + boff) & 1, nfull * AT_KT, true);

        // the row sum, then this pair's output row offsets are fixed before the next pair is set
        float l;
        if (ONES) {
            constexpr int rr = D % 32;
            constexpr int e_l = ((rr >> 3) << 2) | (rr & 3);
            constexpr int fh_l = (rr >> 2) & 1;
            const float mine = o[DB - 1][e_l];
            const float other = __shfl_xor(mine, 32, 64);
            l = (fh == fh_l) ? mine : other;
        } else {
            l = l_run + __shfl_xor(l_run, 32, 64);
        }
        // this pair's rows to LDS (the accumulators die here) ...
        const float inv = 1.0f / l;
        unsigned char* wreg = sO + wave * 32 * OROW;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d0 = db * 32 + 8 * g + 4 * fh;
                if (d0 >= D) continue;
                if constexpr (F8O) {     // saturate_448(o * oqs) as OCP e4m3 (bf_attention_fp8out)
                    const float sc = inv * oqs;
                    float a[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) a[i] = fminf(fmaxf(o[db][4 * g + i] * sc, -448.f), 448.f);
                    int pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[0], a[1], 0, false);
                    pk = __builtin_amdgcn_cvt_pk_fp8_f32(a[2], a[3], pk, true);
                    *reinterpret_cast<int*>(wreg + fr * OROW + d0) = pk;
                } else {
                    V64 w;
                    w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                    w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                    *reinterpret_cast<V64*>(wreg + fr * OROW + 2 * d0) = w;
                }
            }
        const __amdgpu_buffer_rsrc_t ro = rsrc(reinterpret_cast<unsigned char*>(O) + EB * (bc_off(b) + h * D), 0x7FFFFFFF);
        // ... the next pair's Q and first tile go out (older than this pair's stores) ...
        const int pn = p + (int)gridDim.x;
        const bool next = pn < npairs;                          // uniform
        if (next) {
            set_pair(pn);
            load_q();
            stage_load(0);
        }
        // ... and this pair's rows leave as whole 2D-byte head rows
#pragma unroll
        for (int j = 0; j < (32 * OCH + 63) / 64; ++j) {
            const int c = lane + 64 * j;
            const int cc = min(c, 32 * OCH - 1);
            const int r = cc / OCH, col = cc % OCH;
            const int qr = wave * 32 + r;
            const u32x4 val = *reinterpret_cast<const u32x4*>(wreg + r * OROW + 16 * col);
            // rows past sq (and the surplus lanes of a partial last pass): an offset past num_records,
            // the store is dropped -- every lane issues every store, so the waitcnt pass counts them
            // exactly and the next pair's first wait leaves them in flight
            const int off = (qr < sq && c < 32 * OCH) ? EB * qr * o_rs + 16 * col : (int)0x80000000;
            __builtin_amdgcn_raw_buffer_store_b128(val, ro, off, 0, 0);
        }
        if (!next) break;
        boff = (ntiles + boff) & 1;                             // the buffer the last tile did not use
        stage_store(boff);
        __syncthreads();
        p = pn;
    }
}

// ------------------------------------------------------------------------------------------
// k_attn5: short heads (<= 5 key tiles, 5..9 query blocks: CLIP's 257 tokens), every K / V tile of
// the (batch, head) resident in LDS and filled by LDS-DMA (1-KiB pieces, per-lane source rows; the
// V padding chunks -- the ones column at d = D and zeros -- DMA'd from a 32-B constant).  Tile 0
// has arrays of its own, so the waits the compiler derives for its reads cover only tile 0's
// pieces: the waves compute tile 0 while tiles 1..4 land, wait once, and run the remaining tiles
// with no barrier at all (the waves of a SIMD drift apart, so one wave's softmax issues beside
// another's MFMAs).  Per query the arithmetic is k_attn2's (bit-identical output).
// ------------------------------------------------------------------------------------------

template <int D, int NW, bool KPF = false>
__global__ void __launch_bounds__(NW * 64, 1) k_attn5(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                     const u16* __restrict__ V, u16* __restrict__ O,
                                                     int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                     int o_rs, long long q_bs, long long k_bs,
                                                     long long v_bs, long long o_bs, float scale_log2,
                                                     const int32_t* __restrict__ o_map) {
    constexpr int KS = D / 16;
    constexpr int DB = (D + 31) / 32;
    constexpr bool ONES = (D % 32) != 0;
    constexpr int KROW = D + 8;
    constexpr int VROW = attn_vrow_bytes(D) / 2;
    constexpr int KTILE = AT_KT * KROW;
    constexpr int VTILE = AT_KT * VROW;
    constexpr int CPR = D / 8;
    constexpr int NTILE = 5;
    constexpr int KP = KTILE * 2 / 1024, VP = VTILE * 2 / 1024;     // 1-KiB pieces per tile
    static_assert(KP * 1024 == KTILE * 2 && VP * 1024 == VTILE * 2, "tiles of whole pieces");
    constexpr int PT = KP + VP, NPIECE = NTILE * PT;
    constexpr int PW = (NPIECE + NW - 1) / NW;
    __shared__ __attribute__((aligned(16))) u16 sK0[KTILE];
    __shared__ __attribute__((aligned(16))) u16 sV0[VTILE];
    __shared__ __attribute__((aligned(16))) u16 sKr[(NTILE - 1) * KTILE];
    __shared__ __attribute__((aligned(16))) u16 sVr[(NTILE - 1) * VTILE];
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(3))) s16x4* lds_s4;
    typedef short s16x8 __attribute__((ext_vector_type(8)));

    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const AttnBlk blk = attn_block(1);
    const int h = blk.h, b = blk.b;
    const int fr = lane & 31, fh = lane >> 5;
    const int g16 = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int q = wave * 32 + fr;
    const u16* Qb = Q + b * q_bs + h * D;
    const u16* Kb = K + b * k_bs + h * D;
    const u16* Vb = V + b * v_bs + h * D;

    // Q^T fragments by inline-asm loads: the compiler's waitcnt pass does not see them (it would
    // otherwise wait for every outstanding DMA piece before the first MFMA); the counted wait
    // before the first barrier covers them (they are older than every piece)
    typedef unsigned u32x4q __attribute__((ext_vector_type(4)));
    u32x4q qraw[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
        asm volatile("global_load_dwordx4 %0, %1, off"
                     : "=v"(qraw[ks])
                     : "v"(Qb + (size_t)min(q, sq - 1) * q_rs + 16 * ks + 8 * fh)
                     : "memory");

    // wave w DMAs pieces j = w, w + NW, w + 2 NW (< PT) of every tile, tile by tile; the lane's
    // source row / column of each of those pieces is the same in every tile (+ 64 keys per tile)
    constexpr int MJ = (PT + NW - 1) / NW;
    int prow[MJ], pcol[MJ];
    bool pv_[MJ], pconst[MJ];
#pragma unroll
    for (int m = 0; m < MJ; ++m) {
        const int j = wave + NW * m;
        pv_[m] = j >= KP;
        const int pc = pv_[m] ? j - KP : j;
        const int u = pc * 64 + lane;                    // 16-B chunk of the tile image
        const int cpr = pv_[m] ? VROW / 8 : KROW / 8;
        prow[m] = u / cpr;
        const int c = u % cpr;
        pconst[m] = pv_[m] && c >= CPR;
        pcol[m] = c < CPR ? 8 * c : (ONES && c == CPR ? 0 : 8);   // pads: offset in the 32-B constant
    }
    int after0 = 0;                                       // this wave's pieces of tiles 1..4
#pragma unroll
    for (int tt = 0; tt < NTILE; ++tt) {
#pragma unroll
        for (int m = 0; m < MJ; ++m) {
            const int j = wave + NW * m;
            if (j >= PT) continue;                        // uniform
            const int key = min(tt * AT_KT + prow[m], sk - 1);
            const u16* src = !pv_[m] ? Kb + (size_t)key * k_rs + pcol[m]
                                     : (pconst[m] ? g_attn_vpad5 + pcol[m] : Vb + (size_t)key * v_rs + pcol[m]);
            const int pc = pv_[m] ? j - KP : j;
            u16* dst = tt == 0 ? (pv_[m] ? sV0 : sK0) : (pv_[m] ? sVr + (tt - 1) * VTILE : sKr + (tt - 1) * KTILE);
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(dst + pc * 512), 16, 0, 0);
            after0 += tt > 0;
        }
    }

    f32x16 o[DB];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    const int ntiles = (sk + AT_KT - 1) / AT_KT;

    bf16x8 qf[KS];
    auto tile_body = [&](const u16* kt, const u16* vt, int k0, bool mask) {
        const bool sub1 = !mask || (k0 + 32 < sk);
        f32x16 s[2];
        if (KPF && sub1) {
            bf16x8 kf[2][KS];
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    kf[sub][ks] = *reinterpret_cast<const bf16x8*>(kt + (sub * 32 + fr) * KROW + 16 * ks + 8 * fh);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int sub = 0; sub < 2; ++sub)
                    s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[sub][ks], qf[ks], ks == 0 ? f32x16{} : s[sub], 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * KS, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2 * KS, 0);
        } else
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            if (sub == 1 && !sub1) {
#pragma unroll
                for (int e = 0; e < 16; ++e) s[1][e] = -INFINITY;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (sub * 32 + fr) * KROW + 16 * ks + 8 * fh);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], ks == 0 ? f32x16{} : s[sub], 0, 0, 0);
            }
        }
        bf16x8 pf[2][2];
        attn2_softmax<D, DB, ONES>(s, sub1, mask, k0, sk, fh, scale_log2, m_run, l_run, o, pf);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const int d0 = db * 32 + g16 * 16 + 4 * p4;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    if (sub == 1 && !sub1) continue;
                    const int kb = 32 * sub + 16 * ss + 4 * fh + q4;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + kb * VROW + d0));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(vt + (kb + 8) * VROW + d0));
                    const s16x8 lohi = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, lohi), pf[sub][ss], o[db], 0, 0, 0);
                }
        }
    };

    // raw barriers: __syncthreads() would add vmcnt(0) and drain the later tiles' DMA
    attn_wait_vm(after0);                             // this wave's tile-0 pieces (and Q) landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, qraw[ks]);
    if (ntiles == 1) tile_body(sK0, sV0, 0, true);
    else tile_body(sK0, sV0, 0, false);
    attn_wait_vm(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int tile = 1; tile < ntiles; ++tile)
        tile_body(sKr + (tile - 1) * KTILE, sVr + (tile - 1) * VTILE, tile * AT_KT, tile == ntiles - 1);

    float l;
    if (ONES) {
        constexpr int rr = D % 32;
        constexpr int e_l = ((rr >> 3) << 2) | (rr & 3);
        constexpr int fh_l = (rr >> 2) & 1;
        const float mine = o[DB - 1][e_l];
        const float other = __shfl_xor(mine, 32, 64);
        l = (fh == fh_l) ? mine : other;
    } else {
        l = l_run + __shfl_xor(l_run, 32, 64);
    }
    const long long o_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
    if (q < sq && o_off >= 0) {
        const float inv = 1.0f / l;
        u16* orow = O + o_off + h * D;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d0 = db * 32 + 8 * g + 4 * fh;
                if (d0 >= D) continue;
                V64 w;
                w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                *reinterpret_cast<V64*>(orow + d0) = w;
            }
    }
}

// ------------------------------------------------------------------------------------------
// Resident variant for short sequences (k_attn_r, sk <= 64*NTILE: CLIP's 257 tokens): the whole
// K and V of the (batch, head) go to LDS as [keys][D] images by LDS-DMA (global_load_lds, 1-KiB
// pieces, per-lane source rows), every piece issued up front after the Q loads; key tile t waits
// only for its own pieces with a counted vmcnt (the pieces of later tiles stay in flight under
// this tile's MFMAs), then one barrier.  No buffer is reused, so there is no WAR hazard.
// Rows past sk are clamped copies (their scores are masked); a zeroed slack after V covers the
// padded head-dim columns that the last O^T row block reads past the last key row.
// ------------------------------------------------------------------------------------------

template <int D, int NW, int NTILE>
__global__ void __launch_bounds__(NW * 64) k_attn_r(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                       const u16* __restrict__ V, u16* __restrict__ O,
                                                       int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                       int o_rs, long long q_bs, long long k_bs,
                                                       long long v_bs, long long o_bs, float scale_log2,
                                                     const int32_t* __restrict__ o_map) {
    constexpr int KS = D / 16;
    constexpr int DB = (D + 31) / 32;
    constexpr int ROWS = NTILE * AT_KT;
    constexpr int OPB = ROWS * D * 2;                // bytes of one operand image
    constexpr int PPT = AT_KT * D * 2 / 1024;        // 1-KiB pieces per operand per tile
    constexpr int QP = NW * 32 * D * 2 / 1024;       // pieces of the Q image (all NW*32 queries)
    constexpr int NPIECE = QP + NTILE * 2 * PPT;     // issue order: Q, then tile, operand, piece
    constexpr int SLACK = 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char at_smem[];
    u16* sQ = reinterpret_cast<u16*>(at_smem);
    u16* sK = reinterpret_cast<u16*>(at_smem + QP * 1024);
    u16* sV = reinterpret_cast<u16*>(at_smem + QP * 1024 + OPB);
    static_assert(PPT * 1024 == AT_KT * D * 2, "tile must be whole 1-KiB pieces");
    static_assert(QP * 1024 == NW * 32 * D * 2, "Q image must be whole 1-KiB pieces");

    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int h = blockIdx.y, b = blockIdx.z;
    const int fr = lane & 31, fh = lane >> 5;
    const int q = blockIdx.x * (NW * 32) + wave * 32 + fr;
    const int q_base = blockIdx.x * (NW * 32);
    const u16* Qb = Q + b * q_bs + h * D;
    const u16* Kb = K + b * k_bs + h * D;
    const u16* Vb = V + b * v_bs + h * D;

    if (t < SLACK / 2) reinterpret_cast<u16*>(at_smem + QP * 1024 + 2 * OPB)[t] = 0;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    // Q, K and V all arrive by LDS-DMA (no plain global loads in the kernel, so the compiler adds
    // no waits of its own); every wave issues exactly PW pieces (a surplus slot repeats the
    // wave's last piece: same bytes, same place)
    constexpr int PW = (NPIECE + NW - 1) / NW;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        int g = wave + i * NW;
        if (g >= NPIECE) g -= NW;
        const u16* src;
        int dst;
        if (g < QP) {
            const int e = g * 512 + lane * 8;
            src = Qb + (size_t)min(q_base + e / D, sq - 1) * q_rs + e % D;
            dst = g * 1024;
        } else {
            const int gg = g - QP;
            const int tile = gg / (2 * PPT), rem = gg % (2 * PPT);
            const int op = rem / PPT, pc = tile * PPT + rem % PPT;  // piece within the operand
            const int e = pc * 512 + lane * 8;
            const int row = min(e / D, sk - 1), col = e % D;
            src = (op ? Vb + (size_t)row * v_rs : Kb + (size_t)row * k_rs) + col;
            dst = QP * 1024 + op * OPB + pc * 1024;
        }
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(at_smem + dst), 16, 0, 0);
    }

    f32x16 o[DB];
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    const int g16 = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    const int ntiles = (sk + AT_KT - 1) / AT_KT;
    bf16x8 qf[KS];
    // this wave's slots issued after its last piece of `tile` (issue order = tile order)
    for (int tile = 0; tile < ntiles; ++tile) {
        const int k0 = tile * AT_KT;
        const int last = QP + (tile + 1) * 2 * PPT;                   // first piece of the next tile
        const int mine_upto = last > wave ? (last - wave + NW - 1) / NW : 0;
        attn_wait_vm(PW - mine_upto);
        // raw barrier: __syncthreads() would add vmcnt(0) and drain the later tiles' DMA
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (tile == 0) {      // Q^T fragments (B operand) from the Q image
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                qf[ks] = *reinterpret_cast<const bf16x8*>(sQ + (wave * 32 + fr) * D + 16 * ks + 8 * fh);
        }
        const u16* kt = sK + k0 * D;
        const u16* vt = sV + k0 * D;
        f32x16 s[2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (sub * 32 + fr) * D + 16 * ks + 8 * fh);
                s[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], ks == 0 ? f32x16{} : s[sub], 0, 0, 0);
            }
        }
        bf16x8 pf[2][2];
        attn_softmax_tile<DB>(s, k0, sk, fh, scale_log2, m_run, l_run, o, pf);
        // V^T fragments: transposed reads in inline asm (the builtin makes the compiler drain
        // every pending LDS-DMA first), retired by an explicit lgkmcnt before their MFMAs
        typedef unsigned long long u64;
        const unsigned vbase = (unsigned)(size_t)(__attribute__((address_space(3))) u16*)vt;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const int d0 = db * 32 + g16 * 16 + 4 * p4;
            u64 lo[2][2], hi[2][2];
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const int kb = 32 * sub + 16 * ss + 4 * fh + q4;
                    const unsigned a0 = vbase + (unsigned)((kb * D + d0) * 2);
                    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[sub][ss]) : "v"(a0));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[sub][ss]) : "v"(a0), "i"(8 * D * 2));
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    asm volatile("" : "+v"(lo[sub][ss]), "+v"(hi[sub][ss]));
                    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                    const u64x2 lh = {lo[sub][ss], hi[sub][ss]};
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, lh),
                                                                   pf[sub][ss], o[db], 0, 0, 0);
                }
        }
    }
    const long long o_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
    if (q < sq && o_off >= 0) {
        const float inv = 1.0f / l_run;
        u16* orow = O + o_off + h * D;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d0 = db * 32 + 8 * g + 4 * fh;
                if (d0 >= D) continue;
                V64 w;
                w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                *reinterpret_cast<V64*>(orow + d0) = w;
            }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outstanding at exit
}

template <int D, int NW, int NTILE>
static void launch_attn_r(dim3 grid, hipStream_t st, const void* q, const void* k, const void* v, void* o,
                          int sq, int sk, int q_rs, int k_rs, int v_rs, int o_rs, long long q_bs,
                          long long k_bs, long long v_bs, long long o_bs, float sl2,
                          const int32_t* o_map) {
    constexpr size_t lds = (size_t)NW * 32 * D * 2 + 2 * (size_t)NTILE * AT_KT * D * 2 + 64;
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_attn_r<D, NW, NTILE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL((k_attn_r<D, NW, NTILE>), grid, dim3(NW * 64), lds, st, (const u16*)q,
                       (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs,
                       k_bs, v_bs, o_bs, sl2, o_map);
}

// ------------------------------------------------------------------------------------------
// k_attn_p: persistent short-head attention (CLIP: S = 257, D = 80) on an LDS-DMA ring.
// The per-(batch, head) workgroup of k_attn2 (one 9-wave workgroup per CU: 164 VGPRs) runs its
// Q load and first K/V tile with nothing to compute beside them, and keeps only one 20-KB K/V tile
// in flight per CU.  Here one workgroup per CU walks (batch, head) pairs p = blockIdx.x + j *
// gridDim.x as one continuous stream of 64-key steps, and every byte arrives by LDS-DMA
// (global_load_lds, 1-KiB wave pieces, per-lane source rows) three steps ahead:
//   * ring of 4 step slots: K image [64 keys][10 chunks] x 16 B, chunk order swizzled per row
//     (atp_pos: conflict-free ds_read_b128 of the S^T = K Q^T A operand, coalesced DMA rows),
//     V image row-major [64 keys][96] (192-B rows:
//     conflict-free ds_read_b64_tr_b16; d = 80 is a ones column, 81..95 zeros, both DMA'd from a
//     32-B constant) -> 22 pieces per step;
//   * one Q image [288 queries][10 chunks] x 16 B, swizzled like K (45 pieces): pair i+1's Q is issued during
//     steps 1..2 of pair i (after every wave has read pair i's Q fragments at step 0) and retired
//     by the step-0 wait of pair i+1;
//   * batch B_s (issued at step s) = K/V of step s+3 (+ Q pieces); the wait at step s leaves
//     B_{s-1} and B_{s-2} in flight (counted vmcnt: loads, stores and LDS-DMA retire in issue
//     order), then a raw s_barrier (no vmcnt(0));
//   * the tile body is k_attn2's (deferred-max softmax, ones row for l); a pair's output rows are
//     stored right after its last step, under the next pair's DMA.
// Requires 193 <= sk <= 320, sq <= 288 (4 or 5 key steps, queries in one workgroup).
// ------------------------------------------------------------------------------------------
__device__ const uint16_t g_attn_vpad[16] = {0x3F80, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

// K and Q images are dense 160-B rows (so a DMA piece reads whole rows: coalesced) with the 16-B
// chunk order rotated by one in rows 16..31 of every 32: the ds_read_b128 lane groups of the
// fragment reads ({0-3,12-15,20-27}, {4-11,16-19,28-31}) then hit 16 distinct 4-bank groups
__device__ __forceinline__ int atp_pos(int row, int c) { const int p = c + ((row >> 4) & 1); return p >= 10 ? p - 10 : p; }
__device__ __forceinline__ int atp_chunk(int row, int pos) { const int c = pos - ((row >> 4) & 1); return c < 0 ? c + 10 : c; }

#define ATP_NQ 288
#define ATP_QPIECES 45                    // 10 chunks x 288 queries x 16 B / 1 KiB
#define ATP_KPIECES 10
#define ATP_VPIECES 12
#define ATP_KV (ATP_KPIECES + ATP_VPIECES)
#define ATP_SLOT ((ATP_KPIECES + ATP_VPIECES) * 1024)
#define ATP_LDS (ATP_QPIECES * 1024 + 4 * ATP_SLOT)

template <int NW>
__global__ void __launch_bounds__(NW * 64) k_attn_p(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                     const u16* __restrict__ V, u16* __restrict__ O,
                                                     int heads, int npairs, int sq, int sk, int q_rs,
                                                     int k_rs, int v_rs, int o_rs, long long q_bs,
                                                     long long k_bs, long long v_bs, long long o_bs,
                                                     float scale_log2, const int32_t* __restrict__ o_map) {
    constexpr int D = 80, KS = 5, DB = 3, VROWB = 192;
    static_assert(NW * 32 == ATP_NQ, "one workgroup holds every query");
    extern __shared__ __attribute__((aligned(16))) unsigned char at_smem[];
    unsigned char* sQ = at_smem;
    unsigned char* sR = at_smem + ATP_QPIECES * 1024;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;

    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int fr = lane & 31, fh = lane >> 5;
    const int g16 = (lane >> 4) & 1, q4 = (lane & 15) >> 2, p4 = lane & 3;
    // pair j of this workgroup = wg + j * G; wg is XCD-major (blockIdx % 8 = XCD) so that the
    // workgroups of one XCD walk adjacent heads together (their 160-B rows share cache lines)
    const int G = gridDim.x;
    const int wg = (G % 8 == 0) ? ((int)blockIdx.x % 8) * (G / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int nmine = wg < npairs ? (npairs - wg + G - 1) / G : 0;
    const int NTL = (sk + AT_KT - 1) / AT_KT;
    const int total = nmine * NTL;
    const int q = wave * 32 + fr;

    const int n_kv_mine = wave < ATP_KV ? (ATP_KV - wave + NW - 1) / NW : 0;
    // element offsets of a pair's rows fit in 32 bits (checked on the host): fewer live SGPRs
    auto pair_off = [&](int j, long long bs) {
        const int pp = wg + j * G;
        return (pp / heads) * (int)bs + (pp % heads) * D;
    };
    auto issue_kv = [&](int koff, int voff, int k0, int slot) {
        unsigned char* base = sR + slot * ATP_SLOT;
        int ln = lane;                                // opaque: keeps the address math in the step
        asm volatile("" : "+v"(ln));                  // (hoisted, it would pin 20+ VGPRs)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (j < n_kv_mine) {
                const int g = wave + NW * j;          // this wave's pieces: g = wave + 9 j
                const void* src;
                if (g < ATP_KPIECES) {                // K rows, swizzled chunk order (atp_pos)
                    const int sl = g * 64 + ln, r = sl / 10;
                    src = K + koff + min(k0 + r, sk - 1) * k_rs + atp_chunk(r, sl - r * 10) * 8;
                } else {                              // V rows: 12 chunks per key, 10..11 padding
                    const int sl = (g - ATP_KPIECES) * 64 + ln, r = sl / 12, ch = sl - r * 12;
                    src = ch < 10 ? (const void*)(V + voff + min(k0 + r, sk - 1) * v_rs + ch * 8)
                                  : (const void*)(g_attn_vpad + (ch - 10) * 8);
                }
                __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(base + g * 1024), 16, 0, 0);
            }
        }
        return n_kv_mine;
    };
    auto issue_q = [&](int qoff, int ql, int qh) {   // Q pieces [ql, qh): pc = wave mod 9
        int cnt = 0;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        for (int pc = ql + ((wave - ql % NW + NW) % NW); pc < qh; pc += NW) {
            const int sl = pc * 64 + ln, qq = sl / 10;
            const void* src = Q + qoff + min(qq, sq - 1) * q_rs + atp_chunk(qq, sl - qq * 10) * 8;
            __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(sQ + pc * 1024), 16, 0, 0);
            ++cnt;
        }
        return cnt;
    };

    // K/V issue cursor (pair j3, step t3), three steps ahead of the compute cursor (i, tt)
    int j3 = 0, t3 = 0;
    int Kb3 = pair_off(0, k_bs), Vb3 = pair_off(0, v_bs);
    auto advance3 = [&]() {
        if (++t3 == NTL) {
            t3 = 0;
            ++j3;
            if (j3 < nmine) { Kb3 = pair_off(j3, k_bs); Vb3 = pair_off(j3, v_bs); }
        }
    };
    int c_m2 = 0, c_m1 = 0;
    if (total > 0) {
        // B_-3 = Q of pair 0 + K/V of step 0; B_-2, B_-1 = K/V of steps 1, 2
        int c0 = issue_q(pair_off(0, q_bs), 0, ATP_QPIECES) + issue_kv(Kb3, Vb3, 0, 0);
        advance3();
        c_m2 = total > 1 ? issue_kv(Kb3, Vb3, t3 * AT_KT, 1) : 0;
        if (total > 1) advance3();
        c_m1 = total > 2 ? issue_kv(Kb3, Vb3, t3 * AT_KT, 2) : 0;
        if (total > 2) advance3();
        (void)c0;
    }
    int Qn = nmine > 1 ? pair_off(1, q_bs) : 0;     // the next pair's Q rows

    f32x16 o[DB];
    float m_run = -INFINITY, l_run = 0.f;
    bf16x8 qf[KS];
    int i = 0, tt = 0;
    for (int s = 0; s < total; ++s) {
        attn_wait_vm(c_m2 + c_m1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        int c_now = 0;
        if (s + 3 < total) {
            c_now += issue_kv(Kb3, Vb3, t3 * AT_KT, (s + 3) & 3);
            advance3();
        }
        if (i + 1 < nmine) {
            if (NTL == 5 && tt == 1) c_now += issue_q(Qn, 0, 23);
            else if (NTL == 5 && tt == 2) c_now += issue_q(Qn, 23, ATP_QPIECES);
            else if (NTL == 4 && tt == 1) c_now += issue_q(Qn, 0, ATP_QPIECES);
        }
        c_m2 = c_m1;
        c_m1 = c_now;
        if (tt == 0) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                qf[ks] = *reinterpret_cast<const bf16x8*>(sQ + (q * 10 + atp_pos(q, 2 * ks + fh)) * 16);
#pragma unroll
            for (int db = 0; db < DB; ++db)
#pragma unroll
                for (int e = 0; e < 16; ++e) o[db][e] = 0.f;
            m_run = -INFINITY;
            l_run = 0.f;
        }
        const unsigned char* kt = sR + (s & 3) * ATP_SLOT;
        const unsigned char* vt = kt + ATP_KPIECES * 1024;
        const int k0 = tt * AT_KT;
        const bool mask = k0 + AT_KT > sk;
        const bool sub1 = k0 + 32 < sk;
        f32x16 sc[2];
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            if (sub == 1 && !sub1) {
#pragma unroll
                for (int e = 0; e < 16; ++e) sc[1][e] = -INFINITY;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int kr = sub * 32 + fr;
                const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kt + (kr * 10 + atp_pos(kr, 2 * ks + fh)) * 16);
                sc[sub] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], ks == 0 ? f32x16{} : sc[sub], 0, 0, 0);
            }
        }
        bf16x8 pf[2][2];
        attn2_softmax<D, DB, true>(sc, sub1, mask, k0, sk, fh, scale_log2, m_run, l_run, o, pf);
        typedef unsigned long long u64;
        const unsigned vbase = (unsigned)(size_t)(__attribute__((address_space(3))) const unsigned char*)vt;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
            const int d0 = db * 32 + g16 * 16 + 4 * p4;
            u64 lo[2][2], hi[2][2];
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    const int kb = 32 * sub + 16 * ss + 4 * fh + q4;
                    const unsigned a0 = vbase + (unsigned)(kb * VROWB + d0 * 2);
                    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[sub][ss]) : "v"(a0));
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi[sub][ss]) : "v"(a0), "i"(8 * VROWB));
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int sub = 0; sub < 2; ++sub)
#pragma unroll
                for (int ss = 0; ss < 2; ++ss) {
                    if (sub == 1 && !sub1) continue;
                    asm volatile("" : "+v"(lo[sub][ss]), "+v"(hi[sub][ss]));
                    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                    const u64x2 lh = {lo[sub][ss], hi[sub][ss]};
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, lh), pf[sub][ss],
                                                                   o[db], 0, 0, 0);
                }
        }
        if (tt == NTL - 1) {
            // row sum from the ones row d = 80 of O^T: block 2, row 16 -> register 8 of lane half 0
            const float mine_l = o[DB - 1][8];
            const float other = __shfl_xor(mine_l, 32, 64);
            const float l = fh == 0 ? mine_l : other;
            const int p = wg + i * G;
            const int b = p / heads, h = p % heads;
            const long long o_off = attn_out_offset(o_map, b, q, sq, o_bs, o_rs);
            if (q < sq && o_off >= 0) {
                const float inv = 1.0f / l;
                u16* orow = O + o_off + h * D;
#pragma unroll
                for (int db = 0; db < DB; ++db)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int d0 = db * 32 + 8 * g + 4 * fh;
                        if (db * 32 + 8 * g >= D) continue;
                        V64 w;
                        w.x = (uint32_t)at_f2bf(o[db][4 * g + 0] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 1] * inv) << 16);
                        w.y = (uint32_t)at_f2bf(o[db][4 * g + 2] * inv) | ((uint32_t)at_f2bf(o[db][4 * g + 3] * inv) << 16);
                        *reinterpret_cast<V64*>(orow + d0) = w;
                    }
            }
        }
        if (++tt == NTL) {
            tt = 0;
            ++i;
            if (i + 1 < nmine) Qn = pair_off(i + 1, q_bs);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outstanding at exit
}

BF_API int bf_gemm_get_cu_budget(void);
// CUs a persistent attention grid may assume: the device's, or the budget set for CU-masked
// launch streams (bf_gemm_set_cu_budget: rank 0 at N > 1 reserves CUs for the fusion stream; a
// grid wider than the stream's CUs would run its surplus workgroups after whole walks finish)
static int attn_num_cus() {
    static int n = [] {
        int dev = 0, c = 0;
        hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        return c;
    }();
    const int budget = bf_gemm_get_cu_budget();
    return budget > 0 && budget < n ? budget : n;
}

static int launch_attn_p(hipStream_t st, const void* q, const void* k, const void* v, void* o, int batch,
                         int heads, int sq, int sk, int q_rs, int k_rs, int v_rs, int o_rs, long long q_bs,
                         long long k_bs, long long v_bs, long long o_bs, float sl2, const int32_t* o_map) {
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)k_attn_p<9>, hipFuncAttributeMaxDynamicSharedMemorySize, ATP_LDS);
        attr = true;
    }
    const int npairs = batch * heads;
    const long long span = (long long)(batch - 1) * std::max(std::max(q_bs, k_bs), v_bs) + (long long)heads * 80 +
                           (long long)ATP_NQ * std::max(std::max(q_rs, k_rs), v_rs);
    if (span >= (1ll << 31)) return BF_ERR_UNSUPPORTED;      // 32-bit element offsets in the kernel
    const int grid = npairs < attn_num_cus() ? npairs : attn_num_cus();
    hipLaunchKernelGGL((k_attn_p<9>), dim3(grid), dim3(9 * 64), ATP_LDS, st, (const u16*)q, (const u16*)k,
                       (const u16*)v, (u16*)o, heads, npairs, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs,
                       o_bs, sl2, o_map);
    return bf_check_launch();
}

// 6 (default): k_attn2 with the LDS-staged whole-row output stores (27: the same kernel with the
// per-lane fragment stores; 26: k_attn6, persistent; 16: k_attn4, one wave per SIMD with two query
// blocks; 17 / 18: k_attn5, all K / V tiles resident by LDS-DMA; 12: k_attn2 PP, ping-pong tiles);
// 7 / 8: k_attn2 with two 5-wave / three 3-wave workgroups per short head;
// 1/2: k_attn_s (with / without the XCD block order), 3: k_attn_r for short sequences, 4/5:
// k_attn_s with 5/3 waves per workgroup for short sequences, 0: k_attn.  Env BF_ATTN_VARIANT.
// 9: k_attn_p (persistent, LDS-DMA ring 3 steps deep, next head's Q prefetched), 10: k_attn2 XQ
// (8 MFMA waves + the 257th query in VALU), 11: k_attn2 LW (8 MFMA waves + a ninth wave of 16
// queries on 16x16x32 MFMAs).
// Measured (scripts/attn_bench.py, one MI355X): CLIP 128x16x257x80 k_attn_s 153.7 us -> k_attn2
// 128.6 us; CuTR windows 72x12x512x64 122.0 -> 109.9; CuTR global 8x12x1600x64 124.8 -> 105.0.
// CLIP, this round: v6 130.9-132.5 us, v9 131.0 (equal: same FETCH, +9 M SALU / +7 M VALU for
// the DMA address math), v10 146.9 (8 waves hide less latency than 9: 41 % of wave cycles at
// waitcnt / barrier, 32 % issue-stalled; a 3-slot ring issuing tile t+1's S^T MFMAs beside tile
// t's softmax on top of it: 149.7, dropped).  scripts/attn_rounds.py: 17 us per round of 256
// (batch, head) workgroups from 1 to 16 rounds, also with every operand MALL-resident -- the
// per-workgroup chain, not HBM, sets the time.  v11 130.9 us vs v6 130.8 in the same process
// (the ninth wave's halved MFMA work is not on the critical path either); 16-byte epilogue
// stores (halves of a query swapping 4-value chunks): 132.6, not kept.  Softmax + P.V per 32-key
// sub-tile (sub-tile 0's P.V MFMAs issued before sub-tile 1's exp work): 134.1-141.8 vs v6
// 132.5-133.3 in three interleaved runs, not kept.  s_setprio 1 over the MFMA blocks: 129.2-133.1
// vs 131.7-133.1 (the first variant in a run reads ~2 % slow: order bias), not kept.
static int g_attn_variant = [] {
    const char* e = getenv("BF_ATTN_VARIANT");
    return e ? atoi(e) : 6;
}();
BF_API void bf_attention_set_variant(int v) { g_attn_variant = v; }

BF_API int bf_attention_bf16_omap(const void* q, const void* k, const void* v, void* o, int batch,
                                  int heads, int sq, int sk, int head_dim, int q_rs, int k_rs,
                                  int v_rs, int o_rs, long long q_bs, long long k_bs, long long v_bs,
                                  long long o_bs, float scale, const int32_t* o_map, void* stream) {
    if (!q || !k || !v || !o || batch <= 0 || heads <= 0 || sq <= 0 || sk <= 0) return BF_ERR_ARG;
    if ((q_rs | k_rs | v_rs) % 8 != 0 || o_rs % 4 != 0) return BF_ERR_UNSUPPORTED;
    const float sl2 = scale * 1.4426950408889634f;
    // short sequences (CLIP: 257 tokens) run every query of a (batch, head) in ONE workgroup of
    // ceil(sq/32) waves, so K/V are staged once and no 128-query tile is almost empty
    const int nw_one = (sq + 31) / 32;
    // variant 3: short sequences with all queries in one workgroup, resident K/V filled by
    // LDS-DMA (measured slower than the streaming ring on CLIP's shape; kept as an alternative)
    if (g_attn_variant == 3 && nw_one > 4 && nw_one <= 9 && sk <= 5 * AT_KT &&
        (head_dim == 80 || head_dim == 64)) {
        const dim3 grid(1, heads, batch);
        if (head_dim == 80)
            launch_attn_r<80, 9, 5>(grid, bf_stream(stream), q, k, v, o, sq, sk, q_rs, k_rs, v_rs, o_rs,
                                    q_bs, k_bs, v_bs, o_bs, sl2, o_map);
        else
            launch_attn_r<64, 9, 5>(grid, bf_stream(stream), q, k, v, o, sq, sk, q_rs, k_rs, v_rs, o_rs,
                                    q_bs, k_bs, v_bs, o_bs, sl2, o_map);
        return bf_check_launch();
    }
    // variant 9: the persistent LDS-DMA ring (k_attn_p) for D = 80 heads of 193..320 keys and
    // <= 288 queries (CLIP ViT-H: 257); other shapes take k_attn2
    if (g_attn_variant == 9 && head_dim == 80 && sq <= ATP_NQ && sk >= 193 && sk <= 5 * AT_KT &&
        batch * heads < (1 << 30))
        return launch_attn_p(bf_stream(stream), q, k, v, o, batch, heads, sq, sk, q_rs, k_rs, v_rs, o_rs,
                             q_bs, k_bs, v_bs, o_bs, sl2, o_map);
    // variant 10: short heads with sq = 257-like (32*8 + 1): 8 MFMA waves + the last query in
    // VALU beside them (k_attn2 XQ), one workgroup per (batch, head)
    if (g_attn_variant == 10 && nw_one == 9 && sq % 32 == 1 && (head_dim == 80 || head_dim == 64)) {
        if (head_dim == 80)
            hipLaunchKernelGGL((k_attn2<80, 8, false, false, true>), dim3(1, heads, batch), dim3(512), 0,
                               bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk,
                               q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map, 1.f);
        else
            hipLaunchKernelGGL((k_attn2<64, 8, false, false, true>), dim3(1, heads, batch), dim3(512), 0,
                               bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk,
                               q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map, 1.f);
        return bf_check_launch();
    }
    // variant 12: short heads (5..9 query blocks, one 9-wave workgroup per (batch, head)), the
    // ping-pong tile order (k_attn2 PP)
    if (g_attn_variant == 12 && nw_one > 4 && nw_one <= 9 && (head_dim == 80 || head_dim == 64)) {
        if (head_dim == 80)
            hipLaunchKernelGGL((k_attn2<80, 9, false, false, false, false, true>), dim3(1, heads, batch),
                               dim3(9 * 64), 0, bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v,
                               (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map, 1.f);
        else
            hipLaunchKernelGGL((k_attn2<64, 9, false, false, false, false, true>), dim3(1, heads, batch),
                               dim3(9 * 64), 0, bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v,
                               (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map, 1.f);
        return bf_check_launch();
    }
    // variant 26: short heads (5..9 query blocks), k_attn6 -- persistent, output rows through LDS,
    // the next pair's loads issued before the current pair's stores (bit-identical; CLIP 126.3 ->
    // 116.6 us in the bench's re-run, but with rank 0's fusion of 8 ranks beside it, 132.6-137.9 vs
    // 142.4-142.7 frames/s: the walk holds every CU, so the fusion stream's kernels wait)
    if (g_attn_variant == 26 && nw_one > 4 && nw_one <= 9 && (head_dim == 80 || head_dim == 64) &&
        o_map == nullptr && (long long)batch * heads < (1LL << 30) &&
        2LL * ((long long)sq * (q_rs > o_rs ? q_rs : o_rs) + (long long)sk * (k_rs > v_rs ? k_rs : v_rs)) < (1LL << 31)) {
        const int npairs = batch * heads;
        int grid = attn_num_cus();
        grid = grid < npairs ? grid : npairs;
        if (head_dim == 80)
            hipLaunchKernelGGL((k_attn6<80, 9>), dim3(grid), dim3(9 * 64), 0, bf_stream(stream), (const u16*)q,
                               (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs,
                               k_bs, v_bs, o_bs, sl2, heads, npairs);
        else
            hipLaunchKernelGGL((k_attn6<64, 9>), dim3(grid), dim3(9 * 64), 0, bf_stream(stream), (const u16*)q,
                               (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs,
                               k_bs, v_bs, o_bs, sl2, heads, npairs);
        return bf_check_launch();
    }
    // variant 16: CLIP-like short heads (D = 80, 193..272 queries, 129..320 keys): k_attn4, one wave
    // per SIMD, two query blocks per wave
    if (g_attn_variant == 16 && head_dim == 80 && sq > 192 && sq <= 272 && sk > 2 * AT_KT && sk <= 5 * AT_KT) {
        hipLaunchKernelGGL((k_attn4<80>), dim3(1, heads, batch), dim3(256), 0, bf_stream(stream),
                           (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs,
                           q_bs, k_bs, v_bs, o_bs, sl2, o_map);
        return bf_check_launch();
    }
    // variant 17: short heads (5..9 query blocks, <= 320 keys): k_attn5, resident K / V by LDS-DMA,
    // barrier-free after tile 0
    if (g_attn_variant == 17 && nw_one > 4 && nw_one <= 9 && sk <= 5 * AT_KT && (head_dim == 80 || head_dim == 64)) {
        if (head_dim == 80)
            hipLaunchKernelGGL((k_attn5<80, 9>), dim3(1, heads, batch), dim3(9 * 64), 0, bf_stream(stream),
                               (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs,
                               o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map);
        else
            hipLaunchKernelGGL((k_attn5<64, 9>), dim3(1, heads, batch), dim3(9 * 64), 0, bf_stream(stream),
                               (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs,
                               o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map);
        return bf_check_launch();
    }
    // variant 18: k_attn5 with every K fragment of a tile read before its first S^T MFMA
    if (g_attn_variant == 18 && head_dim == 80 && nw_one > 4 && nw_one <= 9 && sk <= 5 * AT_KT) {
        hipLaunchKernelGGL((k_attn5<80, 9, true>), dim3(1, heads, batch), dim3(9 * 64), 0, bf_stream(stream),
                           (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs,
                           o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map);
        return bf_check_launch();
    }
    // variant 11: CLIP-like short heads (D = 80, 257..272 queries): 8 full waves + the light ninth
    if (g_attn_variant == 11 && head_dim == 80 && nw_one == 9 && sq <= 8 * 32 + 16) {
        hipLaunchKernelGGL((k_attn2<80, 9, false, false, false, true>), dim3(1, heads, batch), dim3(9 * 64), 0,
                           bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk,
                           q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map, 1.f);
        return bf_check_launch();
    }
    if ((g_attn_variant >= 6 && g_attn_variant <= 11) || g_attn_variant == 27) {
#define LAUNCH_2(DD, NWV)                                                                         \
    hipLaunchKernelGGL((k_attn2<DD, NWV>), dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch),    \
                       dim3(NWV * 64), 0, bf_stream(stream), (const u16*)q, (const u16*)k,          \
                       (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs,    \
                       o_bs, sl2, o_map)
        // short sequences (<= 288 queries): 6 = one 9-wave workgroup per (batch, head), 7 = two
        // 5-wave workgroups, 8 = three 3-wave workgroups (several workgroups per CU, independent
        // barriers; K / V re-read from L2); longer ones: 4-wave workgroups of 128 queries
        const bool short_s = nw_one > 4 && nw_one <= 9;
        const int var = g_attn_variant;      // (`v` is the V operand)
        // <= 64 queries per (batch, head) (CLIP's last block: the class token only): 2-wave
        // workgroups, so no idle waves compute empty query blocks
#define LAUNCH_2L(DD)                                                                             \
    hipLaunchKernelGGL((k_attn2<DD, 9, false, false, false, false, false, true>), dim3(1, heads, batch), \
                       dim3(576), 0, bf_stream(stream), (const u16*)q, (const u16*)k,               \
                       (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs,    \
                       o_bs, sl2, o_map, 1.f)
#define LAUNCH_2L4(DD)                                                                            \
    hipLaunchKernelGGL((k_attn2<DD, 4, false, false, false, false, false, true>),                  \
                       dim3((sq + 127) / 128, heads, batch), dim3(256), 0, bf_stream(stream),       \
                       (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs,    \
                       v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map, 1.f)
#define LAUNCH_2D(DD)                                                                             \
    if (nw_one <= 2) { LAUNCH_2(DD, 2); }                                                          \
    else if (!short_s && var == 6) { LAUNCH_2L4(DD); }                                             \
    else if (!short_s) { LAUNCH_2(DD, 4); }                                                        \
    else if (var == 7) { LAUNCH_2(DD, 5); }                                                        \
    else if (var == 8) { LAUNCH_2(DD, 3); }                                                        \
    else if (var == 6) { LAUNCH_2L(DD); }                                                          \
    else { LAUNCH_2(DD, 9); }
        switch (head_dim) {
            case 32: LAUNCH_2D(32); break;
            case 64: LAUNCH_2D(64); break;
            case 80: LAUNCH_2D(80); break;
            case 128: LAUNCH_2(128, 4); break;
            default: return BF_ERR_UNSUPPORTED;
        }
#undef LAUNCH_2D
#undef LAUNCH_2L
#undef LAUNCH_2L4
#undef LAUNCH_2
        return bf_check_launch();
    }
    if (g_attn_variant >= 1) {
#define LAUNCH_S(DD, NWV)                                                                         \
    hipLaunchKernelGGL((k_attn_s<DD, NWV>), dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch),   \
                       dim3(NWV * 64), 0, bf_stream(stream), (const u16*)q, (const u16*)k,          \
                       (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs,    \
                       o_bs, sl2, o_map, g_attn_variant == 2 ? 0 : 1)
#define LAUNCH_SD(DD)                                                                             \
    if (nw_one > 4 && nw_one <= 9) {                                                              \
        if (g_attn_variant == 4) { LAUNCH_S(DD, 5); }                                             \
        else if (g_attn_variant == 5) { LAUNCH_S(DD, 3); }                                        \
        else { LAUNCH_S(DD, 9); }                                                                 \
    } else { LAUNCH_S(DD, 4); }
        switch (head_dim) {
            case 32: LAUNCH_SD(32); break;
            case 64: LAUNCH_SD(64); break;
            case 80: LAUNCH_SD(80); break;
            case 128: LAUNCH_S(128, 4); break;     // 9 waves would spill at D = 128
            default: return BF_ERR_UNSUPPORTED;
        }
#undef LAUNCH_SD
#undef LAUNCH_S
        return bf_check_launch();
    }
#define LAUNCH_NW(DD, NWV, NTV)                                                                   \
    hipLaunchKernelGGL((k_attn<DD, NWV, NTV>), dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch), \
                       dim3(NWV * 64), 0, bf_stream(stream), (const u16*)q, (const u16*)k,          \
                       (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs,    \
                       o_bs, sl2, o_map)
#define LAUNCH(DD)                                                                                \
    if (nw_one > 4 && nw_one <= 9 && sk <= 5 * AT_KT) { LAUNCH_NW(DD, 9, 5); }                     \
    else if (nw_one > 4 && nw_one <= 9) { LAUNCH_NW(DD, 9, 1); }                                  \
    else { LAUNCH_NW(DD, 4, 1); }
#define LAUNCH_STREAM(DD)                                                                         \
    if (nw_one > 4 && nw_one <= 9) { LAUNCH_NW(DD, 9, 1); } else { LAUNCH_NW(DD, 4, 1); }
    switch (head_dim) {
        case 32: LAUNCH(32); break;
        case 64: LAUNCH(64); break;
        case 80: LAUNCH(80); break;
        case 128: LAUNCH_STREAM(128); break;   // resident K/V would exceed the 160 KiB LDS
        default: return BF_ERR_UNSUPPORTED;
    }
#undef LAUNCH
#undef LAUNCH_STREAM
#undef LAUNCH_NW
    return bf_check_launch();
}

BF_API int bf_attention_bf16(const void* q, const void* k, const void* v, void* o, int batch,
                             int heads, int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs,
                             int o_rs, long long q_bs, long long k_bs, long long v_bs,
                             long long o_bs, float scale, void* stream) {
    return bf_attention_bf16_omap(q, k, v, o, batch, heads, sq, sk, head_dim, q_rs, k_rs, v_rs, o_rs,
                                  q_bs, k_bs, v_bs, o_bs, scale, nullptr, stream);
}

// the same attention (k_attn2, the default schedule) with an fp8 e4m3 output
// saturate_448(o * out_qscale); o_rs / o_bs in elements = bytes, o_rs % 4 == 0
BF_API int bf_attention_fp8out(const void* q, const void* k, const void* v, void* o, int batch,
                               int heads, int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs,
                               int o_rs, long long q_bs, long long k_bs, long long v_bs, long long o_bs,
                               float scale, float out_qscale, void* stream) {
    if (!q || !k || !v || !o || batch <= 0 || heads <= 0 || sq <= 0 || sk <= 0 || !(out_qscale > 0.f))
        return BF_ERR_ARG;
    if ((q_rs | k_rs | v_rs) % 8 != 0 || o_rs % 4 != 0 || o_bs % 4 != 0) return BF_ERR_UNSUPPORTED;
    const float sl2 = scale * 1.4426950408889634f;
    const int nw_one = (sq + 31) / 32;
    // k_attn6 (the bf16 default's persistent short-head kernel) with the fp8 row store
    const bool k6_ok = (long long)batch * heads < (1LL << 30) &&
                       (long long)sq * o_rs + 2LL * ((long long)sq * q_rs + (long long)sk * (k_rs > v_rs ? k_rs : v_rs)) < (1LL << 31);
    const int k6_grid = attn_num_cus() < batch * heads ? attn_num_cus() : batch * heads;
#define LAUNCH_8(DD, NWV)                                                                         \
    if (g_attn_variant == 6)                                                                      \
        hipLaunchKernelGGL((k_attn2<DD, NWV, true, false, false, false, false, true>),             \
                           dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch), dim3(NWV * 64), 0, \
                           bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, \
                           sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2,           \
                           (const int32_t*)nullptr, out_qscale);                                  \
    else                                                                                          \
    hipLaunchKernelGGL((k_attn2<DD, NWV, true>), dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch), \
                       dim3(NWV * 64), 0, bf_stream(stream), (const u16*)q, (const u16*)k,          \
                       (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs,    \
                       o_bs, sl2, (const int32_t*)nullptr, out_qscale)
#define LAUNCH_8D(DD)                                                                             \
    if (g_attn_variant == 10 && nw_one == 9 && sq % 32 == 1) {                                    \
        hipLaunchKernelGGL((k_attn2<DD, 8, true, false, true>), dim3(1, heads, batch), dim3(512), 0,  \
                           bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, \
                           sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2,                 \
                           (const int32_t*)nullptr, out_qscale);                                    \
    } else if (DD == 80 && g_attn_variant == 11 && nw_one == 9 && sq <= 8 * 32 + 16) {            \
        hipLaunchKernelGGL((k_attn2<80, 9, true, false, false, true>), dim3(1, heads, batch), dim3(576), 0, \
                           bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, \
                           sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2,                 \
                           (const int32_t*)nullptr, out_qscale);                                    \
    } else if (nw_one > 4 && nw_one <= 9 && g_attn_variant == 26 && k6_ok) {                             \
        hipLaunchKernelGGL((k_attn6<DD, 9, true>), dim3(k6_grid), dim3(576), 0, bf_stream(stream),        \
                           (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, \
                           o_rs, q_bs, k_bs, v_bs, o_bs, sl2, heads, batch * heads, out_qscale);           \
    } else if (nw_one > 4 && nw_one <= 9) { LAUNCH_8(DD, 9); } else { LAUNCH_8(DD, 4); }
    switch (head_dim) {
        case 64: LAUNCH_8D(64); break;
        case 80: LAUNCH_8D(80); break;
        default: return BF_ERR_UNSUPPORTED;
    }
#undef LAUNCH_8D
#undef LAUNCH_8
    return bf_check_launch();
}

// causal self-attention (sq == sk == s): the CLIP text tower (open_clip TextTransformer's attn_mask,
// precompute_class_features.py:37 encode_text); same k_attn2 body, keys after the query masked
BF_API int bf_attention_causal(const void* q, const void* k, const void* v, void* o, int batch, int heads,
                               int s, int head_dim, int q_rs, int k_rs, int v_rs, int o_rs, long long q_bs,
                               long long k_bs, long long v_bs, long long o_bs, float scale, void* stream) {
    if (!q || !k || !v || !o || batch <= 0 || heads <= 0 || s <= 0) return BF_ERR_ARG;
    if ((q_rs | k_rs | v_rs) % 8 != 0 || o_rs % 4 != 0) return BF_ERR_UNSUPPORTED;
    const float sl2 = scale * 1.4426950408889634f;
#define LAUNCH_C(DD)                                                                              \
    hipLaunchKernelGGL((k_attn2<DD, 4, false, true>), dim3((s + 127) / 128, heads, batch), dim3(256), \
                       0, bf_stream(stream), (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, s, s, \
                       q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, (const int32_t*)nullptr, 1.f)
    switch (head_dim) {
        case 64: LAUNCH_C(64); break;
        case 80: LAUNCH_C(80); break;
        default: return BF_ERR_UNSUPPORTED;
    }
#undef LAUNCH_C
    return bf_check_launch();
}
