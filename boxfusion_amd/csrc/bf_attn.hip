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

// NW waves of 32 queries per workgroup; NT key tiles resident in LDS at once: NT == 1 streams
// the keys tile by tile, NT > 1 (short sequences, sk <= 64*NT) stages every key and V^T column
// of the (batch, head) once and runs the whole key loop without barriers.
template <int D, int NW, int NT>
__global__ void __launch_bounds__(NW * 64) k_attn(const u16* __restrict__ Q, const u16* __restrict__ K,
                                                     const u16* __restrict__ V, u16* __restrict__ O,
                                                     int sq, int sk, int q_rs, int k_rs, int v_rs,
                                                     int o_rs, long long q_bs, long long k_bs,
                                                     long long v_bs, long long o_bs, float scale_log2) {
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
    if (q < sq) {
        const float inv = 1.0f / l_run;
        u16* orow = O + b * o_bs + (size_t)q * o_rs + h * D;
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

BF_API int bf_attention_bf16(const void* q, const void* k, const void* v, void* o, int batch,
                             int heads, int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs,
                             int o_rs, long long q_bs, long long k_bs, long long v_bs,
                             long long o_bs, float scale, void* stream) {
    if (!q || !k || !v || !o || batch <= 0 || heads <= 0 || sq <= 0 || sk <= 0) return BF_ERR_ARG;
    if ((q_rs | k_rs | v_rs) % 8 != 0 || o_rs % 4 != 0) return BF_ERR_UNSUPPORTED;
    const float sl2 = scale * 1.4426950408889634f;
    // short sequences (CLIP: 257 tokens) run every query of a (batch, head) in ONE workgroup of
    // ceil(sq/32) waves, so K/V are staged once and no 128-query tile is almost empty
    const int nw_one = (sq + 31) / 32;
#define LAUNCH_NW(DD, NWV, NTV)                                                                   \
    hipLaunchKernelGGL((k_attn<DD, NWV, NTV>), dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch), \
                       dim3(NWV * 64), 0, bf_stream(stream), (const u16*)q, (const u16*)k,          \
                       (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs,    \
                       o_bs, sl2)
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
