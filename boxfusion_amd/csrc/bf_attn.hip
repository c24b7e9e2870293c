// bf_attn.hip — fused multi-head attention (flash-style online softmax) on gfx950 MFMA.
//
// Used for CuTR's joint RGB+depth window attention (vit.py:170-203: 512 keys per window, the
// row softmax spans all concatenated keys, so it is exact joint attention), its global blocks
// (1600 tokens), CLIP ViT-H/14 (257 tokens, head_dim 80; tools/utils.py:383-403) and the CLIP
// text tower's causal attention (precompute_class_features.py:37).
//
// Element (b, h, s, d) of X in {Q, K, V, O} lives at X + b*x_bs + s*x_rs + h*D + d (token-major,
// straight out of / into the QKV and proj GEMMs; no transposes in HBM).
//
// One kernel, k_attn2 (per workgroup: NW wave64, 32 queries per wave, one (batch, head)):
//   * Q^T fragments stay in registers for the whole key loop;
//   * key tiles of 64 stream through a double-buffered LDS ring: K rows padded to D+8 elements
//     (conflict-free ds_read_b128 fragments), V row-major with a row pitch of 64 or 192 mod 256
//     bytes, read transposed by ds_read_b64_tr_b16 as the A operand of O^T = V^T P^T;
//   * S^T = K Q^T via v_mfma_f32_32x32x16_bf16 -> the query sits on the lane, keys in the 16
//     accumulator registers (+ the lane half), so the row max/sum is an in-lane reduction plus one
//     cross-half exchange, and the rescale of O^T is a per-lane scalar;
//   * the S^T accumulator, converted to bf16, is directly the B operand of O^T = V^T P^T;
//   * softmax in f32 with exp2 (scale*log2e folded), O normalised once at the end.
// Earlier structures (resident K/V, persistent walks, one wave per SIMD with two query blocks,
// an eighth-wave VALU query, ping-pong tiles, 3- and 5-wave short-head splits) all measured
// slower on CLIP's shape or no faster; they are in the git history.
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

typedef short s16x4 __attribute__((ext_vector_type(4)));


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

// ------------------------------------------------------------------------------------------
// k_attn2, restructured for the VALU budget of short heads
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
// LSTQ: output rows staged through LDS and stored as whole head rows (the default for non-causal
// launches; LSTQ = false keeps the per-lane fragment stores)
// The D = 64 4-wave form (CuTR's windows and global blocks, the text tower) is held to 3 waves per
// SIMD (163 registers instead of 200 and 64 AGPRs, no spills): 3 workgroups per CU instead of 2
// take 15-18 % off its shapes (joint windows 105.5-110 -> 86.5-89.8 us, global 97.6-100.5 ->
// 84.3-84.5; scripts/probe/attn_cutr_probe.py, profiles/r05_attn_cutr_probe.log).  4 waves per
// SIMD (<= 128 registers) is out of the allocator's reach.  ATTN_WPE64 = 1 rebuilds the old form.
#ifndef ATTN_WPE64
#define ATTN_WPE64 3
#endif
// The D = 80 4-wave form (CLIP's 257-query heads as three workgroups of 128 / 128 / 1 queries, the
// last one's three empty waves skipping the MFMA work) takes the same bound (166-168 registers
// instead of 248): 112.8-116.0 vs 117.6-118.7 us for the 9-wave form; 140 us without the bound.
// Not the causal instantiation (it spills at 168).
#ifndef ATTN_WPE80
#define ATTN_WPE80 3
#endif
template <int D, int NW, bool F8O = false, bool CAUSAL = false, bool LSTQ = false>
__global__ void __launch_bounds__(NW * 64, (D == 64 && NW == 4) ? ATTN_WPE64 : (D == 80 && NW == 4 && !CAUSAL) ? ATTN_WPE80 : 1)
k_attn2(const u16* __restrict__ Q, const u16* __restrict__ K,
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
    constexpr int NBUF = 2;
    __shared__ __attribute__((aligned(16))) u16 sK[NBUF * KTILE];
    __shared__ __attribute__((aligned(16))) u16 sV[NBUF * VTILE];
    // LST (the default for one-workgroup short heads): the bf16 output rows go through a per-wave
    // LDS region of their own and leave as whole 2D-byte head rows (16 B per lane along the row)
    // instead of 8-byte fragments of 32 rows per store instruction (CLIP: 122.8 -> 115.8 us)
    // (8- and 9-wave workgroups: an LDS region of their own, free at one workgroup per CU; 4-wave ones
    // reuse the K ring after a barrier, so their occupancy is unchanged)
    constexpr bool LST = LSTQ && !CAUSAL && D % 16 == 0;
    constexpr int EB = F8O ? 1 : 2;                                 // output bytes per element
    constexpr int OROW = ((EB * D + 16) / 32) * 32 + 16;           // bytes per staged row (16-B aligned)
    constexpr bool OWN = NW >= 8;
    static_assert(!LST || OWN || NW * 32 * OROW <= NBUF * KTILE * 2, "staged rows fit the K ring");
    __shared__ __attribute__((aligned(16))) unsigned char sO[LST && OWN ? NW * 32 * OROW : 16];

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const AttnBlk blk = attn_block(1);
    const int h = blk.h, b = blk.b;
    const int fr = lane & 31, fh = lane >> 5;
    const int q = blk.qb * (NW * 32) + wave * 32 + fr;
    // a wave whose 32 queries all lie past sq (the last query tile of a head) stages K / V and
    // meets every barrier but skips the MFMA / softmax work (wave-uniform)
    const bool idle = blk.qb * (NW * 32) + wave * 32 >= sq;
    const u16* Qb = Q + b * q_bs + h * D;
    const u16* Kb = K + b * k_bs + h * D;
    const u16* Vb = V + b * v_bs + h * D;

    bf16x8 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
        qf[ks] = *reinterpret_cast<const bf16x8*>(Qb + (size_t)min(q, sq - 1) * q_rs + 16 * ks + 8 * fh);
    // V padding columns: a ones column at d = D (the row sum), zeros after it
    if (VROW > D)
        for (int i = t; i < NBUF * AT_KT * (VROW - D); i += NT) {
            const int r = i / (VROW - D), c = i % (VROW - D);
            sV[r * VROW + D + c] = (ONES && c == 0) ? (u16)0x3F80 : (u16)0;
        }

    static_assert(CH % 64 == 0 && NT % 64 == 0, "wave-uniform staging guard");
    constexpr int NTS = NT;
    const int ts = t;
    constexpr int NSO = (CH + NTS - 1) / NTS;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 stk[NSO], stv[NSO];
    int srow[NSO], scol[NSO];
#pragma unroll
    for (int i = 0; i < NSO; ++i) {
        const int c = min(ts + i * NTS, CH - 1);
        srow[i] = c / CPR;
        scol[i] = (c % CPR) * 8;
    }
    auto stage_load = [&](int k0_) {
#pragma unroll
        for (int i = 0; i < NSO; ++i) {
            const int key = min(k0_ + srow[i], sk - 1);
            stk[i] = *reinterpret_cast<const u32x4*>(Kb + (size_t)key * k_rs + scol[i]);
            stv[i] = *reinterpret_cast<const u32x4*>(Vb + (size_t)key * v_rs + scol[i]);
        }
    };
    auto stage_store = [&](int buf_) {
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
    };
    auto tile_body = [&](int tile, auto mask_tag) {
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
    } else {
        for (int tile = 0; tile < nfull; ++tile) {
            const bool more = tile + 1 < ntiles;
            if (more) stage_load((tile + 1) * AT_KT);          // in flight during this tile
            if (!idle) tile_body(tile, std::false_type{});
            if (more) stage_store((tile + 1) % NBUF);
            __syncthreads();
        }
        if (nfull < ntiles && !idle) tile_body(nfull, std::true_type{});
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
        if (idle) return;
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
// Per-call variant (bf_attention_bf16_ex / bf_attention_fp8out_ex; 0 = 6): 6 (default) k_attn2 with
// the LDS-staged whole-row output stores for non-causal launches; 27 the same kernel with the
// per-lane fragment stores (A/B reference; bit-identical); 28: 129-288 queries on 9 waves (the
// round-4 dispatch), 29 / 30: 129-256 queries on 4 / 8 waves, 31: 129-288 on 4 waves, for every
// head dim; 33: 449-512 queries at D = 64 on 4 waves (A/B references; bit-identical).
BF_API int bf_attention_bf16_ex(const void* q, const void* k, const void* v, void* o, int batch,
                                int heads, int sq, int sk, int head_dim, int q_rs, int k_rs,
                                int v_rs, int o_rs, long long q_bs, long long k_bs, long long v_bs,
                                long long o_bs, float scale, const int32_t* o_map, int variant,
                                void* stream) {
    const int av = variant == 0 ? 6 : variant;
    if (!q || !k || !v || !o || batch <= 0 || heads <= 0 || sq <= 0 || sk <= 0) return BF_ERR_ARG;
    if ((q_rs | k_rs | v_rs) % 8 != 0 || o_rs % 4 != 0) return BF_ERR_UNSUPPORTED;
    const float sl2 = scale * 1.4426950408889634f;
    // short sequences (CLIP: 257 tokens) run every query of a (batch, head) in ONE workgroup of
    // ceil(sq/32) <= 9 waves, so K/V are staged once and no 128-query tile is almost empty; longer
    // ones 4-wave workgroups of 128 queries; <= 64 queries (CLIP's last block: the class token
    // only) 2-wave workgroups
    const int nw_one = (sq + 31) / 32;
    const bool short_s = nw_one > 4 && nw_one <= 9;
    const bool lst = av != 27;
    // 129-256 queries (CuTR's rgb-only and last-depth windows: 256): a ninth wave would hold no
    // query.  D = 64 and 80 take 4-wave workgroups of 128 queries (3 per CU at the forms' 3 waves
    // per SIMD: rgb windows 37.3 -> 28.2 us against 8 waves, last-depth 55.8 -> 43.7, CLIP-shaped
    // 256-query heads 108 -> 92), other head dims 8 waves (profiles/r05_attn_cutr_probe.log).
    // Variants 28 / 29 / 30: 9 / 4 / 8 waves for every D (A/B references; every form gives the same
    // bits).
    // 257-288 queries (CLIP: 257): 9 waves, at D = 80 4-wave workgroups (ATTN_WPE80 above).
    // Variant 28 restores 9 waves for all of 129-288, 31 takes 4 waves for all of it.
    const int mid = av == 28 ? 9 : av == 29 ? 4 : av == 30 ? 8
                  : (head_dim == 64 || head_dim == 80) ? 4 : 8;
    const bool four_all = av == 31;
    const int top = av == 28 ? 9 : (four_all || head_dim == 80) ? 4 : 9;
    const bool eight = short_s && nw_one <= 8 && mid == 8 && !four_all;
    const bool nine = short_s && !four_all && (nw_one <= 8 ? mid == 9 : top == 9);
    // 449-512 queries at D = 64 (CuTR's joint windows: 512) on two 8-wave workgroups per head
    // instead of four 4-wave ones: K / V staged twice instead of four times, 76.9-79.0 vs 86.3-89.8
    // us (the 1600-token global blocks and the 256-query windows are faster on 4 waves).  Variant
    // 33: the 4-wave form (A/B; the same bits).
    const bool wide8 = head_dim == 64 && sq > 448 && sq <= 512 && av != 33;
    const hipStream_t st = bf_stream(stream);
#define LAUNCH_2(DD, NWV, LS)                                                                     \
    hipLaunchKernelGGL((k_attn2<DD, NWV, false, false, LS>), dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch), \
                       dim3(NWV * 64), 0, st, (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, \
                       q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, o_map, 1.f)
#define LAUNCH_2D(DD)                                                                             \
    if (nw_one <= 2) { LAUNCH_2(DD, 2, false); }                                                  \
    else if (eight) { if (lst) { LAUNCH_2(DD, 8, true); } else { LAUNCH_2(DD, 8, false); } }      \
    else if (nine) { if (lst) { LAUNCH_2(DD, 9, true); } else { LAUNCH_2(DD, 9, false); } }       \
    else if (wide8) { if (lst) { LAUNCH_2(DD, 8, true); } else { LAUNCH_2(DD, 8, false); } }      \
    else { if (lst) { LAUNCH_2(DD, 4, true); } else { LAUNCH_2(DD, 4, false); } }
    switch (head_dim) {
        case 32: LAUNCH_2D(32); break;
        case 64: LAUNCH_2D(64); break;
        case 80: LAUNCH_2D(80); break;
        case 128: LAUNCH_2(128, 4, false); break;
        default: return BF_ERR_UNSUPPORTED;
    }
#undef LAUNCH_2D
#undef LAUNCH_2
    return bf_check_launch();
}

BF_API int bf_attention_bf16_omap(const void* q, const void* k, const void* v, void* o, int batch,
                                  int heads, int sq, int sk, int head_dim, int q_rs, int k_rs,
                                  int v_rs, int o_rs, long long q_bs, long long k_bs, long long v_bs,
                                  long long o_bs, float scale, const int32_t* o_map, void* stream) {
    return bf_attention_bf16_ex(q, k, v, o, batch, heads, sq, sk, head_dim, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs,
                                v_bs, o_bs, scale, o_map, 0, stream);
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
BF_API int bf_attention_fp8out_ex(const void* q, const void* k, const void* v, void* o, int batch,
                                  int heads, int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs,
                                  int o_rs, long long q_bs, long long k_bs, long long v_bs, long long o_bs,
                                  float scale, float out_qscale, int variant, void* stream) {
    const int av = variant == 0 ? 6 : variant;
    if (!q || !k || !v || !o || batch <= 0 || heads <= 0 || sq <= 0 || sk <= 0 || !(out_qscale > 0.f))
        return BF_ERR_ARG;
    if ((q_rs | k_rs | v_rs) % 8 != 0 || o_rs % 4 != 0 || o_bs % 4 != 0) return BF_ERR_UNSUPPORTED;
    const float sl2 = scale * 1.4426950408889634f;
    const int nw_one = (sq + 31) / 32;
    const bool lst = av != 27;
    const hipStream_t st = bf_stream(stream);
#define LAUNCH_8(DD, NWV, LS)                                                                     \
    hipLaunchKernelGGL((k_attn2<DD, NWV, true, false, LS>), dim3((sq + NWV * 32 - 1) / (NWV * 32), heads, batch), \
                       dim3(NWV * 64), 0, st, (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, sq, sk, \
                       q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs, sl2, (const int32_t*)nullptr, out_qscale)
    // 257-288 queries at D = 80 (CLIP) on 4-wave workgroups as in bf_attention_bf16 (variant 28: 9)
    const bool nine = nw_one > 4 && nw_one <= 9 && !(head_dim == 80 && nw_one == 9 && av != 28);
#define LAUNCH_8D(DD)                                                                             \
    if (nine) { if (lst) { LAUNCH_8(DD, 9, true); } else { LAUNCH_8(DD, 9, false); } }             \
    else { if (lst) { LAUNCH_8(DD, 4, true); } else { LAUNCH_8(DD, 4, false); } }
    switch (head_dim) {
        case 64: LAUNCH_8D(64); break;
        case 80: LAUNCH_8D(80); break;
        default: return BF_ERR_UNSUPPORTED;
    }
#undef LAUNCH_8D
#undef LAUNCH_8
    return bf_check_launch();
}

BF_API int bf_attention_fp8out(const void* q, const void* k, const void* v, void* o, int batch,
                               int heads, int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs,
                               int o_rs, long long q_bs, long long k_bs, long long v_bs, long long o_bs,
                               float scale, float out_qscale, void* stream) {
    return bf_attention_fp8out_ex(q, k, v, o, batch, heads, sq, sk, head_dim, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs,
                                  v_bs, o_bs, scale, out_qscale, 0, stream);
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
