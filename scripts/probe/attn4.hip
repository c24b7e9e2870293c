// Probe: k_attn4 (one wave per SIMD, two 32-query blocks per wave; git 5045105) with the O^T
// accumulators pinned in AGPRs ("+a"-constrained MFMAs) -- against the shipped k_attn2 on CLIP heads.
#include "../../boxfusion_amd/csrc/bf_attn.hip"

#ifndef A4_FENCES
#define A4_FENCES 0
#endif
#if A4_FENCES
#define A4_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define A4_FENCE() do {} while (0)
#endif
#ifndef A4_PIN
#define A4_PIN 1
#endif
#if A4_PIN
#define A4_MFMA32(ACC, A_, B_) asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(A_), "v"(B_))
#define A4_MFMA16(ACC, A_, B_) asm("v_mfma_f32_16x16x16_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(A_), "v"(B_))
// wait states between an MFMA's AGPR result and a VALU access to it (and back): the compiler does
// not price the inline-asm producers
#define A4_HAZ() asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory")
#else
#define A4_MFMA32(ACC, A_, B_) ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A_, B_, ACC, 0, 0, 0)
#define A4_MFMA16(ACC, A_, B_) ACC = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A_, B_, ACC, 0, 0, 0)
#define A4_HAZ() do {} while (0)
#endif
// attn2_softmax with the O^T rescale fenced by wait states (O^T may sit in AGPRs written by asm MFMAs)
template <int D, int DB>
__device__ __forceinline__ void attn4_softmax(f32x16 (&s)[2], bool sub1, bool mask, int k0, int sk,
                                              int fh, float c, float& m_run, f32x16 (&o)[DB], bf16x8 (&pf)[2][2]) {
    if (mask) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int key = k0 + sub * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
                s[sub][e] = (key <= sk - 1) ? s[sub][e] : -INFINITY;
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
    if (__any(mt > m_run + AT2_THR)) {
        const float m_new = fmaxf(m_run, mt);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        A4_HAZ();
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[db][e] *= alpha;
        A4_HAZ();
    }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
        if (sub == 1 && !sub1) {
#pragma unroll
            for (int e = 0; e < 16; ++e) pf[1][e >> 3][e & 7] = (__bf16)0.0f;
            continue;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) pf[sub][e >> 3][e & 7] = (__bf16)__builtin_amdgcn_exp2f(fmaf(s[sub][e], c, -m_run));
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
                    A4_MFMA32(o[db], __builtin_bit_cast(bf16x8, lohi), pf[sub][ss]);
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
    float ma = -INFINITY, mb = -INFINITY;
    bf16x8 pa[2][2], pb[2][2];

    qk(0, qa, sa, true);
    attn4_softmax<D, DB>(sa, true, false, 0, sk, fh, scale_log2, ma, oa, pa);
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
        attn4_softmax<D, DB>(sb, sub1_t, LAST, k0, sk, fh, scale_log2, mb, ob, pb);
        pv(tile, pa, oa, sub1_t);
        A4_FENCE();
        if (!LAST) {
            qk(tile + 1, qa, sa, sub1_n);
            A4_FENCE();
            attn4_softmax<D, DB>(sa, sub1_n, NEXT_TAIL, k1, sk, fh, scale_log2, ma, oa, pa);
        }
        pv(tile, pb, ob, sub1_t);
        A4_FENCE();
        if (!LAST) qk(tile + 1, qb, sb, sub1_n);
        A4_FENCE();
        if (hasC) c_tile(tile);
        A4_FENCE();
        if (stage) {                                         // tile + 2 landed, slot tile - 1 free
            attn_wait_vm(0);
            raw_barrier();
        }
    };
    for (int tile = 0; tile < nt - 2; ++tile) body(tile, std::false_type{}, std::false_type{});
    body(nt - 2, std::true_type{}, std::false_type{});
    body(nt - 1, std::false_type{}, std::true_type{});

    A4_HAZ();
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


extern "C" int attn4_launch(const void* q, const void* k, const void* v, void* o, int batch, int heads, int sq, int sk,
                            int q_rs, int k_rs, int v_rs, int o_rs, long long q_bs, long long k_bs, long long v_bs,
                            long long o_bs, float scale, void* stream) {
    if (!(sq > 192 && sq <= 272 && sk > 2 * AT_KT && sk <= 5 * AT_KT)) return -1;
    hipLaunchKernelGGL((k_attn4<80>), dim3(1, heads, batch), dim3(256), 0, (hipStream_t)stream, (const u16*)q,
                       (const u16*)k, (const u16*)v, (u16*)o, sq, sk, q_rs, k_rs, v_rs, o_rs, q_bs, k_bs, v_bs, o_bs,
                       scale * 1.4426950408889634f, (const int32_t*)nullptr);
    return (int)hipGetLastError();
}
