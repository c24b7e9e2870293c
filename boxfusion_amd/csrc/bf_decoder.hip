// bf_decoder.hip — the CuTR decoder's global cross-attention bias on gfx950 (f32, HBM-bound).
//
// GlobalCrossAttention (cubify_transformer.py:93-190 of the reference; boxfusion_amd
// cubify_transformer.py GlobalCrossAttention) adds a relative position bias to the box queries'
// attention logits before the softmax:
//   ref  = (cx - w/2, cy - h/2, cx + w/2, cy + h/2) of each box query's reference box
//   rx[b,q,x,:] = cpb_mlp1((ref_x0, ref_x1) - pos_x[x]),  ry[b,q,y,:] = cpb_mlp2(... - pos_y[y])
//                 (Linear(2,512) + ReLU + Linear(512,heads, no bias))
//   attn[b,h,q,y*w+x] += rx[b,q,x,h] + ry[b,q,y,h];  attn = clip(attn, f32 min, f32 max);
//   attn = softmax(attn, -1)
// In torch that is a [B*nq*w, 512] hidden activation per axis, a broadcast [B,nq,h,w,heads] bias,
// an index_put add, a clip and a softmax over [B,heads,Nq,h*w] — about 1.6 GB of HBM traffic per
// decoder layer.  Here:
//   k_cpb_mlp_r    the reference width (hidden 512, 8 heads): one wave per 4 positions, every weight
//                  in registers, a butterfly reduce-scatter of the 32 head sums; 28 us vs 57 us for
//                  the LDS form at 8 x 300 x 40 (scripts/cpb_bench.py); writes rx / ry [B,nq,n,heads]
//   k_cpb_mlp      other widths: 8 lanes per (b, q, position), each over 1/8 of the hidden layer
//                  (weights in LDS, broadcast reads), xor-shuffle reduction
//   k_rpe_softmax  one wave per attention row: the row's two 1-D bias tables into LDS, the row
//                  read once, bias + clip + softmax, written once (in place)
// Numerics: f32 throughout; the sums run in a fixed order (not the BLAS blocking of the torch
// path), so results match the torch decoder to f32 rounding (tests compare with a tolerance).
#include "bf_common.h"
#include <cstdlib>

#define CPB_MAX_HIDDEN 512
#define CPB_MAX_HEADS 16
#define RPE_MAX_SIDE 256

// ------------------------------------------------------------------------------------------
// rx / ry tables
// ------------------------------------------------------------------------------------------
// 8 lanes per output position, each over hidden/8 units of the hidden layer; per unit one
// 16-B LDS read of (w1[j,0], w1[j,1], b1[j], 0) and the unit's heads-wide column of W2
// (transposed in LDS); the 8 partial head sums are combined with xor shuffles.
#define CPB_LANES 8
#define CPB_W2S (CPB_MAX_HEADS + 4)   // W2^T row stride (floats): 8 adjacent rows hit disjoint banks
#define CPB_BLOCKS 768                 // persistent (3 x 256 CUs at 41 KB LDS): weights staged once per WG
__global__ void __launch_bounds__(256) k_cpb_mlp(const float* __restrict__ ref, int B, int nq,
                                                 const float* __restrict__ pos, int n, int axis,
                                                 const float* __restrict__ w1,
                                                 const float* __restrict__ b1,
                                                 const float* __restrict__ w2, int hidden,
                                                 int heads, float* __restrict__ out) {
    __shared__ float4 s_l1[CPB_MAX_HIDDEN];                     // (w1a, w1b, b1, 0) per unit
    __shared__ float s_w2t[CPB_MAX_HIDDEN * CPB_W2S];           // [unit][head], 80-B rows
    for (int j = threadIdx.x; j < hidden; j += blockDim.x)
        s_l1[j] = make_float4(w1[2 * j], w1[2 * j + 1], b1[j], 0.f);
    for (int i = threadIdx.x; i < heads * hidden; i += blockDim.x) {
        const int hd = i / hidden, j = i % hidden;
        s_w2t[j * CPB_W2S + hd] = w2[i];
    }
    __syncthreads();
    const long long total = (long long)B * nq * n;
    const int sub = threadIdx.x % CPB_LANES;
    const long long step = (long long)gridDim.x * blockDim.x / CPB_LANES;
    // the 8 lanes of a position share e: the loop and the shuffles are uniform per lane group
    for (long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / CPB_LANES; e < total;
         e += step) {
    const long long ee = e;
    const int p = (int)(ee % n);
    const long long bq = ee / n;
    const float* r = ref + bq * 4;
    // (c - wh/2, c + wh/2) on this axis, minus the position
    const float c = r[axis], half = r[2 + axis] / 2;
    const float in0 = (c - half) - pos[p];
    const float in1 = (c + half) - pos[p];
    float acc[CPB_MAX_HEADS];
#pragma unroll
    for (int hd = 0; hd < CPB_MAX_HEADS; ++hd) acc[hd] = 0.f;
    const int per = hidden / CPB_LANES;                          // hidden % 8 == 0 (host check)
#pragma unroll 4
    for (int jj = 0; jj < per; ++jj) {
        const int j = jj * CPB_LANES + sub;      // the 8 lanes read 8 adjacent units: no bank conflicts
        const float4 l1 = s_l1[j];
        float hv = in0 * l1.x + in1 * l1.y + l1.z;
        hv = hv > 0.f ? hv : 0.f;
        const float4* w = reinterpret_cast<const float4*>(s_w2t + j * CPB_W2S);
#pragma unroll
        for (int q = 0; q < CPB_MAX_HEADS / 4; ++q) {
            if (4 * q < heads) {
                const float4 wv = w[q];
                acc[4 * q + 0] += wv.x * hv;
                acc[4 * q + 1] += wv.y * hv;
                acc[4 * q + 2] += wv.z * hv;
                acc[4 * q + 3] += wv.w * hv;
            }
        }
    }
#pragma unroll
    for (int hd = 0; hd < CPB_MAX_HEADS; ++hd) {
        if (hd < heads) {
#pragma unroll
            for (int o = CPB_LANES / 2; o > 0; o >>= 1) acc[hd] += __shfl_xor(acc[hd], o, 64);
        }
    }
    if (sub == 0) {
        float* o = out + e * heads;
#pragma unroll
        for (int hd = 0; hd < CPB_MAX_HEADS; ++hd)
            if (hd < heads) o[hd] = acc[hd];
    }
    }
}

// The reference shape (hidden 512, 8 heads): one wave per group of 4 positions, every weight in
// registers (lane l owns hidden units l + 64 u, u < 8: w1, b1 and its 8 W2 entries = 88 VGPRs), no
// LDS traffic in the loop.  Each lane accumulates the 4 x 8 partial head sums of its 8 units; a
// butterfly reduce-scatter over the 64 lanes (xor 32 .. 2, then xor 1) leaves lane l with the total
// of value (l >> 1) = (position (l >> 4), head (l >> 1) & 7), and the even lanes store the group's
// 32 contiguous outputs.
// one reduce-scatter step: lanes with (lane & SEL) keep values HALF..2 HALF-1, the others 0..HALF-1,
// each adding its xor-SEL partner's copy of the values it keeps
template <int HALF, int SEL>
__device__ __forceinline__ void cpb_halve(float* acc, int lane) {
    const bool up = (lane & SEL) != 0;
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
        const float keep = up ? acc[i + HALF] : acc[i];
        const float give = up ? acc[i] : acc[i + HALF];
        acc[i] = keep + __shfl_xor(give, SEL, 64);
    }
}
#define CPB_R_UNITS 8
#define CPB_R_HEADS 8
#define CPB_R_POS 4
__global__ void __launch_bounds__(256) k_cpb_mlp_r(const float* __restrict__ ref, long long total, int n,
                                                   const float* __restrict__ pos, int axis,
                                                   const float* __restrict__ w1,
                                                   const float* __restrict__ b1,
                                                   const float* __restrict__ w2, float* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float wa[CPB_R_UNITS], wb[CPB_R_UNITS], bb[CPB_R_UNITS], wt[CPB_R_UNITS][CPB_R_HEADS];
#pragma unroll
    for (int u = 0; u < CPB_R_UNITS; ++u) {
        const int j = lane + 64 * u;
        wa[u] = w1[2 * j];
        wb[u] = w1[2 * j + 1];
        bb[u] = b1[j];
#pragma unroll
        for (int hd = 0; hd < CPB_R_HEADS; ++hd) wt[u][hd] = w2[hd * 64 * CPB_R_UNITS + j];
    }
    const long long ngroups = (total + CPB_R_POS - 1) / CPB_R_POS;
    const int last_bq = (int)((total - 1) / n), last_p = (int)((total - 1) % n);
    for (long long g = (long long)blockIdx.x * 4 + wave; g < ngroups; g += (long long)gridDim.x * 4) {
        float in0[CPB_R_POS], in1[CPB_R_POS];
        // (box, position) of the group's first element by one division, then stepped (total < 2^31)
        const int e0 = (int)g * CPB_R_POS;
        int bq = e0 / n, p = e0 - bq * n;
#pragma unroll
        for (int pp = 0; pp < CPB_R_POS; ++pp) {
            const bool live = e0 + pp < total;           // the tail group repeats the last element
            const int pq = live ? p : last_p;
            const float* r = ref + (size_t)(live ? bq : last_bq) * 4;
            const float c = r[axis], half = r[2 + axis] / 2;
            in0[pp] = (c - half) - pos[pq];
            in1[pp] = (c + half) - pos[pq];
            if (++p == n) { p = 0; ++bq; }
        }
        float acc[CPB_R_POS * CPB_R_HEADS];
#pragma unroll
        for (int i = 0; i < CPB_R_POS * CPB_R_HEADS; ++i) acc[i] = 0.f;
#pragma unroll
        for (int u = 0; u < CPB_R_UNITS; ++u)
#pragma unroll
            for (int pp = 0; pp < CPB_R_POS; ++pp) {
                float hv = in0[pp] * wa[u] + in1[pp] * wb[u] + bb[u];
                hv = hv > 0.f ? hv : 0.f;
#pragma unroll
                for (int hd = 0; hd < CPB_R_HEADS; ++hd) acc[pp * CPB_R_HEADS + hd] += wt[u][hd] * hv;
            }
        // reduce-scatter: at width w, lanes with bit (lane & sel) keep the upper half of the values
        static_assert(CPB_R_POS * CPB_R_HEADS == 32, "five halving steps");
        cpb_halve<16, 32>(acc, lane);
        cpb_halve<8, 16>(acc, lane);
        cpb_halve<4, 8>(acc, lane);
        cpb_halve<2, 4>(acc, lane);
        cpb_halve<1, 2>(acc, lane);
        const float tot = acc[0] + __shfl_xor(acc[0], 1, 64);
        const long long e = g * CPB_R_POS + (lane >> 4);
        if ((lane & 1) == 0 && e < total) out[e * CPB_R_HEADS + ((lane >> 1) & 7)] = tot;
    }
}

BF_API int bf_cpb_mlp(const float* ref, int B, int nq, const float* pos, int n, int axis,
                      const float* w1, const float* b1, const float* w2, int hidden, int heads,
                      float* out, void* stream) {
    if (!ref || !pos || !w1 || !b1 || !w2 || !out || B < 0 || nq < 0 || n <= 0 || (axis != 0 && axis != 1))
        return BF_ERR_ARG;
    if (hidden <= 0 || hidden > CPB_MAX_HIDDEN || hidden % CPB_LANES || heads <= 0 ||
        heads > CPB_MAX_HEADS)
        return BF_ERR_CAPACITY;
    const long long total = (long long)B * nq * n;
    if (total == 0) return BF_OK;
    static const int use_r = [] { const char* e = getenv("BF_CPB_VARIANT"); return e ? atoi(e) : 1; }();
    if (use_r && hidden == 64 * CPB_R_UNITS && heads == CPB_R_HEADS && total < (1LL << 31) - CPB_R_POS) {
        const long long groups = (total + CPB_R_POS - 1) / CPB_R_POS;
        const long long blocks = (groups + 3) / 4;
        hipLaunchKernelGGL(k_cpb_mlp_r, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0,
                           bf_stream(stream), ref, total, n, pos, axis, w1, b1, w2, out);
        return bf_check_launch();
    }
    const long long blocks = (total * CPB_LANES + 255) / 256;
    hipLaunchKernelGGL(k_cpb_mlp, dim3((unsigned)(blocks < CPB_BLOCKS ? blocks : CPB_BLOCKS)), dim3(256), 0,
                       bf_stream(stream), ref, B, nq, pos, n, axis, w1, b1, w2, hidden, heads, out);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// bias + clip + softmax over one attention row per wave (in place)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int NPL>   // float4 per lane (row length <= 256 * NPL)
__global__ void __launch_bounds__(256) k_rpe_softmax(float* __restrict__ attn, int rows, int Nq,
                                                     int H, int q0, const float* __restrict__ rx,
                                                     const float* __restrict__ ry, int hh, int ww) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const int N = hh * ww;                                // multiple of 4
    const int q = row % Nq;
    const int bh = row / Nq;
    const int hd = bh % H, b = bh / H;
    const bool biased = q >= q0;
    const int nqb = Nq - q0;
    // this row's 1-D bias tables (ww + hh values, stride H in HBM) into LDS once
    __shared__ float s_bias[4][RPE_MAX_SIDE * 2];
    float* bx = s_bias[threadIdx.x >> 6];
    float* by = bx + RPE_MAX_SIDE;
    if (biased) {
        const float* rxr = rx + ((size_t)(b * nqb + (q - q0)) * ww) * H + hd;
        const float* ryr = ry + ((size_t)(b * nqb + (q - q0)) * hh) * H + hd;
        for (int i = lane; i < ww; i += 64) bx[i] = rxr[(size_t)i * H];
        for (int i = lane; i < hh; i += 64) by[i] = ryr[(size_t)i * H];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    float* a = attn + (size_t)row * N;
    const float fmax_ = 3.40282347e38f;
    float4 v[NPL];
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int c = (i * 64 + lane) * 4;
        if (c < N) {
            float4 x = *reinterpret_cast<const float4*>(a + c);
            float* xs = reinterpret_cast<float*>(&x);
            if (biased) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int nn = c + k, y = nn / ww, xx = nn - y * ww;
                    xs[k] = xs[k] + (bx[xx] + by[y]);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                xs[k] = fminf(fmaxf(xs[k], -fmax_), fmax_);   // clip(min=finfo.min, max=finfo.max)
                m = fmaxf(m, xs[k]);
            }
            v[i] = x;
        }
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int c = (i * 64 + lane) * 4;
        if (c < N) {
            float* xs = reinterpret_cast<float*>(&v[i]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                xs[k] = expf(xs[k] - m);
                s += xs[k];
            }
        }
    }
    s = wave_sum(s);
    const float inv = 1.0f / s;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int c = (i * 64 + lane) * 4;
        if (c < N) {
            float* xs = reinterpret_cast<float*>(&v[i]);
#pragma unroll
            for (int k = 0; k < 4; ++k) xs[k] *= inv;
            *reinterpret_cast<float4*>(a + c) = v[i];
        }
    }
}

BF_API int bf_rpe_softmax(float* attn, int B, int H, int Nq, int q0, const float* rx,
                          const float* ry, int hh, int ww, void* stream) {
    if (!attn || B < 0 || H <= 0 || Nq < 0 || q0 < 0 || q0 > Nq || hh <= 0 || ww <= 0)
        return BF_ERR_ARG;
    if (q0 < Nq && (!rx || !ry)) return BF_ERR_ARG;
    const int N = hh * ww;
    if (N % 4) return BF_ERR_ARG;
    if (hh > RPE_MAX_SIDE || ww > RPE_MAX_SIDE) return BF_ERR_CAPACITY;
    const int rows = B * H * Nq;
    if (rows == 0) return BF_OK;
    const unsigned grid = (unsigned)((rows + 3) / 4);
    hipStream_t s = bf_stream(stream);
    if (N <= 256 * 4) {
        hipLaunchKernelGGL(k_rpe_softmax<4>, dim3(grid), dim3(256), 0, s, attn, rows, Nq, H, q0, rx, ry, hh, ww);
    } else if (N <= 256 * 8) {
        hipLaunchKernelGGL(k_rpe_softmax<8>, dim3(grid), dim3(256), 0, s, attn, rows, Nq, H, q0, rx, ry, hh, ww);
    } else if (N <= 256 * 16) {
        hipLaunchKernelGGL(k_rpe_softmax<16>, dim3(grid), dim3(256), 0, s, attn, rows, Nq, H, q0, rx, ry, hh, ww);
    } else {
        return BF_ERR_CAPACITY;
    }
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// Fused global cross-attention (GlobalCrossAttention.forward after the q / k / v projections,
// cubify_transformer.py:93-190 of the reference), f32 end to end:
//   s[q,j] = (scale q_q) . k_j  (+ rx[b,q-q0,x_j,h] + ry[b,q-q0,y_j,h] for q >= q0, j = y*ww + x)
//   s = clip(s, -FLT_MAX, FLT_MAX);  out[q] = sum_j softmax_j(s)[j] v_j
// replacing the two batched f32 GEMMs, the [B,H,Nq,N] logits round trip through HBM and the
// head permutes of the torch path.  Head dim 32.  Workgroup = (32 queries, head, batch), 4 waves
// splitting the keys; per 32-key block one wave runs S^T = K Q^T (16 v_mfma_f32_32x32x2_f32: the
// query on the lane, exact f32 FMA chains) and O^T += V^T P^T (16 more, P straight from the S
// accumulator: k-step s of lane half h is the key S^T register s holds), with an online softmax
// (expf, f32) in between; the 4 waves' (max, sum, O) combine through LDS.  The bias tables of the
// workgroup's 32 queries sit in LDS as [position][query] (a half-wave reads 32 consecutive floats).
// Summation order differs from the torch path (f32 rounding; tests compare with a tolerance).
// ------------------------------------------------------------------------------------------
#define XA_MAX_SIDE 128
#define XA_WAVES 4
typedef float xa_f32x16 __attribute__((ext_vector_type(16)));

// SELF: the decoder's masked self-attention (nn.MultiheadAttention with the block mask of
// CubifyTransformer.decode: the q0 metric queries see only the q0 metric keys, the box queries
// only the box keys): no bias tables, keys = queries (N = Nq), key j valid for query i iff
// (j < q0) == (i < q0).
template <bool SELF>
__global__ void __launch_bounds__(XA_WAVES * 64) k_xattn(
    const float* __restrict__ q, int ldq, const float* __restrict__ k, int ldk,
    const float* __restrict__ v, int ldv, const float* __restrict__ rx, const float* __restrict__ ry,
    float* __restrict__ out, int ldo, int H, int Nq, int N, int q0, int hh, int ww, float scale) {
    __shared__ float s_bx[XA_MAX_SIDE * 32], s_by[XA_MAX_SIDE * 32];
    __shared__ float s_m[XA_WAVES][32], s_l[XA_WAVES][32];
    __shared__ float s_o[XA_WAVES][32][33];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int jq = lane & 31, hf = lane >> 5;
    const int qb = blockIdx.x, hd = blockIdx.y, b = blockIdx.z;
    const int qg = qb * 32 + jq;                       // this lane's query
    const int nqb = Nq - q0;
    // bias tables of the 32 queries: [x][query], [y][query] (0 for metric / absent queries)
    if (!SELF) {
        for (int i = t; i < ww * 32; i += XA_WAVES * 64) {
            const int x = i >> 5, j = i & 31, qq = qb * 32 + j;
            s_bx[i] = (qq >= q0 && qq < Nq) ? rx[(((size_t)b * nqb + (qq - q0)) * ww + x) * H + hd] : 0.f;
        }
        for (int i = t; i < hh * 32; i += XA_WAVES * 64) {
            const int y = i >> 5, j = i & 31, qq = qb * 32 + j;
            s_by[i] = (qq >= q0 && qq < Nq) ? ry[(((size_t)b * nqb + (qq - q0)) * hh + y) * H + hd] : 0.f;
        }
    }
    // Q^T fragments: k-step s of lane half hf is dim 16*hf + s (any order agreeing with K's)
    float qf[16];
    {
        const float* qp = q + ((size_t)b * Nq + min(qg, Nq - 1)) * ldq + hd * 32 + 16 * hf;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const float4 x = *reinterpret_cast<const float4*>(qp + 4 * s4);
            qf[4 * s4 + 0] = qg < Nq ? x.x * scale : 0.f;
            qf[4 * s4 + 1] = qg < Nq ? x.y * scale : 0.f;
            qf[4 * s4 + 2] = qg < Nq ? x.z * scale : 0.f;
            qf[4 * s4 + 3] = qg < Nq ? x.w * scale : 0.f;
        }
    }
    __syncthreads();
    const int nblk = (N + 31) / 32;
    const int kb0 = wave * nblk / XA_WAVES, kb1 = (wave + 1) * nblk / XA_WAVES;
    const float* kbase = k + (size_t)b * N * ldk + hd * 32;
    const float* vbase = v + (size_t)b * N * ldv + hd * 32;
    xa_f32x16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    const float FMAX = 3.40282347e38f;
    for (int kb = kb0; kb < kb1; ++kb) {
        // K fragment: key kb*32 + jq, dims 16*hf + [0,16).  (Loading the next block's K / V a
        // block ahead cost occupancy and measured slower: 96.7 -> 108.9 us per decoder layer; the
        // next K alone, 123 VGPRs: 97.9-98.0 vs 98.0-99.2 us, bit-identical, not kept --
        // scripts/xattn_bench.py.)
        float kf[16];
        {
            const int key = min(kb * 32 + jq, N - 1);
            const float* kp = kbase + (size_t)key * ldk + 16 * hf;
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const float4 x = *reinterpret_cast<const float4*>(kp + 4 * s4);
                kf[4 * s4 + 0] = x.x; kf[4 * s4 + 1] = x.y; kf[4 * s4 + 2] = x.z; kf[4 * s4 + 3] = x.w;
            }
        }
        // V^T fragment per k-step s: V[key of S^T register s in half hf][dim jq]
        float vf[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int key = min(kb * 32 + (s & 3) + 8 * (s >> 2) + 4 * hf, N - 1);
            vf[s] = vbase[(size_t)key * ldv + jq];
        }
        xa_f32x16 sc;
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.f;
#pragma unroll
        for (int s = 0; s < 16; ++s) sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[s], qf[s], sc, 0, 0, 0);
        // bias, clip, mask; register r holds key kb*32 + (r&3) + 8*(r>>2) + 4*hf
        float mt = -INFINITY;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int key0 = kb * 32 + 8 * g + 4 * hf;
            if (SELF) {
                const bool qmetric = qg < q0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 4 * g + i, key = key0 + i;
                    const float sv = (key < N && ((key < q0) == qmetric)) ? sc[r] : -INFINITY;
                    sc[r] = sv;
                    mt = fmaxf(mt, sv);
                }
                continue;
            }
            int y = key0 / ww, x = key0 - y * ww;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * g + i;
                float sv = sc[r] + (s_bx[x * 32 + jq] + s_by[min(y, hh - 1) * 32 + jq]);
                sv = sv > FMAX ? FMAX : (sv < -FMAX ? -FMAX : sv);
                sv = (key0 + i < N) ? sv : -INFINITY;
                sc[r] = sv;
                mt = fmaxf(mt, sv);
                if (++x == ww) { x = 0; ++y; }
            }
        }
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        if (mt > m_run) {
            const float alpha = expf(m_run - mt);        // m_run = -inf -> 0
            l_run *= alpha;
#pragma unroll
            for (int r = 0; r < 16; ++r) o[r] *= alpha;
            m_run = mt;
        }
        // a query with no valid key in this block so far (SELF: the metric queries) keeps
        // m_run = -inf: its probabilities are 0, not exp(-inf + inf)
        const float m_ref = m_run == -INFINITY ? 0.f : m_run;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float p = expf(sc[r] - m_ref);
            l_run += p;
            sc[r] = p;
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) o = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[s], sc[s], o, 0, 0, 0);
    }
    // combine the 4 waves: O^T lane (jq, hf) register r = dim (r&3) + 8*(r>>2) + 4*hf of query jq
    l_run += __shfl_xor(l_run, 32, 64);
    if (hf == 0) { s_m[wave][jq] = m_run; s_l[wave][jq] = l_run; }
#pragma unroll
    for (int r = 0; r < 16; ++r) s_o[wave][(r & 3) + 8 * (r >> 2) + 4 * hf][jq] = o[r];
    __syncthreads();
    {
        const int j = t & 31, d0 = (t >> 5) * 4;      // 8 threads per query, 4 dims each
        const int qq = qb * 32 + j;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < XA_WAVES; ++w) M = fmaxf(M, s_m[w][j]);
        float L = 0.f, e[XA_WAVES];
#pragma unroll
        for (int w = 0; w < XA_WAVES; ++w) {
            e[w] = s_m[w][j] == -INFINITY ? 0.f : expf(s_m[w][j] - M);
            L += s_l[w][j] * e[w];
        }
        const float inv = 1.0f / L;
        float r4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float acc = 0.f;
#pragma unroll
            for (int w = 0; w < XA_WAVES; ++w) acc += s_o[w][d0 + i][j] * e[w];
            r4[i] = acc * inv;
        }
        if (qq < Nq)
            *reinterpret_cast<float4*>(out + ((size_t)b * Nq + qq) * ldo + hd * 32 + d0) =
                make_float4(r4[0], r4[1], r4[2], r4[3]);
    }
}

BF_API int bf_xattn_f32(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                        const float* rx, const float* ry, float* out, int ldo, int B, int H, int Nq,
                        int q0, int hh, int ww, float scale, void* stream) {
    if (!q || !k || !v || !out || B < 0 || H <= 0 || Nq < 0 || q0 < 0 || q0 > Nq || hh <= 0 || ww <= 0)
        return BF_ERR_ARG;
    if (q0 < Nq && (!rx || !ry)) return BF_ERR_ARG;
    if (ldq % 4 || ldo % 4 || ldq < H * 32 || ldk < H * 32 || ldv < H * 32 || ldo < H * 32 ||
        (uintptr_t)q % 16 || (uintptr_t)k % 16 || (uintptr_t)out % 16 || ldk % 4)
        return BF_ERR_UNSUPPORTED;
    if (hh > XA_MAX_SIDE || ww > XA_MAX_SIDE || ww < 4) return BF_ERR_CAPACITY;
    if (B == 0 || Nq == 0) return BF_OK;
    const int N = hh * ww;
    hipLaunchKernelGGL(k_xattn<false>, dim3((Nq + 31) / 32, H, B), dim3(XA_WAVES * 64), 0, bf_stream(stream), q,
                       ldq, k, ldk, v, ldv, rx, ry, out, ldo, H, Nq, N, q0, hh, ww, scale);
    return bf_check_launch();
}

// the decoder self-attention (PreNormGlobalDecoderLayer.self_attn with CubifyTransformer.decode's
// block mask): q / k / v f32 [B, N, H*32] (row strides ldq / ldk / ldv, batches packed), q0 =
// number of metric queries, scale = head_dim^-0.5 applied to q (nn.MultiheadAttention)
BF_API int bf_self_attn_f32(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                            float* out, int ldo, int B, int H, int N, int q0, float scale, void* stream) {
    if (!q || !k || !v || !out || B < 0 || H <= 0 || N < 0 || q0 < 0 || q0 > N) return BF_ERR_ARG;
    if (ldq % 4 || ldo % 4 || ldk % 4 || ldq < H * 32 || ldk < H * 32 || ldv < H * 32 || ldo < H * 32 ||
        (uintptr_t)q % 16 || (uintptr_t)k % 16 || (uintptr_t)out % 16)
        return BF_ERR_UNSUPPORTED;
    if (B == 0 || N == 0) return BF_OK;
    hipLaunchKernelGGL(k_xattn<true>, dim3((N + 31) / 32, H, B), dim3(XA_WAVES * 64), 0, bf_stream(stream), q,
                       ldq, k, ldk, v, ldv, nullptr, nullptr, out, ldo, H, N, N, q0, 1, 1, scale);
    return bf_check_launch();
}
