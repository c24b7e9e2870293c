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
//   k_cpb_mlp      one thread per (b, q, position): the 512-wide hidden layer stays in registers
//                  (weights in LDS, broadcast reads), writes rx / ry [B,nq,n,heads] only
//   k_rpe_softmax  one wave per attention row: reads the row once, adds the bias built from the
//                  two small tables, clips, softmax, writes the row once (in place)
// Numerics: f32 throughout; the sums run in a fixed order (not the BLAS blocking of the torch
// path), so results match the torch decoder to f32 rounding (tests compare with a tolerance).
#include "bf_common.h"

#define CPB_MAX_HIDDEN 512
#define CPB_MAX_HEADS 16

// ------------------------------------------------------------------------------------------
// rx / ry tables
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_cpb_mlp(const float* __restrict__ ref, int B, int nq,
                                                 const float* __restrict__ pos, int n, int axis,
                                                 const float* __restrict__ w1,
                                                 const float* __restrict__ b1,
                                                 const float* __restrict__ w2, int hidden,
                                                 int heads, float* __restrict__ out) {
    __shared__ float s_w1[2 * CPB_MAX_HIDDEN], s_b1[CPB_MAX_HIDDEN];
    __shared__ float s_w2[CPB_MAX_HEADS * CPB_MAX_HIDDEN];
    for (int i = threadIdx.x; i < 2 * hidden; i += blockDim.x) s_w1[i] = w1[i];
    for (int i = threadIdx.x; i < hidden; i += blockDim.x) s_b1[i] = b1[i];
    for (int i = threadIdx.x; i < heads * hidden; i += blockDim.x) s_w2[i] = w2[i];
    __syncthreads();
    const long long total = (long long)B * nq * n;
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int p = (int)(e % n);
    const long long bq = e / n;
    const float* r = ref + bq * 4;
    // (c - wh/2, c + wh/2) on this axis, minus the position
    const float c = r[axis], half = r[2 + axis] / 2;
    const float in0 = (c - half) - pos[p];
    const float in1 = (c + half) - pos[p];
    float acc[CPB_MAX_HEADS];
#pragma unroll
    for (int hd = 0; hd < CPB_MAX_HEADS; ++hd) acc[hd] = 0.f;
    for (int j = 0; j < hidden; ++j) {
        float hv = in0 * s_w1[2 * j] + in1 * s_w1[2 * j + 1] + s_b1[j];
        hv = hv > 0.f ? hv : 0.f;
#pragma unroll
        for (int hd = 0; hd < CPB_MAX_HEADS; ++hd)
            if (hd < heads) acc[hd] += s_w2[hd * hidden + j] * hv;
    }
    float* o = out + e * heads;
#pragma unroll
    for (int hd = 0; hd < CPB_MAX_HEADS; ++hd)
        if (hd < heads) o[hd] = acc[hd];
}

BF_API int bf_cpb_mlp(const float* ref, int B, int nq, const float* pos, int n, int axis,
                      const float* w1, const float* b1, const float* w2, int hidden, int heads,
                      float* out, void* stream) {
    if (!ref || !pos || !w1 || !b1 || !w2 || !out || B < 0 || nq < 0 || n <= 0 || (axis != 0 && axis != 1))
        return BF_ERR_ARG;
    if (hidden <= 0 || hidden > CPB_MAX_HIDDEN || heads <= 0 || heads > CPB_MAX_HEADS)
        return BF_ERR_CAPACITY;
    const long long total = (long long)B * nq * n;
    if (total == 0) return BF_OK;
    hipLaunchKernelGGL(k_cpb_mlp, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
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
    const float* rxr = biased ? rx + ((size_t)(b * nqb + (q - q0)) * ww) * H + hd : nullptr;
    const float* ryr = biased ? ry + ((size_t)(b * nqb + (q - q0)) * hh) * H + hd : nullptr;
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
                    xs[k] = xs[k] + (rxr[(size_t)xx * H] + ryr[(size_t)y * H]);
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
