// bf_vit_ops.hip — memory-bound companions of the MFMA kernels (gfx950):
//   bf_layernorm      LayerNorm f32 -> bf16 with optional row scatter (window partition, pad rows
//                     left to the caller's zero-fill) — vit.py:283-291,326 / open_clip ln_1/ln_2
//   bf_im2col_rgb8    Preprocessor.normalize + ImageList pad + PatchEmbed im2col in one pass
//                     (preprocessor.py:131-144, imagelist.py:55-115, vit.py:102-128)
//   bf_im2col_f32     the same for the standardised depth map (1 channel)
//   bf_crop_resize_im2col  tools/utils.py:405-403 crop -> 224x224 bilinear -> CLIP normalise ->
//                     14x14 patch im2col (K padded with zeros to a multiple of 64)
// One wave per LayerNorm row; im2col writes 16-B bf16x8 chunks (coalesced).
#include "bf_common.h"
#include "bf_cv2.h"

typedef unsigned short u16;

#ifndef LN_PRELOAD_GB
#define LN_PRELOAD_GB 1         // 0: gamma / beta read after the reductions (38.9 vs 36.9 us, CLIP 32896 x 1280)
#endif

__device__ __forceinline__ u16 vf2bf(float f) {
    __bf16 b = (__bf16)f;
    return *reinterpret_cast<u16*>(&b);
}

struct alignas(16) W128 {
    uint32_t x, y, z, w;
};

// ------------------------------------------------------------------------------------------
// LayerNorm: one wave per row, C <= 4096, C % 4 == 0
// ------------------------------------------------------------------------------------------
// OUTK 0: bf16 output, 1: f32, 2: fp8 e4m3 (OCP) = sat448(y * qs) (the CLIP fp8 path's GEMM input)
template <int NPL, int OUTK>  // float4 per lane
__global__ void __launch_bounds__(256) k_layernorm(const float* __restrict__ x, int ldx,
                                                   const float* __restrict__ g,
                                                   const float* __restrict__ bb, float eps,
                                                   void* __restrict__ out_, int ldo,
                                                   const int32_t* __restrict__ row_map, int M,
                                                   int C, float qs = 1.f) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= M) return;
    const float* xr = x + (size_t)row * ldx;
    float4 v[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        int c = (lane + 64 * i) * 4;
        v[i] = *reinterpret_cast<const float4*>(xr + min(c, C - 4));   // address always in-row
    }
#if LN_PRELOAD_GB
    // gamma / beta fetched beside the row, not after the two reductions
    float4 gpre[NPL], bpre[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int c = min((lane + 64 * i) * 4, C - 4);
        gpre[i] = *reinterpret_cast<const float4*>(g + c);
        bpre[i] = *reinterpret_cast<const float4*>(bb + c);
    }
#endif
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        int c = (lane + 64 * i) * 4;
        if (c >= C) v[i] = make_float4(0, 0, 0, 0);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        int c = (lane + 64 * i) * 4;
        if (c < C) {
            float a = v[i].x - mean, b2 = v[i].y - mean, c2 = v[i].z - mean, d = v[i].w - mean;
            q += (a * a + b2 * b2) + (c2 * c2 + d * d);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q / (float)C + eps);
    const int orow = row_map ? row_map[row] : row;
    if (orow < 0) return;
    if (OUTK == 2) {
        unsigned char* yr = static_cast<unsigned char*>(out_) + (size_t)orow * ldo;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            int c = (lane + 64 * i) * 4;
            if (c < C) {
#if LN_PRELOAD_GB
                const float4 gg = gpre[i], be = bpre[i];
#else
                float4 gg = *reinterpret_cast<const float4*>(g + c);
                float4 be = *reinterpret_cast<const float4*>(bb + c);
#endif
                const float y0 = fminf(fmaxf(((v[i].x - mean) * rstd * gg.x + be.x) * qs, -448.f), 448.f);
                const float y1 = fminf(fmaxf(((v[i].y - mean) * rstd * gg.y + be.y) * qs, -448.f), 448.f);
                const float y2 = fminf(fmaxf(((v[i].z - mean) * rstd * gg.z + be.z) * qs, -448.f), 448.f);
                const float y3 = fminf(fmaxf(((v[i].w - mean) * rstd * gg.w + be.w) * qs, -448.f), 448.f);
                int p = __builtin_amdgcn_cvt_pk_fp8_f32(y0, y1, 0, false);
                p = __builtin_amdgcn_cvt_pk_fp8_f32(y2, y3, p, true);
                *reinterpret_cast<int*>(yr + c) = p;
            }
        }
        return;
    }
    if (OUTK == 1) {      // (in place allowed: the row is in registers before the first store)
        float* yr = static_cast<float*>(out_) + (size_t)orow * ldo;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            int c = (lane + 64 * i) * 4;
            if (c < C) {
#if LN_PRELOAD_GB
                const float4 gg = gpre[i], be = bpre[i];
#else
                float4 gg = *reinterpret_cast<const float4*>(g + c);
                float4 be = *reinterpret_cast<const float4*>(bb + c);
#endif
                *reinterpret_cast<float4*>(yr + c) =
                    make_float4((v[i].x - mean) * rstd * gg.x + be.x, (v[i].y - mean) * rstd * gg.y + be.y,
                                (v[i].z - mean) * rstd * gg.z + be.z, (v[i].w - mean) * rstd * gg.w + be.w);
            }
        }
        return;
    }
    u16* yr = static_cast<u16*>(out_) + (size_t)orow * ldo;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        int c = (lane + 64 * i) * 4;
        if (c < C) {
#if LN_PRELOAD_GB
            const float4 gg = gpre[i], be = bpre[i];
#else
            float4 gg = *reinterpret_cast<const float4*>(g + min(c, C - 4));
            float4 be = *reinterpret_cast<const float4*>(bb + min(c, C - 4));
#endif
            uint32_t lo = (uint32_t)vf2bf((v[i].x - mean) * rstd * gg.x + be.x) |
                          ((uint32_t)vf2bf((v[i].y - mean) * rstd * gg.y + be.y) << 16);
            uint32_t hi = (uint32_t)vf2bf((v[i].z - mean) * rstd * gg.z + be.z) |
                          ((uint32_t)vf2bf((v[i].w - mean) * rstd * gg.w + be.w) << 16);
            *reinterpret_cast<uint2*>(yr + c) = make_uint2(lo, hi);
        }
    }
}

BF_API int bf_layernorm_out(const float* x, int ldx, const float* gamma, const float* beta, float eps,
                            void* out, int ldo, int out_f32, const int32_t* row_map, int M, int C,
                            void* stream) {
    if (!x || !gamma || !beta || !out || M < 0 || C <= 0 || C % 4 || ldx % 4 || ldo % 4)
        return BF_ERR_ARG;
    if (M == 0) return BF_OK;
    dim3 grid((M + 3) / 4), block(256);
    const int npl = (C / 4 + 63) / 64;
#define LN(N)                                                                                      \
    if (out_f32) hipLaunchKernelGGL((k_layernorm<N, 1>), grid, block, 0, bf_stream(stream), x,     \
                                    ldx, gamma, beta, eps, out, ldo, row_map, M, C, 1.f);          \
    else hipLaunchKernelGGL((k_layernorm<N, 0>), grid, block, 0, bf_stream(stream), x, ldx,        \
                            gamma, beta, eps, out, ldo, row_map, M, C, 1.f)
    if (npl <= 1) LN(1);
    else if (npl <= 2) LN(2);
    else if (npl <= 3) LN(3);
    else if (npl <= 4) LN(4);
    else if (npl <= 5) LN(5);
    else if (npl <= 8) LN(8);
    else if (npl <= 16) LN(16);
    else return BF_ERR_UNSUPPORTED;
#undef LN
    return bf_check_launch();
}

BF_API int bf_layernorm(const float* x, int ldx, const float* gamma, const float* beta, float eps,
                        void* out, int ldo, const int32_t* row_map, int M, int C, void* stream) {
    return bf_layernorm_out(x, ldx, gamma, beta, eps, out, ldo, 0, row_map, M, C, stream);
}

BF_API int bf_layernorm_fp8(const float* x, int ldx, const float* gamma, const float* beta, float eps,
                            void* out, int ldo, float qscale, int M, int C, void* stream) {
    if (!x || !gamma || !beta || !out || M < 0 || C <= 0 || C % 4 || ldx % 4 || ldo % 4 ||
        !(qscale > 0.f))
        return BF_ERR_ARG;
    if (M == 0) return BF_OK;
    dim3 grid((M + 3) / 4), block(256);
    const int npl = (C / 4 + 63) / 64;
#define LN8(N) hipLaunchKernelGGL((k_layernorm<N, 2>), grid, block, 0, bf_stream(stream), x, ldx, gamma, \
                                  beta, eps, out, ldo, (const int32_t*)nullptr, M, C, qscale)
    if (npl <= 2) LN8(2);
    else if (npl <= 4) LN8(4);
    else if (npl <= 5) LN8(5);
    else if (npl <= 8) LN8(8);
    else if (npl <= 16) LN8(16);
    else return BF_ERR_UNSUPPORTED;
#undef LN8
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// RGB u8 HWC -> normalised, zero-padded to a square of `pad`, patch im2col (K = 3*p*p ordered
// c, ky, kx like the Conv2d weight), bf16.  One thread per 8 consecutive K elements (same c, ky).
// ------------------------------------------------------------------------------------------
// pixel (b, c, y, x) at img[b*sb + c*sc + y*sy + x*sx]: HWC frames (sc = 1, sx = 3) as decoded,
// or CHW (sx = 1, sc = H*W) as the reference's capture stream hands them over (capture_stream.py:221)
__global__ void __launch_bounds__(256) k_im2col_rgb8(const uint8_t* __restrict__ img, int B, int H,
                                                     int W, long long sb, long long sc, long long sy,
                                                     int sx, int pad, int p, float m0, float m1,
                                                     float m2, float s0, float s1, float s2,
                                                     u16* __restrict__ out, int ldo) {
    const int np = pad / p;
    const int K = 3 * p * p;
    const int chunks = K / 8;
    const long long total = (long long)B * np * np * chunks;
    long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= total) return;
    const int ch = (int)(id % chunks);
    const long long prow = id / chunks;           // b*np*np + py*np + px
    const int b = (int)(prow / (np * np));
    const int pp = (int)(prow % (np * np));
    const int py = pp / np, px = pp % np;
    const int k0 = ch * 8;
    const int c = k0 / (p * p), rem = k0 % (p * p);
    const int ky = rem / p, kx0 = rem % p;
    const int y = py * p + ky;
    const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
    const float sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
    u16 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int x = px * p + kx0 + i;
        const float px_v = (float)img[b * sb + c * sc + min(y, H - 1) * sy + (long long)min(x, W - 1) * sx];
        v[i] = vf2bf((y < H && x < W) ? (px_v - mean) / sd : 0.f);
    }
    W128 w = {(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
              (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16)};
    *reinterpret_cast<W128*>(out + (size_t)prow * ldo + k0) = w;
}

BF_API int bf_im2col_rgb8_chw(const uint8_t* img, int B, int H, int W, int chw, int pad, int patch,
                              const float* mean3, const float* std3, void* out, int ldo, void* stream) {
    if (!img || !out || !mean3 || !std3 || B <= 0 || H <= 0 || W <= 0 || pad % patch ||
        (3 * patch * patch) % 8 || ldo % 8 || H > pad || W > pad)
        return BF_ERR_ARG;
    const int np = pad / patch;
    const long long total = (long long)B * np * np * (3 * patch * patch / 8);
    const long long hw = (long long)H * W;
    const long long sb = 3 * hw, sc = chw ? hw : 1, sy = chw ? W : 3 * (long long)W;
    const int sx = chw ? 1 : 3;
    hipLaunchKernelGGL(k_im2col_rgb8, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       bf_stream(stream), img, B, H, W, sb, sc, sy, sx, pad, patch, mean3[0],
                       mean3[1], mean3[2], std3[0], std3[1], std3[2], (u16*)out, ldo);
    return bf_check_launch();
}

BF_API int bf_im2col_rgb8(const uint8_t* img, int B, int H, int W, int pad, int patch,
                          const float* mean3, const float* std3, void* out, int ldo, void* stream) {
    return bf_im2col_rgb8_chw(img, B, H, W, 0, pad, patch, mean3, std3, out, ldo, stream);
}

// single-channel f32 (standardised depth) -> zero-padded square -> im2col (K = p*p)
__global__ void __launch_bounds__(256) k_im2col_f32(const float* __restrict__ x, int B, int H,
                                                    int W, int pad, int p, u16* __restrict__ out,
                                                    int ldo) {
    const int np = pad / p;
    const int chunks = p * p / 8;
    const long long total = (long long)B * np * np * chunks;
    long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= total) return;
    const int ch = (int)(id % chunks);
    const long long prow = id / chunks;
    const int b = (int)(prow / (np * np));
    const int pp = (int)(prow % (np * np));
    const int py = pp / np, px = pp % np;
    const int k0 = ch * 8;
    const int ky = k0 / p, kx0 = k0 % p;
    const int y = py * p + ky;
    u16 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int xx = px * p + kx0 + i;
        const float dv = x[((size_t)b * H + min(y, H - 1)) * W + min(xx, W - 1)];
        v[i] = vf2bf((y < H && xx < W) ? dv : 0.f);
    }
    W128 w = {(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
              (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16)};
    *reinterpret_cast<W128*>(out + (size_t)prow * ldo + k0) = w;
}

BF_API int bf_im2col_f32(const float* x, int B, int H, int W, int pad, int patch, void* out,
                         int ldo, void* stream) {
    if (!x || !out || B <= 0 || pad % patch || (patch * patch) % 8 || ldo % 8) return BF_ERR_ARG;
    const int np = pad / patch;
    const long long total = (long long)B * np * np * (patch * patch / 8);
    hipLaunchKernelGGL(k_im2col_f32, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       bf_stream(stream), x, B, H, W, pad, patch, (u16*)out, ldo);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// CLIP crops: for crop n with integer box (x1,y1,x2,y2) of frame img_idx[n] (u8 HWC RGB):
//   crop = img[y1:y2, x1:x2] (empty -> zeros, tools/utils.py:385), cv2.resize(crop, (S, S)) with
//   OpenCV's u8 INTER_LINEAR fixed-point arithmetic (bf_cv2.h; a u8 image, as the reference's),
//   /255, (x - mean_c)/std_c, then p x p patch im2col with K padded to ldo (zeros).
//   Output rows: n*(S/p)^2 + patch.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_crop_im2col(const uint8_t* __restrict__ img, int H, int W,
                                                     const int32_t* __restrict__ boxes,
                                                     const int32_t* __restrict__ img_idx, int N,
                                                     int S, int p, float m0, float m1, float m2,
                                                     float s0, float s1, float s2,
                                                     u16* __restrict__ out, int ldo) {
    const int np = S / p;
    const int chunks = ldo / 8;
    const long long total = (long long)N * np * np * chunks;
    long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= total) return;
    const int ch = (int)(id % chunks);
    const long long prow = id / chunks;
    const int n = (int)(prow / (np * np));
    const int pp = (int)(prow % (np * np));
    const int py = pp / np, px = pp % np;
    const int K = 3 * p * p;
    // numpy slice semantics for the (non-negative) box: clamp into the frame
    const int x1 = min(max(boxes[4 * n], 0), W), y1 = min(max(boxes[4 * n + 1], 0), H);
    const int x2 = min(max(boxes[4 * n + 2], x1), W), y2 = min(max(boxes[4 * n + 3], y1), H);
    const int cw = x2 - x1, chh = y2 - y1;
    const bool nonempty = cw > 0 && chh > 0;
    const uint8_t* crop = img + (size_t)max(img_idx ? img_idx[n] : 0, 0) * H * W * 3 + ((size_t)y1 * W + x1) * 3;
    const double sxs = nonempty ? cv2_scale(cw, S) : 1.0, sys = nonempty ? cv2_scale(chh, S) : 1.0;
    u16 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int k = ch * 8 + i;
        const int kk = min(k, K - 1);
        const int c = kk / (p * p), rem = kk % (p * p);
        const int oy = py * p + rem / p, ox = px * p + rem % p;
        const int val = nonempty ? cv2_resize_u8_at(crop, W * 3, chh, cw, 3, c, S, S, oy, ox, c, sxs, sys) : 0;
        const float mean = c == 0 ? m0 : (c == 1 ? m1 : m2);
        const float sd = c == 0 ? s0 : (c == 1 ? s1 : s2);
        const float f = ((float)val / 255.f - mean) / sd;
        v[i] = vf2bf(k < K ? f : 0.f);
    }
    W128 w = {(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16),
              (uint32_t)v[4] | ((uint32_t)v[5] << 16), (uint32_t)v[6] | ((uint32_t)v[7] << 16)};
    *reinterpret_cast<W128*>(out + (size_t)prow * ldo + ch * 8) = w;
}

BF_API int bf_crop_resize_im2col(const uint8_t* img, int H, int W, const int32_t* boxes,
                                 const int32_t* img_idx, int N, int size, int patch,
                                 const float* mean3, const float* std3, void* out, int ldo,
                                 void* stream) {
    if (!img || !boxes || !out || !mean3 || !std3 || N < 0 || size % patch || ldo % 8 ||
        ldo < 3 * patch * patch)
        return BF_ERR_ARG;
    if (N == 0) return BF_OK;
    const int np = size / patch;
    const long long total = (long long)N * np * np * (ldo / 8);
    hipLaunchKernelGGL(k_crop_im2col, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       bf_stream(stream), img, H, W, boxes, img_idx, N, size, patch, mean3[0],
                       mean3[1], mean3[2], std3[0], std3[1], std3[2], (u16*)out, ldo);
    return bf_check_launch();
}
