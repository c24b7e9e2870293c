// bf_ingest.hip — GPU frame ingestion: the per-frame host work of the
// reference's capture streams (capture_stream.py:194-311 ScanNet, :402-529 CA-1M) after image
// decode, in one launch per frame batch:
//   color: cv2.cvtColor(BGR -> RGB) (:201), cv2.resize(color, (W_d, H_d)) (:206, u8 INTER_LINEAR,
//          bf_cv2.h), np.moveaxis(-1, 0) (:228, CHW), rotate_tensor (:285, torch.rot90 k, dims
//          (-2, -1));
//   depth: u16 PNG -> astype(float32) / depth_scale (:203, f32 division), cv2.resize to the same
//          size (:247, cv::resize's copy), rotate_tensor (:287).
// The decoded frames (BGR u8 [F, Hc, Wc, 3], depth u16 [F, Hd, Wd]) are the inputs; JPEG / PNG
// decoding itself stays on the host.
#include "bf_cv2.h"

// pre-rotation pixel (y, x) of the H x W image that lands at (i, j) of torch.rot90(img, k)
__device__ __forceinline__ void rot90_src(int k, int H, int W, int i, int j, int& y, int& x) {
    switch (k & 3) {
        case 0: y = i; x = j; break;
        case 1: y = j; x = W - 1 - i; break;           // out [W, H]
        case 2: y = H - 1 - i; x = W - 1 - j; break;
        default: y = H - 1 - j; x = i; break;          // k = 3 / -1, out [W, H]
    }
}

// one thread per output pixel (all three colour channels and the depth value)
__global__ void __launch_bounds__(256) k_ingest_rgbd(const uint8_t* __restrict__ bgr, int Hc, int Wc,
                                                     const uint16_t* __restrict__ depth, int Hd, int Wd,
                                                     int F, float depth_scale, int rot_k, int src_bgr,
                                                     double sx_scale, double sy_scale,
                                                     uint8_t* __restrict__ rgb_out, float* __restrict__ depth_out) {
    const int Ho = (rot_k & 1) ? Wd : Hd, Wo = (rot_k & 1) ? Hd : Wd;
    const long long per = (long long)Ho * Wo;
    const long long total = per * F;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const int f = (int)(e / per);
        const int p = (int)(e - (long long)f * per);
        const int i = p / Wo, j = p - i * Wo;
        int y, x;
        rot90_src(rot_k, Hd, Wd, i, j, y, x);
        const uint8_t* src = bgr + (size_t)f * Hc * Wc * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            // RGB channel c is BGR channel 2 - c; it sits at row position x*3 + c of the RGB image cv2 resizes
            const int v = cv2_resize_u8_at(src, Wc * 3, Hc, Wc, 3, src_bgr ? 2 - c : c, Hd, Wd, y, x, c, sx_scale,
                                           sy_scale);
            rgb_out[((size_t)f * 3 + c) * per + p] = (uint8_t)v;
        }
        if (depth) {
            const float d = (float)depth[(size_t)f * Hd * Wd + (size_t)y * Wd + x];
            depth_out[(size_t)f * per + p] = d / depth_scale;
        }
    }
}

BF_API int bf_ingest_rgbd(const uint8_t* bgr, int Hc, int Wc, const uint16_t* depth, int Hd, int Wd, int F,
                          float depth_scale, int rot_k, int src_bgr, uint8_t* rgb_out, float* depth_out,
                          void* stream) {
    if (!bgr || !rgb_out || Hc <= 0 || Wc <= 0 || Hd <= 0 || Wd <= 0 || F < 0 || (depth && !depth_out) ||
        (depth && !(depth_scale > 0.f)))
        return BF_ERR_ARG;
    if ((long long)Hc * Wc * 3 >= (1ll << 31) || (long long)Hd * Wd >= (1ll << 31)) return BF_ERR_CAPACITY;
    if (F == 0) return BF_OK;
    const long long total = (long long)Hd * Wd * F;
    const unsigned g = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_ingest_rgbd, dim3(g), dim3(256), 0, bf_stream(stream), bgr, Hc, Wc, depth, Hd, Wd, F,
                       depth_scale, ((rot_k % 4) + 4) % 4, src_bgr, cv2_scale(Wc, Wd), cv2_scale(Hc, Hd), rgb_out,
                       depth_out);
    return bf_check_launch();
}

// the cv2 resize alone (u8, cn channels, HWC), for tests and for callers that only resize:
// src [F, Hs, Ws, cn] -> dst [F, Hd, Wd, cn]
__global__ void __launch_bounds__(256) k_cv2_resize_u8(const uint8_t* __restrict__ src, int Hs, int Ws, int cn,
                                                       int Hd, int Wd, int F, double sx_scale, double sy_scale,
                                                       uint8_t* __restrict__ dst) {
    const long long per = (long long)Hd * Wd * cn;
    const long long total = per * F;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const int f = (int)(e / per);
        const long long r = e - (long long)f * per;
        const int c = (int)(r % cn);
        const int px = (int)(r / cn);
        const int y = px / Wd, x = px - y * Wd;
        dst[e] = (uint8_t)cv2_resize_u8_at(src + (size_t)f * Hs * Ws * cn, Ws * cn, Hs, Ws, cn, c, Hd, Wd, y, x,
                                           c, sx_scale, sy_scale);
    }
}

BF_API int bf_cv2_resize_u8(const uint8_t* src, int Hs, int Ws, int cn, int Hd, int Wd, int F, uint8_t* dst,
                            void* stream) {
    if (!src || !dst || Hs <= 0 || Ws <= 0 || Hd <= 0 || Wd <= 0 || cn <= 0 || cn > 4 || F < 0)
        return BF_ERR_ARG;
    if (F == 0) return BF_OK;
    const long long total = (long long)Hd * Wd * cn * F;
    const unsigned g = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_cv2_resize_u8, dim3(g), dim3(256), 0, bf_stream(stream), src, Hs, Ws, cn, Hd, Wd, F,
                       cv2_scale(Ws, Wd), cv2_scale(Hs, Hd), dst);
    return bf_check_launch();
}
