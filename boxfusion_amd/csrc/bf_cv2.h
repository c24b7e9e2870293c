// bf_cv2.h — OpenCV's u8 INTER_LINEAR resize, element by element, for the kernels that replace the
// reference's cv2.resize calls (capture_stream.py:206,418 frame ingestion; tools/utils.py:385 the
// 224x224 CLIP crops).  Restated from OpenCV 4.x imgproc/src/resize.cpp (cv2 is absent here, so
// the bits are pinned to this restatement and to oracle/bf_oracle.c's copy of it, not to a cv2 run):
//   * scale = 1 / (dst / src) in double; per output column fx = (float)((dx + 0.5) * scale - 0.5),
//     sx = floor(fx), fx -= sx; sx < 0 -> (sx, fx) = (0, 0); sx >= src - 1 -> (src - 1, 0); the
//     columns with sx + 1 >= src take S[sx] * 2048 (HResizeLinear's border), the others
//     S[sx] * a0 + S[sx + 1] * a1 with a = lrint({1 - fx, fx} * 2048) (INTER_RESIZE_COEF_BITS 11);
//   * rows: the same fy / sy without the clamp (rows clipped to [0, src - 1]), b = lrint(.. * 2048);
//   * vertical pass (VResizeLinear<uchar, int, short>): the 128-bit SIMD body
//     sat_u8((mulhi(S0 >> 4, b0) + mulhi(S1 >> 4, b1) + 2) >> 2) covers the first 16*floor(w/16)
//     elements of a row (w = dst width * channels) plus 8 more when w % 16 > 8; the scalar tail
//     is sat_u8((S0*b0 + S1*b1 + 2^21) >> 22);
//   * dst size == src size is a plain copy (cv::resize's early exit).
#pragma once
#include "bf_common.h"

struct Cv2Tap {
    int s0, s1;     // source indices (s1 clipped)
    int w0, w1;     // fixed-point weights (2048 = 1)
    bool border;    // x only: the S[s0] * 2048 border form
};

__device__ __forceinline__ float cv2_src_coord(int d, double scale) {
#pragma clang fp contract(off)
    const double t = ((double)d + 0.5) * scale;
    return (float)(t - 0.5);
}

__device__ __forceinline__ Cv2Tap cv2_tap_x(int dx, double scale, int nsrc) {
    float f = cv2_src_coord(dx, scale);
    int s = (int)floorf(f);
    f -= (float)s;
    if (s < 0) { f = 0.f; s = 0; }
    Cv2Tap t;
    t.border = s + 1 >= nsrc;
    if (s >= nsrc - 1) { f = 0.f; s = nsrc - 1; }
    t.s0 = s;
    t.s1 = min(s + 1, nsrc - 1);
    t.w0 = (int)rintf((1.f - f) * 2048.f);
    t.w1 = (int)rintf(f * 2048.f);
    return t;
}

__device__ __forceinline__ Cv2Tap cv2_tap_y(int dy, double scale, int nsrc) {
    float f = cv2_src_coord(dy, scale);
    const int s = (int)floorf(f);
    f -= (float)s;
    Cv2Tap t;
    t.border = false;
    t.s0 = min(max(s, 0), nsrc - 1);
    t.s1 = min(max(s + 1, 0), nsrc - 1);
    t.w0 = (int)rintf((1.f - f) * 2048.f);
    t.w1 = (int)rintf(f * 2048.f);
    return t;
}

// index (within a row of w = dst_width * cn elements) below which the SIMD vertical body runs
__host__ __device__ __forceinline__ int cv2_simd_end(int w) {
    const int q = w & ~15, r = w - q;
    return q + (r > 8 ? 8 : 0);
}

__device__ __forceinline__ int cv2_vmix(int h0, int h1, int b0, int b1, bool simd) {
    if (simd) {
        const int a0 = min(max(h0 >> 4, -32768), 32767), a1 = min(max(h1 >> 4, -32768), 32767);
        const int t0 = (a0 * b0) >> 16, t1 = (a1 * b1) >> 16;
        const int s = min(max(t0 + t1, -32768), 32767);
        return min(max((s + 2) >> 2, 0), 255);
    }
    return min(max((h0 * b0 + h1 * b1 + (1 << 21)) >> 22, 0), 255);
}

// one element: channel c of output pixel (dy, dx) of the src (Hs x Ws, cn channels, row stride
// `ld` bytes, channel ch_src read for output channel c) resized to Hd x Wd
__device__ __forceinline__ int cv2_resize_u8_at(const uint8_t* src, int ld, int Hs, int Ws, int cn,
                                                int ch_src, int Hd, int Wd, int dy, int dx, int c,
                                                double sx_scale, double sy_scale) {
    if (Hs == Hd && Ws == Wd) return src[(size_t)dy * ld + dx * cn + ch_src];
    const Cv2Tap tx = cv2_tap_x(dx, sx_scale, Ws), ty = cv2_tap_y(dy, sy_scale, Hs);
    const uint8_t* r0 = src + (size_t)ty.s0 * ld;
    const uint8_t* r1 = src + (size_t)ty.s1 * ld;
    int h0, h1;
    if (tx.border) {
        h0 = (int)r0[tx.s0 * cn + ch_src] * 2048;
        h1 = (int)r1[tx.s0 * cn + ch_src] * 2048;
    } else {
        h0 = (int)r0[tx.s0 * cn + ch_src] * tx.w0 + (int)r0[tx.s1 * cn + ch_src] * tx.w1;
        h1 = (int)r1[tx.s0 * cn + ch_src] * tx.w0 + (int)r1[tx.s1 * cn + ch_src] * tx.w1;
    }
    return cv2_vmix(h0, h1, ty.w0, ty.w1, dx * cn + c < cv2_simd_end(Wd * cn));
}

// cv::resize's scale factors: inv_scale = dst / src, scale = 1 / inv_scale (both double)
__host__ __device__ __forceinline__ double cv2_scale(int src, int dst) {
    const double inv = (double)dst / (double)src;
    return 1.0 / inv;
}
