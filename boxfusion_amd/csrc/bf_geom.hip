// bf_geom.hip — per-box and per-pixel geometry on gfx950 (HBM/latency-bound, no MFMA).
//   bf_box_corners          boxes.py:725-778   GeneralInstance3DBoxes.corners
//   bf_box_transform2world  boxes.py:825-833   GeneralInstance3DBoxes.transform2world
//   bf_project_boxes        instances.py:333-369 Instances3D.project_3d_boxes
//   bf_backproject          tools/utils.py:232-287 unproject / get_camera_coords
//   bf_depth_standardize    preprocessor.py:97-129 Preprocessor.standardize_depth_map
// Built with -ffp-contract=off so every f32 product/sum rounds like the reference's CPU path.
#include "bf_common.h"

// ------------------------------------------------------------------------------------------
// corners: one thread per (box, corner)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_box_corners(const float* __restrict__ b,
                                                     const float* __restrict__ R, int n,
                                                     float* __restrict__ out) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 8) return;
    int i = t >> 3, c = t & 7;
    const float* x = b + 6 * i;
    const float* r = R + 9 * i;
    float hl = x[3] / 2, hh = x[4] / 2, hw = x[5] / 2;
    float v0 = bf_vsign_x(c) > 0 ? hl : -hl;
    float v1 = bf_vsign_y(c) > 0 ? hh : -hh;
    float v2 = bf_vsign_z(c) > 0 ? hw : -hw;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        float s = r[3 * j + 0] * v0;
        s = s + r[3 * j + 1] * v1;
        s = s + r[3 * j + 2] * v2;
        out[24 * i + 3 * c + j] = s + x[j];
    }
}

BF_API int bf_box_corners(const float* xyzlhw, const float* R, int n, float* corners,
                          void* stream) {
    if (n < 0 || (n > 0 && (!xyzlhw || !R || !corners))) return BF_ERR_ARG;
    if (n == 0) return BF_OK;
    hipLaunchKernelGGL(k_box_corners, dim3(bf_cdiv(n * 8, 256)), dim3(256), 0, bf_stream(stream),
                       xyzlhw, R, n, corners);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// transform2world, in place: xyz <- Rc xyz + tc ; R <- Rc R
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_box_t2w(float* __restrict__ b, float* __restrict__ R,
                                                 const float* __restrict__ P, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* p = P + 16 * i;
    float x[3] = {b[6 * i], b[6 * i + 1], b[6 * i + 2]};
    float r[9];
    for (int k = 0; k < 9; ++k) r[k] = R[9 * i + k];
    for (int j = 0; j < 3; ++j) {
        float s = p[4 * j] * x[0];
        s = s + p[4 * j + 1] * x[1];
        s = s + p[4 * j + 2] * x[2];
        b[6 * i + j] = s + p[4 * j + 3];
    }
    for (int j = 0; j < 3; ++j)
        for (int c = 0; c < 3; ++c) {
            float s = p[4 * j] * r[c];
            s = s + p[4 * j + 1] * r[3 + c];
            s = s + p[4 * j + 2] * r[6 + c];
            R[9 * i + 3 * j + c] = s;
        }
}

BF_API int bf_box_transform2world(float* xyzlhw, float* R, const float* cam_pose, int n,
                                  void* stream) {
    if (n < 0 || (n > 0 && (!xyzlhw || !R || !cam_pose))) return BF_ERR_ARG;
    if (n == 0) return BF_OK;
    hipLaunchKernelGGL(k_box_t2w, dim3(bf_cdiv(n, 256)), dim3(256), 0, bf_stream(stream), xyzlhw, R,
                       cam_pose, n);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// project: one thread per (box, corner); pose inverse per box (f64 cofactors)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_project(const float* __restrict__ corners,
                                                 const float* __restrict__ P,
                                                 const float* __restrict__ K, int n, float W,
                                                 float H, float* __restrict__ uv) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 8) return;
    int i = t >> 3, c = t & 7;
    float pinv[16];
    bf_inv4(P + 16 * i, pinv);
    const float* q = corners + 24 * i + 3 * c;
    float h[4] = {q[0], q[1], q[2], 1.0f};
    float cam[3];
    for (int r = 0; r < 3; ++r) {
        float s = pinv[4 * r] * h[0];
        s = s + pinv[4 * r + 1] * h[1];
        s = s + pinv[4 * r + 2] * h[2];
        s = s + pinv[4 * r + 3] * h[3];
        cam[r] = s;
    }
    float u = (K[0] * cam[0] / cam[2]) + K[2];
    float v = (K[4] * cam[1] / cam[2]) + K[5];
    u = fminf(fmaxf(u, 0.f), W);
    v = fminf(fmaxf(v, 0.f), H);
    uv[16 * i + 2 * c] = u;
    uv[16 * i + 2 * c + 1] = v;
}

BF_API int bf_project_boxes(const float* corners, const float* cam_pose, const float* K, int n,
                            float W, float H, float* uv, void* stream) {
    if (n < 0 || (n > 0 && (!corners || !cam_pose || !K || !uv))) return BF_ERR_ARG;
    if (n == 0) return BF_OK;
    hipLaunchKernelGGL(k_project, dim3(bf_cdiv(n * 8, 256)), dim3(256), 0, bf_stream(stream),
                       corners, cam_pose, K, n, W, H, uv);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// back-projection: one thread per pixel, K^-1 and RT in registers
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_backproject(const float* __restrict__ d,
                                                     const float* __restrict__ K,
                                                     const float* __restrict__ RT, int h, int w,
                                                     float max_depth, float* __restrict__ xyz,
                                                     uint8_t* __restrict__ valid) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= h * w) return;
    float K4[16] = {K[0], K[1], K[2], 0.f, K[3], K[4], K[5], 0.f, K[6], K[7], K[8], 0.f,
                    0.f, 0.f, 0.f, 1.f};
    float Ki[16];
    bf_inv4(K4, Ki);
    float dv = d[p];
    int u = p % w, v = p / w;
    float uvd[4] = {(float)u * dv, (float)v * dv, dv, 1.0f};
    float cam[4];
    for (int r = 0; r < 4; ++r) {
        float s = Ki[4 * r] * uvd[0];
        s = s + Ki[4 * r + 1] * uvd[1];
        s = s + Ki[4 * r + 2] * uvd[2];
        s = s + Ki[4 * r + 3] * uvd[3];
        cam[r] = s;
    }
    for (int r = 0; r < 3; ++r) {
        float s = RT[4 * r] * cam[0];
        s = s + RT[4 * r + 1] * cam[1];
        s = s + RT[4 * r + 2] * cam[2];
        s = s + RT[4 * r + 3] * cam[3];
        xyz[3 * p + r] = s;
    }
    bool ok = dv > 0.f;
    if (max_depth > 0.f) ok = ok && (dv < max_depth);
    valid[p] = ok ? 1 : 0;
}

BF_API int bf_backproject(const float* depth, const float* K, const float* RT, int h, int w,
                          float max_depth, float* xyz, uint8_t* valid, void* stream) {
    if (h <= 0 || w <= 0 || !depth || !K || !RT || !xyz || !valid) return BF_ERR_ARG;
    hipLaunchKernelGGL(k_backproject, dim3(bf_cdiv(h * w, 256)), dim3(256), 0, bf_stream(stream),
                       depth, K, RT, h, w, max_depth, xyz, valid);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// detection filters of demo.py:138-148 (box_manager.py:217-245) over a batch of frames' top-k
// instances, one thread per instance: keep = score >= thr & uv inside [gap, size - gap] & !floor
// & !large.  Every comparison in f32 like the reference's torch ops on f32 tensors (a python
// scalar operand is rounded to f32); bits 1..4 of `bits` record each filter's own mask.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_detection_filter(const float* __restrict__ scores,
                                                          const float* __restrict__ proj_xy,
                                                          const float* __restrict__ box3d, int n,
                                                          bf_filter_cfg cfg, uint8_t* __restrict__ keep,
                                                          uint8_t* __restrict__ bits) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool s_ok = scores[i] >= cfg.score_thresh;
    const float u = proj_xy[2 * i], v = proj_xy[2 * i + 1];
    const bool uv_ok = (u > (float)cfg.gap_w) & (u < (float)(cfg.W - cfg.gap_w)) &
                       (v > (float)cfg.gap_h) & (v < (float)(cfg.H - cfg.gap_h));
    const float a = box3d[6 * i + 3], b = box3d[6 * i + 4], c = box3d[6 * i + 5];
    const float mx = fmaxf(fmaxf(a, b), c), mn = fminf(fminf(a, b), c);
    // second largest of three (torch.sort(descending)[:, 1])
    const float second = fmaxf(fminf(a, b), fminf(fmaxf(a, b), c));
    const float q = mx / mn;
    bool floor_m = q > cfg.floor_ratio;
    floor_m |= (q > cfg.floor_half) & (mx / second > cfg.floor_half) & (second / mn < 2.0f) &
               (second < 0.15f) & (mn < 0.15f);
    const bool large_m = mx > cfg.size_max;
    bool k = true;
    if (cfg.use_score) k &= s_ok;
    if (cfg.use_uv) k &= uv_ok;
    if (cfg.use_floor) k &= !floor_m;
    if (cfg.use_large) k &= !large_m;
    keep[i] = k ? 1 : 0;
    if (bits) bits[i] = (uint8_t)((s_ok ? 2 : 0) | (uv_ok ? 4 : 0) | (floor_m ? 8 : 0) | (large_m ? 16 : 0));
}

BF_API int bf_detection_filter(const float* scores, const float* proj_xy, const float* box3d, int n,
                               const bf_filter_cfg* cfg, uint8_t* keep, uint8_t* bits, void* stream) {
    if (!scores || !proj_xy || !box3d || !cfg || !keep || n < 0) return BF_ERR_ARG;
    if (n == 0) return BF_OK;
    hipLaunchKernelGGL(k_detection_filter, dim3(bf_cdiv(n, 256)), dim3(256), 0, bf_stream(stream),
                       scores, proj_xy, box3d, n, *cfg, keep, bits);
    return bf_check_launch();
}
