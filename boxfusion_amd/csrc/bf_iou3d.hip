// bf_iou3d.hip — pairwise sampled 3-D OBB IoU (instances.py:493-613) on gfx950.
//
// Semantics (reference Instances3D.obb_iou):
//   gate: any of the 20 points of A (8 corners + 12 f32 edge midpoints) inside hull(B) or vice
//         versa, "inside" = n.p + d <= 1e-6 for all 12 triangulated hull facets;
//   grid: 25^3 linspace points over the union AABB of the 16 corners, counted against both hulls;
//   IoU = n12 / (n1 + n2 - n12 + 1e-6).
// The 12 qhull facets are reproduced in closed form (each face split along its convex diagonal,
// unit outward normal in f64 from the f32 corners) — verified bit-exact against scipy/qhull on
// the golden pairs.
//
// Layout: k_obb_prep writes per-box planes (12 x f64[4]) and gate points (20 x f32[3]) to the
// workspace; k_obb_pairs runs one 256-thread workgroup per unordered pair (i<j): the gate is one
// wave-wide ballot, the grid is 15625 points striped over 256 lanes (f64 VALU, no MFMA).
#include "bf_common.h"

#define IOU_THREADS 256

__constant__ int c_face[6][4] = {{0, 3, 7, 4}, {1, 2, 6, 5}, {0, 1, 5, 4},
                                 {3, 2, 6, 7}, {0, 1, 2, 3}, {4, 5, 6, 7}};
__constant__ int c_edge[12][2] = {{0, 1}, {0, 4}, {1, 5}, {4, 5}, {2, 3}, {2, 6},
                                  {6, 7}, {3, 7}, {0, 3}, {4, 7}, {1, 2}, {5, 6}};

struct BoxPrep {
    double pl[12][4];  // unit outward planes
    float pt[20][3];   // gate points
    float mn[3], mx[3];
    float pad[2];
};

__device__ void tri_plane(const double* p0, const double* p1, const double* p2, const double* cen,
                          double* pl) {
    double a0 = p1[0] - p0[0], a1 = p1[1] - p0[1], a2 = p1[2] - p0[2];
    double b0 = p2[0] - p0[0], b1 = p2[1] - p0[1], b2 = p2[2] - p0[2];
    double nx = a1 * b2 - a2 * b1;
    double ny = a2 * b0 - a0 * b2;
    double nz = a0 * b1 - a1 * b0;
    double nn = sqrt(nx * nx + ny * ny + nz * nz);
    nx /= nn; ny /= nn; nz /= nn;
    double d = -(nx * p0[0] + ny * p0[1] + nz * p0[2]);
    if (nx * cen[0] + ny * cen[1] + nz * cen[2] + d > 0) { nx = -nx; ny = -ny; nz = -nz; d = -d; }
    pl[0] = nx; pl[1] = ny; pl[2] = nz; pl[3] = d;
}

__global__ void __launch_bounds__(64) k_obb_prep(const float* __restrict__ corners, int n,
                                                 BoxPrep* __restrict__ prep) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* c = corners + 24 * i;
    double p[8][3], cen[3] = {0, 0, 0};
    for (int q = 0; q < 8; ++q)
        for (int k = 0; k < 3; ++k) { p[q][k] = c[3 * q + k]; cen[k] += p[q][k]; }
    for (int k = 0; k < 3; ++k) cen[k] /= 8.0;
    BoxPrep& o = prep[i];
    for (int f = 0; f < 6; ++f) {
        const double* a = p[c_face[f][0]];
        const double* b = p[c_face[f][1]];
        const double* cc = p[c_face[f][2]];
        const double* d = p[c_face[f][3]];
        double t[4];
        tri_plane(a, b, cc, cen, t);
        if (t[0] * d[0] + t[1] * d[1] + t[2] * d[2] + t[3] <= 0) {
            tri_plane(a, b, cc, cen, o.pl[2 * f]);
            tri_plane(a, cc, d, cen, o.pl[2 * f + 1]);
        } else {
            tri_plane(a, b, d, cen, o.pl[2 * f]);
            tri_plane(b, cc, d, cen, o.pl[2 * f + 1]);
        }
    }
    for (int q = 0; q < 8; ++q)
        for (int k = 0; k < 3; ++k) o.pt[q][k] = c[3 * q + k];
    for (int e = 0; e < 12; ++e)
        for (int k = 0; k < 3; ++k)
            o.pt[8 + e][k] = (c[3 * c_edge[e][0] + k] + c[3 * c_edge[e][1] + k]) / 2;
    for (int k = 0; k < 3; ++k) {
        float lo = c[k], hi = c[k];
        for (int q = 1; q < 8; ++q) {
            lo = fminf(lo, c[3 * q + k]);
            hi = fmaxf(hi, c[3 * q + k]);
        }
        o.mn[k] = lo;
        o.mx[k] = hi;
    }
}

__device__ __forceinline__ bool inside12(double x, double y, double z, const double (*pl)[4]) {
    bool in = true;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        double v = ((x * pl[k][0] + y * pl[k][1]) + z * pl[k][2]) + pl[k][3];
        in = in && (v <= 1e-6);
    }
    return in;
}

// linear pair index -> (i, j), i < j, row-major upper triangle
__device__ __forceinline__ void pair_of(long long p, int n, int* i, int* j) {
    // row i holds n-1-i pairs; solve with f64 sqrt then fix up
    double nn = (double)n;
    long long r = (long long)((2.0 * nn - 1.0 - sqrt((2.0 * nn - 1.0) * (2.0 * nn - 1.0) - 8.0 * (double)p)) / 2.0);
    if (r < 0) r = 0;
    auto start = [&](long long rr) { return rr * (2LL * n - rr - 1) / 2; };
    while (r > 0 && start(r) > p) --r;
    while (start(r + 1) <= p) ++r;
    *i = (int)r;
    *j = (int)(p - start(r) + r + 1);
}

__global__ void __launch_bounds__(IOU_THREADS) k_obb_pairs(const BoxPrep* __restrict__ prep, int n,
                                                           double* __restrict__ iou) {
    int i, j;
    pair_of((long long)blockIdx.x, n, &i, &j);
    __shared__ double pl[2][12][4];
    __shared__ double g[3][25];
    __shared__ int s_gate;
    __shared__ long long s_red[3][IOU_THREADS / 64];
    const int t = threadIdx.x;
    const BoxPrep& A = prep[i];
    const BoxPrep& B = prep[j];
    if (t < 48) pl[0][t >> 2][t & 3] = A.pl[t >> 2][t & 3];
    else if (t < 96) pl[1][(t - 48) >> 2][(t - 48) & 3] = B.pl[(t - 48) >> 2][(t - 48) & 3];
    if (t == 0) s_gate = 0;
    __syncthreads();
    // gate: lanes 0..19 test A's points against B, lanes 20..39 B's against A (first wave)
    if (t < 64) {
        bool in = false;
        if (t < 20) in = inside12(A.pt[t][0], A.pt[t][1], A.pt[t][2], pl[1]);
        else if (t < 40) in = inside12(B.pt[t - 20][0], B.pt[t - 20][1], B.pt[t - 20][2], pl[0]);
        unsigned long long m = __ballot(in);
        if (t == 0) s_gate = (m != 0ull) ? 1 : 0;
    }
    __syncthreads();
    if (!s_gate) {
        if (t == 0) {
            iou[(size_t)i * n + j] = 0.0;
            iou[(size_t)j * n + i] = 0.0;
        }
        return;
    }
    // numpy.linspace(f64(min), f64(max), 25) per axis over the union AABB
    if (t < 75) {
        int ax = t / 25, k = t % 25;
        float lo = fminf(A.mn[ax], B.mn[ax]);
        float hi = fmaxf(A.mx[ax], B.mx[ax]);
        double start = lo, stop = hi;
        double step = (stop - start) / 24.0;
        g[ax][k] = (k == 24) ? stop : (double)k * step + start;
    }
    __syncthreads();
    // A grid point more than 1e-3 outside a box's (f32) AABB is outside its hull: some facet plane
    // is then at a signed distance >= 1e-3/sqrt(3) >> the 1e-6 tolerance, so skipping the 12
    // f64 plane tests there changes no count (the tests themselves are unchanged).
    const double m = 1e-3;
    const double alo0 = A.mn[0] - m, alo1 = A.mn[1] - m, alo2 = A.mn[2] - m;
    const double ahi0 = A.mx[0] + m, ahi1 = A.mx[1] + m, ahi2 = A.mx[2] + m;
    const double blo0 = B.mn[0] - m, blo1 = B.mn[1] - m, blo2 = B.mn[2] - m;
    const double bhi0 = B.mx[0] + m, bhi1 = B.mx[1] + m, bhi2 = B.mx[2] + m;
    // both plane sets in registers (96 f64): read from LDS once, not 96 broadcast reads per point
    double pa[12][4], pb[12][4];
#pragma unroll
    for (int k = 0; k < 12; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) { pa[k][c] = pl[0][k][c]; pb[k][c] = pl[1][k][c]; }
    long long n1 = 0, n2 = 0, n12 = 0;
    for (int p = t; p < 15625; p += IOU_THREADS) {
        int ix = p / 625, iy = (p / 25) % 25, iz = p % 25;
        double x = g[0][ix], y = g[1][iy], z = g[2][iz];
        const bool ina = x >= alo0 && x <= ahi0 && y >= alo1 && y <= ahi1 && z >= alo2 && z <= ahi2;
        const bool inb = x >= blo0 && x <= bhi0 && y >= blo1 && y <= bhi1 && z >= blo2 && z <= bhi2;
        bool a = ina && inside12(x, y, z, pa);
        bool b = inb && inside12(x, y, z, pb);
        n1 += a;
        n2 += b;
        n12 += (a && b);
    }
    n1 = bf_wave_sum_i64(n1);
    n2 = bf_wave_sum_i64(n2);
    n12 = bf_wave_sum_i64(n12);
    if (bf_lane() == 0) {
        s_red[0][t >> 6] = n1;
        s_red[1][t >> 6] = n2;
        s_red[2][t >> 6] = n12;
    }
    __syncthreads();
    if (t == 0) {
        long long a = 0, b = 0, c = 0;
        for (int w = 0; w < IOU_THREADS / 64; ++w) { a += s_red[0][w]; b += s_red[1][w]; c += s_red[2][w]; }
        double v = (double)c / ((double)(a + b - c) + 1e-6);
        iou[(size_t)i * n + j] = v;
        iou[(size_t)j * n + i] = v;
    }
}

__global__ void k_iou_diag(double* iou, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) iou[(size_t)i * n + i] = 1.0;
}

BF_API size_t bf_obb_iou_workspace_size(int n) { return (size_t)(n > 0 ? n : 0) * sizeof(BoxPrep); }

BF_API int bf_obb_iou_matrix(const float* corners, int n, double* iou, void* workspace,
                             void* stream) {
    if (n < 0 || (n > 0 && (!corners || !iou || !workspace))) return BF_ERR_ARG;
    if (n == 0) return BF_OK;
    hipStream_t s = bf_stream(stream);
    BoxPrep* prep = reinterpret_cast<BoxPrep*>(workspace);
    hipLaunchKernelGGL(k_obb_prep, dim3(bf_cdiv(n, 64)), dim3(64), 0, s, corners, n, prep);
    hipLaunchKernelGGL(k_iou_diag, dim3(bf_cdiv(n, 256)), dim3(256), 0, s, iou, n);
    long long pairs = (long long)n * (n - 1) / 2;
    if (pairs > 0) {
        if (pairs > 0x7fffffffLL) return BF_ERR_CAPACITY;
        hipLaunchKernelGGL(k_obb_pairs, dim3((unsigned)pairs), dim3(IOU_THREADS), 0, s, prep, n, iou);
    }
    return bf_check_launch();
}
