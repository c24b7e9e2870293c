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

// device-side work list of the split form (k_obb_gate / k_obb_grid)
struct ObbWork {
    int n_gated;      // pairs that passed the gate
    int grid_done;    // k_obb_grid workgroups finished (the last one divides)
    int pad[2];
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

// 8 lanes per box (the f64 plane fits are long dependent chains: one lane per box left a single
// latency-bound wave, 30 us at n ~ 60): lanes 0-5 fit face f's two planes, lane 6 writes the gate
// points, lane 7 the AABB; every value is computed by the same expression sequence as before
__global__ void __launch_bounds__(64) k_obb_prep(const float* __restrict__ corners, int n,
                                                 BoxPrep* __restrict__ prep, double* __restrict__ iou,
                                                 ObbWork* __restrict__ w) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0 && w) { w->n_gated = 0; w->grid_done = 0; }
    const int i = t >> 3, sub = t & 7;
    if (i >= n) return;
    const float* c = corners + 24 * i;
    BoxPrep& o = prep[i];
    if (sub < 6) {
        if (sub == 0) iou[(size_t)i * n + i] = 1.0;      // diagonal (pairs fill the rest)
        double p[8][3], cen[3] = {0, 0, 0};
        for (int q = 0; q < 8; ++q)
            for (int k = 0; k < 3; ++k) { p[q][k] = c[3 * q + k]; cen[k] += p[q][k]; }
        for (int k = 0; k < 3; ++k) cen[k] /= 8.0;
        const int f = sub;
        const double* a = p[c_face[f][0]];
        const double* b = p[c_face[f][1]];
        const double* cc = p[c_face[f][2]];
        const double* d = p[c_face[f][3]];
        double tt[4];
        tri_plane(a, b, cc, cen, tt);
        if (tt[0] * d[0] + tt[1] * d[1] + tt[2] * d[2] + tt[3] <= 0) {
            tri_plane(a, b, cc, cen, o.pl[2 * f]);
            tri_plane(a, cc, d, cen, o.pl[2 * f + 1]);
        } else {
            tri_plane(a, b, d, cen, o.pl[2 * f]);
            tri_plane(b, cc, d, cen, o.pl[2 * f + 1]);
        }
    } else if (sub == 6) {
        for (int q = 0; q < 8; ++q)
            for (int k = 0; k < 3; ++k) o.pt[q][k] = c[3 * q + k];
        for (int e = 0; e < 12; ++e)
            for (int k = 0; k < 3; ++k)
                o.pt[8 + e][k] = (c[3 * c_edge[e][0] + k] + c[3 * c_edge[e][1] + k]) / 2;
    } else {
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

// ------------------------------------------------------------------------------------------
// Split form (default): the gate and the grid count are separate launches, so the grid count
// only runs for the pairs that pass the gate and spreads each over OBB_SPLIT workgroups.  One
// workgroup per pair (k_obb_pairs above) leaves most of the chip idle behind a few long
// workgroups and, on the fusion stream's CU partition, queues thousands of short ones.
//   k_obb_gate   one wave per pair: 40-lane gate ballot; IoU 0 written for gated-out pairs,
//                the others appended to a device list (order-free: each pair owns its entries)
//   k_obb_grid   persistent: item = (gated pair, split), 15625 / OBB_SPLIT grid points each,
//                integer counts added atomically (exact, order-free)
//                the last workgroup to finish divides: IoU = n12 / ((n1 + n2 - n12) + 1e-6)
//   (k_obb_prep also writes the diagonal and resets the work list: 3 launches per matrix)
// ------------------------------------------------------------------------------------------
#ifndef OBB_SPLIT
#define OBB_SPLIT 2         // (a diagnostic build sets 0: one workgroup per pair, k_obb_pairs)
#endif
#define OBB_GRID_WGS 512
#ifndef OBB_LAST_BLOCK
// 0 (default): the division as its own launch (k_obb_final); 1 (diagnostic build): the grid's
// last workgroup divides (one launch less, but every workgroup's release fence writes back L2,
// which costs more than the launch under the detect load)
#define OBB_LAST_BLOCK 0
#endif


__global__ void __launch_bounds__(256) k_obb_gate(const BoxPrep* __restrict__ prep, int n,
                                                  long long pairs, double* __restrict__ iou,
                                                  ObbWork* __restrict__ w, int* __restrict__ gated,
                                                  int* __restrict__ cnt) {
    const long long p = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= pairs) return;                                  // wave-uniform
    const int t = threadIdx.x & 63;
    int i, j;
    pair_of(p, n, &i, &j);
    const BoxPrep& A = prep[i];
    const BoxPrep& B = prep[j];
    bool in = false;
    if (t < 20) in = inside12(A.pt[t][0], A.pt[t][1], A.pt[t][2], B.pl);
    else if (t < 40) in = inside12(B.pt[t - 20][0], B.pt[t - 20][1], B.pt[t - 20][2], A.pl);
    const unsigned long long m = __ballot(in);
    if (t == 0) {
        if (m == 0ull) {
            iou[(size_t)i * n + j] = 0.0;
            iou[(size_t)j * n + i] = 0.0;
        } else {
            const int slot = atomicAdd(&w->n_gated, 1);
            gated[slot] = (int)p;
            cnt[3 * slot + 0] = 0;
            cnt[3 * slot + 1] = 0;
            cnt[3 * slot + 2] = 0;
        }
    }
}

__global__ void __launch_bounds__(IOU_THREADS) k_obb_grid(const BoxPrep* __restrict__ prep, int n,
                                                          ObbWork* __restrict__ w,
                                                          const int* __restrict__ gated,
                                                          int* __restrict__ cnt,
                                                          double* __restrict__ iou) {
    __shared__ double pl[2][12][4];
    __shared__ double g[3][25];
    __shared__ int s_red[3][IOU_THREADS / 64];
    const int t = threadIdx.x;
    constexpr int SPLIT = OBB_SPLIT > 0 ? OBB_SPLIT : 1;
    const int items = w->n_gated * SPLIT;
    constexpr int PER = (15625 + SPLIT - 1) / SPLIT;
    for (int it = blockIdx.x; it < items; it += gridDim.x) {
        const int slot = it / SPLIT, part = it % SPLIT;
        int i, j;
        pair_of((long long)gated[slot], n, &i, &j);
        const BoxPrep& A = prep[i];
        const BoxPrep& B = prep[j];
        __syncthreads();                                     // previous item's LDS reads done
        if (t < 48) pl[0][t >> 2][t & 3] = A.pl[t >> 2][t & 3];
        else if (t < 96) pl[1][(t - 48) >> 2][(t - 48) & 3] = B.pl[(t - 48) >> 2][(t - 48) & 3];
        else if (t < 96 + 75) {
            // numpy.linspace(f64(min), f64(max), 25) per axis over the union AABB
            const int ax = (t - 96) / 25, k = (t - 96) % 25;
            float lo = fminf(A.mn[ax], B.mn[ax]);
            float hi = fmaxf(A.mx[ax], B.mx[ax]);
            double start = lo, stop = hi;
            double step = (stop - start) / 24.0;
            g[ax][k] = (k == 24) ? stop : (double)k * step + start;
        }
        __syncthreads();
        // points outside a box's AABB by > 1e-3 skip its plane tests (see k_obb_pairs)
        const double m = 1e-3;
        const double alo0 = A.mn[0] - m, alo1 = A.mn[1] - m, alo2 = A.mn[2] - m;
        const double ahi0 = A.mx[0] + m, ahi1 = A.mx[1] + m, ahi2 = A.mx[2] + m;
        const double blo0 = B.mn[0] - m, blo1 = B.mn[1] - m, blo2 = B.mn[2] - m;
        const double bhi0 = B.mx[0] + m, bhi1 = B.mx[1] + m, bhi2 = B.mx[2] + m;
        int n1 = 0, n2 = 0, n12 = 0;
        const int p0 = part * PER, p1 = min(p0 + PER, 15625);
        for (int p = p0 + t; p < p1; p += IOU_THREADS) {
            int ix = p / 625, iy = (p / 25) % 25, iz = p % 25;
            double x = g[0][ix], y = g[1][iy], z = g[2][iz];
            const bool ina = x >= alo0 && x <= ahi0 && y >= alo1 && y <= ahi1 && z >= alo2 && z <= ahi2;
            const bool inb = x >= blo0 && x <= bhi0 && y >= blo1 && y <= bhi1 && z >= blo2 && z <= bhi2;
            bool a = ina && inside12(x, y, z, pl[0]);
            bool b = inb && inside12(x, y, z, pl[1]);
            n1 += a;
            n2 += b;
            n12 += (a && b);
        }
        n1 = bf_wave_sum_i32(n1);
        n2 = bf_wave_sum_i32(n2);
        n12 = bf_wave_sum_i32(n12);
        if (bf_lane() == 0) {
            s_red[0][t >> 6] = n1;
            s_red[1][t >> 6] = n2;
            s_red[2][t >> 6] = n12;
        }
        __syncthreads();
        if (t < 3) {
            int s = 0;
            for (int q = 0; q < IOU_THREADS / 64; ++q) s += s_red[t][q];
            atomicAdd(&cnt[3 * slot + t], s);
        }
    }
    if (!OBB_LAST_BLOCK) return;
    // the last workgroup to finish divides: IoU = n12 / ((n1 + n2 - n12) + 1e-6)
    __shared__ int s_last;
    __threadfence();
    __syncthreads();
    if (t == 0)
        s_last = __hip_atomic_fetch_add(&w->grid_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                 (int)gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    const int ng = __hip_atomic_load(&w->n_gated, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int slot = t; slot < ng; slot += IOU_THREADS) {
        int i, j;
        pair_of((long long)gated[slot], n, &i, &j);
        const long long a = __hip_atomic_load(&cnt[3 * slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const long long b = __hip_atomic_load(&cnt[3 * slot + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const long long c = __hip_atomic_load(&cnt[3 * slot + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const double v = (double)c / ((double)(a + b - c) + 1e-6);
        iou[(size_t)i * n + j] = v;
        iou[(size_t)j * n + i] = v;
    }
}




// ------------------------------------------------------------------------------------------
// Column form (default, OBB_COLS 1): one lane per grid column (ix, iy), 25 z points each.
// Along a column x, y and the plane's partial sum S = x*a + y*b are fixed, z_k = linspace(k) is
// non-decreasing in k, and v(k) = (S + z_k*c) + d is a chain of monotone roundings of z_k*c, so
// the test v <= 1e-6 holds on a prefix of k (c > 0), a suffix (c < 0) or all / none (c == 0 or
// NaN: v does not depend on z).  Each of the 12 plane tests is therefore a 5-step binary search
// for its boundary and the box's inside set on the column is the interval they cut out,
// intersected with the AABB cull's interval (the same two monotone z tests the point form
// makes).  Counts: n1 = |I_A|, n2 = |I_B|, n12 = |I_A ∩ I_B| — the point form's counts exactly,
// in ≈ 140 instead of ≈ 25·12·3 f64 operations per column and box.  A pair whose z step is not
// >= 0 or whose planes are not all finite takes the point-by-point loop over its 25 z values.
// ------------------------------------------------------------------------------------------
#ifndef OBB_COLS
#define OBB_COLS 1
#endif
#define OBB_COL_CHUNKS 10          // 64-column chunks per pair (625 columns)

struct ZLine {
    double start, step, stop;
    __device__ __forceinline__ double at(int k) const { return k == 24 ? stop : (double)k * step + start; }
};

// number of leading k in [0, 25) with pred(k) (pred true on a prefix)
template <class F>
__device__ __forceinline__ int lead_true(F pred) {
    int K = 0;
#pragma unroll
    for (int st = 16; st >= 1; st >>= 1)
        if (K + st <= 25 && pred(K + st - 1)) K += st;
    return K;
}

// number of trailing k in [0, 25) with pred(k) (pred true on a suffix)
template <class F>
__device__ __forceinline__ int trail_true(F pred) {
    int T = 0;
#pragma unroll
    for (int st = 16; st >= 1; st >>= 1)
        if (T + st <= 25 && pred(25 - T - st)) T += st;
    return T;
}

// the box's inside interval [lo, hi) of z indices on column (x, y) (empty when hi <= lo)
__device__ __forceinline__ void col_interval(double x, double y, const ZLine& z, const BoxPrep& P,
                                             int* lo_out, int* hi_out) {
    const double m = 1e-3;
    const double lo0 = P.mn[0] - m, lo1 = P.mn[1] - m, lo2 = P.mn[2] - m;
    const double hi0 = P.mx[0] + m, hi1 = P.mx[1] + m, hi2 = P.mx[2] + m;
    int lo = 0, hi = 0;
    if (x >= lo0 && x <= hi0 && y >= lo1 && y <= hi1) {
        // AABB cull in z: z >= lo2 on a suffix, z <= hi2 on a prefix
        lo = 25 - trail_true([&](int k) { return z.at(k) >= lo2; });
        hi = lead_true([&](int k) { return z.at(k) <= hi2; });
#pragma unroll 1
        for (int q = 0; q < 12; ++q) {
            const double a = P.pl[q][0], b = P.pl[q][1], c = P.pl[q][2], d = P.pl[q][3];
            const double S = x * a + y * b;
            auto in = [&](int k) { return ((S + z.at(k) * c) + d) <= 1e-6; };
            if (c > 0) hi = min(hi, lead_true(in));
            else if (c < 0) lo = max(lo, 25 - trail_true(in));
            else if (!in(0)) hi = 0;
        }
    }
    *lo_out = lo;
    *hi_out = hi;
}

__device__ __forceinline__ bool prep_finite(const BoxPrep& P) {
    bool f = true;
#pragma unroll 1
    for (int q = 0; q < 12; ++q)
        for (int c = 0; c < 4; ++c) f = f && isfinite(P.pl[q][c]);
    return f;
}

// persistent: item = (gated pair, 64-column chunk), one wave per item, 4 waves per workgroup
__global__ void __launch_bounds__(256) k_obb_cols(const BoxPrep* __restrict__ prep, int n,
                                                  const ObbWork* __restrict__ w,
                                                  const int* __restrict__ gated, int* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int items = w->n_gated * OBB_COL_CHUNKS;
    for (int it = blockIdx.x * 4 + (threadIdx.x >> 6); it < items; it += gridDim.x * 4) {
        const int slot = it / OBB_COL_CHUNKS, chunk = it % OBB_COL_CHUNKS;
        int i, j;
        pair_of((long long)gated[slot], n, &i, &j);
        const BoxPrep& A = prep[i];
        const BoxPrep& B = prep[j];
        // numpy.linspace(f64(min), f64(max), 25) per axis over the union AABB (as k_obb_grid)
        const ZLine gx{(double)fminf(A.mn[0], B.mn[0]), 0.0, (double)fmaxf(A.mx[0], B.mx[0])};
        const ZLine gy{(double)fminf(A.mn[1], B.mn[1]), 0.0, (double)fmaxf(A.mx[1], B.mx[1])};
        ZLine gz{(double)fminf(A.mn[2], B.mn[2]), 0.0, (double)fmaxf(A.mx[2], B.mx[2])};
        ZLine lx = gx, ly = gy;
        lx.step = (gx.stop - gx.start) / 24.0;
        ly.step = (gy.stop - gy.start) / 24.0;
        gz.step = (gz.stop - gz.start) / 24.0;
        const int col = chunk * 64 + lane;
        int n1 = 0, n2 = 0, n12 = 0;
        if (col < 625) {
            const double x = lx.at(col / 25), y = ly.at(col % 25);
            if (gz.step >= 0 && prep_finite(A) && prep_finite(B)) {
                int la, ha, lb, hb;
                col_interval(x, y, gz, A, &la, &ha);
                col_interval(x, y, gz, B, &lb, &hb);
                n1 = max(ha - la, 0);
                n2 = max(hb - lb, 0);
                n12 = max(min(ha, hb) - max(la, lb), 0);
            } else {
                const double m = 1e-3;
#pragma unroll 1
                for (int k = 0; k < 25; ++k) {
                    const double z = gz.at(k);
                    const bool ina = x >= A.mn[0] - m && x <= A.mx[0] + m && y >= A.mn[1] - m &&
                                     y <= A.mx[1] + m && z >= A.mn[2] - m && z <= A.mx[2] + m;
                    const bool inb = x >= B.mn[0] - m && x <= B.mx[0] + m && y >= B.mn[1] - m &&
                                     y <= B.mx[1] + m && z >= B.mn[2] - m && z <= B.mx[2] + m;
                    const bool a = ina && inside12(x, y, z, A.pl);
                    const bool b = inb && inside12(x, y, z, B.pl);
                    n1 += a;
                    n2 += b;
                    n12 += (a && b);
                }
            }
        }
        n1 = bf_wave_sum_i32(n1);
        n2 = bf_wave_sum_i32(n2);
        n12 = bf_wave_sum_i32(n12);
        if (lane == 0) {
            atomicAdd(&cnt[3 * slot + 0], n1);
            atomicAdd(&cnt[3 * slot + 1], n2);
            atomicAdd(&cnt[3 * slot + 2], n12);
        }
    }
}

__global__ void __launch_bounds__(256) k_obb_final(int n, const ObbWork* __restrict__ w,
                                                   const int* __restrict__ gated,
                                                   const int* __restrict__ cnt,
                                                   double* __restrict__ iou) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= w->n_gated) return;
    int i, j;
    pair_of((long long)gated[slot], n, &i, &j);
    const long long a = cnt[3 * slot], b = cnt[3 * slot + 1], c = cnt[3 * slot + 2];
    const double v = (double)c / ((double)(a + b - c) + 1e-6);
    iou[(size_t)i * n + j] = v;
    iou[(size_t)j * n + i] = v;
}

static size_t obb_prep_bytes(int n) { return ((size_t)n * sizeof(BoxPrep) + 255) & ~(size_t)255; }

BF_API size_t bf_obb_iou_workspace_size(int n) {
    if (n <= 0) return 0;
    const size_t pairs = (size_t)n * (n - 1) / 2;
    // prep | work header | gated pair list | 3 counts per gated pair
    return obb_prep_bytes(n) + 256 + sizeof(int) * pairs + sizeof(int) * 3 * pairs;
}

BF_API int bf_obb_iou_matrix(const float* corners, int n, double* iou, void* workspace,
                             void* stream) {
    if (n < 0 || (n > 0 && (!corners || !iou || !workspace))) return BF_ERR_ARG;
    if (n == 0) return BF_OK;
    hipStream_t s = bf_stream(stream);
    BoxPrep* prep = reinterpret_cast<BoxPrep*>(workspace);
    char* ws = reinterpret_cast<char*>(workspace) + obb_prep_bytes(n);
    ObbWork* w = reinterpret_cast<ObbWork*>(ws);
    long long pairs = (long long)n * (n - 1) / 2;
    int* gated = reinterpret_cast<int*>(ws + 256);
    int* cnt = gated + pairs;
    if (pairs > 0x7fffffffLL / 4) return BF_ERR_CAPACITY;
    hipLaunchKernelGGL(k_obb_prep, dim3(bf_cdiv(8 * n, 64)), dim3(64), 0, s, corners, n, prep, iou, w);
    if (pairs > 0) {
        if (OBB_SPLIT == 0) {
            hipLaunchKernelGGL(k_obb_pairs, dim3((unsigned)pairs), dim3(IOU_THREADS), 0, s, prep, n, iou);
        } else {
            hipLaunchKernelGGL(k_obb_gate, dim3((unsigned)((pairs + 3) / 4)), dim3(256), 0, s, prep, n,
                               pairs, iou, w, gated, cnt);
            if (OBB_COLS) {
                const long long waves = pairs * OBB_COL_CHUNKS;
                const unsigned gw = (unsigned)std::min<long long>((waves + 3) / 4, OBB_GRID_WGS);
                hipLaunchKernelGGL(k_obb_cols, dim3(gw), dim3(256), 0, s, prep, n, w, gated, cnt);
            } else {
                const unsigned gw = (unsigned)(pairs * (OBB_SPLIT > 0 ? OBB_SPLIT : 1) < OBB_GRID_WGS
                                                   ? pairs * (OBB_SPLIT > 0 ? OBB_SPLIT : 1) : OBB_GRID_WGS);
                hipLaunchKernelGGL(k_obb_grid, dim3(gw), dim3(IOU_THREADS), 0, s, prep, n, w, gated, cnt,
                                   iou);
            }
            if (OBB_COLS || !OBB_LAST_BLOCK)
                hipLaunchKernelGGL(k_obb_final, dim3(bf_cdiv((unsigned)pairs, 256)), dim3(256), 0, s, n,
                                   w, gated, cnt, iou);
        }
    }
    return bf_check_launch();
}
