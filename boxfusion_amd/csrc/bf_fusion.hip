// bf_fusion.hip — multi-view box fusion (particle-swarm refinement) on gfx950.
//
// Reference: BoxFusion.boxfusion (box_fusion.py:622-724).  The reference launches its CUDA
// kernel compute_iou_value (:264-405) once per iteration per box, with a host round trip, a
// Python loop over 1023 particles (cal_transform :475-535) and host scalar updates (update_PST
// :537-563, momentum :685-706).  Here one call refines every job with all iterations on the
// device (no host round trip): per iteration one launch evaluates every (job, view, particle)
// pair across the chip and one launch per job does the sequential update:
//
//   per iteration:  fitness[p] = sum_v |1 - IoU2D(hull(proj_v(box (+) PST[p]*s)), hull(tc_v))|
//                                / (V + 1e-6)            (views summed in order: deterministic,
//                                                         unlike the reference's atomicAdd)
//                   accepted = first `max_accept` particles j >= 1 with fitness[j] < fitness[0]
//                              (block ballot prefix, order-preserving)
//                   weighted sums in reference order on 8 lanes (f64 or f32 per promotion mode)
//                   lane 0: cal_transform / update_PST / momentum / accept, exactly as the host
//
// Arithmetic follows the reference kernel's float32 (+ f64 line intersection) expression by
// expression; compiled with -ffp-contract=off.  Hull buffers have fixed capacity; inputs that
// would overflow the reference's own fixed buffers (corners_i[36], convex_inter[8]) set
// BF_DEV_HULL_OVERFLOW (the result is still the mathematically intended one); more candidates
// than this kernel's own 64 slots set BF_DEV_HULL_TRUNC (never seen: two convex 8-gons give at
// most 16 vertices + 32 crossings; the host raises on it).
#include "bf_common.h"

#define FUSE_MAX_VIEWS 32
#ifndef FUSE_SPLIT_ITER
// 1: terms and step as two launches per iteration (default: measured faster under the detect
// load — the one-launch form's device-scope fences write back L2 in every workgroup);
// 0 (diagnostic build): k_fuse_iter, one launch per iteration
#define FUSE_SPLIT_ITER 1
#endif
#define FUSE_MAX_PST 1024
#define CAND_CAP 64

struct P2 {
    float x, y;
};

__device__ __forceinline__ float cross2(P2 o, P2 a, P2 b) {
    return (a.x - o.x) * (b.y - o.y) - (a.y - o.y) * (b.x - o.x);
}

// convex_hull (box_fusion.py:95-145): exchange sort by (x, y), monotone chain, pop on cross <= 0
template <int CAP>
__device__ int convex_hull(P2* in, int n, P2* out) {
    if (n == 0) return 0;
    for (int i = 0; i < n - 1; ++i)
        for (int j = i + 1; j < n; ++j)
            if (in[i].x > in[j].x || (in[i].x == in[j].x && in[i].y > in[j].y)) {
                P2 tt = in[i]; in[i] = in[j]; in[j] = tt;
            }
    P2 lower[CAP], upper[CAP];
    int nl = 0, nu = 0;
    for (int i = 0; i < n; ++i) {
        while (nl >= 2 && cross2(lower[nl - 2], lower[nl - 1], in[i]) <= 0) nl--;
        lower[nl++] = in[i];
    }
    for (int i = n - 1; i >= 0; --i) {
        while (nu >= 2 && cross2(upper[nu - 2], upper[nu - 1], in[i]) <= 0) nu--;
        upper[nu++] = in[i];
    }
    nl--; nu--;
    for (int i = 0; i < nl; ++i) out[i] = lower[i];
    for (int i = 0; i < nu; ++i) out[nl + i] = upper[i];
    return nl + nu;
}

__device__ __forceinline__ float polygon_area(const P2* p, int n) {
    float a = 0.0f;
    for (int i = 0; i < n; ++i) {
        P2 p1 = p[i], p2 = p[(i + 1) % n];
        a += p1.x * p2.y - p2.x * p1.y;
    }
    return (float)(fabs((double)a) / 2.0);
}

__device__ __forceinline__ bool line_intersection(P2 a1, P2 a2, P2 b1, P2 b2, P2* out) {
    double dx1 = a2.x - a1.x, dy1 = a2.y - a1.y, dx2 = b2.x - b1.x, dy2 = b2.y - b1.y;
    double den = dx1 * dy2 - dy1 * dx2;
    if (fabs(den) < 1e-8) return false;
    double tt = (dx2 * (a1.y - b1.y) + dy2 * (b1.x - a1.x)) / den;
    double s = (dx1 * (a1.y - b1.y) + dy1 * (b1.x - a1.x)) / den;
    if (tt >= -1e-8 && tt <= 1.00000001 && s >= -1e-8 && s <= 1.00000001) {
        out->x = (float)(a1.x + tt * dx1);
        out->y = (float)(a1.y + tt * dy1);
        return true;
    }
    return false;
}

__device__ __forceinline__ bool point_in_polygon(P2 p, const P2* poly, int n) {
    bool in = false;
    for (int i = 0; i < n; ++i) {
        P2 p1 = poly[i], p2 = poly[(i + 1) % n];
        if ((p1.y > p.y) != (p2.y > p.y)) {
            float xi = ((p.y - p1.y) * (p2.x - p1.x) / (p2.y - p1.y)) + p1.x;
            if (p.x < xi) in = !in;
        }
    }
    return in;
}

// segments whose bounding boxes are more than 1e-3 px apart cannot produce an accepted
// intersection: line_intersection accepts parameters in [-1e-8, 1 + 1e-8], i.e. at most
// ~1e-5 px outside a segment of an image-sized extent.  Skipping them changes no result and
// avoids the two f64 divisions.
__device__ __forceinline__ bool seg_boxes_apart(P2 a1, P2 a2, P2 b1, P2 b2) {
    const float m = 1e-3f;
    return fmaxf(a1.x, a2.x) + m < fminf(b1.x, b2.x) || fmaxf(b1.x, b2.x) + m < fminf(a1.x, a2.x) ||
           fmaxf(a1.y, a2.y) + m < fminf(b1.y, b2.y) || fmaxf(b1.y, b2.y) + m < fminf(a1.y, a2.y);
}

// IoU of hull(c0) with a precomputed hull ht[nt] (polygon_intersection :202-261 + :374-396)
__device__ float iou_hull_pre(P2* c0, const P2* ht, int nt, float at, int* flags) {
    P2 h0[8];
    int n0 = convex_hull<8>(c0, 8, h0);
    P2 cand[CAND_CAP];
    int nc = 0;
    for (int i = 0; i < n0; ++i)
        if (point_in_polygon(h0[i], ht, nt)) {
            if (nc < CAND_CAP) cand[nc++] = h0[i];
            else *flags |= BF_DEV_HULL_TRUNC;
        }
    for (int i = 0; i < nt; ++i)
        if (point_in_polygon(ht[i], h0, n0)) {
            if (nc < CAND_CAP) cand[nc++] = ht[i];
            else *flags |= BF_DEV_HULL_TRUNC;
        }
    for (int i = 0; i < n0; ++i)
        for (int j = 0; j < nt; ++j) {
            const P2 a1 = h0[i], a2 = h0[(i + 1) % n0], b1 = ht[j], b2 = ht[(j + 1) % nt];
            if (seg_boxes_apart(a1, a2, b1, b2)) continue;
            P2 pt;
            if (line_intersection(a1, a2, b1, b2, &pt)) {
                if (nc < CAND_CAP) cand[nc++] = pt;
                else *flags |= BF_DEV_HULL_TRUNC;
            }
        }
    if (nc > 36) *flags |= BF_DEV_HULL_OVERFLOW;
    P2 hi[CAND_CAP];
    int ni = convex_hull<CAND_CAP>(cand, nc, hi);
    if (ni > 8) *flags |= BF_DEV_HULL_OVERFLOW;
    float inter = polygon_area(hi, ni);
    float a0 = polygon_area(h0, n0);
    float uni = a0 + at - inter;
    float iou = 0;
    if (uni > 0) iou = (float)((double)inter / ((double)uni + 0.00001));
    return iou;
}

// IoU of the hulls of two 8-point sets
__device__ float iou_hulls(P2* c0, P2* ct, int* flags) {
    P2 ht[8];
    const int nt = convex_hull<8>(ct, 8, ht);
    return iou_hull_pre(c0, ht, nt, polygon_area(ht, nt), flags);
}

// ------------------------------------------------------------------------------------------
// LDS form of iou_hull_pre for the refinement loop (same arithmetic, same results).
// The scratch form keeps ~2 KB of per-thread arrays (hull stacks, 64 candidates) that spill
// to L2 at this kernel's occupancy; here one wave's stacks live in LDS, element e of lane l
// at [e * 64 + l], and the 8 projected corners are sorted in registers by a 19-comparator
// network (any correct sort gives the exchange sort's order: equal keys are equal points).
// Lanes with more than FAST_CAND candidates (never seen on real boxes: two convex 8-gons give
// at most 16 vertices + 16 crossings in general position) take the scratch path.
// ------------------------------------------------------------------------------------------
#ifndef FAST_CAND
#define FAST_CAND 32   // (a diagnostic build lowers it to exercise the scratch path)
#endif
struct HullLds {
    P2 cand[FAST_CAND * 64];   // candidates, sorted; then the lower chain in place
    P2 up[FAST_CAND * 64];     // upper chain of the candidate hull
    P2 lo0[8 * 64];            // lower chain of hull(c0)
    P2 up0[8 * 64];            // upper chain of hull(c0)
};

__device__ __forceinline__ bool p2_greater(P2 a, P2 b) {
    return a.x > b.x || (a.x == b.x && a.y > b.y);
}

__device__ __forceinline__ void p2_cswap(P2& a, P2& b) {
    const bool g = p2_greater(a, b);
    const P2 lo = g ? b : a, hi = g ? a : b;
    a = lo;
    b = hi;
}

// hull vertex i of a monotone-chain hull stored as lower[0..nl-1) ++ upper[0..nu-1)
#define HULL_AT(lo, up, nl1, i) ((i) < (nl1) ? (lo)[(i) * 64] : (up)[((i) - (nl1)) * 64])

__device__ float iou_hull_lds(const P2* c0in, const P2* ht, int nt, float at, HullLds& L,
                              int lane, int* flags) {
    P2 c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = c0in[j];
    p2_cswap(c[0], c[2]); p2_cswap(c[1], c[3]); p2_cswap(c[4], c[6]); p2_cswap(c[5], c[7]);
    p2_cswap(c[0], c[4]); p2_cswap(c[1], c[5]); p2_cswap(c[2], c[6]); p2_cswap(c[3], c[7]);
    p2_cswap(c[0], c[1]); p2_cswap(c[2], c[3]); p2_cswap(c[4], c[5]); p2_cswap(c[6], c[7]);
    p2_cswap(c[2], c[4]); p2_cswap(c[3], c[5]);
    p2_cswap(c[1], c[4]); p2_cswap(c[3], c[6]);
    p2_cswap(c[1], c[2]); p2_cswap(c[3], c[4]); p2_cswap(c[5], c[6]);
    // hull(c0): convex_hull's two monotone chains
    P2* lo0 = L.lo0 + lane;
    P2* up0 = L.up0 + lane;
    int nl = 0, nu = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        while (nl >= 2 && cross2(lo0[(nl - 2) * 64], lo0[(nl - 1) * 64], c[i]) <= 0) nl--;
        lo0[(nl++) * 64] = c[i];
    }
#pragma unroll
    for (int i = 7; i >= 0; --i) {
        while (nu >= 2 && cross2(up0[(nu - 2) * 64], up0[(nu - 1) * 64], c[i]) <= 0) nu--;
        up0[(nu++) * 64] = c[i];
    }
    const int nl1 = nl - 1;
    const int n0 = nl1 + (nu - 1);
    // candidates
    P2* cand = L.cand + lane;
    int nc = 0;
    bool slow = false;
    for (int i = 0; i < n0; ++i) {
        const P2 p = HULL_AT(lo0, up0, nl1, i);
        if (point_in_polygon(p, ht, nt)) {
            if (nc < FAST_CAND) cand[(nc++) * 64] = p;
            else slow = true;
        }
    }
    for (int i = 0; i < nt; ++i) {
        // point_in_polygon(ht[i], h0, n0)
        const P2 p = ht[i];
        bool in = false;
        for (int k = 0; k < n0; ++k) {
            const P2 p1 = HULL_AT(lo0, up0, nl1, k);
            const P2 p2 = HULL_AT(lo0, up0, nl1, (k + 1) % n0);
            if ((p1.y > p.y) != (p2.y > p.y)) {
                float xi = ((p.y - p1.y) * (p2.x - p1.x) / (p2.y - p1.y)) + p1.x;
                if (p.x < xi) in = !in;
            }
        }
        if (in) {
            if (nc < FAST_CAND) cand[(nc++) * 64] = p;
            else slow = true;
        }
    }
    for (int i = 0; i < n0 && !slow; ++i) {
        const P2 a1 = HULL_AT(lo0, up0, nl1, i);
        const P2 a2 = HULL_AT(lo0, up0, nl1, (i + 1) % n0);
        for (int j = 0; j < nt; ++j) {
            const P2 b1 = ht[j], b2 = ht[(j + 1) % nt];
            if (seg_boxes_apart(a1, a2, b1, b2)) continue;
            P2 pt;
            if (line_intersection(a1, a2, b1, b2, &pt)) {
                if (nc < FAST_CAND) cand[(nc++) * 64] = pt;
                else { slow = true; break; }
            }
        }
    }
    if (slow) {   // scratch path from the original corners (rare)
        P2 cc[8];
        for (int j = 0; j < 8; ++j) cc[j] = c0in[j];
        return iou_hull_pre(cc, ht, nt, at, flags);
    }
    float a0 = 0.0f;
    for (int i = 0; i < n0; ++i) {
        const P2 p1 = HULL_AT(lo0, up0, nl1, i), p2 = HULL_AT(lo0, up0, nl1, (i + 1) % n0);
        a0 += p1.x * p2.y - p2.x * p1.y;
    }
    a0 = (float)(fabs((double)a0) / 2.0);
    // hull(cand): sort (insertion: same order as the exchange sort), upper chain into `up`,
    // then the lower chain in place over the sorted candidates (it writes index <= i only)
    for (int i = 1; i < nc; ++i) {
        const P2 x = cand[i * 64];
        int j = i - 1;
        while (j >= 0 && p2_greater(cand[j * 64], x)) { cand[(j + 1) * 64] = cand[j * 64]; --j; }
        cand[(j + 1) * 64] = x;
    }
    P2* up = L.up + lane;
    int ni = 0, cl1 = 0;
    if (nc > 0) {
        int mu = 0;
        for (int i = nc - 1; i >= 0; --i) {
            const P2 x = cand[i * 64];
            while (mu >= 2 && cross2(up[(mu - 2) * 64], up[(mu - 1) * 64], x) <= 0) mu--;
            up[(mu++) * 64] = x;
        }
        int ml = 0;
        for (int i = 0; i < nc; ++i) {
            const P2 x = cand[i * 64];
            while (ml >= 2 && cross2(cand[(ml - 2) * 64], cand[(ml - 1) * 64], x) <= 0) ml--;
            cand[(ml++) * 64] = x;
        }
        cl1 = ml - 1;
        ni = cl1 + (mu - 1);
    }
    if (ni > 8) *flags |= BF_DEV_HULL_OVERFLOW;
    float inter = 0.0f;
    for (int i = 0; i < ni; ++i) {
        const P2 p1 = HULL_AT(cand, up, cl1, i), p2 = HULL_AT(cand, up, cl1, (i + 1) % ni);
        inter += p1.x * p2.y - p2.x * p1.y;
    }
    inter = (float)(fabs((double)inter) / 2.0);
    float uni = a0 + at - inter;
    float iou = 0;
    if (uni > 0) iou = (float)((double)inter / ((double)uni + 0.00001));
    return iou;
}

// ------------------------------------------------------------------------------------------
// Four lanes per (particle, view) pair (the refinement's terms kernel): the same IoU as
// iou_hull_lds, with the pair's work split where it is independent.  Each lane projects two of
// the eight corners; all four run the corner sort and hull(c0) (identical values on identical LDS
// slots); the candidate tests (hull(c0) vertices in the target, target vertices in hull(c0), the
// n0 x nt edge crossings) go round-robin over the four lanes and append to the pair's list with
// an LDS atomic; the list is then ordered by rank (key (x, y), ties by list position -- equal keys
// are equal points, so every arrival order gives the exchange sort's sequence) with each lane
// ranking a quarter of it, and all four run the candidate hull's chains and the areas.  Every
// arithmetic expression is the one iou_hull_lds evaluates, so the terms are bit-identical; the
// dependent-LDS chain of one lane shrinks to the two hulls' monotone chains.
// ------------------------------------------------------------------------------------------
#define G4_PAIRS 16                      // pairs per one-wave workgroup
struct HullG4 {
    P2 c0[8 * G4_PAIRS];                 // the projected corners, [j * 16 + pair]
    P2 lo0[8 * G4_PAIRS];                // hull(c0) chains, [e * 16 + pair]
    P2 up0[8 * G4_PAIRS];
    P2 cand[FAST_CAND * G4_PAIRS];       // candidates in arrival order
    P2 srt[FAST_CAND * G4_PAIRS];        // sorted candidates; then the lower chain in place
    P2 up[FAST_CAND * G4_PAIRS];         // upper chain of the candidate hull
    int cnt[G4_PAIRS];
};
#define HULL_AT16(lo, up, nl1, i) ((i) < (nl1) ? (lo)[(i) * G4_PAIRS] : (up)[((i) - (nl1)) * G4_PAIRS])

__device__ __forceinline__ bool p2_less(P2 a, P2 b) { return a.x < b.x || (a.x == b.x && a.y < b.y); }
__device__ __forceinline__ bool p2_equal(P2 a, P2 b) { return a.x == b.x && a.y == b.y; }

// c0in: this pair's 8 projected corners (all four lanes); returns the IoU (all four lanes)
__device__ float iou_hull_g4(const P2* c0in, const P2* ht, int nt, float at, HullG4& L, int pr,
                             int g, int* flags) {
    P2 c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = c0in[j];
    p2_cswap(c[0], c[2]); p2_cswap(c[1], c[3]); p2_cswap(c[4], c[6]); p2_cswap(c[5], c[7]);
    p2_cswap(c[0], c[4]); p2_cswap(c[1], c[5]); p2_cswap(c[2], c[6]); p2_cswap(c[3], c[7]);
    p2_cswap(c[0], c[1]); p2_cswap(c[2], c[3]); p2_cswap(c[4], c[5]); p2_cswap(c[6], c[7]);
    p2_cswap(c[2], c[4]); p2_cswap(c[3], c[5]);
    p2_cswap(c[1], c[4]); p2_cswap(c[3], c[6]);
    p2_cswap(c[1], c[2]); p2_cswap(c[3], c[4]); p2_cswap(c[5], c[6]);
    P2* lo0 = L.lo0 + pr;
    P2* up0 = L.up0 + pr;
    int nl = 0, nu = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        while (nl >= 2 && cross2(lo0[(nl - 2) * G4_PAIRS], lo0[(nl - 1) * G4_PAIRS], c[i]) <= 0) nl--;
        lo0[(nl++) * G4_PAIRS] = c[i];
    }
#pragma unroll
    for (int i = 7; i >= 0; --i) {
        while (nu >= 2 && cross2(up0[(nu - 2) * G4_PAIRS], up0[(nu - 1) * G4_PAIRS], c[i]) <= 0) nu--;
        up0[(nu++) * G4_PAIRS] = c[i];
    }
    const int nl1 = nl - 1;
    const int n0 = nl1 + (nu - 1);
    // candidates, round-robin over the pair's lanes
    P2* cand = L.cand + pr;
    int* cnt = L.cnt + pr;
    if (g == 0) *cnt = 0;
    __syncthreads();
    for (int i = g; i < n0; i += 4) {
        const P2 p = HULL_AT16(lo0, up0, nl1, i);
        if (point_in_polygon(p, ht, nt)) {
            const int k = atomicAdd(cnt, 1);
            if (k < FAST_CAND) cand[k * G4_PAIRS] = p;
        }
    }
    for (int i = g; i < nt; i += 4) {
        const P2 p = ht[i];
        bool in = false;
        for (int k = 0; k < n0; ++k) {
            const P2 p1 = HULL_AT16(lo0, up0, nl1, k);
            const P2 p2 = HULL_AT16(lo0, up0, nl1, (k + 1) % n0);
            if ((p1.y > p.y) != (p2.y > p.y)) {
                float xi = ((p.y - p1.y) * (p2.x - p1.x) / (p2.y - p1.y)) + p1.x;
                if (p.x < xi) in = !in;
            }
        }
        if (in) {
            const int k = atomicAdd(cnt, 1);
            if (k < FAST_CAND) cand[k * G4_PAIRS] = p;
        }
    }
    for (int q = g; q < n0 * nt; q += 4) {
        const int i = q / nt, j = q - i * nt;
        const P2 a1 = HULL_AT16(lo0, up0, nl1, i);
        const P2 a2 = HULL_AT16(lo0, up0, nl1, (i + 1) % n0);
        const P2 b1 = ht[j], b2 = ht[(j + 1) % nt];
        if (seg_boxes_apart(a1, a2, b1, b2)) continue;
        P2 pt;
        if (line_intersection(a1, a2, b1, b2, &pt)) {
            const int k = atomicAdd(cnt, 1);
            if (k < FAST_CAND) cand[k * G4_PAIRS] = pt;
        }
    }
    __syncthreads();
    // (the barriers below are reached by every lane: a pair on the scratch path skips the work,
    // not the barriers)
    const bool slow = *cnt > FAST_CAND;
    const int nc = slow ? 0 : *cnt;
    float iou_slow = 0.f;
    if (slow && g == 0) {     // scratch path from the original corners (rare): lane 0 of the pair
        P2 cc[8];
        for (int j = 0; j < 8; ++j) cc[j] = c0in[j];
        iou_slow = iou_hull_pre(cc, ht, nt, at, flags);
    }
    float a0 = 0.0f;
    for (int i = 0; i < n0; ++i) {
        const P2 p1 = HULL_AT16(lo0, up0, nl1, i), p2 = HULL_AT16(lo0, up0, nl1, (i + 1) % n0);
        a0 += p1.x * p2.y - p2.x * p1.y;
    }
    a0 = (float)(fabs((double)a0) / 2.0);
    // rank order of the candidates (each lane a quarter of them)
    P2* srt = L.srt + pr;
    for (int k = g; k < nc; k += 4) {
        const P2 x = cand[k * G4_PAIRS];
        int r = 0;
        for (int m = 0; m < nc; ++m) {
            const P2 y = cand[m * G4_PAIRS];
            r += p2_less(y, x) || (m < k && p2_equal(y, x));
        }
        srt[r * G4_PAIRS] = x;
    }
    __syncthreads();
    P2* up = L.up + pr;
    int ni = 0, cl1 = 0;
    if (nc > 0) {
        int mu = 0;
        for (int i = nc - 1; i >= 0; --i) {
            const P2 x = srt[i * G4_PAIRS];
            while (mu >= 2 && cross2(up[(mu - 2) * G4_PAIRS], up[(mu - 1) * G4_PAIRS], x) <= 0) mu--;
            up[(mu++) * G4_PAIRS] = x;
        }
        int ml = 0;
        for (int i = 0; i < nc; ++i) {
            const P2 x = srt[i * G4_PAIRS];
            while (ml >= 2 && cross2(srt[(ml - 2) * G4_PAIRS], srt[(ml - 1) * G4_PAIRS], x) <= 0) ml--;
            srt[(ml++) * G4_PAIRS] = x;
        }
        cl1 = ml - 1;
        ni = cl1 + (mu - 1);
    }
    if (slow) return iou_slow;
    if (ni > 8) *flags |= BF_DEV_HULL_OVERFLOW;
    float inter = 0.0f;
    for (int i = 0; i < ni; ++i) {
        const P2 p1 = HULL_AT16(srt, up, cl1, i), p2 = HULL_AT16(srt, up, cl1, (i + 1) % ni);
        inter += p1.x * p2.y - p2.x * p1.y;
    }
    inter = (float)(fabs((double)inter) / 2.0);
    float uni = a0 + at - inter;
    float iou = 0;
    if (uni > 0) iou = (float)((double)inter / ((double)uni + 0.00001));
    return iou;
}

struct FuseViews {
    float pose[FUSE_MAX_VIEWS][16];
    float tc[FUSE_MAX_VIEWS][16];
};

// fitness of one particle (box already perturbed into its 8 corners) over all views
__device__ float particle_fitness(const float* corners, const FuseViews& V, int nv,
                                  const bf_fuse_cfg& cfg, int* flags) {
    float val = 0.0f, cnt = 0.0f;
    for (int v = 0; v < nv; ++v) {
        const float* P = V.pose[v];
        P2 c0[8], ct[8];
        for (int j = 0; j < 8; ++j) {
            float vx = corners[3 * j] - P[3], vy = corners[3 * j + 1] - P[7], vz = corners[3 * j + 2] - P[11];
            float cx = P[0] * vx + P[4] * vy + P[8] * vz;
            float cy = P[1] * vx + P[5] * vy + P[9] * vz;
            float cz = P[2] * vx + P[6] * vy + P[10] * vz;
            float px = ((cx * cfg.K[0]) / cz + cfg.K[2]);
            float py = ((cy * cfg.K[5]) / cz + cfg.K[6]);
            c0[j].x = (px > cfg.img_w) ? cfg.img_w : (px < 0) ? 0 : px;
            c0[j].y = (py > cfg.img_h) ? cfg.img_h : (py < 0) ? 0 : py;
            ct[j].x = V.tc[v][2 * j];
            ct[j].y = V.tc[v][2 * j + 1];
        }
        float iou = iou_hulls(c0, ct, flags);
        val += fabsf(1 - iou);
        cnt += 1.0f;
    }
    return val / (cnt + 1e-6f);
}

// compute_iou_value's box perturbation + corners (box_fusion.py:289-331)
__device__ __forceinline__ void particle_corners(const float* box, const float* R, const float* prow,
                                                 const float* ss, float* corners) {
    float x = box[0] + prow[0] * ss[0];
    float y = box[1] + prow[1] * ss[1];
    float z = box[2] + prow[2] * ss[2];
    float w = box[5] + prow[5] * ss[5];
    float h = box[4] + prow[4] * ss[4];
    float l = box[3] + prow[3] * ss[3];
    w = fmaxf(w, 0.01f);
    h = fmaxf(h, 0.01f);
    l = fmaxf(l, 0.01f);
    const float xyz[3] = {x, y, z};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float v[3] = {bf_vsign_x(c) > 0 ? l / 2 : -l / 2, bf_vsign_y(c) > 0 ? h / 2 : -h / 2,
                            bf_vsign_z(c) > 0 ? w / 2 : -w / 2};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float s = 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k) s += R[j * 3 + k] * v[k];
            s += xyz[j];
            corners[3 * c + j] = s;
        }
    }
}

// ------------------------------------------------------------------------------------------
// single evaluation (evaluate_iou) — used by tests and by callers that drive their own loop
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_fitness(const float* __restrict__ box,
                                                  const float* __restrict__ R, int nv,
                                                  const float* __restrict__ vpose,
                                                  const float* __restrict__ vtc,
                                                  const float* __restrict__ pst, int np_,
                                                  const float* __restrict__ ss, bf_fuse_cfg cfg,
                                                  float* __restrict__ fitness) {
    __shared__ FuseViews V;
    for (int q = threadIdx.x; q < nv * 16; q += blockDim.x) {
        V.pose[q / 16][q % 16] = vpose[q];
        V.tc[q / 16][q % 16] = vtc[q];
    }
    __syncthreads();
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np_) return;
    float b[6], r[9], s[6], corners[24];
    for (int k = 0; k < 6; ++k) { b[k] = box[k]; s[k] = ss[k]; }
    for (int k = 0; k < 9; ++k) r[k] = R[k];
    particle_corners(b, r, pst + 6 * p, s, corners);
    int flags = 0;
    fitness[p] = particle_fitness(corners, V, nv, cfg, &flags);
}

BF_API int bf_fusion_fitness(const float* box, const float* R, int n_views, const float* view_pose,
                             const float* view_tc, const float* pst, int pst_size,
                             const float* search_size, const bf_fuse_cfg* cfg, float* fitness,
                             void* stream) {
    if (!cfg || !box || !R || !view_pose || !view_tc || !pst || !search_size || !fitness)
        return BF_ERR_ARG;
    if (n_views <= 0 || n_views > FUSE_MAX_VIEWS || pst_size <= 0) return BF_ERR_CAPACITY;
    hipLaunchKernelGGL(k_fitness, dim3(bf_cdiv(pst_size, 256)), dim3(256), 0, bf_stream(stream), box,
                       R, n_views, view_pose, view_tc, pst, pst_size, search_size, *cfg, fitness);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// full refinement: per iteration two launches over all jobs
//   k_fuse_terms  grid (pairs/256, job): thread = (view, particle), |1 - IoU2D| of that pair.
//                 A job's V*P independent pairs spread over many CUs (the single-workgroup
//                 form ran every particle of a job on one CU and was latency-bound).
//   k_fuse_step   one workgroup per job: fitness[p] = (sum of the V terms in view order)
//                 / (V + 1e-6) (the reference kernel's per-particle f32 accumulation order),
//                 accepted-set prefix, cal_transform sums, update_PST / momentum / accept.
// A job that stopped (3 consecutive failures) skips the remaining launches.
// ------------------------------------------------------------------------------------------
struct FuseState {
    double x[6];        // global_xyzlwh (f64, box_fusion.py:655)
    float ss[6];        // search_size (f32)
    float prev[6];      // previous_search_size (f32)
    float R[9];         // mean_rot
    float box32[6];     // x cast to f32 for the kernel
    int nv, off;
    int prev_success, fails, need_update, stop, iters_done, flags;
};

__global__ void __launch_bounds__(64) k_fuse_init(const int32_t* __restrict__ view_off,
                                                  const int32_t* __restrict__ n_views, int max_views,
                                                  const float* __restrict__ vbox,
                                                  const float* __restrict__ vR,
                                                  const float* __restrict__ vscore,
                                                  bf_fuse_cfg cfg, FuseState* __restrict__ states) {
    const int job = blockIdx.x;
    if (threadIdx.x != 0) return;
    FuseState& S = states[job];
    const int nv = n_views[job];
    const int off = view_off[job];
    S.nv = nv;
    S.off = off;
    S.prev_success = 0; S.fails = 0; S.need_update = 0; S.iters_done = 0; S.flags = 0;
    if (nv <= 0 || nv > FUSE_MAX_VIEWS || nv > max_views) {
        S.stop = 1;
        S.flags = BF_DEV_VIEW_OVERFLOW;
        for (int k = 0; k < 6; ++k) { S.x[k] = 0.0; S.box32[k] = 0.f; }
        return;
    }
    S.stop = 0;
    // init_opt_params (box_fusion.py:566-600)
    const float* vb = vbox + (size_t)off * 6;
    const float* vs = vscore + off;
    int best = 0;
    for (int v = 1; v < nv; ++v)
        if (vs[v] > vs[best]) best = v;
    for (int k = 0; k < 3; ++k) {
        float s = vb[k];
        for (int v = 1; v < nv; ++v) s = s + vb[6 * v + k];
        S.x[k] = (double)(s / (float)nv);
    }
    const float* bd = vb + 6 * best + 3;
    int si[3] = {0, 1, 2};
    for (int i = 1; i < 3; ++i) {
        int tt = si[i], j = i - 1;
        while (j >= 0 && bd[si[j]] > bd[tt]) { si[j + 1] = si[j]; --j; }
        si[j + 1] = tt;
    }
    int rank[3];
    for (int r = 0; r < 3; ++r) rank[si[r]] = r;
    float acc[3] = {0, 0, 0};
    for (int v = 0; v < nv; ++v) {
        float d[3] = {vb[6 * v + 3], vb[6 * v + 4], vb[6 * v + 5]};
        for (int i = 1; i < 3; ++i) {
            float tt = d[i];
            int j = i - 1;
            while (j >= 0 && d[j] > tt) { d[j + 1] = d[j]; --j; }
            d[j + 1] = tt;
        }
        for (int k = 0; k < 3; ++k) acc[k] = (v == 0) ? d[rank[k]] : acc[k] + d[rank[k]];
    }
    for (int k = 0; k < 3; ++k) S.x[3 + k] = (double)(acc[k] / (float)nv);
    for (int k = 0; k < 9; ++k) S.R[k] = vR[(size_t)(off + best) * 9 + k];
    for (int k = 0; k < 3; ++k) {
        S.ss[k] = (float)cfg.center_init;
        S.ss[3 + k] = (float)cfg.shape_init;
        S.prev[k] = 0.f;
        S.prev[3 + k] = 0.f;
    }
    for (int k = 0; k < 6; ++k) S.box32[k] = (float)S.x[k];
}

// target hull of every (job, view): fixed over the iterations, built once per call
struct TargetHull {
    P2 h[8];
    int n;
    float area;
};

__global__ void __launch_bounds__(64) k_fuse_targets(const float* __restrict__ vtc,
                                                     const FuseState* __restrict__ states,
                                                     int max_views, TargetHull* __restrict__ th) {
    const int job = blockIdx.x, v = threadIdx.x;
    const FuseState& S = states[job];
    if (v >= max_views) return;
    TargetHull& T = th[(size_t)job * max_views + v];
    if (S.stop || v >= S.nv) { T.n = 0; T.area = 0.f; return; }
    P2 ct[8], ht[8];
    const float* tc = vtc + ((size_t)S.off + v) * 16;
    for (int j = 0; j < 8; ++j) { ct[j].x = tc[2 * j]; ct[j].y = tc[2 * j + 1]; }
    const int nt = convex_hull<8>(ct, 8, ht);
    for (int j = 0; j < 8; ++j) T.h[j] = ht[j];
    T.n = nt;
    T.area = polygon_area(ht, nt);
}

#define TERM_THREADS 64   // one wave per workgroup (k_fuse_iter: its hull stacks take 40 KB of LDS)
// one wave = G4_PAIRS (particle, view) pairs x 4 lanes (iou_hull_g4); the pairs of a workgroup
// share the view (P % 64 == 0)
__global__ void __launch_bounds__(TERM_THREADS) k_fuse_terms(const float* __restrict__ vpose,
                                                             const TargetHull* __restrict__ th,
                                                             const float* __restrict__ pst,
                                                             bf_fuse_cfg cfg,
                                                             FuseState* __restrict__ states,
                                                             float* __restrict__ terms, int max_views) {
    const int job = blockIdx.y;
    const FuseState& S = states[job];
    if (S.stop) return;                                   // uniform per workgroup
    const int P = cfg.pst_size;                           // multiple of 64
    const int lane = threadIdx.x;
    const int pr = lane >> 2, g = lane & 3;
    const int pair = blockIdx.x * G4_PAIRS + pr;
    const int v = pair / P, p = pair % P;                 // v uniform per workgroup
    if (v >= S.nv) return;
    __shared__ float s_pose[16];
    __shared__ TargetHull s_th;
    __shared__ HullG4 s_hull;
    const size_t vi = (size_t)S.off + v;
    if (lane < 16) s_pose[lane] = vpose[vi * 16 + lane];
    else if (lane < 16 + 18) reinterpret_cast<float*>(&s_th)[lane - 16] =
        reinterpret_cast<const float*>(th + (size_t)job * max_views + v)[lane - 16];
    // this lane's two corners of the pair's particle box (particle_corners' expressions)
    float b[6], r[9], ss[6];
    for (int k = 0; k < 6; ++k) { b[k] = S.box32[k]; ss[k] = S.ss[k]; }
    for (int k = 0; k < 9; ++k) r[k] = S.R[k];
    const float* prow = pst + 6 * p;
    float x = b[0] + prow[0] * ss[0];
    float y = b[1] + prow[1] * ss[1];
    float z = b[2] + prow[2] * ss[2];
    float w = b[5] + prow[5] * ss[5];
    float h = b[4] + prow[4] * ss[4];
    float l = b[3] + prow[3] * ss[3];
    w = fmaxf(w, 0.01f);
    h = fmaxf(h, 0.01f);
    l = fmaxf(l, 0.01f);
    const float xyz[3] = {x, y, z};
    __syncthreads();
    const float* Pm = s_pose;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
        const int c = 2 * g + cc;
        const float vv[3] = {bf_vsign_x(c) > 0 ? l / 2 : -l / 2, bf_vsign_y(c) > 0 ? h / 2 : -h / 2,
                             bf_vsign_z(c) > 0 ? w / 2 : -w / 2};
        float cn[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float sacc = 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k) sacc += r[j * 3 + k] * vv[k];
            sacc += xyz[j];
            cn[j] = sacc;
        }
        float vx = cn[0] - Pm[3], vy = cn[1] - Pm[7], vz = cn[2] - Pm[11];
        float cx = Pm[0] * vx + Pm[4] * vy + Pm[8] * vz;
        float cy = Pm[1] * vx + Pm[5] * vy + Pm[9] * vz;
        float cz = Pm[2] * vx + Pm[6] * vy + Pm[10] * vz;
        float px = ((cx * cfg.K[0]) / cz + cfg.K[2]);
        float py = ((cy * cfg.K[5]) / cz + cfg.K[6]);
        P2 q;
        q.x = (px > cfg.img_w) ? cfg.img_w : (px < 0) ? 0 : px;
        q.y = (py > cfg.img_h) ? cfg.img_h : (py < 0) ? 0 : py;
        s_hull.c0[c * G4_PAIRS + pr] = q;
    }
    __syncthreads();
    P2 c0[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c0[j] = s_hull.c0[j * G4_PAIRS + pr];
    int flags = 0;
    const float iou = iou_hull_g4(c0, s_th.h, s_th.n, s_th.area, s_hull, pr, g, &flags);
    if (g == 0) terms[((size_t)job * max_views + v) * P + p] = fabsf(1 - iou);
    if (flags) atomicOr(&states[job].flags, flags);
}

// the sequential update of one job after an iteration's terms (any block size, multiple of 64)
struct StepLds {
    float fit[FUSE_MAX_PST];
    int acc[FUSE_MAX_PST];
    float prod[FUSE_MAX_PST * 8];   // accepted particle k: 6 weighted offsets, w, fit*w
};

__device__ void fuse_step_body(int job, const float* __restrict__ pst, const bf_fuse_cfg& cfg,
                               FuseState* __restrict__ states, const float* __restrict__ terms,
                               int max_views, int it, float* __restrict__ trace, StepLds& L) {
    const int t = threadIdx.x;
    const int P = cfg.pst_size;
    FuseState* G = states + job;
    if (G->stop) return;
    float* s_fit = L.fit;
    int* s_acc = L.acc;
    float* s_prod = L.prod;
    __shared__ int s_wave[16];
    __shared__ double s_dsum[8];
    __shared__ float s_fsum[8];
    const int nv = G->nv;
    const int NT = blockDim.x;
    // ---- fitness: the reference's per-particle loop `val += |1 - iou|; cnt += 1` -------------
    for (int p = t; p < P; p += NT) {
        float val = 0.0f, cnt = 0.0f;
        const float* tp = terms + (size_t)job * max_views * P + p;
        for (int v = 0; v < nv; ++v) {
            val += tp[(size_t)v * P];
            cnt += 1.0f;
        }
        const float f = val / (cnt + 1e-6f);
        s_fit[p] = f;
        if (trace) trace[((size_t)job * cfg.iters + it) * P + p] = f;
    }
    __syncthreads();
    // ---- accepted particles: j >= 1, fit[j] < fit[0], first max_accept in index order ------
    // (chunks of NT particles in index order; within a chunk a block ballot prefix)
    const float f0 = s_fit[0];
    int base = 0;
    for (int c0 = 0; c0 < P; c0 += NT) {
        const int p = c0 + t;
        const bool flag = (p >= 1) && (p < P) && (s_fit[p] < f0);
        const unsigned long long m = __ballot(flag);
        if (bf_lane() == 0) s_wave[t >> 6] = __popcll(m);
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < (NT >> 6); ++w) {
            if (w < (t >> 6)) before += s_wave[w];
            tot += s_wave[w];
        }
        const int rnk = base + before + bf_lanes_below(m);
        if (flag && rnk < cfg.max_accept) s_acc[rnk] = p;
        base += tot;
        __syncthreads();
    }
    const int n_acc = base < cfg.max_accept ? base : cfg.max_accept;
    // ---- cal_transform sums in reference order (8 independent sequential sums) -------------
    // the f32 products of every accepted particle are formed in parallel into LDS first, so
    // the 8 sequential sums below only chain adds (not a dependent global load per step)
    for (int k = t; k < n_acc; k += NT) {
        const int j = s_acc[k];
        const float fj = s_fit[j];
        const float w = f0 - fj;
        const float* pj = pst + 6 * j;
#pragma unroll
        for (int c = 0; c < 6; ++c) s_prod[8 * k + c] = pj[c] * w;
        s_prod[8 * k + 6] = w;
        s_prod[8 * k + 7] = fj * w;
    }
    __syncthreads();
    if (t < 8) {
        double ds = 0.0;
        float fs = 0.0f;
        if (cfg.legacy_promotion)
            for (int k = 0; k < n_acc; ++k) ds += (double)s_prod[8 * k + t];
        else
            for (int k = 0; k < n_acc; ++k) fs = fs + s_prod[8 * k + t];
        s_dsum[t] = ds;
        s_fsum[t] = fs;
    }
    __syncthreads();
    // ---- lane 0: cal_transform tail, update_PST, momentum, accept ----------------------------
    if (t == 0) {
        FuseState S = *G;
        const bool success = n_acc > 0;
        float mt[6] = {0, 0, 0, 0, 0, 0};
        double iou_d = 0;
        float iou_f = 0;
        if (!success) {
            iou_d = f0;
            iou_f = f0;
        } else if (cfg.legacy_promotion) {
            iou_d = s_dsum[7] / s_dsum[6];
            for (int k = 0; k < 6; ++k) mt[k] = (float)((s_dsum[k] / s_dsum[6]) * (double)S.ss[k]);
        } else {
            iou_f = s_fsum[7] / s_fsum[6];
            for (int k = 0; k < 6; ++k) mt[k] = (s_fsum[k] / s_fsum[6]) * S.ss[k];
        }
        if (cfg.legacy_promotion) {
            double sc[6];
            for (int k = 0; k < 6; ++k) sc[k] = fabs((double)mt[k]) + cfg.min_scale;
            double nrm = sc[0] * sc[0];
            for (int k = 1; k < 6; ++k) nrm = nrm + sc[k] * sc[k];
            nrm = sqrt(nrm);
            for (int k = 3; k < 6; ++k) S.ss[k] = (float)(cfg.shape_coef * iou_d * (sc[k] / nrm) + cfg.min_scale);
            for (int k = 0; k < 3; ++k) S.ss[k] = (float)(cfg.center_coef * iou_d * (sc[k] / nrm) + cfg.min_scale);
        } else {
            const float ms = (float)cfg.min_scale;
            float sc[6];
            for (int k = 0; k < 6; ++k) sc[k] = fabsf(mt[k]) + ms;
            float nrm = sc[0] * sc[0];
            for (int k = 1; k < 6; ++k) nrm = nrm + sc[k] * sc[k];
            nrm = sqrtf(nrm);
            for (int k = 3; k < 6; ++k) S.ss[k] = (float)cfg.shape_coef * iou_f * (sc[k] / nrm) + ms;
            for (int k = 0; k < 3; ++k) S.ss[k] = (float)cfg.center_coef * iou_f * (sc[k] / nrm) + ms;
        }
        if (S.prev_success && success) {
            for (int k = 0; k < 6; ++k) {
                if (cfg.legacy_promotion)
                    S.ss[k] = (float)(cfg.beta * (double)S.ss[k] + (1.0 - cfg.beta) * (double)S.prev[k]);
                else
                    S.ss[k] = (float)cfg.beta * S.ss[k] + (float)(1.0 - cfg.beta) * S.prev[k];
            }
        }
        if (success) {
            S.need_update = 1;
            S.prev_success = 1;
            S.fails = 0;
            for (int k = 0; k < 6; ++k) S.x[k] += (double)mt[k];
            for (int k = 0; k < 6; ++k) S.prev[k] = S.ss[k];
        } else {
            S.fails++;
            S.prev_success = 0;
        }
        S.iters_done = it + 1;
        if (S.fails >= 3) S.stop = 1;
        for (int k = 0; k < 6; ++k) S.box32[k] = (float)S.x[k];
        S.flags = G->flags;                       // term kernels may have OR-ed flags in
        *G = S;
    }
}

// One launch per iteration: the terms of every (job, view, particle) as k_fuse_terms, then the
// job's workgroup that finishes last (device-scope counter per job) runs the job's sequential
// update — half the launches of the terms + step pair, on a path that is launch-latency bound.
// The step reuses the hull stacks' LDS (dead by then).
union IterLds {
    HullLds hull;
    StepLds step;
};

__global__ void __launch_bounds__(TERM_THREADS) k_fuse_iter(const float* __restrict__ vpose,
                                                            const TargetHull* __restrict__ th,
                                                            const float* __restrict__ pst,
                                                            bf_fuse_cfg cfg,
                                                            FuseState* __restrict__ states,
                                                            float* __restrict__ terms, int max_views,
                                                            int it, float* __restrict__ trace,
                                                            int* __restrict__ done) {
    __shared__ IterLds U;
    __shared__ float s_pose[16];
    __shared__ TargetHull s_th;
    __shared__ int s_last;
    const int job = blockIdx.y;
    const FuseState& S = states[job];
    const int P = cfg.pst_size;                           // multiple of 64
    const int pair = blockIdx.x * TERM_THREADS + threadIdx.x;
    const int v = pair / P, p = pair % P;                 // v uniform per (one-wave) workgroup
    const int lane = threadIdx.x;
    if (!S.stop && v < S.nv) {
        const size_t vi = (size_t)S.off + v;
        if (lane < 16) s_pose[lane] = vpose[vi * 16 + lane];
        else if (lane < 16 + 18) reinterpret_cast<float*>(&s_th)[lane - 16] =
            reinterpret_cast<const float*>(th + (size_t)job * max_views + v)[lane - 16];
        __syncthreads();
        float b[6], r[9], ss[6], corners[24];
        for (int k = 0; k < 6; ++k) { b[k] = S.box32[k]; ss[k] = S.ss[k]; }
        for (int k = 0; k < 9; ++k) r[k] = S.R[k];
        particle_corners(b, r, pst + 6 * p, ss, corners);
        const float* Pm = s_pose;
        P2 c0[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float vx = corners[3 * j] - Pm[3], vy = corners[3 * j + 1] - Pm[7], vz = corners[3 * j + 2] - Pm[11];
            float cx = Pm[0] * vx + Pm[4] * vy + Pm[8] * vz;
            float cy = Pm[1] * vx + Pm[5] * vy + Pm[9] * vz;
            float cz = Pm[2] * vx + Pm[6] * vy + Pm[10] * vz;
            float px = ((cx * cfg.K[0]) / cz + cfg.K[2]);
            float py = ((cy * cfg.K[5]) / cz + cfg.K[6]);
            c0[j].x = (px > cfg.img_w) ? cfg.img_w : (px < 0) ? 0 : px;
            c0[j].y = (py > cfg.img_h) ? cfg.img_h : (py < 0) ? 0 : py;
        }
        int flags = 0;
        const float iou = iou_hull_lds(c0, s_th.h, s_th.n, s_th.area, U.hull, lane, &flags);
        terms[((size_t)job * max_views + v) * P + p] = fabsf(1 - iou);
        if (flags) atomicOr(&states[job].flags, flags);
    }
    // the job's last workgroup to finish runs the update
    __threadfence();
    __syncthreads();
    if (lane == 0)
        s_last = __hip_atomic_fetch_add(&done[job], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                 (int)gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    if (lane == 0) done[job] = 0;                          // for the next iteration's launch
    fuse_step_body(job, pst, cfg, states, terms, max_views, it, trace, U.step);
}

__global__ void __launch_bounds__(1024) k_fuse_step(const float* __restrict__ pst, bf_fuse_cfg cfg,
                                                    FuseState* __restrict__ states,
                                                    const float* __restrict__ terms, int max_views,
                                                    int it, float* __restrict__ trace) {
    __shared__ StepLds L;
    fuse_step_body(blockIdx.x, pst, cfg, states, terms, max_views, it, trace, L);
}

__global__ void __launch_bounds__(64) k_fuse_final(const FuseState* __restrict__ states, int n_jobs,
                                                   float* __restrict__ out_box,
                                                   int32_t* __restrict__ out_updated,
                                                   int32_t* __restrict__ out_iters,
                                                   int32_t* __restrict__ status) {
    const int job = blockIdx.x * blockDim.x + threadIdx.x;
    if (job >= n_jobs) return;
    FuseState S = states[job];
    for (int k = 3; k < 6; ++k)
        if (S.x[k] < 0.01) S.x[k] = 0.01;
    for (int k = 0; k < 6; ++k) out_box[6 * job + k] = (float)S.x[k];
    out_updated[job] = S.need_update;
    out_iters[job] = S.iters_done;
    if (S.flags) atomicOr(status, S.flags);
}

// BoxFusion.boxfusion's write-back (box_fusion.py:716-724): rows of the refined boxes whose job
// updated get xyz + lhw (R unchanged); target f32 rows of `ld` floats (xyzlhw first)
__global__ void __launch_bounds__(64) k_fuse_writeback(const float* __restrict__ out_box,
                                                       const int32_t* __restrict__ updated,
                                                       const int32_t* __restrict__ rows, int n_jobs,
                                                       float* __restrict__ target, int ld) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_jobs * 6) return;
    const int job = e / 6, k = e % 6;
    if (updated[job]) target[(size_t)rows[job] * ld + k] = out_box[6 * job + k];
}

BF_API int bf_fusion_writeback(const float* out_box, const int32_t* updated, const int32_t* rows,
                               int n_jobs, float* target, int ld, void* stream) {
    if (n_jobs < 0 || ld < 6) return BF_ERR_ARG;
    if (n_jobs == 0) return BF_OK;
    if (!out_box || !updated || !rows || !target) return BF_ERR_ARG;
    hipLaunchKernelGGL(k_fuse_writeback, dim3(bf_cdiv(n_jobs * 6, 64)), dim3(64), 0,
                       bf_stream(stream), out_box, updated, rows, n_jobs, target, ld);
    return bf_check_launch();
}

static size_t fuse_states_bytes(int n_jobs) {
    return ((size_t)n_jobs * sizeof(FuseState) + 255) & ~(size_t)255;
}
static size_t fuse_targets_bytes(int n_jobs, int max_views) {
    return ((size_t)n_jobs * max_views * sizeof(TargetHull) + 255) & ~(size_t)255;
}

static size_t fuse_done_bytes(int n_jobs) { return ((size_t)n_jobs * sizeof(int) + 255) & ~(size_t)255; }

BF_API size_t bf_fusion_fit_workspace_size(int n_jobs, int max_views, int pst_size) {
    if (n_jobs <= 0 || max_views <= 0 || pst_size <= 0) return 0;
    return fuse_states_bytes(n_jobs) + fuse_targets_bytes(n_jobs, max_views) + fuse_done_bytes(n_jobs) +
           (size_t)n_jobs * max_views * pst_size * sizeof(float);
}

BF_API int bf_fusion_fit(const int32_t* view_off, const int32_t* n_views, int n_jobs,
                         int max_views, const float* view_box, const float* view_R,
                         const float* view_score, const float* view_pose, const float* view_tc,
                         const float* pst, const bf_fuse_cfg* cfg, float* out_box,
                         int32_t* out_updated, int32_t* out_iters, float* trace,
                         int32_t* status, void* workspace, void* stream) {
    if (!cfg || n_jobs < 0) return BF_ERR_ARG;
    if (n_jobs == 0) return BF_OK;
    if (!view_off || !n_views || !view_box || !view_R || !view_score || !view_pose || !view_tc ||
        !pst || !out_box || !out_updated || !out_iters || !status || !workspace)
        return BF_ERR_ARG;
    if (max_views <= 0 || max_views > FUSE_MAX_VIEWS) return BF_ERR_CAPACITY;
    if (cfg->pst_size <= 0 || cfg->pst_size > FUSE_MAX_PST || (cfg->pst_size % 64) != 0)
        return BF_ERR_CAPACITY;
    hipStream_t s = bf_stream(stream);
    FuseState* states = reinterpret_cast<FuseState*>(workspace);
    char* ws = reinterpret_cast<char*>(workspace) + fuse_states_bytes(n_jobs);
    TargetHull* th = reinterpret_cast<TargetHull*>(ws);
    int* done = reinterpret_cast<int*>(ws + fuse_targets_bytes(n_jobs, max_views));
    float* terms = reinterpret_cast<float*>(reinterpret_cast<char*>(done) + fuse_done_bytes(n_jobs));
    if (hipMemsetAsync(done, 0, sizeof(int) * (size_t)n_jobs, s) != hipSuccess) return BF_ERR_LAUNCH;
    const int P = cfg->pst_size;
    hipLaunchKernelGGL(k_fuse_init, dim3(n_jobs), dim3(64), 0, s, view_off, n_views, max_views,
                       view_box, view_R, view_score, *cfg, states);
    hipLaunchKernelGGL(k_fuse_targets, dim3(n_jobs), dim3(64), 0, s, view_tc, states, max_views, th);
    const dim3 tgrid((unsigned)bf_cdiv(max_views * P, TERM_THREADS), (unsigned)n_jobs);
    const dim3 tgrid4((unsigned)bf_cdiv(max_views * P, G4_PAIRS), (unsigned)n_jobs);
    for (int it = 0; it < cfg->iters; ++it) {
#if FUSE_SPLIT_ITER
        hipLaunchKernelGGL(k_fuse_terms, tgrid4, dim3(TERM_THREADS), 0, s, view_pose, th, pst,
                           *cfg, states, terms, max_views);
        hipLaunchKernelGGL(k_fuse_step, dim3(n_jobs), dim3(P), 0, s, pst, *cfg, states, terms,
                           max_views, it, trace);
#else
        hipLaunchKernelGGL(k_fuse_iter, tgrid, dim3(TERM_THREADS), 0, s, view_pose, th, pst, *cfg,
                           states, terms, max_views, it, trace, done);
#endif
    }
    hipLaunchKernelGGL(k_fuse_final, dim3(bf_cdiv(n_jobs, 64)), dim3(64), 0, s, states, n_jobs,
                       out_box, out_updated, out_iters, status);
    return bf_check_launch();
}
