// bf_assoc.hip — spatial and correspondence association on gfx950.
//
//   k_nms_scan    nms_3d (instances.py:22-101) + BoxManager.record (box_manager.py:40-88)
//   k_corr_assoc  correspondence_association (instances.py:411-490), project_3d_to_2d_box
//                 (:670-717), IoU_2D_box (:643-668), BoxManager.record_corr (box_manager.py:90-129)
//
// Both are inherently serial state machines (each greedy step depends on the previous one), so
// each runs as ONE 256-thread workgroup: the per-step data-parallel part (IoU threshold tests of
// the remaining candidates, order-preserving compaction, 2-D projection and IoU, argmax) uses all
// four waves with ballot/prefix primitives; the bookkeeping (fusion lists, keep edits) runs on
// lane 0 exactly in the reference's order.  Fusion lists live in global memory as fixed-capacity
// rows (cap from the config, overflow -> BF_DEV_FUSION_LIST_OVERFLOW).
#include "bf_common.h"

#define SCAN_THREADS 256
#define SCAN_WAVES (SCAN_THREADS / 64)

// --- order-preserving block compaction helper ---------------------------------------------
// Each thread contributes one flag; returns its exclusive rank among set flags of the block and
// writes the block total to *total (all threads).
__device__ __forceinline__ int block_rank(bool f, int* s_wave, int* total) {
    unsigned long long m = __ballot(f);
    int w = threadIdx.x >> 6;
    if (bf_lane() == 0) s_wave[w] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
    for (int k = 0; k < SCAN_WAVES; ++k) {
        if (k < w) off += s_wave[k];
        tot += s_wave[k];
    }
    __syncthreads();
    *total = tot;
    return off + bf_lanes_below(m);
}

__device__ int fl_append_sorted(int32_t* row, int32_t* len, int cap, const int32_t* vals, int nv) {
    if (*len + nv > cap) return BF_DEV_FUSION_LIST_OVERFLOW;
    for (int v = 0; v < nv; ++v) row[(*len)++] = vals[v];
    for (int i = 1; i < *len; ++i) {
        int32_t x = row[i];
        int j = i - 1;
        while (j >= 0 && row[j] > x) { row[j + 1] = row[j]; --j; }
        row[j + 1] = x;
    }
    return 0;
}

// fl_append_sorted by the 64 lanes of one wave (a wave-uniform call): lane l holds entry l of
// the appended row and writes it at its rank (smaller values, ties by position) -- the order the
// insertion sort produces, in one pass instead of lane 0's O(L^2) LDS chain
__device__ int fl_append_sorted_w(int32_t* row, int32_t* len, int cap, const int32_t* vals, int nv) {
    const int L0 = *len, Ln = L0 + nv;
    if (Ln > cap) return BF_DEV_FUSION_LIST_OVERFLOW;
    const int l = threadIdx.x & 63;
    if (Ln > 64) {                                   // (list capacity above a wave: lane 0)
        int st = 0;
        if (l == 0) st = fl_append_sorted(row, len, cap, vals, nv);
        return st;
    }
    const int v = l < L0 ? row[l] : (l < Ln ? vals[l - L0] : 0);
    int r = 0;
    for (int k = 0; k < Ln; ++k) {
        const int x = __shfl(v, k, 64);
        r += (x < v) || (x == v && k < l);
    }
    if (l < Ln) row[r] = v;
    if (l == 0) *len = Ln;
    return 0;
}

// keep.remove(cur); keep.append(idx) when cur is in keep (record()'s branch-2 edit), by one wave
__device__ void keep_replace_w(int* keep, int nk, int cur, int idx) {
    const int l = threadIdx.x & 63;
    int pos = nk;
    for (int b = 0; b < nk; b += 64) {
        const unsigned long long m = __ballot(b + l < nk && keep[b + l] == cur);
        if (m) { pos = b + __ffsll((long long)m) - 1; break; }
    }
    if (pos >= nk) return;
    for (int b = pos; b < nk - 1; b += 64) {        // shift left: chunk reads precede its writes
        const int q = b + l;
        const int x = q + 1 < nk ? keep[q + 1] : 0;
        if (q < nk - 1) keep[q] = x;
    }
    if (l == 0) keep[nk - 1] = idx;
}

__device__ __forceinline__ void box_center(const float* corners, int i, float* c) {
    for (int k = 0; k < 3; ++k) {
        float s = corners[24 * i + k];
        for (int q = 1; q < 8; ++q) s = s + corners[24 * i + 3 * q + k];
        c[k] = s / 8.0f;
    }
}

// global -> LDS copy with 8 independent loads in flight per lane (a plain strided loop waits for
// every load before the next: one memory latency per 64 elements)
template <typename T, int F = 8>
__device__ __forceinline__ void stage_lds(T* dst, const T* __restrict__ src, int count, int t, int nt) {
    int q = t;
    for (; q + (F - 1) * nt < count; q += F * nt) {
        T v[F];
#pragma unroll
        for (int k = 0; k < F; ++k) v[k] = src[q + k * nt];
#pragma unroll
        for (int k = 0; k < F; ++k) dst[q + k * nt] = v[k];
    }
    for (; q < count; q += nt) dst[q] = src[q];
}

// rank sort of distinct int values in LDS (ascending), in place via a scratch buffer
__device__ void block_sort_distinct(int* a, int* tmp, int n) {
    for (int q = threadIdx.x; q < n; q += SCAN_THREADS) tmp[q] = a[q];
    __syncthreads();
    for (int q = threadIdx.x; q < n; q += SCAN_THREADS) {
        int v = tmp[q], r = 0;
        for (int k = 0; k < n; ++k) r += tmp[k] < v;
        a[r] = v;
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------
// NMS scan
// ------------------------------------------------------------------------------------------
#define NMS_IOU_LDS_N 120                                   // n <= 120: IoU matrix (<=113 KB) in LDS
#define NMS_IOU_LDS_MAX (NMS_IOU_LDS_N * NMS_IOU_LDS_N)
__global__ void __launch_bounds__(SCAN_THREADS) k_nms_scan(
    const double* __restrict__ iou, const float* __restrict__ corners,
    const float* __restrict__ scores, const int32_t* __restrict__ init_id,
    const float* __restrict__ poses, int n, int32_t* __restrict__ fl, int32_t* __restrict__ fl_len,
    float* __restrict__ valid_num, int32_t* __restrict__ keep_out, int32_t* __restrict__ n_keep,
    int32_t* __restrict__ succ_out, int32_t* __restrict__ n_succ, int32_t* __restrict__ events,
    int32_t* __restrict__ n_events, int32_t* __restrict__ status, bf_nms_cfg cfg) {
    extern __shared__ __attribute__((aligned(16))) double dsmem[];
    // small problems stage the IoU matrix in LDS: the scan reads one row per kept box
    const bool iou_lds = (size_t)n * n <= NMS_IOU_LDS_MAX;
    double* iou_s = dsmem;
    int* smem = reinterpret_cast<int*>(dsmem + (iou_lds ? (size_t)n * n : 0));
    int* bufA = smem;             // order (ping)
    int* bufB = bufA + n + 1;     // order (pong)
    int* supp = bufB + n + 1;     // suppressed list of the current step
    int* keep = supp + n + 1;     // python-list image of `keep`
    int* succ = keep + n + 2;     // success_nms
    float* cen = reinterpret_cast<float*>(succ + n + 2);   // box centres [n][3] (nms_3d:49)
    __shared__ int s_wave[SCAN_WAVES];
    __shared__ int s_no, s_nk, s_ns, s_nsupp;
    const int t = threadIdx.x;
    const int cap = cfg.list_capacity;

    for (int i = t; i < n; i += SCAN_THREADS) box_center(corners, i, cen + 3 * i);
    if (iou_lds) stage_lds(iou_s, iou, n * n, t, SCAN_THREADS);
    const double* I = iou_lds ? iou_s : iou;
    // order = scores.argsort()[::-1]: descending, ties -> higher index first
    for (int i = t; i < n; i += SCAN_THREADS) {
        float si = scores[i];
        int r = 0;
        for (int j = 0; j < n; ++j) {
            float sj = scores[j];
            r += (sj > si) || (sj == si && j > i);
        }
        bufA[r] = i;
    }
    if (t == 0) { s_no = n; s_nk = 0; s_ns = 0; }
    __syncthreads();
    int* order = bufA;
    int* rest = bufB;
    int nev = 0, st = 0;  // lane-0 private
    while (true) {
        int no = s_no;
        if (no <= 0) break;
        const int i = order[0];
        if (t == 0) keep[s_nk++] = i;
        int nrest = 0, nsupp = 0;
        for (int base = 1; base < no; base += SCAN_THREADS) {
            int q = base + t;
            const bool live = q < no;
            const int j = order[live ? q : no - 1];          // valid index: the load is always safe
            const double v = live ? I[(size_t)i * n + j] : 0.0;
            bool fr = (q < no) && (v <= cfg.iou_threshold);
            bool fs = (q < no) && (v > cfg.iou_threshold);
            int tr, ts;
            int pr = block_rank(fr, s_wave, &tr);
            int ps = block_rank(fs, s_wave, &ts);
            if (fr) rest[nrest + pr] = j;
            if (fs) supp[nsupp + ps] = j;
            nrest += tr;
            nsupp += ts;
        }
        __syncthreads();
        if (nsupp > 0 && t == 0) {
            valid_num[i] += 1.0f;
            succ[s_ns++] = i;
            // BoxManager.record(cur=i, fusion_inds=supp)
            const int cur = i;
            const float* ccur = cen + 3 * cur;
            for (int s = 0; s < nsupp; ++s) {
                const int idx = supp[s];
                const float* cidx = cen + 3 * idx;
                float dx = ccur[0] - cidx[0], dy = ccur[1] - cidx[1], dz = ccur[2] - cidx[2];
                float cd = sqrtf((dx * dx + dy * dy) + dz * dz);
                int branch;
                if (fl_len[idx] == 1) {
                    branch = 1;
                    int cnt = 0;
                    // a caller-supplied length past the row capacity reads no further than the
                    // row (the one-wave scan's clamp) and is reported
                    const int L = min(fl_len[cur], cap);
                    if (fl_len[cur] > cap) st |= BF_DEV_FUSION_LIST_OVERFLOW;
                    for (int q = 0; q < L; ++q) {
                        int pi = fl[(size_t)cur * cap + q];
                        float b, a;
                        bf_pose_disparity(poses + 16 * (size_t)pi, poses + 16 * (size_t)init_id[idx], &b, &a);
                        if ((b > cfg.translation_gap || a > cfg.rotation_gap) || (double)cd > cfg.center_gap) cnt++;
                    }
                    if (cnt == L && L < cfg.max_list) {
                        int32_t v = init_id[idx];
                        st |= fl_append_sorted(fl + (size_t)cur * cap, fl_len + cur, cap, &v, 1);
                    }
                } else {
                    branch = 2;
                    int cnt = 0;
                    const int L = min(fl_len[idx], cap);
                    if (fl_len[idx] > cap) st |= BF_DEV_FUSION_LIST_OVERFLOW;
                    for (int q = 0; q < L; ++q) {
                        int pi = fl[(size_t)idx * cap + q];
                        float b, a;
                        bf_pose_disparity(poses + 16 * (size_t)pi, poses + 16 * (size_t)init_id[cur], &b, &a);
                        if ((b > cfg.translation_gap || a > cfg.rotation_gap) || (double)cd > cfg.center_gap) cnt++;
                    }
                    if (cnt == L && L < cfg.max_list) {
                        // fl[cur] += fl[idx]  (copy first: rows are distinct, cur != idx)
                        st |= fl_append_sorted(fl + (size_t)cur * cap, fl_len + cur, cap,
                                               fl + (size_t)idx * cap, L);
                    } else {
                        int nk = s_nk, pos = -1;
                        for (int q = 0; q < nk; ++q)
                            if (keep[q] == cur) { pos = q; break; }
                        if (pos >= 0) {
                            for (int q = pos; q + 1 < nk; ++q) keep[q] = keep[q + 1];
                            keep[nk - 1] = idx;
                        }
                    }
                }
                events[3 * nev + 0] = cur;
                events[3 * nev + 1] = idx;
                events[3 * nev + 2] = branch;
                nev++;
            }
        }
        if (t == 0) s_no = nrest;
        __syncthreads();
        int* tmp = order; order = rest; rest = tmp;
        if (nrest == 1) {
            if (t == 0) keep[s_nk++] = order[0];
            __syncthreads();
            break;
        }
    }
    __syncthreads();
    const int nk = s_nk, ns = s_ns;
    // sort keep / success (distinct indices) using the free order buffers as scratch
    block_sort_distinct(keep, bufA == order ? bufB : bufA, nk);
    block_sort_distinct(succ, bufA == order ? bufB : bufA, ns);
    for (int q = t; q < nk; q += SCAN_THREADS) keep_out[q] = keep[q];
    for (int q = t; q < ns; q += SCAN_THREADS) succ_out[q] = succ[q];
    if (t == 0) {
        *n_keep = nk;
        *n_succ = ns;
        *n_events = nev;
        *status |= st;
    }
}

// ------------------------------------------------------------------------------------------
// Single-wave NMS scan for small problems (n <= NMS_FAST_N and every operand fits in LDS).
// The IoU matrix, fusion lists, init ids, valid_num, scores and box centres are staged in LDS;
// the compaction of the remaining candidates is a wave ballot (no workgroup barriers); the
// pose-disparity tests of one suppression over a fusion list run on the list's lanes at once
// (record() only counts them: order-free).  The list / keep edits stay on lane 0 in the
// reference's order, so the results are those of k_nms_scan.
// ------------------------------------------------------------------------------------------
#ifndef NMS_FAST_N
#define NMS_FAST_N 96       // (a diagnostic build sets 0 to run k_nms_scan everywhere)
#endif
#define NMS_FAST_LDS_MAX (150 * 1024)

__device__ __forceinline__ unsigned long long lanes_lt_mask() {
    const int l = threadIdx.x & 63;
    return l == 0 ? 0ull : ((1ull << l) - 1ull);
}

// LDS pose cache of the scan: a direct-mapped table of NMS_PC camera poses keyed by frame id
// (tag = the frame, -1 empty), filled before the scan with the poses record() can test (the
// boxes' init ids and their fusion-list entries); a lookup whose slot holds another frame reads
// the pose from global memory instead, so every pose value is the same either way.
#define NMS_PC 256
#ifndef NMS_DIAG_NORECORD
#define NMS_DIAG_NORECORD 0     // timing diagnostic only (wrong results): the scan without record()
#endif
__device__ __forceinline__ const float* nms_pose(const float* poses, const int* ptag, const float* pcache,
                                                 int f) {
    const int slot = f & (NMS_PC - 1);
    return ptag[slot] == f ? pcache + 16 * slot : poses + 16 * (size_t)f;
}

// entries q < L of `row` whose pose is far from pose pj (record()'s count, box_manager.py:51-80)
__device__ __forceinline__ int nms_count_far(const int* row, int L, const float* poses, const int* ptag,
                                             const float* pcache, int pj, float cd,
                                             const bf_nms_cfg& cfg) {
    int cnt = 0;
    const float* Pj = nms_pose(poses, ptag, pcache, pj);
    for (int base = 0; base < L; base += 64) {
        const int q = base + (int)threadIdx.x;
        bool f = false;
        if (q < L) {
            float b, a;
            bf_pose_disparity(nms_pose(poses, ptag, pcache, row[q]), Pj, &b, &a);
            f = (b > cfg.translation_gap || a > cfg.rotation_gap) || (double)cd > cfg.center_gap;
        }
        cnt += __popcll(__ballot(f));
    }
    return cnt;
}

// 64-bit words per row of a threshold bit mask
__host__ __device__ inline int nms_words(int n) { return (n + 63) / 64; }

static size_t nms_fast_lds(int n, int cap, bool bits) {
    return sizeof(float) * 16 * NMS_PC + sizeof(int) * NMS_PC   // pose cache + tags
           + (bits ? sizeof(unsigned long long) * 2 * (size_t)n * nms_words(n)   // masks
                   : sizeof(double) * (size_t)n * n)            // IoU
           + sizeof(int) * ((size_t)n * cap + 2 * (size_t)n)     // lists, lengths, init ids
           + sizeof(float) * 5 * (size_t)n                       // valid_num, scores, centres
           + sizeof(int) * (5 * (size_t)n + 8);                  // order x2, supp, keep, succ
}

// the scan reads the IoU matrix only through the two tests iou <= t (stays in `order`) and
// iou > t (suppressed; a NaN passes neither and leaves the order), so for large n it runs on
// these two bit masks, [2][n][words]: row i, word c, bit l <-> column 64c + l
__global__ void __launch_bounds__(256) k_nms_bits(const double* __restrict__ iou, int n, int words,
                                                  double thr, unsigned long long* __restrict__ bits) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= n * words) return;                                 // wave-uniform
    const int lane = threadIdx.x & 63;
    const int i = w / words, c = w % words, j = 64 * c + lane;
    const bool live = j < n;
    const double v = live ? iou[(size_t)i * n + j] : 0.0;
    const unsigned long long r = __ballot(live && v <= thr);
    const unsigned long long sp = __ballot(live && v > thr);
    if (lane == 0) {
        bits[(size_t)i * words + c] = r;
        bits[(size_t)n * words + (size_t)i * words + c] = sp;
    }
}

template <bool BITS>
__global__ void __launch_bounds__(64) k_nms_scan_w(
    const double* __restrict__ iou, const float* __restrict__ corners,
    const float* __restrict__ scores, const int32_t* __restrict__ init_id,
    const float* __restrict__ poses, int n, int32_t* __restrict__ fl, int32_t* __restrict__ fl_len,
    float* __restrict__ valid_num, int32_t* __restrict__ keep_out, int32_t* __restrict__ n_keep,
    int32_t* __restrict__ succ_out, int32_t* __restrict__ n_succ, int32_t* __restrict__ events,
    int32_t* __restrict__ n_events, int32_t* __restrict__ status, bf_nms_cfg cfg,
    const unsigned long long* __restrict__ bits) {
    extern __shared__ __attribute__((aligned(16))) double wsm[];
    const int cap = cfg.list_capacity;
    const int t = threadIdx.x;
    const int words = nms_words(n);
    float* pcache = reinterpret_cast<float*>(wsm);                // [NMS_PC][16]
    int* ptag = reinterpret_cast<int*>(pcache + 16 * NMS_PC);    // [NMS_PC]
    double* I = reinterpret_cast<double*>(ptag + NMS_PC);         // IoU matrix, or the masks:
    unsigned long long* Bm = reinterpret_cast<unsigned long long*>(I);
    int* fls = BITS ? reinterpret_cast<int*>(Bm + 2 * (size_t)n * words)
                    : reinterpret_cast<int*>(I + (size_t)n * n);
    int* fll = fls + (size_t)n * cap;
    int* iid = fll + n;
    float* vn = reinterpret_cast<float*>(iid + n);
    float* sc = vn + n;
    float* cen = sc + n;
    int* bufA = reinterpret_cast<int*>(cen + 3 * n);
    int* bufB = bufA + n + 1;
    int* supp = bufB + n + 1;
    int* keep = supp + n + 1;
    int* succ = keep + n + 2;
    // list lengths clamped to the row capacity (a longer input length would read and write past
    // the row); such an input sets the overflow status bit
    int in_over = 0;
    for (int q = t; q < n; q += 64) {
        fll[q] = min(fl_len[q], cap);
        in_over |= fl_len[q] > cap;
        iid[q] = init_id[q];
        vn[q] = valid_num[q];
        sc[q] = scores[q];
        box_center(corners, q, cen + 3 * q);
    }
    if (BITS) stage_lds<unsigned long long, 16>(Bm, bits, 2 * n * words, t, 64);
    else stage_lds<double, 16>(I, iou, n * n, t, 64);
    // the fusion lists: only each row's live entries (the scan never reads past a row's length),
    // a lane's row loads in flight together
    for (int r = t; r < n; r += 64) {
        const int L = min(fl_len[r], cap);
        const int32_t* src = fl + (size_t)r * cap;
        int* dst = fls + (size_t)r * cap;
        for (int e0 = 0; e0 < L; e0 += 8) {
            int v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = e0 + k < L ? src[e0 + k] : 0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (e0 + k < L) dst[e0 + k] = v[k];
        }
    }
    __syncthreads();
    // pose cache: claim slots with the frames record()'s disparity tests can read (the boxes'
    // init ids and list entries; one claimant per slot wins), then the winners' poses are loaded
    // (16 float4 loads per lane in flight at once)
    for (int q = t; q < NMS_PC; q += 64) ptag[q] = -1;
    __syncthreads();
    for (int r = t; r < n; r += 64) {
        ptag[iid[r] & (NMS_PC - 1)] = iid[r];
        const int L = fll[r] < cap ? fll[r] : cap;
        for (int e = 0; e < L; ++e) {
            const int f = fls[(size_t)r * cap + e];
            ptag[f & (NMS_PC - 1)] = f;
        }
    }
    __syncthreads();
    {
        float4 pv[NMS_PC / 64][4];
#pragma unroll
        for (int k = 0; k < NMS_PC / 64; ++k) {
            const int f = ptag[t + 64 * k];
#pragma unroll
            for (int c = 0; c < 4; ++c)
                pv[k][c] = f >= 0 ? reinterpret_cast<const float4*>(poses + 16 * (size_t)f)[c]
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < NMS_PC / 64; ++k)
#pragma unroll
            for (int c = 0; c < 4; ++c) reinterpret_cast<float4*>(pcache + 16 * (t + 64 * k))[c] = pv[k][c];
    }
    // order = scores.argsort()[::-1]: descending, ties -> higher index first
    for (int i = t; i < n; i += 64) {
        const float si = sc[i];
        int r = 0;
        for (int j = 0; j < n; ++j) {
            const float sj = sc[j];
            r += (sj > si) || (sj == si && j > i);
        }
        bufA[r] = i;
    }
    __syncthreads();
    int* order = bufA;
    int* rest = bufB;
    int no = n, nk = 0, ns = 0, nev = 0;           // wave-uniform counters (st: lane 0)
    int st = __any(in_over) ? BF_DEV_FUSION_LIST_OVERFLOW : 0;
    while (no > 0) {
        const int i = order[0];
        if (t == 0) keep[nk] = i;
        nk++;
        int nrest = 0, nsupp = 0;
        for (int base = 1; base < no; base += 64) {
            const int q = base + t;
            const bool live = q < no;
            const int j = order[live ? q : no - 1];
            bool fr, fs;
            if (BITS) {
                const size_t wi = (size_t)i * words + (j >> 6);
                fr = live && ((Bm[wi] >> (j & 63)) & 1ull);
                fs = live && ((Bm[(size_t)n * words + wi] >> (j & 63)) & 1ull);
            } else {
                const double v = live ? I[(size_t)i * n + j] : 0.0;
                fr = live && (v <= cfg.iou_threshold);
                fs = live && (v > cfg.iou_threshold);
            }
            const unsigned long long mr = __ballot(fr), ms = __ballot(fs);
            if (fr) rest[nrest + __popcll(mr & lanes_lt_mask())] = j;
            if (fs) supp[nsupp + __popcll(ms & lanes_lt_mask())] = j;
            nrest += __popcll(mr);
            nsupp += __popcll(ms);
        }
        __syncthreads();
        if (nsupp > 0) {
            if (t == 0) {
                vn[i] += 1.0f;
                succ[ns] = i;
            }
            ns++;
            // BoxManager.record(cur=i, fusion_inds=supp)
            const int cur = i;
            const float* ccur = cen + 3 * cur;
            for (int s = 0; s < (NMS_DIAG_NORECORD ? 0 : nsupp); ++s) {
                const int idx = supp[s];
                const float* cidx = cen + 3 * idx;
                float dx = ccur[0] - cidx[0], dy = ccur[1] - cidx[1], dz = ccur[2] - cidx[2];
                float cd = sqrtf((dx * dx + dy * dy) + dz * dz);
                int branch;
                if (fll[idx] == 1) {
                    branch = 1;
                    const int L = fll[cur];
                    const int cnt = nms_count_far(fls + (size_t)cur * cap, L, poses, ptag, pcache, iid[idx], cd, cfg);
                    if (cnt == L && L < cfg.max_list) {
                        const int32_t v = iid[idx];
                        st |= fl_append_sorted_w(fls + (size_t)cur * cap, fll + cur, cap, &v, 1);
                    }
                } else {
                    branch = 2;
                    const int L = fll[idx];
                    const int cnt = nms_count_far(fls + (size_t)idx * cap, L, poses, ptag, pcache, iid[cur], cd, cfg);
                    if (cnt == L && L < cfg.max_list) {
                        // fl[cur] += fl[idx]  (rows are distinct, cur != idx)
                        st |= fl_append_sorted_w(fls + (size_t)cur * cap, fll + cur, cap,
                                                 fls + (size_t)idx * cap, L);
                    } else {
                        keep_replace_w(keep, nk, cur, idx);
                    }
                }
                if (t == 0) {
                    events[3 * nev + 0] = cur;
                    events[3 * nev + 1] = idx;
                    events[3 * nev + 2] = branch;
                }
                nev++;
                __syncthreads();   // lane 0's LDS edits before the next suppression reads them
            }
        }
        no = nrest;
        int* tmp = order; order = rest; rest = tmp;
        if (nrest == 1) {
            if (t == 0) keep[nk] = order[0];
            nk++;
            break;
        }
    }
    __syncthreads();
    // sort keep / success (distinct indices) by rank into the outputs
    for (int q = t; q < nk; q += 64) {
        const int v = keep[q];
        int r = 0;
        for (int k = 0; k < nk; ++k) r += keep[k] < v;
        keep_out[r] = v;
    }
    for (int q = t; q < ns; q += 64) {
        const int v = succ[q];
        int r = 0;
        for (int k = 0; k < ns; ++k) r += succ[k] < v;
        succ_out[r] = v;
    }
    for (int r = t; r < n; r += 64)        // the live entries (rows only grow)
        for (int e = 0; e < fll[r]; ++e) fl[(size_t)r * cap + e] = fls[(size_t)r * cap + e];
    for (int q = t; q < n; q += 64) {
        fl_len[q] = fll[q];
        valid_num[q] = vn[q];
    }
    if (t == 0) {
        *n_keep = nk;
        *n_succ = ns;
        *n_events = nev;
        *status |= st;
    }
}

BF_API size_t bf_nms_scan_workspace_size(int n) {
    return n > 0 ? sizeof(unsigned long long) * 2 * (size_t)n * nms_words(n) : 0;
}

BF_API int bf_nms_scan(const double* iou, const float* corners, const float* scores,
                       const int32_t* init_id, const float* cam_poses, int n, int32_t* fl_items,
                       int32_t* fl_len, float* valid_num, int32_t* keep, int32_t* n_keep,
                       int32_t* success, int32_t* n_success, int32_t* events, int32_t* n_events,
                       int32_t* status, const bf_nms_cfg* cfg, void* stream) {
    return bf_nms_scan_ws(iou, corners, scores, init_id, cam_poses, n, fl_items, fl_len, valid_num, keep,
                          n_keep, success, n_success, events, n_events, status, cfg, nullptr, stream);
}

BF_API int bf_nms_scan_ws(const double* iou, const float* corners, const float* scores,
                          const int32_t* init_id, const float* cam_poses, int n, int32_t* fl_items,
                          int32_t* fl_len, float* valid_num, int32_t* keep, int32_t* n_keep,
                          int32_t* success, int32_t* n_success, int32_t* events, int32_t* n_events,
                          int32_t* status, const bf_nms_cfg* cfg, void* workspace, void* stream) {
    if (!cfg || n < 0) return BF_ERR_ARG;
    if (n > BF_MAX_BOXES) return BF_ERR_CAPACITY;
    if (n == 0) return BF_OK;
    if (!iou || !corners || !scores || !init_id || !cam_poses || !fl_items || !fl_len ||
        !valid_num || !keep || !n_keep || !success || !n_success || !events || !n_events || !status)
        return BF_ERR_ARG;
    static bool attr_w = false;
    if (!attr_w) {
        (void)hipFuncSetAttribute((const void*)k_nms_scan_w<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            NMS_FAST_LDS_MAX);
        (void)hipFuncSetAttribute((const void*)k_nms_scan_w<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            NMS_FAST_LDS_MAX);
        attr_w = true;
    }
    hipStream_t st = bf_stream(stream);
    if (n <= NMS_FAST_N && nms_fast_lds(n, cfg->list_capacity, false) <= NMS_FAST_LDS_MAX) {
        hipLaunchKernelGGL(k_nms_scan_w<false>, dim3(1), dim3(64), nms_fast_lds(n, cfg->list_capacity, false),
                           st, iou, corners, scores, init_id, cam_poses, n, fl_items, fl_len, valid_num,
                           keep, n_keep, success, n_success, events, n_events, status, *cfg, nullptr);
        return bf_check_launch();
    }
    if (workspace && NMS_FAST_N > 0 && nms_fast_lds(n, cfg->list_capacity, true) <= NMS_FAST_LDS_MAX) {
        const int words = nms_words(n);
        auto* bits = static_cast<unsigned long long*>(workspace);
        hipLaunchKernelGGL(k_nms_bits, dim3(bf_cdiv(n * words, 4)), dim3(256), 0, st, iou, n, words,
                           cfg->iou_threshold, bits);
        hipLaunchKernelGGL(k_nms_scan_w<true>, dim3(1), dim3(64), nms_fast_lds(n, cfg->list_capacity, true),
                           st, iou, corners, scores, init_id, cam_poses, n, fl_items, fl_len, valid_num,
                           keep, n_keep, success, n_success, events, n_events, status, *cfg, bits);
        return bf_check_launch();
    }
    size_t lds = sizeof(int) * (size_t)(5 * n + 8) + sizeof(float) * 3 * (size_t)n;
    if ((size_t)n * n <= NMS_IOU_LDS_MAX) lds += sizeof(double) * (size_t)n * n;
    static bool attr_set = false;
    if (!attr_set) {
        const size_t big = sizeof(int) * (5 * BF_MAX_BOXES + 8) + sizeof(float) * 3 * BF_MAX_BOXES;
        const size_t small = sizeof(double) * NMS_IOU_LDS_MAX + 32 * (size_t)NMS_IOU_LDS_N;
        hipFuncSetAttribute((const void*)k_nms_scan, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(big > small ? big : small));
        attr_set = true;
    }
    hipLaunchKernelGGL(k_nms_scan, dim3(1), dim3(SCAN_THREADS), lds, bf_stream(stream), iou,
                       corners, scores, init_id, cam_poses, n, fl_items, fl_len, valid_num, keep,
                       n_keep, success, n_success, events, n_events, status, *cfg);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// correspondence association
// ------------------------------------------------------------------------------------------
__device__ void project_2d_box(const float* c, const float* pinv, const float* K, double W,
                               double H, double* box) {
    double u[8], v[8], Z[8];
    bool any_valid = false;
    for (int q = 0; q < 8; ++q) {
        double h[4] = {c[3 * q], c[3 * q + 1], c[3 * q + 2], 1.0};
        double cam[3];
        for (int r = 0; r < 3; ++r) {
            double s = h[0] * (double)pinv[4 * r + 0];
            s = s + h[1] * (double)pinv[4 * r + 1];
            s = s + h[2] * (double)pinv[4 * r + 2];
            s = s + h[3] * (double)pinv[4 * r + 3];
            cam[r] = s;
        }
        Z[q] = cam[2];
        u[q] = ((double)K[0] * cam[0]) / cam[2] + (double)K[2];
        v[q] = ((double)K[4] * cam[1]) / cam[2] + (double)K[5];
        if (Z[q] > 0 && u[q] > 0 && u[q] < W && v[q] > 0 && v[q] < H) any_valid = true;
    }
    box[0] = box[1] = box[2] = box[3] = 0.0;
    if (!any_valid) return;
    bool have = false;
    double x1 = 0, y1 = 0, x2 = 0, y2 = 0;
    for (int q = 0; q < 8; ++q) {
        if (!(Z[q] > 0 && Z[q] < 8)) continue;
        double uu = u[q] < 0 ? 0 : (u[q] > W ? W : u[q]);
        double vv = v[q] < 0 ? 0 : (v[q] > H ? H : v[q]);
        if (!have) { x1 = x2 = uu; y1 = y2 = vv; have = true; }
        else {
            x1 = uu < x1 ? uu : x1;
            x2 = uu > x2 ? uu : x2;
            y1 = vv < y1 ? vv : y1;
            y2 = vv > y2 ? vv : y2;
        }
    }
    if (!have) return;
    box[0] = x1; box[1] = y1; box[2] = x2; box[3] = y2;
}

__device__ __forceinline__ double iou_2d(const float* a32, const double* b) {
    double ax1 = a32[0], ay1 = a32[1], ax2 = a32[2], ay2 = a32[3];
    double area_a = (ax2 - ax1) * (ay2 - ay1);
    double area_b = (b[2] - b[0]) * (b[3] - b[1]);
    double ix1 = ax1 > b[0] ? ax1 : b[0];
    double iy1 = ay1 > b[1] ? ay1 : b[1];
    double ix2 = ax2 < b[2] ? ax2 : b[2];
    double iy2 = ay2 < b[3] ? ay2 : b[3];
    double iw = ix2 - ix1; iw = iw < 0 ? 0 : iw;
    double ih = iy2 - iy1; ih = ih < 0 ? 0 : ih;
    double inter = iw * ih;
    double uni = area_a + area_b - inter;
    return inter / (uni + 1e-6);
}

__device__ int record_corr(int cur, int idx, const int32_t* init_id, const float* poses, int* keep,
                           int nk, int32_t* fl, int32_t* fl_len, const bf_corr_cfg& cfg,
                           int32_t* events, int* nev) {
    const int cap = cfg.list_capacity;
    int st = 0, branch;
    if (fl_len[idx] == 1) {
        branch = 1;
        int cnt = 0;
        const int L = min(fl_len[cur], cap);
        if (fl_len[cur] > cap) st |= BF_DEV_FUSION_LIST_OVERFLOW;
        for (int q = 0; q < L; ++q) {
            int pi = fl[(size_t)cur * cap + q];
            float b, a;
            bf_pose_disparity(poses + 16 * (size_t)pi, poses + 16 * (size_t)init_id[idx], &b, &a);
            if (a > cfg.rotation_gap || b > cfg.translation_gap) cnt++;
        }
        if (cnt == L && L < cfg.max_list) {
            int32_t v = init_id[idx];
            st |= fl_append_sorted(fl + (size_t)cur * cap, fl_len + cur, cap, &v, 1);
        }
    } else {
        branch = 2;
        int cnt = 0;
        const int L = min(fl_len[idx], cap);
        if (fl_len[idx] > cap) st |= BF_DEV_FUSION_LIST_OVERFLOW;
        for (int q = 0; q < L; ++q) {
            int pi = fl[(size_t)idx * cap + q];
            float b, a;
            bf_pose_disparity(poses + 16 * (size_t)pi, poses + 16 * (size_t)init_id[cur], &b, &a);
            if (a > cfg.rotation_gap || b > cfg.translation_gap) cnt++;
        }
        if (cnt == L && L < cfg.max_list) {
            st |= fl_append_sorted(fl + (size_t)cur * cap, fl_len + cur, cap, fl + (size_t)idx * cap, L);
        } else {
            for (int q = 0; q < nk; ++q)
                if (keep[q] == cur) keep[q] = idx;
        }
    }
    events[3 * *nev + 0] = cur;
    events[3 * *nev + 1] = idx;
    events[3 * *nev + 2] = branch;
    (*nev)++;
    return st;
}

__global__ void __launch_bounds__(SCAN_THREADS) k_corr_assoc(
    const float* __restrict__ corners, const float* __restrict__ dims,
    const float* __restrict__ scores, const float* __restrict__ boxes2d,
    const int32_t* __restrict__ init_id, const float* __restrict__ poses,
    const float* __restrict__ cur_pose, const float* __restrict__ K, int n_all, int n_glo,
    const int32_t* __restrict__ mask, int n_mask, const int32_t* __restrict__ success, int n_success,
    int32_t* __restrict__ fl, int32_t* __restrict__ fl_len, float* __restrict__ valid_num,
    int32_t* __restrict__ keep_out, int32_t* __restrict__ n_keep_out, int32_t* __restrict__ events,
    int32_t* __restrict__ n_events, int32_t* __restrict__ status, bf_corr_cfg cfg,
    const int32_t* __restrict__ n_mask_dev, const int32_t* __restrict__ n_success_dev) {
    // chained after bf_nms_scan: the mask / success counts are that kernel's device outputs
    // (n_mask is then the capacity the LDS was sized for)
    if (n_mask_dev) {
        const int nm = *n_mask_dev;
        n_mask = nm < n_mask ? nm : n_mask;
        n_success = *n_success_dev;
    }
    extern __shared__ __attribute__((aligned(16))) double dsm[];
    double* b2d = dsm;                                  // [ng][4]
    int* keep = reinterpret_cast<int*>(b2d + 4 * (size_t)(n_mask + 1));  // [n_mask]
    int* tmp = keep + n_mask + 1;                       // [n_mask]
    unsigned char* gsmall = reinterpret_cast<unsigned char*>(tmp + n_mask + 1);
    __shared__ float s_pinv[16];
    __shared__ double s_bv[SCAN_WAVES];
    __shared__ int s_bg[SCAN_WAVES];
    __shared__ int s_nk;
    const int t = threadIdx.x;
    // global_keep_idx = mask[mask < n_glo] = prefix of the sorted mask
    int ng = 0;
    for (int q = 0; q < n_mask; ++q) ng += mask[q] < n_glo;
    if (t == 0) { bf_inv4(cur_pose, s_pinv); s_nk = n_mask; }
    for (int q = t; q < n_mask; q += SCAN_THREADS) keep[q] = mask[q];
    __syncthreads();
    const float small_lim = (float)(cfg.small_size + 0.1);
    for (int g = t; g < ng; g += SCAN_THREADS) {
        int gi = mask[g];
        project_2d_box(corners + 24 * (size_t)gi, s_pinv, K, (double)cfg.W, (double)cfg.H, b2d + 4 * g);
        const float* gd = dims + 3 * (size_t)gi;
        float gm = fmaxf(fmaxf(gd[0], gd[1]), gd[2]);
        gsmall[g] = gm < small_lim ? 1 : 0;
    }
    __syncthreads();
    int nev = 0, st = 0;
    for (int q = ng; q < n_mask; ++q) {  // cur_keep_idx, ascending
        const int m = mask[q];
        const float* d = dims + 3 * (size_t)m;
        float mx = d[0];
        if (d[1] > mx) mx = d[1];
        if (d[2] > mx) mx = d[2];
        bool in_succ = false;
        for (int s = 0; s < n_success; ++s) in_succ |= (success[s] == m);
        if ((double)mx > cfg.small_size || in_succ) continue;
        if (ng == 0) continue;
        // argmax over g of iou2d * small_mask (first maximum)
        double bv = -1.0;
        int bg = 0x7fffffff;
        for (int g = t; g < ng; g += SCAN_THREADS) {
            double v = iou_2d(boxes2d + 4 * (size_t)m, b2d + 4 * g) * (gsmall[g] ? 1.0 : 0.0);
            if (v > bv || (v == bv && g < bg)) { bv = v; bg = g; }
        }
        for (int o = 32; o > 0; o >>= 1) {
            double ov = __shfl_xor(bv, o, 64);
            int og = __shfl_xor(bg, o, 64);
            if (ov > bv || (ov == bv && og < bg)) { bv = ov; bg = og; }
        }
        if (bf_lane() == 0) { s_bv[t >> 6] = bv; s_bg[t >> 6] = bg; }
        __syncthreads();
        if (t == 0) {
            bv = s_bv[0]; bg = s_bg[0];
            for (int w = 1; w < SCAN_WAVES; ++w)
                if (s_bv[w] > bv || (s_bv[w] == bv && s_bg[w] < bg)) { bv = s_bv[w]; bg = s_bg[w]; }
            if (bv > cfg.threshold) {
                const int corr = mask[bg];
                int nk = s_nk;
                if (scores[corr] < scores[m]) {
                    int w = 0;
                    for (int k = 0; k < nk; ++k)
                        if (keep[k] != corr) keep[w++] = keep[k];
                    nk = w;
                    valid_num[m] += 1.0f;
                    st |= record_corr(m, corr, init_id, poses, keep, nk, fl, fl_len, cfg, events, &nev);
                } else {
                    int w = 0;
                    for (int k = 0; k < nk; ++k)
                        if (keep[k] != m) keep[w++] = keep[k];
                    nk = w;
                    valid_num[corr] += 1.0f;
                    st |= record_corr(corr, m, init_id, poses, keep, nk, fl, fl_len, cfg, events, &nev);
                }
                s_nk = nk;
            }
        }
        __syncthreads();
    }
    const int nk = s_nk;
    // np.sort(keep_idx): values may repeat after record_corr's replacement -> rank with ties
    for (int q = t; q < nk; q += SCAN_THREADS) tmp[q] = keep[q];
    __syncthreads();
    for (int q = t; q < nk; q += SCAN_THREADS) {
        int v = tmp[q], r = 0;
        for (int k = 0; k < nk; ++k) r += (tmp[k] < v) || (tmp[k] == v && k < q);
        keep_out[r] = v;
    }
    if (t == 0) {
        *n_keep_out = nk;
        *n_events = nev;
        *status |= st;
    }
}

BF_API int bf_corr_assoc(const float* corners, const float* dims, const float* scores,
                         const float* boxes2d, const int32_t* init_id, const float* cam_poses,
                         const float* cur_pose, const float* K, int n_all, int n_glo,
                         const int32_t* mask, int n_mask, const int32_t* success, int n_success,
                         int32_t* fl_items, int32_t* fl_len, float* valid_num, int32_t* keep_out,
                         int32_t* n_keep_out, int32_t* events, int32_t* n_events, int32_t* status,
                         const bf_corr_cfg* cfg, void* stream) {
    if (!cfg || n_all < 0 || n_mask < 0 || n_success < 0) return BF_ERR_ARG;
    if (n_all > BF_MAX_BOXES || n_mask > BF_MAX_BOXES) return BF_ERR_CAPACITY;
    if (n_mask == 0) {
        return hipMemsetAsync(n_keep_out, 0, sizeof(int32_t), bf_stream(stream)) == hipSuccess
                   ? BF_OK : BF_ERR_LAUNCH;
    }
    size_t lds = sizeof(double) * 4 * (size_t)(n_mask + 1) + sizeof(int) * 2 * (size_t)(n_mask + 1) +
                 (size_t)n_mask + 16;
    hipLaunchKernelGGL(k_corr_assoc, dim3(1), dim3(SCAN_THREADS), lds, bf_stream(stream), corners,
                       dims, scores, boxes2d, init_id, cam_poses, cur_pose, K, n_all, n_glo, mask,
                       n_mask, success, n_success, fl_items, fl_len, valid_num, keep_out,
                       n_keep_out, events, n_events, status, *cfg, (const int32_t*)nullptr,
                       (const int32_t*)nullptr);
    return bf_check_launch();
}

BF_API int bf_corr_assoc_chained(const float* corners, const float* dims, const float* scores,
                                 const float* boxes2d, const int32_t* init_id,
                                 const float* cam_poses, const float* cur_pose, const float* K,
                                 int n_all, int n_glo, const int32_t* mask,
                                 const int32_t* n_mask_dev, const int32_t* success,
                                 const int32_t* n_success_dev, int32_t* fl_items, int32_t* fl_len,
                                 float* valid_num, int32_t* keep_out, int32_t* n_keep_out,
                                 int32_t* events, int32_t* n_events, int32_t* status,
                                 const bf_corr_cfg* cfg, void* stream) {
    if (!cfg || n_all < 0 || !n_mask_dev || !n_success_dev || !mask || !success) return BF_ERR_ARG;
    if (n_all > BF_MAX_BOXES) return BF_ERR_CAPACITY;
    if (n_all == 0) {
        return hipMemsetAsync(n_keep_out, 0, sizeof(int32_t), bf_stream(stream)) == hipSuccess
                   ? BF_OK : BF_ERR_LAUNCH;
    }
    const int n_mask = n_all;   // nms keep <= n_all
    size_t lds = sizeof(double) * 4 * (size_t)(n_mask + 1) + sizeof(int) * 2 * (size_t)(n_mask + 1) +
                 (size_t)n_mask + 16;
    hipLaunchKernelGGL(k_corr_assoc, dim3(1), dim3(SCAN_THREADS), lds, bf_stream(stream), corners,
                       dims, scores, boxes2d, init_id, cam_poses, cur_pose, K, n_all, n_glo, mask,
                       n_mask, success, 0, fl_items, fl_len, valid_num, keep_out, n_keep_out,
                       events, n_events, status, *cfg, n_mask_dev, n_success_dev);
    return bf_check_launch();
}
