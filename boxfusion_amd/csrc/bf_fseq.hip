// bf_fseq.hip — the keyframe state machine of demo.py:200-305 as a native sequencer.
//
// FusionStage (fusion_stage.py) drives the reference's per-keyframe sequence from Python: cat of
// the global box set, nms_3d + correspondence association (bf_nms_scan + bf_corr_assoc_chained),
// the kept-row gather, BoxFusion.boxfusion's job selection and bf_fusion_fit.  Each step is a
// few kernel launches, but the Python glue around them (Instances3D field churn, list packing,
// ctypes argument conversion) costs ~0.5 ms per keyframe.  bf_fseq runs the same sequence for a
// whole batch of keyframes in one call: the global box set (all_pred_box) lives in device tables
// owned here, BoxManager's lists (fusion_list, fusion_flag, already_fusion) in host vectors, and
// every kernel is the library's own entry point, launched in the reference's order with the
// reference's arguments, so the results are bit-identical to the Python-driven path (tests:
// test_gpu_pipeline.py runs every FusionStage test through both).
//
// One host synchronisation per keyframe remains: the association's outputs (keep lists, fusion
// lists, flag events) decide the next launches.  The deferred BoxFusion result of keyframe k is
// read back with keyframe k+1's association outputs (same wait), exactly where BoxManager.flush
// applies it in the Python path.
//
// Unlike the stateless entry points, a bf_fseq object owns device memory (stream-ordered
// hipMallocAsync, grown by doubling) and pinned host staging buffers.
#include "bf_common.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace {

// global box table (all_pred_box), field-major: xyzlhw 6 | R 9 | score 1 | box2d 4 | init_id 1 |
// valid_num 1 words per row
constexpr int GF = 6;
constexpr int GW[GF] = {6, 9, 1, 4, 1, 1};
constexpr int GROW_WORDS = 22;

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool pooled = false;     // from hipMallocAsync (stream-ordered free) or hipMalloc
};

void dev_free(DevBuf& b, hipStream_t s) {
    if (b.p) {
        if (b.pooled) hipFreeAsync(b.p, s);
        else hipFree(b.p);
    }
    b = DevBuf();
}

struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
};

struct Table {
    DevBuf mem;
    int cap = 0;     // rows
    float* field(int f) const {
        size_t off = 0;
        for (int k = 0; k < f; ++k) off += (size_t)GW[k] * cap;
        return static_cast<float*>(mem.p) + off;
    }
};

// tail rows of the global table from the per-frame rows of this keyframe (cat(all_pred_box,
// pred), demo.py:245; pred's init_id = box_count + row, valid_num = 0, demo.py:217-219), and the
// dims of every row (boxes.dims, the association kernels' contiguous [n,3] input)
__global__ void __launch_bounds__(64) k_fseq_append(const float* __restrict__ p_box,
                                                    const float* __restrict__ p_R,
                                                    const float* __restrict__ p_score,
                                                    const float* __restrict__ p_box2d, long long base,
                                                    int n_before, int n_all, float* g_box, float* g_R,
                                                    float* g_score, float* g_box2d, int32_t* g_id,
                                                    float* g_vn, float* dims) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_all) return;
    if (r >= n_before) {
        const long long s = base + (r - n_before);
        for (int k = 0; k < 6; ++k) g_box[(size_t)r * 6 + k] = p_box[s * 6 + k];
        for (int k = 0; k < 9; ++k) g_R[(size_t)r * 9 + k] = p_R[s * 9 + k];
        g_score[r] = p_score[s];
        for (int k = 0; k < 4; ++k) g_box2d[(size_t)r * 4 + k] = p_box2d[s * 4 + k];
        g_id[r] = (int32_t)s;
        g_vn[r] = 0.f;
    }
    for (int k = 0; k < 3; ++k) dims[(size_t)r * 3 + k] = g_box[(size_t)r * 6 + 3 + k];
}

}  // namespace

struct bf_fseq {
    hipStream_t stream = nullptr;
    bool inited = false;                 // all_pred_box is not None
    Table g[2];
    int cur = 0;                         // g[cur] holds all_pred_box
    int n = 0;                           // its rows
    std::vector<int32_t> ids;            // their init_id (host mirror)
    DevBuf corners, dims, iou, iou_ws, nms_ws, xch, jobs, packed, views, out_box, fit_ws;
    HostBuf h_in, h_out, h_jobs, h_fit;
    // BoxManager state (box_manager.py:9-20)
    std::vector<std::vector<int32_t>> fusion_list;
    std::vector<int32_t> fusion_flag;
    std::vector<std::vector<int32_t>> already;
    std::set<std::vector<int32_t>> already_set;
    // deferred BoxFusion result (box_fusion.py:716-724 bookkeeping)
    bool pending = false;
    std::vector<int32_t> pend_rows;
    std::vector<std::vector<int32_t>> pend_lists;
    // statistics
    long long suppressed = 0, updated_total = 0, fit_calls = 0, hull_calls = 0, assoc = 0;
    long long last_jobs = 0, last_updated = 0, last_iters = 0, last_views = 0;
    int strict_hull = 0;
    std::string err;
    // BF_FSEQ_PROFILE=1 (diagnostic): per-keyframe host / device phase times, printed every 256
    // association steps
    bool used = false;                   // a call has run (s->stream is the caller's)
    int prof = -1;
    hipEvent_t pev[6] = {};
    bool pev_prev = false;
    double pt[10] = {};
    long long pn = 0;
};

namespace {

int fail(bf_fseq* s, int code, const std::string& msg) {
    s->err = msg;
    return code;
}

int dev_reserve(bf_fseq* s, DevBuf& b, size_t bytes) {
    if (bytes <= b.cap) return BF_OK;
    size_t nc = std::max(bytes, b.cap * 2);
    nc = std::max(nc, (size_t)4096);
    void* q = nullptr;
    bool pooled = true;
    if (hipMallocAsync(&q, nc, s->stream) != hipSuccess) {      // no stream-ordered pool: plain
        (void)hipGetLastError();
        pooled = false;
        if (hipMalloc(&q, nc) != hipSuccess) return fail(s, BF_ERR_LAUNCH, "device allocation failed");
    }
    dev_free(b, s->stream);
    b.p = q;
    b.cap = nc;
    b.pooled = pooled;
    return BF_OK;
}

// Pinned staging buffers come from a process-wide pool and go back to it, never to
// hipHostFree: freeing pinned memory waits for the whole device, i.e. for every detect graph in
// flight on the other streams (measured: 70-190 ms stalls on the first steps of a fresh
// sequencer at --sim-ranks 8).  The pool is never torn down (no exit-order dependence).
struct PinnedPool {
    std::mutex m;
    std::multimap<size_t, void*> free;
};

PinnedPool& pinned_pool() {
    static PinnedPool* p = new PinnedPool();
    return *p;
}

void* pinned_get(size_t bytes, size_t* cap) {
    PinnedPool& P = pinned_pool();
    {
        std::lock_guard<std::mutex> g(P.m);
        auto it = P.free.lower_bound(bytes);
        if (it != P.free.end()) {
            void* q = it->second;
            *cap = it->first;
            P.free.erase(it);
            return q;
        }
    }
    void* q = nullptr;
    if (hipHostMalloc(&q, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    *cap = bytes;
    return q;
}

void pinned_put(void* q, size_t cap) {
    if (!q) return;
    PinnedPool& P = pinned_pool();
    std::lock_guard<std::mutex> g(P.m);
    P.free.emplace(cap, q);
}

// the stream is drained before an old buffer goes back to the pool (its copies may be in flight)
int host_reserve(bf_fseq* s, HostBuf& b, size_t bytes) {
    if (bytes <= b.cap) return BF_OK;
    size_t nc = std::max(bytes, b.cap * 2);
    nc = std::max(nc, (size_t)16384);
    if (b.p) {
        if (hipStreamSynchronize(s->stream) != hipSuccess) return fail(s, BF_ERR_LAUNCH, "stream sync failed");
        pinned_put(b.p, b.cap);
        b.p = nullptr;
        b.cap = 0;
    }
    b.p = pinned_get(nc, &b.cap);
    if (!b.p) return fail(s, BF_ERR_LAUNCH, "hipHostMalloc failed");
    return BF_OK;
}

bf_rows_field field_of(const void* a, long long n_a, const void* b, long long n_b, void* dst, int words) {
    bf_rows_field f;
    f.a = a;
    f.b = b;
    f.dst = dst;
    f.n_a = n_a;
    f.n_b = n_b;
    f.row_bytes = 4 * words;
    f.pad = 0;
    return f;
}

// rows of table `src` (n_src rows) -> table `dst`: idx (device int32) or the identity
int table_gather(bf_fseq* s, const Table& src, int n_src, Table& dst, const int32_t* idx, int n_out) {
    if (n_out == 0) return BF_OK;
    bf_rows_field f[GF];
    for (int k = 0; k < GF; ++k) f[k] = field_of(src.field(k), n_src, nullptr, 0, dst.field(k), GW[k]);
    return bf_rows_gather(f, GF, idx, 1, n_out, nullptr, s->stream);
}

int table_reserve(bf_fseq* s, int rows) {
    if (rows <= s->g[s->cur].cap) return BF_OK;
    const int cap = std::max(4096, 2 * rows);
    Table fresh;
    fresh.cap = cap;
    int rc = dev_reserve(s, fresh.mem, (size_t)cap * GROW_WORDS * 4);
    if (rc) return rc;
    rc = table_gather(s, s->g[s->cur], s->n, fresh, nullptr, s->n);    // keep the current rows
    if (rc) return fail(s, rc, "bf_rows_gather (table growth) failed");
    Table& old = s->g[s->cur];
    dev_free(old.mem, s->stream);
    old = fresh;
    Table& other = s->g[s->cur ^ 1];
    dev_free(other.mem, s->stream);
    other = Table();
    other.cap = cap;
    return dev_reserve(s, other.mem, (size_t)cap * GROW_WORDS * 4);
}

// the deferred BoxFusion result (box_fusion.py:716-724 and the status policy of
// box_fusion.py resolve()); h_fit holds the packed read-back [updated | iterations | status]
int resolve_pending(bf_fseq* s) {
    if (!s->pending) return BF_OK;
    s->pending = false;
    const int nj = (int)s->pend_rows.size();
    const int32_t* h = static_cast<const int32_t*>(s->h_fit.p);
    const int st = h[2 * nj];
    if (getenv("BF_FSEQ_DEBUG")) {
        fprintf(stderr, "fseq resolve: nj %d packed:", nj);
        for (int q = 0; q < 2 * nj + 1; ++q) fprintf(stderr, " %d", h[q]);
        fprintf(stderr, "\n");
    }
    if (st & BF_DEV_VIEW_OVERFLOW)
        return fail(s, BF_ERR_CAPACITY, "bf_fusion_fit: a fusion list has more views than the kernel holds");
    if (st & BF_DEV_INDEX_RANGE)
        return fail(s, BF_ERR_CAPACITY, "boxfusion: a fusion list names a per-frame box that does not exist");
    if (st & BF_DEV_HULL_TRUNC)
        return fail(s, BF_ERR_CAPACITY,
                    "bf_fusion_fit: more 2-D intersection candidates than the kernel holds "
                    "(BF_DEV_HULL_TRUNC): the IoU would not be exact");
    if (st & BF_DEV_HULL_OVERFLOW) {
        s->hull_calls += 1;
        if (s->strict_hull)
            return fail(s, BF_ERR_CAPACITY,
                        "bf_fusion_fit: hull capacity exceeded (BF_DEV_HULL_OVERFLOW): the reference "
                        "kernel overruns its fixed buffers on this input");
    }
    long long upd = 0, iters = 0;
    for (int j = 0; j < nj; ++j) {
        iters += h[nj + j];
        if (!h[j]) continue;
        ++upd;
        const int row = s->pend_rows[j];
        if (row >= 0 && row < (int)s->fusion_flag.size()) s->fusion_flag[row] = 1;   // update_fusion_flag
        s->already.push_back(s->pend_lists[j]);                                       // add_fusion_ind
        s->already_set.insert(s->pend_lists[j]);
    }
    s->last_updated = upd;
    s->last_iters = iters;
    s->updated_total += upd;
    return BF_OK;
}

// replay_flags (box_manager.py:85-86, 126-127): fusion_flag propagation of branch-2 events
void replay(bf_fseq* s, const int32_t* ev, int n_ev) {
    for (int e = 0; e < n_ev; ++e) {
        const int cur = ev[3 * e], idx = ev[3 * e + 1], branch = ev[3 * e + 2];
        if (branch == 2 && idx < (int)s->fusion_flag.size() && s->fusion_flag[idx] == 1)
            s->fusion_flag[cur] = 1;
    }
}

struct PerFrame {
    const float *box, *R, *score, *box2d, *pose, *proj;
    long long rows;
};

// BoxFusion.boxfusion (box_fusion.py:622-724 selection; bf_fusion_fit + write-back on the device)
int boxfusion(bf_fseq* s, const PerFrame& P, const bf_fuse_cfg* fuse, const float* pst) {
    std::vector<int32_t> rows;
    std::vector<const std::vector<int32_t>*> lists;
    std::set<std::vector<int32_t>> seen;
    const int lim = std::min((int)s->fusion_list.size(), s->n);
    for (int i = 0; i < lim; ++i) {
        const std::vector<int32_t>& fl = s->fusion_list[i];
        if (fl.size() < 3 || s->already_set.count(fl) || seen.count(fl)) continue;
        seen.insert(fl);
        rows.push_back(i);
        lists.push_back(&fl);
    }
    const int nj = (int)rows.size();
    long long V = 0;
    int maxv = 1;
    for (auto* l : lists) {
        V += (long long)l->size();
        maxv = std::max(maxv, (int)l->size());
    }
    s->last_jobs = nj;
    s->last_views = V;
    s->last_updated = 0;
    s->last_iters = 0;
    if (nj == 0) return BF_OK;
    s->fit_calls += 1;
    maxv = std::min(maxv, 32);
    // one upload: view offsets | view counts | target rows | flattened view indices
    const size_t words = 3 * (size_t)nj + (size_t)V;
    int rc = host_reserve(s, s->h_jobs, words * 4);
    if (!rc) rc = dev_reserve(s, s->jobs, words * 4);
    if (!rc) rc = dev_reserve(s, s->packed, (2 * (size_t)nj + 1) * 4);
    if (!rc) rc = dev_reserve(s, s->views, (size_t)V * 48 * 4);
    if (!rc) rc = dev_reserve(s, s->out_box, (size_t)nj * 6 * 4);
    const size_t ws = bf_fusion_fit_workspace_size(nj, maxv, fuse->pst_size);
    if (!rc) rc = dev_reserve(s, s->fit_ws, std::max(ws, (size_t)256));
    if (!rc) rc = host_reserve(s, s->h_fit, (2 * (size_t)nj + 1) * 4);
    if (rc) return rc;
    int32_t* h = static_cast<int32_t*>(s->h_jobs.p);
    int32_t off = 0;
    for (int j = 0; j < nj; ++j) {
        h[j] = off;
        h[nj + j] = (int32_t)lists[j]->size();
        h[2 * nj + j] = rows[j];
        std::memcpy(h + 3 * nj + off, lists[j]->data(), lists[j]->size() * 4);
        off += (int32_t)lists[j]->size();
    }
    int32_t* d = static_cast<int32_t*>(s->jobs.p);
    int32_t* packed = static_cast<int32_t*>(s->packed.p);
    if (getenv("BF_FSEQ_DEBUG")) {
        fprintf(stderr, "fseq fit: nj %d V %lld maxv %d iters %d pst %d legacy %d K0 %f h:", nj, V, maxv,
                fuse->iters, fuse->pst_size, fuse->legacy_promotion, fuse->K[0]);
        for (size_t q = 0; q < words; ++q) fprintf(stderr, " %d", h[q]);
        fprintf(stderr, "\n");
    }
    if (hipMemcpyAsync(d, h, words * 4, hipMemcpyHostToDevice, s->stream) != hipSuccess ||
        hipMemsetAsync(packed, 0, (2 * (size_t)nj + 1) * 4, s->stream) != hipSuccess)
        return fail(s, BF_ERR_LAUNCH, "boxfusion upload failed");
    // every view's box, rotation, score, pose and 2-D hull in one gather (status: packed[2nj])
    float* vb = static_cast<float*>(s->views.p);
    float* vr = vb + (size_t)V * 6;
    float* vs = vr + (size_t)V * 9;
    float* vp = vs + (size_t)V;
    float* vt = vp + (size_t)V * 16;
    bf_rows_field f[5] = {field_of(P.box, P.rows, nullptr, 0, vb, 6), field_of(P.R, P.rows, nullptr, 0, vr, 9),
                          field_of(P.score, P.rows, nullptr, 0, vs, 1),
                          field_of(P.pose, P.rows, nullptr, 0, vp, 16),
                          field_of(P.proj, P.rows, nullptr, 0, vt, 16)};
    rc = bf_rows_gather(f, 5, d + 3 * nj, 1, (int)V, packed + 2 * nj, s->stream);
    if (rc) return fail(s, rc, "bf_rows_gather (fusion views) failed");
    float* ob = static_cast<float*>(s->out_box.p);
    rc = bf_fusion_fit(d, d + nj, nj, maxv, vb, vr, vs, vp, vt, pst, fuse, ob, packed, packed + nj,
                       nullptr, packed + 2 * nj, s->fit_ws.p, s->stream);
    if (rc) return fail(s, rc, "bf_fusion_fit failed");
    rc = bf_fusion_writeback(ob, packed, d + 2 * nj, nj, s->g[s->cur].field(0), 6, s->stream);
    if (rc) return fail(s, rc, "bf_fusion_writeback failed");
    if (hipMemcpyAsync(s->h_fit.p, packed, (2 * (size_t)nj + 1) * 4, hipMemcpyDeviceToHost, s->stream) !=
        hipSuccess)
        return fail(s, BF_ERR_LAUNCH, "boxfusion read-back failed");
    s->pending = true;
    s->pend_rows = rows;
    s->pend_lists.clear();
    for (auto* l : lists) s->pend_lists.push_back(*l);
    return BF_OK;
}

double now_us() {
    return 1e-3 * (double)std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now().time_since_epoch()).count();
}

void prof_mark(bf_fseq* s, int k) {
    if (s->prof > 0) hipEventRecord(s->pev[k], s->stream);
}

// after the association read-back: device phases of this keyframe (events 0-3), the device gap
// since the previous keyframe's last launch (event 5 -> 0)
void prof_collect(bf_fseq* s, double t_entry, double t_sync0, double t_sync1) {
    float ms[5] = {};
    for (int k = 0; k < 3; ++k) hipEventElapsedTime(&ms[k], s->pev[k], s->pev[k + 1]);
    if (s->pev_prev) {
        hipEventElapsedTime(&ms[3], s->pev[5], s->pev[0]);
        hipEventElapsedTime(&ms[4], s->pev[4], s->pev[5]);
    }
    s->pt[0] += t_sync0 - t_entry;                 // host: prework + enqueue
    s->pt[1] += t_sync1 - t_sync0;                 // host: wait in hipStreamSynchronize
    s->pt[2] += 1e3 * ms[0];                       // device: append .. obb matrix
    s->pt[3] += 1e3 * ms[1];                       // device: nms scan
    s->pt[4] += 1e3 * ms[2];                       // device: corr assoc + read-back
    s->pt[5] += 1e3 * ms[3];                       // device: previous keyframe's tail -> this start
    s->pt[7] += 1e3 * ms[4];                       // device: previous keyframe's gather + fit
    s->pn += 1;
    if (s->pn % 256 == 0)
        fprintf(stderr, "fseq profile (%lld kf, us/kf): host pre %.1f wait %.1f post %.1f | dev obb %.1f nms %.1f "
                "corr+rb %.1f fit %.1f gap %.1f\n", s->pn, s->pt[0] / s->pn, s->pt[1] / s->pn, s->pt[6] / s->pn,
                s->pt[2] / s->pn, s->pt[3] / s->pn, s->pt[4] / s->pn, s->pt[7] / s->pn, s->pt[5] / s->pn);
}

// one keyframe with n > 0 boxes at per-frame rows [base, base + n)
int keyframe(bf_fseq* s, const bf_fseq_cfg* cfg, const PerFrame& P, long long base, int n,
             const float* K, const float* pst) {
    if (!s->inited) {        // first keyframe: all_pred_box = pred (demo.py:226-241)
        int rc = table_reserve(s, n);
        if (!rc) rc = dev_reserve(s, s->dims, (size_t)std::max(n, 1) * 12);
        if (rc) return rc;
        Table& G = s->g[s->cur];
        hipLaunchKernelGGL(k_fseq_append, dim3(bf_cdiv(n, 64)), dim3(64), 0, s->stream, P.box, P.R,
                           P.score, P.box2d, base, 0, n, G.field(0), G.field(1), G.field(2), G.field(3),
                           reinterpret_cast<int32_t*>(G.field(4)), G.field(5),
                           static_cast<float*>(s->dims.p));
        if (bf_check_launch()) return fail(s, BF_ERR_LAUNCH, "k_fseq_append failed");
        s->n = n;
        s->ids.resize(n);
        for (int i = 0; i < n; ++i) {
            s->ids[i] = (int32_t)(base + i);
            s->fusion_list.push_back({i});          // init_new_predictions(n, 0)
            s->fusion_flag.push_back(0);
        }
        s->inited = true;
        return BF_OK;
    }
    // init_new_predictions(n, len(per_frame_ins)) (demo.py:244)
    for (int i = 0; i < n; ++i) {
        s->fusion_list.push_back({(int32_t)(base + i)});
        s->fusion_flag.push_back(0);
    }
    if (s->prof < 0) {
        const char* e = getenv("BF_FSEQ_PROFILE");
        s->prof = e && atoi(e) > 0;
        if (s->prof > 0)
            for (hipEvent_t& ev : s->pev) hipEventCreate(&ev);
    }
    const double t_entry = s->prof > 0 ? now_us() : 0.0;
    const int n_glo = s->n, n_all = s->n + n;
    if (n_all > BF_MAX_BOXES) return fail(s, BF_ERR_CAPACITY, "more global boxes than BF_MAX_BOXES");
    if ((int)s->fusion_list.size() != n_all)
        return fail(s, BF_ERR_ARG, "fusion_list rows differ from all_pred_box rows");
    const int cap = cfg->nms.list_capacity;
    const size_t x_words = (size_t)n_all * cap + n_all + 7 + 9 * ((size_t)n_all + 1);
    const size_t in_words = (size_t)n_all * cap + n_all + 7;
    int rc = table_reserve(s, n_all);
    if (!rc) rc = dev_reserve(s, s->dims, (size_t)n_all * 12);
    if (!rc) rc = dev_reserve(s, s->corners, (size_t)n_all * 96);
    if (!rc) rc = dev_reserve(s, s->iou, (size_t)n_all * n_all * 8);
    if (!rc) rc = dev_reserve(s, s->iou_ws, std::max(bf_obb_iou_workspace_size(n_all), (size_t)256));
    if (!rc) rc = dev_reserve(s, s->nms_ws, std::max(bf_nms_scan_workspace_size(n_all), (size_t)256));
    if (!rc) rc = dev_reserve(s, s->xch, x_words * 4);
    if (!rc) rc = host_reserve(s, s->h_in, in_words * 4);
    if (!rc) rc = host_reserve(s, s->h_out, x_words * 4);
    if (rc) return rc;
    Table& G = s->g[s->cur];
    prof_mark(s, 0);
    // cat(all_pred_box, pred) + dims
    hipLaunchKernelGGL(k_fseq_append, dim3(bf_cdiv(n_all, 64)), dim3(64), 0, s->stream, P.box, P.R,
                       P.score, P.box2d, base, n_glo, n_all, G.field(0), G.field(1), G.field(2),
                       G.field(3), reinterpret_cast<int32_t*>(G.field(4)), G.field(5),
                       static_cast<float*>(s->dims.p));
    if (bf_check_launch()) return fail(s, BF_ERR_LAUNCH, "k_fseq_append failed");
    float* corners = static_cast<float*>(s->corners.p);
    rc = bf_box_corners(G.field(0), G.field(1), n_all, corners, s->stream);
    if (!rc) rc = bf_obb_iou_matrix(corners, n_all, static_cast<double*>(s->iou.p), s->iou_ws.p, s->stream);
    if (rc) return fail(s, rc, "corners / obb iou failed");
    prof_mark(s, 1);
    // fusion lists in (BoxManager.pack_host), counts zeroed
    int32_t* hi = static_cast<int32_t*>(s->h_in.p);
    for (int i = 0; i < n_all; ++i) {
        const std::vector<int32_t>& fl = s->fusion_list[i];
        if ((int)fl.size() > cap) {
            char m[160];
            snprintf(m, sizeof m, "fusion list of %d > capacity %d; raise box_fusion.list_capacity",
                     (int)fl.size(), cap);
            return fail(s, BF_ERR_CAPACITY, m);
        }
        int32_t* row = hi + (size_t)i * cap;
        std::memcpy(row, fl.data(), fl.size() * 4);
        for (int k = (int)fl.size(); k < cap; ++k) row[k] = -1;
        hi[(size_t)n_all * cap + i] = (int32_t)fl.size();
    }
    std::memset(hi + (size_t)n_all * cap + n_all, 0, 7 * 4);
    int32_t* X = static_cast<int32_t*>(s->xch.p);
    if (hipMemcpyAsync(X, hi, in_words * 4, hipMemcpyHostToDevice, s->stream) != hipSuccess)
        return fail(s, BF_ERR_LAUNCH, "list upload failed");
    int32_t* items = X;
    int32_t* lens = items + (size_t)n_all * cap;
    int32_t* counts = lens + n_all;          // n_keep, n_success, n_events, status
    int32_t* ccounts = counts + 4;           // n_keep, n_events, status
    int32_t* keep = ccounts + 3;
    int32_t* succ = keep + n_all + 1;
    int32_t* events = succ + n_all + 1;
    int32_t* ckeep = events + 3 * (n_all + 1);
    int32_t* cevents = ckeep + n_all + 1;
    const int32_t* gid = reinterpret_cast<const int32_t*>(G.field(4));
    rc = bf_nms_scan_ws(static_cast<double*>(s->iou.p), corners, G.field(2), gid, P.pose, n_all, items, lens,
                        G.field(5), keep, counts, succ, counts + 1, events, counts + 2, counts + 3, &cfg->nms,
                        s->nms_ws.p, s->stream);
    if (rc) return fail(s, rc, "bf_nms_scan failed");
    prof_mark(s, 2);
    rc = bf_corr_assoc_chained(corners, static_cast<float*>(s->dims.p), G.field(2), G.field(3), gid, P.pose,
                               P.pose + (size_t)base * 16, K, n_all, n_glo, keep, counts, succ, counts + 1,
                               items, lens, G.field(5), ckeep, ccounts, cevents, ccounts + 1, ccounts + 2,
                               &cfg->corr, s->stream);
    if (rc) return fail(s, rc, "bf_corr_assoc_chained failed");
    if (hipMemcpyAsync(s->h_out.p, X, x_words * 4, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
        return fail(s, BF_ERR_LAUNCH, "association read-back failed");
    prof_mark(s, 3);
    const double t_sync0 = s->prof > 0 ? now_us() : 0.0;
    if (hipStreamSynchronize(s->stream) != hipSuccess) return fail(s, BF_ERR_LAUNCH, "association read-back failed");
    if (s->prof > 0) prof_collect(s, t_entry, t_sync0, now_us());
    const double t_post = s->prof > 0 ? now_us() : 0.0;
    s->assoc += 1;
    const int32_t* ho = static_cast<const int32_t*>(s->h_out.p);
    const int32_t* h_items = ho;
    const int32_t* h_lens = h_items + (size_t)n_all * cap;
    const int32_t* hc = h_lens + n_all;
    const int32_t* hcc = hc + 4;
    const int32_t* h_keep = hcc + 3;
    const int32_t* h_ev = h_keep + 2 * (n_all + 1);
    const int32_t* h_ckeep = h_ev + 3 * (n_all + 1);
    const int32_t* h_cev = h_ckeep + n_all + 1;
    if (hc[3]) {
        char m[96];
        snprintf(m, sizeof m, "bf_nms_scan device status %d (fusion list capacity)", hc[3]);
        return fail(s, BF_ERR_CAPACITY, m);
    }
    if (hcc[2]) {
        char m[96];
        snprintf(m, sizeof m, "bf_corr_assoc device status %d (fusion list capacity)", hcc[2]);
        return fail(s, BF_ERR_CAPACITY, m);
    }
    // unpack_host, then the previous keyframe's fusion result (BoxManager.flush at the first
    // flag read), then the NMS and correspondence events in that order
    for (int i = 0; i < n_all; ++i)
        s->fusion_list[i].assign(h_items + (size_t)i * cap, h_items + (size_t)i * cap + h_lens[i]);
    rc = resolve_pending(s);
    if (rc) return rc;
    replay(s, h_ev, hc[2]);
    replay(s, h_cev, hcc[1]);
    const int n_mask = hc[0];
    bool any_cur = false;
    for (int q = 0; q < n_mask; ++q) any_cur = any_cur || h_keep[q] >= n_glo;
    const int32_t* kidx = any_cur ? h_ckeep : h_keep;
    const int n_keep = any_cur ? hcc[0] : n_mask;
    const int32_t* kdev = any_cur ? ckeep : keep;
    // all_pred_box[keep_idx] (device), BoxManager.update(keep_idx) and the init_id mirror
    Table& D = s->g[s->cur ^ 1];
    rc = table_gather(s, G, n_all, D, kdev, n_keep);
    if (rc) return fail(s, rc, "bf_rows_gather (kept rows) failed");
    s->cur ^= 1;
    std::vector<std::vector<int32_t>> fl(n_keep);
    std::vector<int32_t> ids(n_keep);
    for (int q = 0; q < n_keep; ++q) {
        const int r = kidx[q];
        if (r < 0 || r >= n_all) return fail(s, BF_ERR_CAPACITY, "kept row out of range");
        fl[q].swap(s->fusion_list[r]);
        ids[q] = r < n_glo ? s->ids[r] : (int32_t)(base + (r - n_glo));
    }
    s->fusion_list.swap(fl);
    s->ids.swap(ids);
    s->n = n_keep;
    s->suppressed += hc[1];
    prof_mark(s, 4);
    if (any_cur && cfg->use_fusion) rc = boxfusion(s, P, &cfg->fuse, pst);
    if (s->prof > 0) {
        prof_mark(s, 5);
        s->pev_prev = true;
        s->pt[6] += now_us() - t_post;             // host: unpack, gather, fit selection + enqueue
    }
    return rc;
}

}  // namespace

BF_API int bf_fseq_create(bf_fseq** out) {
    if (!out) return BF_ERR_ARG;
    // keep the stream-ordered pool's memory across synchronisations (a sequencer's buffers are
    // regrown by doubling; the default threshold 0 returns them to the driver at every sync)
    int dev = 0;
    hipMemPool_t mp;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetDefaultMemPool(&mp, dev) == hipSuccess) {
        uint64_t th = UINT64_MAX;
        (void)hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &th);
    }
    (void)hipGetLastError();
    *out = new bf_fseq();
    return BF_OK;
}

BF_API void bf_fseq_destroy(bf_fseq* s) {
    if (!s) return;
    if (s->used) hipStreamSynchronize(s->stream);
    for (Table& t : s->g) dev_free(t.mem, s->stream);
    for (DevBuf* b : {&s->corners, &s->dims, &s->iou, &s->iou_ws, &s->nms_ws, &s->xch, &s->jobs, &s->packed, &s->views,
                      &s->out_box, &s->fit_ws})
        dev_free(*b, s->stream);
    if (s->used) hipStreamSynchronize(s->stream);
    if (s->prof > 0)
        for (hipEvent_t ev : s->pev) hipEventDestroy(ev);
    for (HostBuf* b : {&s->h_in, &s->h_out, &s->h_jobs, &s->h_fit}) pinned_put(b->p, b->cap);
    delete s;
}

BF_API const char* bf_fseq_error(const bf_fseq* s) { return s ? s->err.c_str() : "null bf_fseq"; }

static int use_stream(bf_fseq* s, void* stream) {
    hipStream_t st = bf_stream(stream);
    // earlier work (and frees) on the old stream.  Not before the first call: the initial stream
    // is the null stream, and waiting on it waits for every blocking stream of the process (the
    // detect streams' graphs: a 90 ms stall on a fresh sequencer's first call at --sim-ranks 8)
    if (s->used && s->stream != st) {
        if (hipStreamSynchronize(s->stream) != hipSuccess) return fail(s, BF_ERR_LAUNCH, "stream sync failed");
    }
    s->stream = st;
    s->used = true;
    return BF_OK;
}

BF_API int bf_fseq_keyframes(bf_fseq* s, const bf_fseq_cfg* cfg, int n_kf, const int32_t* sizes,
                             int64_t p_base, int64_t p_rows, const float* p_box, const float* p_R,
                             const float* p_score, const float* p_box2d, const float* p_pose,
                             const float* p_proj, const float* K, const float* pst, void* stream) {
    if (!s || !cfg || n_kf < 0 || (n_kf && !sizes) || p_base < 0 || p_rows < 0) return BF_ERR_ARG;
    int rc = use_stream(s, stream);
    if (rc) return rc;
    s->strict_hull = cfg->strict_hull;
    long long need = p_base;
    for (int j = 0; j < n_kf; ++j) {
        if (sizes[j] < 0) return fail(s, BF_ERR_ARG, "negative keyframe size");
        need += sizes[j];
    }
    if (need > p_rows) return fail(s, BF_ERR_ARG, "keyframe rows beyond the per-frame table");
    if (need > p_base && (!p_box || !p_R || !p_score || !p_box2d || !p_pose || !p_proj || !K || !pst))
        return fail(s, BF_ERR_ARG, "null per-frame field");
    if (cfg->nms.list_capacity != cfg->corr.list_capacity || cfg->nms.list_capacity <= 0)
        return fail(s, BF_ERR_ARG, "list capacities differ");
    const PerFrame P{p_box, p_R, p_score, p_box2d, p_pose, p_proj, p_rows};
    const bool prof_call = s->prof > 0;
    const double t_call = prof_call ? now_us() : 0.0;
    long long base = p_base;
    for (int j = 0; j < n_kf; ++j) {
        const int n = sizes[j];
        if (n == 0) continue;             // demo.py: no boxes -> only num_record (host side)
        rc = keyframe(s, cfg, P, base, n, K, pst);
        if (rc) return rc;
        base += n;
    }
    if (prof_call) {
        s->pt[8] += now_us() - t_call;
        s->pt[9] += 1;
        fprintf(stderr, "fseq call: %d keyframes %.1f us (calls so far %.0f, mean %.1f us)\n", n_kf,
                now_us() - t_call, s->pt[9], s->pt[8] / s->pt[9]);
    }
    return BF_OK;
}

BF_API int bf_fseq_sync(bf_fseq* s) {
    if (!s) return BF_ERR_ARG;
    // (stream may be the null stream: torch's default stream)
    if (s->used && hipStreamSynchronize(s->stream) != hipSuccess)
        return fail(s, BF_ERR_LAUNCH, "stream sync failed");
    return resolve_pending(s);
}

BF_API int bf_fseq_state(bf_fseq* s, int64_t* out) {
    if (!s || !out) return BF_ERR_ARG;
    int rc = bf_fseq_sync(s);
    if (rc) return rc;
    long long fl_items = 0, af_items = 0;
    for (auto& r : s->fusion_list) fl_items += (long long)r.size();
    for (auto& r : s->already) af_items += (long long)r.size();
    const int64_t v[BF_FSEQ_STATE_N] = {s->inited ? s->n : -1, (int64_t)s->fusion_list.size(), fl_items,
                                        (int64_t)s->fusion_flag.size(), (int64_t)s->already.size(), af_items,
                                        s->suppressed, s->updated_total, s->fit_calls, s->hull_calls,
                                        s->last_jobs, s->last_updated, s->last_iters, s->last_views, s->assoc, 0};
    std::memcpy(out, v, sizeof v);
    return BF_OK;
}

BF_API int bf_fseq_lists(bf_fseq* s, int which, int32_t* lens, int32_t* items) {
    if (!s || (which != 0 && which != 1)) return BF_ERR_ARG;
    const auto& L = which == 0 ? s->fusion_list : s->already;
    size_t o = 0;
    for (size_t i = 0; i < L.size(); ++i) {
        if (lens) lens[i] = (int32_t)L[i].size();
        if (items) std::memcpy(items + o, L[i].data(), L[i].size() * 4);
        o += L[i].size();
    }
    return BF_OK;
}

BF_API int bf_fseq_flags(bf_fseq* s, int32_t* flags) {
    if (!s || !flags) return BF_ERR_ARG;
    std::memcpy(flags, s->fusion_flag.data(), s->fusion_flag.size() * 4);
    return BF_OK;
}

BF_API int bf_fseq_global(bf_fseq* s, int32_t* init_id, float* xyzlhw, float* valid_num, void* stream) {
    if (!s) return BF_ERR_ARG;
    int rc = bf_fseq_sync(s);
    if (rc) return rc;
    if (!s->inited || s->n == 0) return BF_OK;
    if (init_id) std::memcpy(init_id, s->ids.data(), (size_t)s->n * 4);
    const Table& G = s->g[s->cur];
    hipStream_t st = bf_stream(stream);
    if ((xyzlhw && hipMemcpyAsync(xyzlhw, G.field(0), (size_t)s->n * 24, hipMemcpyDeviceToDevice, st) != hipSuccess) ||
        (valid_num && hipMemcpyAsync(valid_num, G.field(5), (size_t)s->n * 4, hipMemcpyDeviceToDevice, st) != hipSuccess))
        return fail(s, BF_ERR_LAUNCH, "global row export failed");
    return BF_OK;
}
