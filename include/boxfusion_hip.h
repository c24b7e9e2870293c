/*
 * boxfusion_hip.h — C-ABI of libboxfusion_hip.so, the MI355X (gfx950) hot path of
 * BoxFusion's per-frame detect + multi-view 3D box fusion.
 *
 * Conventions (every entry point):
 *   - All data pointers are CALLER-OWNED DEVICE pointers (e.g. torch tensors' data_ptr()),
 *     contiguous, with the dtype named in the signature.  Nothing here allocates device memory
 *     (except the keyframe sequencer bf_fseq_*, which owns its rows: see its section).
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default stream).
 *   - Every call is asynchronous on `stream` and returns a bf_status (0 = ok, < 0 = error).
 *     Device-side capacity problems are reported through an int32 device status word where the
 *     signature has one (BF_DEV_* flags); the caller reads it after synchronising.
 *   - Functions keep no process-wide state (per-call options travel in caller-owned structs such
 *     as bf_gemm_plan) and are reentrant; concurrent calls on different streams are safe.  The
 *     one stateful object is a bf_fseq sequencer, owned by its caller.
 *
 * Each function cites the reference interface it replaces (paths relative to the reference
 * repository pliam1105/BoxFusion).
 */
#ifndef BOXFUSION_HIP_H
#define BOXFUSION_HIP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    BF_OK = 0,
    BF_ERR_ARG = -1,       /* bad size / null pointer */
    BF_ERR_LAUNCH = -2,    /* hipLaunchKernel / hipGetLastError failure */
    BF_ERR_CAPACITY = -3,  /* host-detectable capacity overflow (e.g. n > BF_MAX_BOXES) */
    BF_ERR_UNSUPPORTED = -4
} bf_status;

/* device status word flags (OR-ed) */
#define BF_DEV_OK 0
#define BF_DEV_FUSION_LIST_OVERFLOW 1   /* a fusion_list row exceeded its capacity */
#define BF_DEV_HULL_OVERFLOW 2          /* a 2-D hull / clip buffer exceeded its capacity */
#define BF_DEV_VIEW_OVERFLOW 4          /* a fusion job has 0 or more than 32 views (skipped) */
#define BF_DEV_INDEX_RANGE 8            /* a gather index outside its source rows (row skipped) */
#define BF_DEV_HULL_TRUNC 16            /* more 2-D intersection candidates than the fitness kernel
                                           holds (64): candidates dropped, the IoU is not exact */

#define BF_MAX_BOXES 4096               /* NMS / association scan limit per call */

/* ------------------------------------------------------------------------------------------
 * Library identity
 * ------------------------------------------------------------------------------------------ */
const char* bf_version(void);
/* returns the number of HIP devices visible (>= 0) or a negative bf_status */
int bf_device_count(void);

/* ------------------------------------------------------------------------------------------
 * Row gather over the fields of a box set (Instances3D.cat / Instances3D.__getitem__,
 * instances.py:155-218 of the reference, one torch.cat / index per field there): every field is
 * a row-major table whose rows are `row_bytes` bytes (a multiple of 4); rows come from the
 * virtual concatenation [a (n_a rows); b (n_b rows)], dst row r = row idx[r] of it (idx == NULL:
 * r itself, i.e. the concatenation; idx is int32 when idx_i32 != 0, else int64).  One launch for all fields.  idx values must lie in
 * [0, n_a + n_b) (checked on the device: out-of-range rows are left unwritten and set
 * BF_DEV_INDEX_RANGE in *status when status != NULL).
 * ------------------------------------------------------------------------------------------ */
#define BF_ROWS_MAX_FIELDS 16
typedef struct {
    const void* a;
    const void* b;           /* may be NULL when n_b == 0 */
    void* dst;
    int64_t n_a, n_b;
    int32_t row_bytes;       /* bytes of a SOURCE row */
    int32_t pad;             /* 0: copy; 1: int64 source -> int32 output (row_bytes % 8 == 0) */
} bf_rows_field;

int bf_rows_gather(const bf_rows_field* fields, int n_fields, const void* idx, int idx_i32,
                   int n_out, int32_t* status, void* stream);

/* ------------------------------------------------------------------------------------------
 * 3-D box geometry  (boxfusion/boxes.py, boxfusion/instances.py)
 * ------------------------------------------------------------------------------------------ */

/* GeneralInstance3DBoxes.corners (boxes.py:725-778).
 * xyzlhw f32[n,6], R f32[n,3,3] -> corners f32[n,8,3] in the reference's v0..v7 order. */
int bf_box_corners(const float* xyzlhw, const float* R, int n, float* corners, void* stream);

/* GeneralInstance3DBoxes.transform2world (boxes.py:825-833), in place.
 * xyz <- Rc*xyz + tc, R <- Rc*R with cam_pose f32[n,4,4] (camera->world). */
int bf_box_transform2world(float* xyzlhw, float* R, const float* cam_pose, int n, void* stream);

/* Instances3D.project_3d_boxes (instances.py:333-369):
 * corners f32[n,8,3], cam_pose f32[n,4,4], K f32[3,3] -> uv f32[n,8,2], clamped to [0,W]x[0,H]
 * (no Z>0 guard, as in the reference). */
int bf_project_boxes(const float* corners, const float* cam_pose, const float* K, int n,
                     float W, float H, float* uv, void* stream);

/* Detection filters of demo.py:138-148 (BoxManager.check_uv_bounds / check_floor_mask /
 * check_large_mask, box_manager.py:217-245, and the score threshold) over n instances:
 * scores f32[n], proj_xy f32[n,2], box3d f32[n,6] (xyz lhw) -> keep u8[n]; bits u8[n] (may be
 * NULL): 2 = score >= thr, 4 = uv inside, 8 = floor mask, 16 = large mask.  Thresholds are the
 * f32 values torch compares with; gap_w / gap_h = int((1 - ratio) * W / H) as in the reference
 * (63 / 47 at 640 x 480, ratio 0.9). */
typedef struct {
    float score_thresh;
    float floor_ratio, floor_half;   /* ratio and ratio / 2 */
    float size_max;
    int32_t gap_w, gap_h, W, H;
    int32_t use_score, use_uv, use_floor, use_large;
} bf_filter_cfg;
int bf_detection_filter(const float* scores, const float* proj_xy, const float* box3d, int n,
                        const bf_filter_cfg* cfg, uint8_t* keep, uint8_t* bits, void* stream);

/* Sampled 3-D OBB IoU of every pair (instances.py:493-613, Instances3D.obb_iou):
 * vertex/edge-midpoint gate against the 12 hull facets (eps 1e-6), then a 25^3 linspace grid over
 * the union AABB.  corners f32[n,8,3] -> iou f64[n,n] (symmetric, diagonal = 1).
 * `workspace` must hold bf_obb_iou_workspace_size(n) bytes. */
size_t bf_obb_iou_workspace_size(int n);
int bf_obb_iou_matrix(const float* corners, int n, double* iou, void* workspace, void* stream);

/* ------------------------------------------------------------------------------------------
 * Spatial association: greedy 3-D NMS with fusion-list bookkeeping
 *   nms_3d (instances.py:22-101) + BoxManager.record (box_manager.py:40-88)
 *   + compute_pose_center_disparity (box_manager.py:188-215)
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    double iou_threshold;    /* cfg box_fusion.nms_threshold (compared with f64 IoU) */
    float translation_gap;   /* cfg association.translation_gap (metres, compared in f32) */
    float rotation_gap;      /* cfg association.rotation_gap (degrees, compared in f32) */
    double center_gap;       /* 0.5 m (box_manager.py:55) */
    int   max_list;          /* 5: a fusion list only grows while shorter than this */
    int   list_capacity;     /* row stride (capacity) of fl_items */
} bf_nms_cfg;

/* One greedy scan over n boxes of all_pred_box.
 *   iou        f64[n,n]  from bf_obb_iou_matrix
 *   corners    f32[n,8,3] (box centres = mean of the 8 corners, as nms_3d:49)
 *   scores     f32[n];  init_id i32[n];  cam_poses f32[M,4,4] indexed by init_id
 *   fl_items   i32[n,cap] / fl_len i32[n]: BoxManager.fusion_list rows (in/out)
 *   valid_num  f32[n] (in/out, +1 for every box that suppressed something)
 * outputs (device): keep i32[n] sorted ascending, n_keep i32[1], success i32[n] sorted, n_success
 *   i32[1], events i32[n,3] = (cur, idx, branch) in scan order, n_events i32[1],
 *   status i32[1] (BF_DEV_* flags). */
int bf_nms_scan(const double* iou, const float* corners, const float* scores,
                const int32_t* init_id, const float* cam_poses, int n,
                int32_t* fl_items, int32_t* fl_len, float* valid_num,
                int32_t* keep, int32_t* n_keep, int32_t* success, int32_t* n_success,
                int32_t* events, int32_t* n_events, int32_t* status,
                const bf_nms_cfg* cfg, void* stream);

/* bf_nms_scan with a caller-owned device workspace of bf_nms_scan_workspace_size(n) bytes
 * (the same nms_3d + record, instances.py:22-101 / box_manager.py:40-88).  With it, scans too
 * large for the IoU matrix to sit in LDS (n > 96) run the single-wave scan on the matrix's two
 * threshold bit masks (iou <= t, iou > t) instead of the 256-thread scan over the f64 matrix in
 * global memory; results are identical.  workspace may be NULL (= bf_nms_scan). */
size_t bf_nms_scan_workspace_size(int n);
int bf_nms_scan_ws(const double* iou, const float* corners, const float* scores,
                   const int32_t* init_id, const float* cam_poses, int n,
                   int32_t* fl_items, int32_t* fl_len, float* valid_num,
                   int32_t* keep, int32_t* n_keep, int32_t* success, int32_t* n_success,
                   int32_t* events, int32_t* n_events, int32_t* status,
                   const bf_nms_cfg* cfg, void* workspace, void* stream);

/* ------------------------------------------------------------------------------------------
 * Cross-view correspondence association for small boxes
 *   Instances3D.correspondence_association (instances.py:411-490) + project_3d_to_2d_box
 *   (:670-717) + IoU_2D_box (:643-668) + BoxManager.record_corr (box_manager.py:90-129)
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    double small_size;       /* cfg box_fusion.small_size */
    double threshold;        /* cfg association.small_threshold (compared with f64 IoU) */
    float translation_gap;
    float rotation_gap;
    float W, H;              /* image size used for the 2-D projection */
    int   max_list;
    int   list_capacity;
} bf_corr_cfg;

/*   n_all boxes = n_glo global boxes followed by the new keyframe's boxes.
 *   corners f32[n_all,8,3], dims f32[n_all,3], scores f32[n_all], boxes2d f32[n_all,4] (xyxy),
 *   init_id i32[n_all], cam_poses f32[M,4,4], cur_pose f32[4,4] (camera->world of this keyframe),
 *   K f32[3,3]; mask i32[n_mask] = sorted NMS keep; success i32[n_success] = sorted success_nms.
 *   In/out: fl_items/fl_len (fusion lists), valid_num f32[n_all].
 *   Out: keep_out i32[n_mask] sorted, n_keep_out i32[1], events i32[n_all,3], n_events,
 *        status i32[1]. */
int bf_corr_assoc(const float* corners, const float* dims, const float* scores,
                  const float* boxes2d, const int32_t* init_id, const float* cam_poses,
                  const float* cur_pose, const float* K, int n_all, int n_glo,
                  const int32_t* mask, int n_mask, const int32_t* success, int n_success,
                  int32_t* fl_items, int32_t* fl_len, float* valid_num,
                  int32_t* keep_out, int32_t* n_keep_out, int32_t* events, int32_t* n_events,
                  int32_t* status, const bf_corr_cfg* cfg, void* stream);

/* bf_corr_assoc chained on the stream right after bf_nms_scan, without the host round trip the
 * reference makes between the two steps (demo.py:243-262: spatial_association returns `mask`
 * and `success` to Python, which slices cur_keep / cur_success and calls
 * correspondence_association).  mask / n_mask_dev and success / n_success_dev are the NMS
 * kernel's device outputs (keep / n_keep, success / n_success), fl_items / fl_len / valid_num
 * the same buffers it updated.  With no new box in `mask` (cur_keep empty: the reference skips
 * the step) the kernel returns keep_out = mask and no events, so the caller may branch after
 * reading both results back once. */
int bf_corr_assoc_chained(const float* corners, const float* dims, const float* scores,
                          const float* boxes2d, const int32_t* init_id, const float* cam_poses,
                          const float* cur_pose, const float* K, int n_all, int n_glo,
                          const int32_t* mask, const int32_t* n_mask_dev,
                          const int32_t* success, const int32_t* n_success_dev,
                          int32_t* fl_items, int32_t* fl_len, float* valid_num,
                          int32_t* keep_out, int32_t* n_keep_out, int32_t* events,
                          int32_t* n_events, int32_t* status, const bf_corr_cfg* cfg,
                          void* stream);

/* ------------------------------------------------------------------------------------------
 * Multi-view box fusion: particle-swarm refinement
 *   BoxFusion.boxfusion (box_fusion.py:622-724), init_opt_params (:566-600),
 *   compute_iou_value CUDA kernel (:264-405), evaluate_iou (:413-461), cal_transform (:475-535),
 *   update_PST (:537-563), init_searchsize (:468-472).  One launch refines every job, all
 *   iterations on the device.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    int   iters;             /* box_fusion.iters (20) */
    int   pst_size;          /* particles, multiple of 64, <= 1024 */
    int   max_accept;        /* 200 (cal_transform early stop) */
    int   legacy_promotion;  /* 1: numpy<2 value-based promotion (pinned numpy 1.26.4, f64 host
                                scalars); 0: NEP 50 promotion (numpy>=2, f32 host scalars) */
    /* host-side Python floats of the reference, kept in f64 so both promotion modes are exact */
    double center_init, shape_init;  /* random_opt.center_init_size / shape_init_size */
    double center_coef, shape_coef;  /* random_opt.*_scaling_coefficient */
    double beta;             /* momentum 0.9 (box_fusion.py:622) */
    double min_scale;        /* 1e-3 (update_PST default) */
    float img_h, img_w;      /* BoxFusion.H / .W */
    float K[16];             /* BoxFusion.K (4x4 row-major) */
} bf_fuse_cfg;

/*   job j fuses views [view_off[j], view_off[j]+n_views[j]) of the view table:
 *   view_box f32[V,6] (xyzlhw, per_frame_box.pred_boxes_3d.tensor rows),
 *   view_R f32[V,3,3], view_score f32[V], view_pose f32[V,4,4], view_tc f32[V,8,2]
 *   (per_frame_box.projected_boxes rows).  pst f32[pst_size,6] (row 0 must be zeros).
 *   out_box f32[n_jobs,6]: refined xyzlhw (lhw >= 0.01), only meaningful where out_updated==1.
 *   out_iters i32[n_jobs]: iterations executed.  trace (nullable) f32[n_jobs, iters, pst_size]
 *   receives every iteration's fitness vector.  max_views (<= 32) bounds every n_views[j] (a job
 *   above it is skipped with BF_DEV_VIEW_OVERFLOW); `workspace` holds
 *   bf_fusion_fit_workspace_size(n_jobs, max_views, pst_size) bytes (per-job state + the
 *   per-iteration |1 - IoU| terms).  Per iteration: one launch over all (job, view, particle)
 *   pairs, one launch per job for the sequential update; no host synchronisation. */
size_t bf_fusion_fit_workspace_size(int n_jobs, int max_views, int pst_size);
int bf_fusion_fit(const int32_t* view_off, const int32_t* n_views, int n_jobs, int max_views,
                  const float* view_box, const float* view_R, const float* view_score,
                  const float* view_pose, const float* view_tc, const float* pst,
                  const bf_fuse_cfg* cfg, float* out_box, int32_t* out_updated,
                  int32_t* out_iters, float* trace, int32_t* status, void* workspace,
                  void* stream);

/* Single evaluation of the reference fitness kernel (compute_iou_value + evaluate_iou):
 *   box f32[6], R f32[9], views as above (n_views), search_size f32[6] -> fitness f32[pst_size]
 *   = (sum over views in order of |1 - IoU2D|) / (n_views + 1e-6f). */
/* The write-back of BoxFusion.boxfusion (box_fusion.py:716-724): for every job j with
 * updated[j] != 0, target[rows[j]][0..6) = out_box[j] (xyz + lhw; R and any further columns of
 * the ld-float target rows untouched).  Rows must be distinct. */
int bf_fusion_writeback(const float* out_box, const int32_t* updated, const int32_t* rows,
                        int n_jobs, float* target, int ld, void* stream);

int bf_fusion_fitness(const float* box, const float* R, int n_views, const float* view_pose,
                      const float* view_tc, const float* pst, int pst_size,
                      const float* search_size, const bf_fuse_cfg* cfg, float* fitness,
                      void* stream);

/* ------------------------------------------------------------------------------------------
 * Keyframe sequencer: the state machine of demo.py:200-305 over a batch of keyframes in one call
 *   (FusionStage.keyframe's per-keyframe sequence: Instances3D.cat (demo.py:245),
 *   init_new_predictions, spatial_association + correspondence_association (:247-262, the
 *   bf_nms_scan / bf_corr_assoc_chained pair), all_pred_box[keep_idx] + BoxManager.update
 *   (:263-268 / :300-304), BoxFusion.boxfusion (:270-299, bf_fusion_fit + write-back)).
 * The exception to "stateless, caller-owned memory": a bf_fseq owns all_pred_box's device rows
 * (stream-ordered allocations that grow by doubling), BoxManager's fusion_list / fusion_flag /
 * already_fusion on the host, and pinned staging buffers.  One host wait per keyframe (the
 * association read-back); a BoxFusion result is applied at the next keyframe's wait or at
 * bf_fseq_sync, where BoxManager.flush applies it in the Python path.
 * ------------------------------------------------------------------------------------------ */
typedef struct bf_fseq bf_fseq;
typedef struct {
    bf_nms_cfg nms;          /* nms_threshold, association gaps, list capacity */
    bf_corr_cfg corr;        /* small_threshold, image size, same list capacity */
    bf_fuse_cfg fuse;        /* BoxFusion's particle search */
    int32_t use_fusion;      /* cfg box_fusion.use */
    int32_t strict_hull;     /* 1: BF_DEV_HULL_OVERFLOW is an error (box_fusion.strict_hull) */
} bf_fseq_cfg;

int bf_fseq_create(bf_fseq** out);
void bf_fseq_destroy(bf_fseq* s);
/* message of the last failing call */
const char* bf_fseq_error(const bf_fseq* s);

/* n_kf keyframes in frame order; keyframe j's detections are the per-frame rows
 * [p_base + sizes[0] + .. + sizes[j-1], + sizes[j]) (sizes[j] = 0: a keyframe without boxes).
 * The per-frame table (per_frame_ins, p_rows rows, the new keyframes' rows already world-space,
 * projected and appended): p_box f32[p_rows,6], p_R f32[p_rows,3,3], p_score f32[p_rows],
 * p_box2d f32[p_rows,4], p_pose f32[p_rows,4,4] (cam_pose), p_proj f32[p_rows,8,2]
 * (projected_boxes).  A row's init_id is its row index.  K f32[3,3], pst f32[pst_size,6]. */
int bf_fseq_keyframes(bf_fseq* s, const bf_fseq_cfg* cfg, int n_kf, const int32_t* sizes,
                      int64_t p_base, int64_t p_rows, const float* p_box, const float* p_R,
                      const float* p_score, const float* p_box2d, const float* p_pose,
                      const float* p_proj, const float* K, const float* pst, void* stream);
/* wait for the sequencer's stream and apply a pending BoxFusion result */
int bf_fseq_sync(bf_fseq* s);
/* (after a sync) [0] all_pred_box rows (-1: None), [1] fusion_list rows, [2] their items,
 * [3] fusion_flag length, [4] already_fusion rows, [5] their items, [6] boxes suppressed,
 * [7] boxes fused (updated), [8] boxfusion calls with jobs, [9] of them with
 * BF_DEV_HULL_OVERFLOW, [10..13] the last call's jobs / updated / iterations / views,
 * [14] association steps, [15] 0 */
#define BF_FSEQ_STATE_N 16
int bf_fseq_state(bf_fseq* s, int64_t* out);
/* which 0: fusion_list, 1: already_fusion -> host lens[rows], items[total] (concatenated) */
int bf_fseq_lists(bf_fseq* s, int which, int32_t* lens, int32_t* items);
int bf_fseq_flags(bf_fseq* s, int32_t* flags);
/* all_pred_box: host init_id[rows] (= per-frame row), device xyzlhw f32[rows,6] (fused rows
 * refined) and valid_num f32[rows], copied on `stream` */
int bf_fseq_global(bf_fseq* s, int32_t* init_id, float* xyzlhw, float* valid_num, void* stream);

/* ------------------------------------------------------------------------------------------
 * Per-frame depth work
 * ------------------------------------------------------------------------------------------ */
/* Preprocessor.standardize_depth_map (preprocessor.py:97-129) for a batch of b frames:
 *   depth f32[b,h,w] -> out f32[b,h,w] standardised (invalid -> mean), params f32[b,2] =
 *   (trunc_mean, trunc_std).  Trimmed order statistics by a 3-level radix select spread over
 *   the whole chip (8192-element slices), no sort.
 *   workspace: bf_depth_standardize_workspace_size(b, h, w) bytes, ZERO-FILLED by the caller
 *   before its first use; every call leaves it zero-filled again (histograms are cleared by the
 *   kernels that consume them).  One workspace per stream (calls sharing one must not overlap). */
size_t bf_depth_standardize_workspace_size(int b, int h, int w);
int bf_depth_standardize(const float* depth, int b, int h, int w, float* out, float* params,
                         void* workspace, void* stream);

/* demo.py:121-131's per-frame depth work in one call: bf_depth_standardize plus, when xyz is not
 * NULL, the back-projection of the same frames (tools/utils.py:232-287, bf_backproject's
 * arithmetic) fused into the normalise pass: K f32[b,3,3] (the depth map's intrinsics),
 * RT f32[b,4,4] (camera -> world), xyz f32[b,h,w,3], valid u8[b,h,w]. */
int bf_depth_preprocess(const float* depth, int b, int h, int w, float* out, float* params,
                        const float* K, const float* RT, float max_depth, float* xyz,
                        uint8_t* valid, void* workspace, void* stream);

/* tools/utils.py unproject + get_camera_coords (:232-287):
 *   depth f32[h,w], K f32[3,3], RT f32[4,4] -> xyz f32[h,w,3], valid u8[h,w]
 *   (valid = d > 0 && d < max_depth; max_depth <= 0 disables the upper bound). */
int bf_backproject(const float* depth, const float* K, const float* RT, int h, int w,
                   float max_depth, float* xyz, uint8_t* valid, void* stream);

/* ------------------------------------------------------------------------------------------
 * MFMA tower kernels: CuTR RGB-D ViT (boxfusion/vit.py, cubify_transformer.py) and the CLIP
 * ViT-H/14 crop tower (tools/utils.py:383-403).  bf16 operands, f32 accumulation.
 * ------------------------------------------------------------------------------------------ */

/* C[orow(r),n] = (resid ? resid[rrow(r),n] : 0) + act(sum_k A[r,k] W[n,k] + bias[n])
 *   A bf16[M,K] (row stride lda), W bf16[N,K] (nn.Linear layout, stride ldw), bias f32[N] or NULL,
 *   resid f32 (stride ldr) or NULL, orow(r) = row_map ? row_map[r] : r (< 0 drops the row),
 *   rrow(r) = resid_mod > 0 ? r % resid_mod : orow(r), C f32 or bf16 (c_bf16), stride ldc,
 *   act 0 none / 1 GELU(erf) / 2 ReLU.  K % 64 == 0, lda/ldw % 8 == 0.
 * Replaces the nn.Linear / 1x1-conv / patch-conv GEMMs of vit.py:102-342 and the open_clip
 * transformer blocks (in_proj, out_proj, c_fc, c_proj, proj). */
int bf_gemm_bf16(const void* A, int lda, const void* W, int ldw, const float* bias,
                 const float* resid, int ldr, int resid_mod, void* C, int ldc, int c_bf16,
                 const int32_t* row_map, int M, int N, int K, int act, void* stream);

/* Kernel choice is a function of the shape and the DEVICE's CU count alone (hand-written kernels
 * only, the same on every box and every rank): few-row problems (the 128 x 128 tiling would feed
 * fewer than half the CUs; N % 32 == 0, K % 256 == 0) run k_gemm_skinny (8 waves split K, partials
 * summed in wave order); large ones the persistent kernels with a tile height of 160 / 192 / 224 /
 * 256 rows picked by the round quantisation of the walk (the height never changes a value).
 *
 * bf_gemm_plan: caller-owned, per-call configuration (no process-wide GEMM state exists; NULL or an
 * all-zero plan = the product defaults):
 *   cu_budget  CUs the persistent grid may assume (0 = every CU of the device): a GEMM launched on a
 *              CU-masked stream passes that stream's CU count.  Sizes the grid and the tile-height
 *              model only, so results are bit-identical under any budget.
 *   tile_rows  0 = the per-shape model; 160 / 192 / 224 / 256 force the height (value-invariant).
 *   The remaining fields are measurement / test hooks (0 = product default):
 *   kernel     1 forces the 128x128 kernel, -1 the persistent kernels (aligned shapes);
 *   variant    persistent kernel variant: 1 = k_gemm256p (staggered 4-phase schedule), 2 = k_gemm256p
 *              unstaggered, 3 / 4 = timing ablations (no epilogue / no global stores: wrong
 *              results), 5 = default (k_gemm256q for bf16 outputs and sub-256-row residual tiles,
 *              k_gemm256p otherwise), 6 = k_gemm256q for every eligible shape;
 *   group_m    row panels per tile group of the persistent tile order (default 8; 1 = row-major);
 *   balanced   0 = default (ceil(tiles / rounds) workgroups when the last round is at least a
 *              quarter full), 1 = one workgroup per CU, 2 = balanced for every multi-round problem.
 * bf_gemm_bf16(...) == bf_gemm_bf16_plan(..., NULL, stream). */
typedef struct {
    int32_t cu_budget;
    int32_t tile_rows;
    int32_t kernel;
    int32_t variant;
    int32_t group_m;
    int32_t balanced;
} bf_gemm_plan;
int bf_gemm_bf16_plan(const void* A, int lda, const void* W, int ldw, const float* bias,
                      const float* resid, int ldr, int resid_mod, void* C, int ldc, int c_bf16,
                      const int32_t* row_map, int M, int N, int K, int act, const bf_gemm_plan* plan,
                      void* stream);
/* 1 if an aligned (16-B rows) problem of this shape runs a 256-column persistent kernel
 * (k_gemm256p/q) under the default plan, 0 if the 128x128 one (k_gemm) -- lets profilers
 * attribute launches to kernels. */
int bf_gemm_large_tiles(int M, int N, int K);

/* fp8 e4m3 (OCP) GEMM of the CLIP ViT-H fp8 path (BASELINE configs[4]; the same open_clip
 * in_proj / c_fc / c_proj linears as bf_gemm_bf16, tools/utils.py:383-403):
 *   C[r,n] = (resid ? resid[r,n] : 0) + act(scale * sum_k A[r,k] W[n,k] + bias[n])
 *   A fp8[M,K] (row stride lda bytes), W fp8[N,K] (stride ldw), scale = activation scale x weight
 *   scale (per-tensor), bias f32[N] or NULL, act 0 none / 1 GELU(erf);
 *   out_kind 0: C f32 (+ resid f32, stride ldr, in place allowed; act 0 only), 1: C bf16,
 *   2: C fp8 = saturate_448(value * out_qscale).  K % 128 == 0, lda/ldw % 16 == 0.
 * Runs on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales. */
int bf_gemm_fp8(const void* A, int lda, const void* W, int ldw, float scale, const float* bias,
                const float* resid, int ldr, void* C, int ldc, int out_kind, float out_qscale,
                int M, int N, int K, int act, void* stream);
/* the same with a per-call plan (cu_budget / tile_rows / variant / group_m / balanced as above) */
int bf_gemm_fp8_plan(const void* A, int lda, const void* W, int ldw, float scale, const float* bias,
                     const float* resid, int ldr, void* C, int ldc, int out_kind, float out_qscale,
                     int M, int N, int K, int act, const bf_gemm_plan* plan, void* stream);

/* softmax(Q K^T * scale) V per (batch, head); X(b,h,s,d) at X + b*x_bs + s*x_rs + h*D + d,
 * bf16 in/out, head_dim in {32, 64, 80, 128}.  Replaces vit.py Attention.forward (:170-203,
 * joint RGB+depth window attention = plain attention over the concatenated 512 tokens) and the
 * open_clip nn.MultiheadAttention of ViT-H/14. */
int bf_attention_bf16(const void* q, const void* k, const void* v, void* o, int batch, int heads,
                      int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs, int o_rs,
                      long long q_bs, long long k_bs, long long v_bs, long long o_bs, float scale,
                      void* stream);
/* the same with an output row map: query q of batch b is stored to row o_map[b*sq + q] of o
 * (o_bs unused; < 0 = not stored).  The window blocks write their outputs back in token order
 * (window_unpartition, vit.py:39-58) with the pad queries dropped. */
int bf_attention_bf16_omap(const void* q, const void* k, const void* v, void* o, int batch,
                           int heads, int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs,
                           int o_rs, long long q_bs, long long k_bs, long long v_bs, long long o_bs,
                           float scale, const int32_t* o_map, void* stream);
/* the same (default kernel) with an fp8 e4m3 output saturate_448(o * out_qscale): the CLIP fp8
 * path's out_proj input (o_rs, o_bs in bytes; head_dim 64 / 80) */
int bf_attention_fp8out(const void* q, const void* k, const void* v, void* o, int batch, int heads,
                        int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs, int o_rs,
                        long long q_bs, long long k_bs, long long v_bs, long long o_bs, float scale,
                        float out_qscale, void* stream);
/* bf_attention_bf16_omap / bf_attention_fp8out with a per-call kernel variant (a test / benchmark
 * hook; 0 or 6 = the default the plain entry points run): 6 = k_attn2 (deferred-max softmax, row
 * sums from a ones row of V on the MFMA; 257-288 queries on 9-wave workgroups, at head dim 80 on
 * 4-wave ones; 129-256 queries on 4-wave workgroups at head dims 64 and 80 and 8-wave ones
 * otherwise; 449-512 queries at head dim 64 on 8-wave workgroups; output rows staged in LDS and
 * stored as whole head rows), 27 = the same kernel with per-lane fragment stores, 28 = 129-288
 * queries on 9 waves, 29 / 30 = 129-256 queries on 4 / 8 waves, 31 = 129-288 queries on 4 waves,
 * for every head dim, 33 = 449-512 queries at head dim 64 on 4 waves (all bit-identical). */
int bf_attention_bf16_ex(const void* q, const void* k, const void* v, void* o, int batch, int heads,
                         int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs, int o_rs,
                         long long q_bs, long long k_bs, long long v_bs, long long o_bs, float scale,
                         const int32_t* o_map, int variant, void* stream);
int bf_attention_fp8out_ex(const void* q, const void* k, const void* v, void* o, int batch, int heads,
                           int sq, int sk, int head_dim, int q_rs, int k_rs, int v_rs, int o_rs,
                           long long q_bs, long long k_bs, long long v_bs, long long o_bs, float scale,
                           float out_qscale, int variant, void* stream);

/* CuTR decoder cross-attention bias (GlobalCrossAttention.rpe + the logits' bias / clip /
 * softmax, cubify_transformer.py:93-190 of the reference), f32:
 *   bf_cpb_mlp: out[b,q,p,:] = W2 relu(W1 ((c - s/2, c + s/2) - pos[p]) + b1), where (c, s) =
 *     (ref[b,q,axis], ref[b,q,2+axis]) of ref f32[B,nq,4] (cx, cy, w, h); W1 f32[hidden,2],
 *     b1 f32[hidden], W2 f32[heads,hidden]; out f32[B,nq,n,heads].  hidden <= 512, heads <= 16.
 *   bf_rpe_softmax: attn f32[B,H,Nq,hh*ww] in place: rows q >= q0 get + (rx[b,q-q0,x,h] +
 *     ry[b,q-q0,y,h]) at column y*ww+x; every row is clipped to the finite f32 range and
 *     softmax-normalised.  hh*ww % 4 == 0, <= 4096. */
int bf_cpb_mlp(const float* ref, int B, int nq, const float* pos, int n, int axis,
               const float* w1, const float* b1, const float* w2, int hidden, int heads,
               float* out, void* stream);
int bf_rpe_softmax(float* attn, int B, int H, int Nq, int q0, const float* rx, const float* ry,
                   int hh, int ww, void* stream);
/* The whole global cross-attention after the projections (GlobalCrossAttention.forward,
 * cubify_transformer.py:170-200 of the reference), f32: out[b,q,h*32+d] = sum_j softmax_j(clip(
 * (scale q[b,q,h]) . k[b,j,h] + bias))[j] v[b,j,h,d] with bias = rx[b,q-q0,x,h] + ry[b,q-q0,y,h]
 * (j = y*ww + x) for q >= q0, 0 otherwise.  q [B,Nq] rows of stride ldq, k / v [B,hh*ww] rows of
 * stride ldk / ldv (e.g. one layer's columns of the all-layer memory projections), head dim 32,
 * hh, ww <= 128.  Replaces the two batched matmuls, bf_rpe_softmax's logits round trip and the
 * head permutes. */
int bf_xattn_f32(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                 const float* rx, const float* ry, float* out, int ldo, int B, int H, int Nq, int q0,
                 int hh, int ww, float scale, void* stream);
/* The decoder self-attention (PreNormGlobalDecoderLayer.self_attn, cubify_transformer.py:
 * 313-352 of the reference, with CubifyTransformer's block mask :1196-1202): q / k / v f32
 * [B, N] rows (strides ldq / ldk / ldv, batches packed), head dim 32, query i sees key j iff
 * (j < q0) == (i < q0) (q0 metric queries), scale applied to q. */
int bf_self_attn_f32(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                     float* out, int ldo, int B, int H, int N, int q0, float scale, void* stream);

/* ---- the CuTR decoder tail, f32 (bf_dec_native.hip; boxfusion_amd.decoder_engine) ----------
 * Replaces the torch / hipBLASLt ops of CubifyTransformer.inference after the backbone
 * (cubify_transformer.py:1172-1227 of the reference).
 * bf_gemm_f32: C[c_map[m]] = resid[c_map[m]] + act(A[a_map[m]] W^T + bias) for m < M on
 *   v_mfma_f32_32x32x2_f32 (act 0 none, 1 GELU(erf), 2 ReLU); A [*,K] row stride lda, W [N,K]
 *   row stride ldw (both % 4, 16-B aligned); a_map / c_map int32 or NULL (identity); a_map < 0
 *   reads a zero row, c_map < 0 drops the row; resid may alias C.  Every nn.Linear / 1x1 and
 *   2x2/2 conv of the decoder tail (cubify_transformer.py:93-352, 812-943, 1128-1170). */
int bf_gemm_f32(const float* A, int lda, const int* a_map, const float* W, int ldw,
                const float* bias, const float* resid, int ldr, float* C, int ldc,
                const int* c_map, int M, int N, int K, int act, void* stream);
/* LayerNorm over rows (C % 256 == 0, <= 1024), optional GELU (LayerNorm2D + GELU of the proposal
 * levels, :858-862), optional second output out2 = y + pos (the decoder's `norm(tgt) +
 * query_pos`, :330-341).  out may alias x. */
int bf_ln_rows_f32(const float* x, int ldx, const float* gamma, const float* beta, float eps,
                   float* out, int ldo, const float* pos, int ldp, float* out2, int ldo2, int M,
                   int C, int gelu, void* stream);
/* GroupNorm(G) of a channel-last map x [B*P, C] (input_proj's GroupNorm, :1131-1136), optional
 * out2 = y + pos (the memory keys' src + pos). */
int bf_groupnorm_cl_f32(const float* x, int ldx, int B, int P, int C, int G, const float* gamma,
                        const float* beta, float eps, float* out, int ldo, const float* pos,
                        int ldp, float* out2, int ldo2, void* stream);
/* space-to-depth rows of a channel-last [B,H,W,C] map for a 2x2 stride-2 Conv2d:
 * out [B*(H/2)*(W/2), 4C], column c*4 + ky*2 + kx (the Conv2d weight order). */
int bf_s2d_f32(const float* x, int ldx, int B, int H, int W, int C, float* out, void* stream);
/* The predictors' output linears (K = 256 / 512, nout <= 8) and transforms, one row per
 * (frame f, query q < nq) of input row f*in_fs + in_off + q: mode 0 ClassPredictor logits
 * (:396-403), 1 DeltaBox2DPredictor + apply_deltas + cxcywh (:478-541; prop / boxes [rows,4]
 * cxcywh, may alias), 2 AbsoluteBox3DPredictor (:592-643; 16 floats per row: proj_xy, z,
 * z_scaled, dims, R_Y(yaw); params [frames,2] = (shift, scale)), 3 ScalePredictor (:545-560;
 * out [frames,2] = exp of the two tokens' linears).  clamp_w / clamp_h: clamp_xy bounds. */
int bf_row_heads_f32(const float* x, int ldx, int in_fs, int in_off, int rows, int nq, int K,
                     const float* w, const float* b, int nout, const float* prop,
                     const float* params, float* out, int ldo, float* boxes, float clamp_w,
                     float clamp_h, float max_ratio, int mode, void* stream);
/* per-frame top-k of v[(f*n + i)*ldv], n <= 4096: idx int32 [frames, k] (and vals), descending,
 * ties -> lower index (torch.topk, :930 / :967). */
int bf_topk_rows_f32(const float* v, int ldv, int frames, int n, int k, int* idx, float* vals,
                     void* stream);
/* the top-k proposals' boxes (ref [frames*k, 4]) and their learned box prompt embedding
 * (Box2DPromptEncoderLearned, :706-737: clamp to [0, max_e], int, 4 tables of ed columns) into
 * qpos row f*qfs + qoff + j. */
int bf_prop_select_f32(const float* boxes, int frames, int n, int k, const int* idx, float* ref,
                       const float* ex, const float* ey, const float* ew, const float* eh, int ed,
                       float max_e, float* qpos, int ldq, int qfs, int qoff, void* stream);
/* inference_single_image (:945-996) for every frame: sigmoid, top-k over (query, class) (nq*nc
 * <= 4096), xyxy boxes clamped to img_wh[f], K^-1 (z u, z v, z), dims reversed, T_gravity R
 * (Tg may be NULL), logits / proj_xy / descriptor rows gathered. */
int bf_infer_select_f32(const float* logits, int frames, int nq, int nc, const float* boxes,
                        const float* b3info, const float* desc, int ld_desc, int desc_fs,
                        int desc_off, int C, const float* Kinv, const float* Tg,
                        const float* img_wh, int k, float* scores, long long* classes,
                        float* out_logits, float* out_boxes, float* out_proj, float* out_b3,
                        float* out_R, float* out_desc, void* stream);
/* CameraRayEmbedding's ray Fourier features of one camera (pos.py:61-186): rays through
 * (fx, fy, cx, cy) at pixel centres, square pad feat*stride, nearest sample every stride pixels,
 * normalised, sin(r_c * scales[k] * pi) -> out [feat*feat, ld] (columns >= 3*nb zeroed). */
int bf_ray_fourier_f32(float fx, float fy, float cx, float cy, int W, int H, int feat, int stride,
                       const float* scales, int nb, float* out, int ld, void* stream);

/* LayerNorm f32[M,C] -> bf16, written to row row_map[r] (NULL = r; < 0 skips). */
int bf_layernorm(const float* x, int ldx, const float* gamma, const float* beta, float eps,
                 void* out, int ldo, const int32_t* row_map, int M, int C, void* stream);
/* the same with an f32 output (out_f32 = 1; x == out in place allowed): CLIP ln_pre / ln_post,
 * CuTR's encoder_norm (vit.py:473) */
int bf_layernorm_out(const float* x, int ldx, const float* gamma, const float* beta, float eps,
                     void* out, int ldo, int out_f32, const int32_t* row_map, int M, int C,
                     void* stream);
/* the same with an fp8 e4m3 output, saturate_448(y * qscale) (ldo in bytes): ln_1 / ln_2 of the
 * CLIP fp8 path feeding bf_gemm_fp8 */
int bf_layernorm_fp8(const float* x, int ldx, const float* gamma, const float* beta, float eps,
                     void* out, int ldo, float qscale, int M, int C, void* stream);

/* Preprocessor.normalize + square zero pad + PatchEmbed im2col (preprocessor.py:131-144,
 * imagelist.py:55-115, vit.py:102-128): img u8[B,H,W,3] -> bf16[B*(pad/p)^2, 3*p*p].
 * mean3/std3 are HOST arrays of 3 floats. */
int bf_im2col_rgb8(const uint8_t* img, int B, int H, int W, int pad, int patch,
                   const float* mean3, const float* std3, void* out, int ldo, void* stream);
/* the same for CHW frames ([B,3,H,W] u8, chw = 1: the layout of the reference's capture stream,
 * capture_stream.py:221 `np.moveaxis(image, -1, 0)`) or HWC (chw = 0) */
int bf_im2col_rgb8_chw(const uint8_t* img, int B, int H, int W, int chw, int pad, int patch,
                       const float* mean3, const float* std3, void* out, int ldo, void* stream);

/* single-channel f32 [B,H,W] -> zero-padded square -> bf16 im2col [B*(pad/p)^2, p*p] */
int bf_im2col_f32(const float* x, int B, int H, int W, int pad, int patch, void* out, int ldo,
                  void* stream);

/* CLIP crop path (tools/utils.py:405-476 crop_image/segment_image + retriev's 224x224 resize):
 * boxes i32[N,4] integer xyxy on frame img_idx[N] of img u8[*,H,W,3] -> cv2.resize(crop, (S, S))
 * (OpenCV u8 INTER_LINEAR fixed point, bit-exact to oracle/bf_oracle.c or_cv2_resize_u8) -> /255 ->
 * (x-mean)/std -> p x p patch im2col bf16 [N*(S/p)^2, ldo] (K = 3p^2 zero-padded to ldo).
 * mean3/std3 are HOST arrays. */
int bf_crop_resize_im2col(const uint8_t* img, int H, int W, const int32_t* boxes,
                          const int32_t* img_idx, int N, int size, int patch, const float* mean3,
                          const float* std3, void* out, int ldo, void* stream);

/* ---- CLIP text tower (reference: boxfusion/precompute_class_features.py:31-43, the open_clip
 * "ViT-H-14" encode_text of its commented path; tools/utils.py:399 renormalises the result) ---- */

/* causal self-attention (open_clip TextTransformer attn_mask: query i sees keys 0..i), sq == sk == s;
 * operands as bf_attention_bf16; head_dim 64 or 80 */
int bf_attention_causal(const void* q, const void* k, const void* v, void* o, int batch, int heads,
                        int s, int head_dim, int q_rs, int k_rs, int v_rs, int o_rs, long long q_bs,
                        long long k_bs, long long v_bs, long long o_bs, float scale, void* stream);

/* token_embedding(ids) + positional_embedding: ids i32 [n_tok] (token t at position t % S),
 * table f32 [vocab, W], pos f32 [S, W] -> out f32 [n_tok, W]; W % 4 == 0.  An id outside
 * [0, vocab) gives a zero embedding row and BF_DEV_INDEX_RANGE in *status (when non-NULL). */
int bf_token_embed(const int32_t* ids, int n_tok, const float* table, int vocab, const float* pos,
                   int S, int W, float* out, int32_t* status, void* stream);

/* text_global_pool 'argmax': out[n] = x[n*S + argmax(ids[n, :S])] (first maximum, torch.argmax);
 * x f32 [N*S, W] -> out f32 [N, W] */
int bf_text_pool(const int32_t* ids, int N, int S, const float* x, int W, float* out, void* stream);

/* out[r] = x[r] / ||x[r]||_2 (precompute_class_features.py:43); in place allowed */
int bf_l2_normalize_rows(const float* x, int rows, int W, float* out, void* stream);

/* ---- GPU frame ingestion (reference: capture_stream.py:194-311 ScanNet / :402-529 CA-1M
 * __iter__ after image decode) ---- */

/* decoded frames -> the sample tensors of the reference's streams, one launch for F frames:
 * bgr u8 [F,Hc,Wc,3] (cv2.imread order; src_bgr = 0: already RGB) -> cvtColor RGB -> cv2.resize to (Wd, Hd) (u8 INTER_LINEAR,
 * OpenCV fixed point) -> CHW -> torch.rot90(k=rot_k, dims (-2,-1)) -> rgb_out u8 [F,3,Ho,Wo];
 * depth u16 [F,Hd,Wd] (PNG, may be NULL) -> f32 / depth_scale -> rot90 -> depth_out f32 [F,Ho,Wo];
 * (Ho, Wo) = (Hd, Wd) for even rot_k, (Wd, Hd) for odd. */
int bf_ingest_rgbd(const uint8_t* bgr, int Hc, int Wc, const uint16_t* depth, int Hd, int Wd, int F,
                   float depth_scale, int rot_k, int src_bgr, uint8_t* rgb_out, float* depth_out,
                   void* stream);

/* cv2.resize(src, (Wd, Hd)) for u8 HWC images with cn <= 4 channels, F images:
 * src [F,Hs,Ws,cn] -> dst [F,Hd,Wd,cn] (INTER_LINEAR, OpenCV's fixed-point arithmetic) */
int bf_cv2_resize_u8(const uint8_t* src, int Hs, int Ws, int cn, int Hd, int Wd, int F, uint8_t* dst,
                     void* stream);

/* ---- depth PNG decode (reference: cv2.imread(depth_path, cv2.IMREAD_UNCHANGED),
 * capture_stream.py:197 ScanNet / :405 CA-1M) ----
 * F PNG files, back to back in device memory: file f = files[offsets[f] .. offsets[f+1]) (offsets
 * int64 [F+1], device; total_file_bytes = offsets[F], max_file_bytes = the largest file, both as the
 * host uploaded them) -> out u16 [F,H,W], the sample values in native order (what cv2 returns).
 * 16-bit greyscale, non-interlaced files of exactly H x W; status int32 [F] (device) gets the
 * BF_PNG_* bits of a file that did not decode (its out rows are then undefined).  The zlib Adler-32
 * is verified; chunk CRCs are not.  work: bf_png_workspace_bytes(F, H, W, total_file_bytes) bytes,
 * caller-owned device memory. */
#define BF_PNG_BAD_SIGNATURE 1
#define BF_PNG_BAD_HEADER 2      /* IHDR missing / invalid */
#define BF_PNG_UNSUPPORTED 4     /* not 16-bit greyscale non-interlaced, or an unknown critical chunk */
#define BF_PNG_BAD_CHUNK 8       /* truncated chunk, no IDAT, a zlib stream of 2 GiB or more */
#define BF_PNG_BAD_ZLIB 16       /* invalid zlib header / deflate block / code / distance */
#define BF_PNG_BAD_ADLER 32
#define BF_PNG_BAD_FILTER 64     /* row filter type > 4 */
#define BF_PNG_SIZE 128          /* IHDR size != (W, H) or inflated length != H x (2W + 1) */
size_t bf_png_workspace_bytes(int F, int H, int W, long long total_file_bytes);
int bf_png_decode_u16(const uint8_t* files, const int64_t* offsets, int F, int H, int W,
                      long long total_file_bytes, long long max_file_bytes, uint16_t* out, void* work,
                      size_t work_bytes, int32_t* status, void* stream);
/* the same decode fused with the streams' depth scaling (capture_stream.py:203 / :410,
 * depth_data.astype(np.float32) / depth_scale, IEEE f32 division): depth_out f32 [F,H,W] */
int bf_png_decode_depth(const uint8_t* files, const int64_t* offsets, int F, int H, int W,
                        long long total_file_bytes, long long max_file_bytes, float depth_scale,
                        float* depth_out, void* work, size_t work_bytes, int32_t* status, void* stream);

/* ---- colour JPEG decode (reference: cv2.imread(color_path), capture_stream.py:194 ScanNet /
 * :402 CA-1M -- libjpeg's default decompression, which PIL's decoder reproduces) ----
 * F baseline (sequential Huffman, 8-bit) JPEG files, back to back in device memory as for the PNG
 * decode, each exactly H x W, 1 or 3 components, chroma at full or half resolution (4:4:4, 4:2:2,
 * 4:2:0), restart markers allowed -> rgb u8 [F,H,W,3] (RGB order; grey files replicated).  islow
 * integer IDCT, fancy upsampling, jdcolor fixed-point YCbCr -> RGB: bit-exact to libjpeg's
 * defaults.  status int32 [F] gets the BF_JPG_* bits of a file that did not decode (its rows are
 * then undefined).  work: bf_jpeg_workspace_bytes(F, H, W) bytes of caller-owned device memory. */
#define BF_JPG_BAD_MARKER 1      /* no SOI, truncated / invalid marker segment, missing tables */
#define BF_JPG_UNSUPPORTED 2     /* progressive / arithmetic / 12-bit / 2 or 4 components / other sampling / multi-scan */
#define BF_JPG_SIZE 4            /* frame size != (W, H) */
#define BF_JPG_BAD_DATA 8        /* invalid Huffman code or coefficient index in the entropy data */
size_t bf_jpeg_workspace_bytes(int F, int H, int W);
int bf_jpeg_decode_rgb(const uint8_t* files, const int64_t* offsets, int F, int H, int W, uint8_t* rgb,
                       void* work, size_t work_bytes, int32_t* status, void* stream);

/* placement probe (diagnostic): n_wg workgroups on `stream`, each spinning `spin` cycles, write
 * out[2b] = HW_ID (CU bits 11:8, SH 12, SE 15:13) and out[2b+1] = XCC id -- which CUs a (CU-masked)
 * stream really runs on */
int bf_cu_probe(int* out, int n_wg, int spin, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BOXFUSION_HIP_H */
