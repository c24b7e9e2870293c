"""ctypes binding of libboxfusion_hip.so (the C-ABI in include/boxfusion_hip.h).

Every wrapper takes/returns torch tensors that live on the HIP device and launches on the current
torch stream.  There is deliberately no CPU fallback: if the shared library is missing or the
tensors are not on the GPU, the call raises.
"""
from __future__ import annotations

import atexit
import ctypes
import threading
import weakref
import sys
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# BF_LIB_PATH: a diagnostic build of the same sources (e.g. one that forces a rare kernel path)
LIB_PATH = os.environ.get("BF_LIB_PATH") or os.path.join(HERE, "libboxfusion_hip.so")
_LIB = None

c_int, c_float, c_double, c_void_p, c_size_t = (ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                                ctypes.c_void_p, ctypes.c_size_t)

BF_DEV_FUSION_LIST_OVERFLOW = 1
BF_DEV_HULL_OVERFLOW = 2
BF_DEV_VIEW_OVERFLOW = 4
BF_DEV_INDEX_RANGE = 8
BF_DEV_HULL_TRUNC = 16


class NmsCfg(ctypes.Structure):
    _fields_ = [("iou_threshold", c_double), ("translation_gap", c_float),
                ("rotation_gap", c_float), ("center_gap", c_double),
                ("max_list", c_int), ("list_capacity", c_int)]


class CorrCfg(ctypes.Structure):
    _fields_ = [("small_size", c_double), ("threshold", c_double),
                ("translation_gap", c_float), ("rotation_gap", c_float),
                ("W", c_float), ("H", c_float), ("max_list", c_int), ("list_capacity", c_int)]


class FuseCfg(ctypes.Structure):
    _fields_ = [("iters", c_int), ("pst_size", c_int), ("max_accept", c_int),
                ("legacy_promotion", c_int),
                ("center_init", c_double), ("shape_init", c_double),
                ("center_coef", c_double), ("shape_coef", c_double),
                ("beta", c_double), ("min_scale", c_double),
                ("img_h", c_float), ("img_w", c_float), ("K", c_float * 16)]


class FilterCfg(ctypes.Structure):
    _fields_ = [("score_thresh", c_float), ("floor_ratio", c_float), ("floor_half", c_float),
                ("size_max", c_float), ("gap_w", ctypes.c_int32), ("gap_h", ctypes.c_int32),
                ("W", ctypes.c_int32), ("H", ctypes.c_int32), ("use_score", ctypes.c_int32),
                ("use_uv", ctypes.c_int32), ("use_floor", ctypes.c_int32), ("use_large", ctypes.c_int32)]


class RowsField(ctypes.Structure):
    _fields_ = [("a", c_void_p), ("b", c_void_p), ("dst", c_void_p), ("n_a", ctypes.c_int64),
                ("n_b", ctypes.c_int64), ("row_bytes", ctypes.c_int32), ("pad", ctypes.c_int32)]


ROWS_MAX_FIELDS = 16


class HipError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise HipError(f"{LIB_PATH} is missing: build it with `python -m boxfusion_amd.build`")
        _LIB = ctypes.CDLL(LIB_PATH)
        _LIB.bf_version.restype = ctypes.c_char_p
        _LIB.bf_obb_iou_workspace_size.restype = c_size_t
        _LIB.bf_obb_iou_workspace_size.argtypes = [c_int]
        _LIB.bf_depth_standardize_workspace_size.restype = c_size_t
        _LIB.bf_depth_standardize_workspace_size.argtypes = [c_int, c_int, c_int]
    return _LIB


def _ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise HipError("boxfusion_amd kernels need device tensors (no CPU fallback)")
    if not t.is_contiguous():
        raise HipError("tensor must be contiguous")
    return c_void_p(t.data_ptr())


def _stream():
    # the raw handle of the calling thread's current stream (torch.cuda.current_stream() builds a
    # Stream object through several device-index lookups: ~10 us per call on the fusion path)
    return c_void_p(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))


def h2d(a, device, dtype=None):
    """host array -> device tensor without blocking the host: staged through pinned memory (torch's
    caching host allocator keeps the block until the copy is done) and copied asynchronously on
    the current stream.  A pageable copy waits until the stream has drained every earlier kernel,
    which on the fusion path is a hidden synchronisation per upload."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.pin_memory().to(device, non_blocking=True)


_SYNC_DEBUG = os.environ.get("BF_SYNC_DEBUG", "0") == "1"


def _check(rc, name):
    if rc != 0:
        raise HipError(f"{name} failed with bf_status {rc}")
    if _SYNC_DEBUG:   # debugging aid: attribute asynchronous faults to the launching entry point
        try:
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            raise HipError(f"{name}: device fault after launch: {e}") from e


def _need(t, dtype, name):
    if t.dtype != dtype:
        raise HipError(f"{name}: expected {dtype}, got {t.dtype}")
    return t


def version():
    return lib().bf_version().decode()


# ------------------------------------------------------------------------------------------
# geometry
# ------------------------------------------------------------------------------------------
def box_corners(xyzlhw, R):
    xyzlhw = _need(xyzlhw.contiguous(), torch.float32, "xyzlhw")
    R = _need(R.contiguous(), torch.float32, "R")
    n = xyzlhw.shape[0]
    out = torch.empty((n, 8, 3), dtype=torch.float32, device=xyzlhw.device)
    _check(lib().bf_box_corners(_ptr(xyzlhw), _ptr(R), c_int(n), _ptr(out), _stream()),
           "bf_box_corners")
    return out


def box_transform2world(xyzlhw, R, cam_pose):
    """in place on xyzlhw / R (both contiguous f32 device tensors)"""
    n = xyzlhw.shape[0]
    _check(lib().bf_box_transform2world(_ptr(xyzlhw), _ptr(R), _ptr(cam_pose.contiguous()),
                                        c_int(n), _stream()), "bf_box_transform2world")


def project_boxes(corners, cam_pose, K, W, H):
    n = corners.shape[0]
    uv = torch.empty((n, 8, 2), dtype=torch.float32, device=corners.device)
    _check(lib().bf_project_boxes(_ptr(corners.contiguous()), _ptr(cam_pose.contiguous()),
                                  _ptr(K.contiguous()), c_int(n), c_float(W), c_float(H), _ptr(uv),
                                  _stream()), "bf_project_boxes")
    return uv


def obb_iou_matrix(corners):
    corners = _need(corners.contiguous(), torch.float32, "corners")
    n = corners.shape[0]
    iou = torch.empty((n, n), dtype=torch.float64, device=corners.device)
    ws = torch.empty(max(1, int(lib().bf_obb_iou_workspace_size(n))), dtype=torch.uint8,
                     device=corners.device)
    _check(lib().bf_obb_iou_matrix(_ptr(corners), c_int(n), _ptr(iou), _ptr(ws), _stream()),
           "bf_obb_iou_matrix")
    return iou


# ------------------------------------------------------------------------------------------
# box-set rows (Instances3D.cat / __getitem__ over every field in one launch)
# ------------------------------------------------------------------------------------------
_ROWS_DT = np.dtype([("a", np.uint64), ("b", np.uint64), ("dst", np.uint64), ("n_a", np.int64),
                     ("n_b", np.int64), ("row_bytes", np.int32), ("pad", np.int32)])


_STATUS = {}


def status_word(device):
    """persistent int32 device word per (device, host thread) that rows_gather launches without a
    caller status OR their BF_DEV_* flags into (an out-of-range index skips its row);
    check_status() reads and clears it -- FusionStage does so at the read-back it already makes
    per keyframe.  One word per thread: the fusion worker's flags never mix with (or get cleared
    by) another thread's reads."""
    import threading
    d = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    key = (d, threading.get_ident())
    if key not in _STATUS:
        _STATUS[key] = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", d))
    return _STATUS[key]


def check_status(device, what="bf_rows_gather"):
    w = status_word(device)
    v = int(w.item())
    if v:
        w.zero_()
        if v & BF_DEV_INDEX_RANGE:
            raise HipError(f"{what}: index out of range (BF_DEV_INDEX_RANGE)")
        raise HipError(f"{what}: device status {v:#x}")


def rows_gather(pairs, idx=None, n_out=None, outs=None, status=None):
    """pairs: [(a, b or None[, narrow])] contiguous device tensors with the same row shape / dtype
    per pair (narrow=True: int64 rows written as int32);
    returns new tensors with rows idx of cat(a, b) (idx: int64 device tensor; None: the whole
    concatenation; int32 or int64); `outs`: write into these contiguous tensors instead (e.g. the
    tail rows of a preallocated table).  One bf_rows_gather launch for up to ROWS_MAX_FIELDS
    fields.  An index outside [0, len(a) + len(b)) sets BF_DEV_INDEX_RANGE in `status` (an int32
    device word the caller reads back), or else in the device's status_word()."""
    if idx is not None:
        n_out = int(idx.shape[0])
    elif n_out is None:
        a, b = pairs[0]
        n_out = a.shape[0] + (0 if b is None else b.shape[0])
    given, outs, recs = outs, [], []
    for k, pr in enumerate(pairs):
        a, b = pr[0], pr[1]
        narrow = len(pr) > 2 and pr[2]                  # int64 rows -> int32 output
        if given is not None:                           # caller's contiguous destinations
            out = given[k]
        else:
            out = torch.empty((n_out,) + a.shape[1:], dtype=torch.int32 if narrow else a.dtype,
                              device=a.device)
        nb = 0 if b is None else b.shape[0]
        # contiguous tensors: stride(0) = elements per row (also for 0-row tensors)
        recs.append((a.data_ptr(), b.data_ptr() if nb else 0, out.data_ptr(), a.shape[0], nb,
                     a.stride(0) * a.element_size() if a.dim() > 1 else a.element_size(),
                     1 if narrow else 0))
        outs.append(out)
    if pairs and n_out:
        arr = np.array(recs, dtype=_ROWS_DT)
        i32 = idx is not None and idx.dtype == torch.int32
        if status is None and idx is not None:
            status = status_word(outs[0].device)
        _check(lib().bf_rows_gather(c_void_p(arr.ctypes.data), c_int(len(pairs)), _ptr(idx), c_int(int(i32)),
                                    c_int(n_out), _ptr(status) if status is not None else None,
                                    _stream()), "bf_rows_gather")
    return outs


# ------------------------------------------------------------------------------------------
# association
# ------------------------------------------------------------------------------------------
def nms_scan(iou, corners, scores, init_id, cam_poses, fl_items, fl_len, valid_num, cfg: NmsCfg,
             out=None):
    """returns device tensors: keep, succ, events, counts (n_keep, n_success, n_events, status);
    `out` = (keep, succ, events, counts) preallocated views (e.g. of one buffer read back once)"""
    dev = iou.device
    n = scores.shape[0]
    i32 = dict(dtype=torch.int32, device=dev)
    if out is not None:
        keep, succ, events, counts = out
    else:
        keep = torch.empty(n + 1, **i32)
        succ = torch.empty(n + 1, **i32)
        events = torch.empty((n + 1, 3), **i32)
        counts = torch.zeros(4, **i32)  # n_keep, n_success, n_events, status
    L = lib()
    L.bf_nms_scan_workspace_size.restype = ctypes.c_size_t
    ws = torch.empty(max(int(L.bf_nms_scan_workspace_size(c_int(n))), 8), dtype=torch.uint8, device=dev)
    _check(L.bf_nms_scan_ws(_ptr(iou), _ptr(corners), _ptr(scores), _ptr(init_id),
                            _ptr(cam_poses), c_int(n), _ptr(fl_items), _ptr(fl_len),
                            _ptr(valid_num), _ptr(keep), _ptr(counts[0:1]), _ptr(succ),
                            _ptr(counts[1:2]), _ptr(events), _ptr(counts[2:3]),
                            _ptr(counts[3:4]), ctypes.byref(cfg), _ptr(ws), _stream()), "bf_nms_scan_ws")
    return keep, succ, events, counts


def corr_assoc(corners, dims, scores, boxes2d, init_id, cam_poses, cur_pose, K, n_glo, mask,
               success, fl_items, fl_len, valid_num, cfg: CorrCfg, out=None):
    """returns device tensors keep, events, counts (n_keep, n_events, status); `out` as nms_scan"""
    dev = corners.device
    n_all = scores.shape[0]
    i32 = dict(dtype=torch.int32, device=dev)
    if out is not None:
        keep, events, counts = out
    else:
        keep = torch.empty(max(1, mask.shape[0]), **i32)
        events = torch.empty((n_all + 1, 3), **i32)
        counts = torch.zeros(3, **i32)  # n_keep, n_events, status
    succ = success if success.numel() else torch.zeros(1, **i32)
    _check(lib().bf_corr_assoc(_ptr(corners), _ptr(dims), _ptr(scores), _ptr(boxes2d),
                               _ptr(init_id), _ptr(cam_poses), _ptr(cur_pose), _ptr(K),
                               c_int(n_all), c_int(n_glo), _ptr(mask), c_int(mask.shape[0]),
                               _ptr(succ), c_int(success.numel()), _ptr(fl_items), _ptr(fl_len),
                               _ptr(valid_num), _ptr(keep), _ptr(counts[0:1]), _ptr(events),
                               _ptr(counts[1:2]), _ptr(counts[2:3]), ctypes.byref(cfg),
                               _stream()), "bf_corr_assoc")
    return keep, events, counts


def corr_assoc_chained(corners, dims, scores, boxes2d, init_id, cam_poses, cur_pose, K, n_glo,
                       mask, n_mask, success, n_success, fl_items, fl_len, valid_num,
                       cfg: CorrCfg, out):
    """bf_corr_assoc_chained: correspondence association on nms_scan's device outputs (mask /
    n_mask = its keep / counts[0:1], success / n_success = its succ / counts[1:2]); `out` =
    (keep [n_all], events [n_all + 1, 3], counts [3]) preallocated device views"""
    keep, events, counts = out
    _check(lib().bf_corr_assoc_chained(
        _ptr(corners), _ptr(dims), _ptr(scores), _ptr(boxes2d), _ptr(init_id), _ptr(cam_poses),
        _ptr(cur_pose), _ptr(K), c_int(scores.shape[0]), c_int(n_glo), _ptr(mask), _ptr(n_mask),
        _ptr(success), _ptr(n_success), _ptr(fl_items), _ptr(fl_len), _ptr(valid_num), _ptr(keep),
        _ptr(counts[0:1]), _ptr(events), _ptr(counts[1:2]), _ptr(counts[2:3]), ctypes.byref(cfg),
        _stream()), "bf_corr_assoc_chained")
    return keep, events, counts


# ------------------------------------------------------------------------------------------
# fusion
# ------------------------------------------------------------------------------------------
def fusion_fit(view_off, n_views, view_box, view_R, view_score, view_pose, view_tc, pst,
               cfg: FuseCfg, trace=False, max_views=None, packed_out=False, packed=None):
    """max_views: host-known bound on n_views (avoids a device read when given).
    packed_out: return (out_box, packed, trace) with packed = int32 [updated(n_jobs),
    iterations(n_jobs), status] (one device->host copy for the caller); `packed` may be given
    (zeroed; its status word may already hold flags of an earlier launch: they are kept)."""
    dev = view_box.device
    n_jobs = view_off.shape[0]
    out_box = torch.empty((n_jobs, 6), dtype=torch.float32, device=dev)
    # updated flags, iteration counts and the status word in one buffer: one read-back
    if packed is None:
        packed = torch.zeros(2 * n_jobs + 1, dtype=torch.int32, device=dev)
    out_upd, out_it, status = packed[:n_jobs], packed[n_jobs:2 * n_jobs], packed[2 * n_jobs:]
    tr = (torch.empty((n_jobs, cfg.iters, cfg.pst_size), dtype=torch.float32, device=dev)
          if trace else None)
    if max_views is None:
        max_views = int(n_views.max().item()) if n_views.numel() else 1
    max_views = max(1, min(int(max_views), 32))
    L = lib()
    L.bf_fusion_fit_workspace_size.restype = ctypes.c_size_t
    nbytes = L.bf_fusion_fit_workspace_size(c_int(n_jobs), c_int(max_views), c_int(cfg.pst_size))
    ws = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
    _check(L.bf_fusion_fit(_ptr(view_off), _ptr(n_views), c_int(n_jobs), c_int(max_views),
                           _ptr(view_box), _ptr(view_R), _ptr(view_score), _ptr(view_pose),
                           _ptr(view_tc), _ptr(pst), ctypes.byref(cfg), _ptr(out_box),
                           _ptr(out_upd), _ptr(out_it), _ptr(tr), _ptr(status), _ptr(ws),
                           _stream()), "bf_fusion_fit")
    if packed_out:
        return out_box, packed, tr
    return out_box, out_upd, out_it, status, tr


def fusion_writeback(out_box, updated, rows, target):
    """target[rows[j], :6] = out_box[j] where updated[j] (bf_fusion_writeback); rows int32"""
    _need(target, torch.float32, "target")
    if not target.is_contiguous():
        raise HipError("fusion_writeback: target must be contiguous")
    _check(lib().bf_fusion_writeback(_ptr(out_box), _ptr(updated), _ptr(rows), c_int(rows.shape[0]),
                                     _ptr(target), c_int(target.shape[1]), _stream()),
           "bf_fusion_writeback")


def fusion_fitness(box, R, view_pose, view_tc, pst, search_size, cfg: FuseCfg):
    nv = view_pose.shape[0]
    out = torch.empty(pst.shape[0], dtype=torch.float32, device=box.device)
    _check(lib().bf_fusion_fitness(_ptr(box), _ptr(R), c_int(nv), _ptr(view_pose),
                                   _ptr(view_tc), _ptr(pst), c_int(pst.shape[0]),
                                   _ptr(search_size), ctypes.byref(cfg), _ptr(out), _stream()),
           "bf_fusion_fitness")
    return out


# ------------------------------------------------------------------------------------------
# keyframe sequencer (bf_fseq_*)
# ------------------------------------------------------------------------------------------
class FseqCfg(ctypes.Structure):
    _fields_ = [("nms", NmsCfg), ("corr", CorrCfg), ("fuse", FuseCfg), ("use_fusion", ctypes.c_int32),
                ("strict_hull", ctypes.c_int32)]


FSEQ_STATE_N = 16


class FusionSequencer:
    """Owner of one bf_fseq: the demo.py:200-305 keyframe sequence over batches of keyframes,
    all_pred_box on the device and BoxManager's lists in the library (include/boxfusion_hip.h).
    Calls launch on the calling thread's current stream."""

    def __init__(self):
        L = lib()
        L.bf_fseq_error.restype = ctypes.c_char_p
        L.bf_fseq_error.argtypes = [c_void_p]
        L.bf_fseq_destroy.restype = None
        L.bf_fseq_destroy.argtypes = [c_void_p]
        self._L = L
        self.h = c_void_p()
        _check(L.bf_fseq_create(ctypes.byref(self.h)), "bf_fseq_create")
        self._state = np.zeros(FSEQ_STATE_N, np.int64)
        _LIVE_SEQUENCERS.add(self)

    def close(self):
        """release the sequencer's device buffers and handle now (idempotent)"""
        h, L = getattr(self, "h", None), getattr(self, "_L", None)
        if h is not None and h.value and L is not None:
            L.bf_fseq_destroy(h)
        self.h = None

    def _rc(self, rc, name):
        if rc != 0:
            raise HipError(f"{name}: {self._L.bf_fseq_error(self.h).decode()} (bf_status {rc})")
        if _SYNC_DEBUG:
            torch.cuda.synchronize()

    def keyframes(self, cfg: FseqCfg, sizes, p_base, fields, K, pst):
        """sizes: int32 [n_kf]; fields: (box, R, score, box2d, pose, proj) of the per-frame table,
        contiguous f32 device tensors with p_rows rows"""
        sizes = np.ascontiguousarray(sizes, np.int32)
        p_rows = int(fields[0].shape[0])
        self._rc(self._L.bf_fseq_keyframes(
            self.h, ctypes.byref(cfg), c_int(len(sizes)), sizes.ctypes.data_as(c_void_p),
            ctypes.c_int64(int(p_base)), ctypes.c_int64(p_rows), *[_ptr(t) for t in fields], _ptr(K),
            _ptr(pst), _stream()), "bf_fseq_keyframes")

    def sync(self):
        self._rc(self._L.bf_fseq_sync(self.h), "bf_fseq_sync")

    def state(self):
        """bf_fseq_state (waits for the stream and applies a pending fusion result)"""
        self._rc(self._L.bf_fseq_state(self.h, self._state.ctypes.data_as(c_void_p)), "bf_fseq_state")
        return self._state.copy()

    def lists(self, which, rows, items):
        lens = np.zeros(max(rows, 1), np.int32)
        flat = np.zeros(max(items, 1), np.int32)
        self._rc(self._L.bf_fseq_lists(self.h, c_int(which), lens.ctypes.data_as(c_void_p),
                                       flat.ctypes.data_as(c_void_p)), "bf_fseq_lists")
        off = np.concatenate([[0], np.cumsum(lens[:rows])])
        fl = flat.tolist()
        return [fl[off[i]:off[i + 1]] for i in range(rows)]

    def flags(self, n):
        out = np.zeros(max(n, 1), np.int32)
        self._rc(self._L.bf_fseq_flags(self.h, out.ctypes.data_as(c_void_p)), "bf_fseq_flags")
        return out[:n].tolist()

    def global_rows(self, n, device):
        """all_pred_box's init_id (host int32), xyzlhw [n,6] and valid_num [n] (device copies)"""
        ids = np.zeros(max(n, 1), np.int32)
        xyz = torch.empty((n, 6), dtype=torch.float32, device=device)
        vn = torch.empty(n, dtype=torch.float32, device=device)
        self._rc(self._L.bf_fseq_global(self.h, ids.ctypes.data_as(c_void_p), _ptr(xyz) if n else None,
                                        _ptr(vn) if n else None, _stream()), "bf_fseq_global")
        return ids[:n], xyz, vn

    def __del__(self, _finalizing=sys.is_finalizing):
        if _finalizing():             # interpreter exit: _shutdown() already released it
            return
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter teardown: the process frees everything
            pass


def filter_cfg(det_cfg, W, H):
    """FilterCfg from a config's `detection` section (demo.py:138-148 keys)"""
    c = FilterCfg()
    c.use_score = 1
    c.score_thresh = float(np.float32(det_cfg.get("score_thresh", 0.0)))
    c.use_uv = int(bool(det_cfg.get("uv_bound", False)))
    ratio = float(det_cfg.get("uv_bound_value", 1.0))
    c.gap_w, c.gap_h = int((1 - ratio) * W), int((1 - ratio) * H)     # python float, as the reference
    c.W, c.H = int(W), int(H)
    c.use_floor = int(bool(det_cfg.get("floor_mask", False)))
    fr = float(det_cfg.get("floor_ratio", 20))
    c.floor_ratio, c.floor_half = float(np.float32(fr)), float(np.float32(fr / 2))
    lg = det_cfg.get("size_max_thres")
    c.use_large = int(bool(lg))
    c.size_max = float(np.float32(lg)) if lg else 0.0
    return c


def detection_filter(scores, proj_xy, box3d, cfg: FilterCfg, with_bits=False):
    """keep mask (bool, shape of scores) of the demo.py:138-148 filters (bf_detection_filter)"""
    n = scores.numel()
    keep = torch.empty(scores.shape, dtype=torch.uint8, device=scores.device)
    bits = torch.empty(scores.shape, dtype=torch.uint8, device=scores.device) if with_bits else None
    _check(lib().bf_detection_filter(_ptr(_need(scores.contiguous(), torch.float32, "scores")),
                                     _ptr(_need(proj_xy.contiguous(), torch.float32, "proj_xy")),
                                     _ptr(_need(box3d.contiguous(), torch.float32, "box3d")),
                                     c_int(n), ctypes.byref(cfg), _ptr(keep), _ptr(bits), _stream()),
           "bf_detection_filter")
    return (keep.bool(), bits) if with_bits else keep.bool()


# ------------------------------------------------------------------------------------------
# per-frame depth
# ------------------------------------------------------------------------------------------
_DS_WS = {}


def depth_workspace(b, h, w, device):
    """zero-filled workspace of bf_depth_standardize / bf_depth_preprocess, one per (device,
    stream, shape): the kernels leave it zeroed, so it is reused as is by stream-ordered calls.
    Not for graph captures: a captured launch keeps the address, so replays on another stream
    would race the eager users of the cached buffer -- depth_preprocess therefore requires an
    explicit caller-owned `ws` (new_depth_workspace) while the current stream is capturing."""
    dev = torch.device(device)
    stream = torch.cuda.current_stream(dev).cuda_stream
    key = (dev.index, stream, b, h, w)
    ws = _DS_WS.get(key)
    if ws is None:
        size = int(lib().bf_depth_standardize_workspace_size(c_int(b), c_int(h), c_int(w)))
        ws = torch.zeros(max(size, 1), dtype=torch.uint8, device=dev)
        _DS_WS[key] = ws
    return ws


def depth_standardize(depth, out=None, params=None):
    """depth f32[b,h,w] -> (standardised f32[b,h,w], params f32[b,2])"""
    return depth_preprocess(depth, out=out, params=params)


def depth_preprocess(depth, K=None, RT=None, max_depth=10.0, out=None, params=None, xyz=None, valid=None,
                     ws=None):
    """demo.py:121-131 per-frame depth work for a batch: depth f32[b,h,w] -> (standardised,
    params f32[b,2]) and, with K f32[b,3,3] / RT f32[b,4,4], the back-projection (xyz f32[b,h,w,3],
    valid bool[b,h,w]) from the same pass.  ws: a zero-filled workspace of
    bf_depth_standardize_workspace_size bytes owned by the caller (default: one per stream)"""
    depth = _need(depth.contiguous(), torch.float32, "depth")
    if not depth.is_cuda:
        raise HipError("bf_depth_preprocess: depth must be a device tensor (no CPU path)")
    b, h, w = depth.shape
    out = torch.empty_like(depth) if out is None else out
    params = torch.empty((b, 2), dtype=torch.float32, device=depth.device) if params is None else params
    bp = K is not None
    if bp:
        K = _need(K.contiguous(), torch.float32, "K")
        RT = _need(RT.contiguous(), torch.float32, "RT")
        if K.shape != (b, 3, 3) or RT.shape != (b, 4, 4):
            raise HipError(f"bf_depth_preprocess: K {tuple(K.shape)} / RT {tuple(RT.shape)} for {b} frames")
        xyz = torch.empty((b, h, w, 3), dtype=torch.float32, device=depth.device) if xyz is None else xyz
        valid = torch.empty((b, h, w), dtype=torch.uint8, device=depth.device) if valid is None else valid
    if ws is None:
        if torch.cuda.is_current_stream_capturing():
            raise HipError("bf_depth_preprocess under graph capture needs a caller-owned ws "
                           "(new_depth_workspace): the per-stream cached workspace is shared")
        ws = depth_workspace(b, h, w, depth.device)
    _check(lib().bf_depth_preprocess(_ptr(depth), c_int(b), c_int(h), c_int(w), _ptr(out), _ptr(params),
                                     _ptr(K) if bp else None, _ptr(RT) if bp else None,
                                     c_float(max_depth if max_depth is not None else 0.0),
                                     _ptr(xyz) if bp else None, _ptr(valid) if bp else None, _ptr(ws),
                                     _stream()), "bf_depth_preprocess")
    if bp:
        return out, params, xyz, valid.view(torch.bool)
    return out, params


def backproject(depth, K, RT, max_depth=10.0):
    h, w = depth.shape
    xyz = torch.empty((h, w, 3), dtype=torch.float32, device=depth.device)
    valid = torch.empty((h, w), dtype=torch.uint8, device=depth.device)
    _check(lib().bf_backproject(_ptr(depth.contiguous()), _ptr(K.contiguous()),
                                _ptr(RT.contiguous()), c_int(h), c_int(w),
                                c_float(max_depth if max_depth is not None else 0.0), _ptr(xyz),
                                _ptr(valid), _stream()), "bf_backproject")
    return xyz, valid.bool()


# ------------------------------------------------------------------------------------------
# MFMA tower kernels
# ------------------------------------------------------------------------------------------
ACT = {None: 0, "none": 0, "gelu": 1, "relu": 2}


class GemmPlan(ctypes.Structure):
    """bf_gemm_plan: per-call GEMM options (include/boxfusion_hip.h); all-zero = product defaults"""
    _fields_ = [("cu_budget", ctypes.c_int32), ("tile_rows", ctypes.c_int32), ("kernel", ctypes.c_int32),
                ("variant", ctypes.c_int32), ("group_m", ctypes.c_int32), ("balanced", ctypes.c_int32)]


# The CU budget a thread's GEMMs pass in their plan (0 = every CU).  Host-side, per thread: the C
# library keeps no GEMM state; the thread that launches on a CU-masked detect stream sets it
# (partition_streams), a fusion worker thread keeps 0.
_TLS = threading.local()


def set_cu_budget(n):
    """CUs the calling thread's GEMMs size their persistent grid for (0 = all)"""
    _TLS.cu_budget = max(int(n), 0)


def cu_budget():
    return getattr(_TLS, "cu_budget", 0)


def set_knobs(**kw):
    """measurement hooks for scripts/ (not used by the product path): per-thread defaults merged into
    the bf_gemm_plan of every GEMM call made without a plan (GemmPlan field names) and into every
    attention call made without a variant (attn_variant=...).  set_knobs() with no arguments clears
    them."""
    _TLS.knobs = {**getattr(_TLS, "knobs", {}), **kw} if kw else {}


def _knobs():
    return getattr(_TLS, "knobs", {})


def _plan(plan):
    if plan is None:
        k = {f: v for f, v in _knobs().items() if f != "attn_variant"}
        b = cu_budget()
        if not b and not k:
            return None
        plan = GemmPlan(**{"cu_budget": b, **k})
    elif isinstance(plan, dict):
        plan = GemmPlan(**{"cu_budget": cu_budget(), **plan})
    return ctypes.byref(plan)


def gemm(a, w, bias=None, act=None, resid=None, resid_mod=0, out=None, out_dtype=torch.bfloat16,
         row_map=None, m=None, plan=None):
    """out[orow(r)] = resid[...] + act(a @ w.T + bias); a bf16 [M,K] (row stride a.stride(0)),
    w bf16 [N,K]. `out` may be given (its row stride is used).  plan: None (defaults + the
    thread's CU budget), a GemmPlan or a dict of its fields (measurement hooks)."""
    _need(a, torch.bfloat16, "a")
    _need(w, torch.bfloat16, "w")
    M = a.shape[0] if m is None else m
    N, K = w.shape
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    c_bf16 = 1 if out.dtype == torch.bfloat16 else 0
    if not c_bf16 and out.dtype != torch.float32:
        raise HipError("gemm output must be bf16 or f32")
    if resid is not None:
        _need(resid, torch.float32, "resid")
    if bias is not None:
        _need(bias, torch.float32, "bias")
    if a.stride(1) != 1 or w.stride(1) != 1 or out.stride(1) != 1:
        raise HipError("gemm operands need unit column stride")
    _check(lib().bf_gemm_bf16_plan(c_void_p(a.data_ptr()), c_int(a.stride(0)), c_void_p(w.data_ptr()),
                                   c_int(w.stride(0)), _ptr(bias) if bias is not None else None,
                                   c_void_p(resid.data_ptr()) if resid is not None else None,
                                   c_int(resid.stride(0) if resid is not None else 0), c_int(resid_mod),
                                   c_void_p(out.data_ptr()), c_int(out.stride(0)), c_int(c_bf16),
                                   _ptr(row_map) if row_map is not None else None, c_int(M), c_int(N),
                                   c_int(K), c_int(ACT[act]), _plan(plan), _stream()), "bf_gemm_bf16")
    return out


def attention(q, k, v, o, batch, heads, sq, sk, head_dim, scale, q_bs=None, k_bs=None, v_bs=None,
              o_bs=None, o_map=None, variant=0):
    """q/k/v/o are 2-D token-major views [batch*S, >= heads*head_dim] (any row stride).
    o_map: int32 [batch*sq] output row of each query (< 0: not stored).  variant: the per-call
    kernel-variant hook of bf_attention_bf16_ex (0 = default)."""
    for x, n in ((q, "q"), (k, "k"), (v, "v"), (o, "o")):
        _need(x, torch.bfloat16, n)
    q_bs = sq * q.stride(0) if q_bs is None else q_bs
    k_bs = sk * k.stride(0) if k_bs is None else k_bs
    v_bs = sk * v.stride(0) if v_bs is None else v_bs
    o_bs = sq * o.stride(0) if o_bs is None else o_bs
    if o_map is not None:
        _need(o_map, torch.int32, "o_map")
        if o_map.numel() < batch * sq:
            raise HipError(f"o_map has {o_map.numel()} rows < batch*sq = {batch * sq}")
    LL = ctypes.c_longlong
    _check(lib().bf_attention_bf16_ex(c_void_p(q.data_ptr()), c_void_p(k.data_ptr()),
                                      c_void_p(v.data_ptr()), c_void_p(o.data_ptr()), c_int(batch),
                                      c_int(heads), c_int(sq), c_int(sk), c_int(head_dim),
                                      c_int(q.stride(0)), c_int(k.stride(0)), c_int(v.stride(0)),
                                      c_int(o.stride(0)), LL(q_bs), LL(k_bs), LL(v_bs), LL(o_bs),
                                      c_float(scale), _ptr(o_map) if o_map is not None else None,
                                      c_int(variant or _knobs().get("attn_variant", 0)), _stream()),
           "bf_attention_bf16_ex")
    return o


def attention_fp8out(q, k, v, o, batch, heads, sq, sk, head_dim, scale, out_qscale, q_bs=None,
                     k_bs=None, v_bs=None, o_bs=None, variant=0):
    """attention() with an fp8 e4m3 output o = saturate(softmax(q k^T) v * out_qscale)"""
    for x, n in ((q, "q"), (k, "k"), (v, "v")):
        _need(x, torch.bfloat16, n)
    _need(o, FP8, "o")
    q_bs = sq * q.stride(0) if q_bs is None else q_bs
    k_bs = sk * k.stride(0) if k_bs is None else k_bs
    v_bs = sk * v.stride(0) if v_bs is None else v_bs
    o_bs = sq * o.stride(0) if o_bs is None else o_bs
    LL = ctypes.c_longlong
    _check(lib().bf_attention_fp8out_ex(c_void_p(q.data_ptr()), c_void_p(k.data_ptr()), c_void_p(v.data_ptr()),
                                        c_void_p(o.data_ptr()), c_int(batch), c_int(heads), c_int(sq),
                                        c_int(sk), c_int(head_dim), c_int(q.stride(0)), c_int(k.stride(0)),
                                        c_int(v.stride(0)), c_int(o.stride(0)), LL(q_bs), LL(k_bs), LL(v_bs),
                                        LL(o_bs), c_float(scale), c_float(out_qscale),
                                        c_int(variant or _knobs().get("attn_variant", 0)), _stream()),
           "bf_attention_fp8out_ex")
    return o


def layernorm(x, weight, bias, eps, out=None, row_map=None, out_dtype=torch.bfloat16):
    """x f32 [M, C] (any row stride) -> LayerNorm rows in bf16 (or f32: out / out_dtype), row r
    written to row_map[r] of out (< 0 skipped)"""
    _need(x, torch.float32, "x")
    M, C = x.shape
    if out is None:
        out = torch.empty((M, C), dtype=out_dtype, device=x.device)
    if out.dtype not in (torch.bfloat16, torch.float32) or x.stride(1) != 1 or out.stride(1) != 1:
        raise HipError("layernorm: f32 in, bf16 / f32 out, unit column stride")
    _check(lib().bf_layernorm_out(c_void_p(x.data_ptr()), c_int(x.stride(0)), _ptr(weight),
                                  _ptr(bias), c_float(eps), c_void_p(out.data_ptr()),
                                  c_int(out.stride(0)), c_int(int(out.dtype == torch.float32)),
                                  _ptr(row_map) if row_map is not None else None, c_int(M), c_int(C),
                                  _stream()), "bf_layernorm_out")
    return out



def attention_causal(q, k, v, o, batch, heads, s, head_dim, scale):
    """causal self-attention (CLIP text tower): q/k/v/o token-major 2-D views [batch*s, >= heads*D]"""
    for x, n in ((q, "q"), (k, "k"), (v, "v"), (o, "o")):
        _need(x, torch.bfloat16, n)
    LL = ctypes.c_longlong
    _check(lib().bf_attention_causal(c_void_p(q.data_ptr()), c_void_p(k.data_ptr()), c_void_p(v.data_ptr()),
                                     c_void_p(o.data_ptr()), c_int(batch), c_int(heads), c_int(s),
                                     c_int(head_dim), c_int(q.stride(0)), c_int(k.stride(0)),
                                     c_int(v.stride(0)), c_int(o.stride(0)), LL(s * q.stride(0)),
                                     LL(s * k.stride(0)), LL(s * v.stride(0)), LL(s * o.stride(0)),
                                     c_float(scale), _stream()), "bf_attention_causal")
    return o


def token_embed(ids, table, pos, out=None, status=None):
    """ids i32 [N, S] -> table[ids] + pos, f32 [N*S, W]; an out-of-range id raises HipError"""
    _need(ids, torch.int32, "ids")
    _need(table, torch.float32, "table")
    _need(pos, torch.float32, "pos")
    N, S = ids.shape
    W = table.shape[1]
    if pos.shape[0] < S or pos.shape[1] != W:
        raise HipError(f"token_embed: positional table {tuple(pos.shape)} for S={S}, W={W}")
    if out is None:
        out = torch.empty((N * S, W), dtype=torch.float32, device=ids.device)
    _need(out, torch.float32, "out")
    own = status is None
    if own:
        status = torch.zeros(1, dtype=torch.int32, device=ids.device)
    _check(lib().bf_token_embed(_ptr(ids), c_int(N * S), _ptr(table), c_int(table.shape[0]), _ptr(pos),
                                c_int(S), c_int(W), _ptr(out), _ptr(status), _stream()), "bf_token_embed")
    if own and int(status.item()) & BF_DEV_INDEX_RANGE:
        raise HipError("bf_token_embed: a token id outside the vocabulary (BF_DEV_INDEX_RANGE)")
    return out


def text_pool(ids, x, out=None):
    """x f32 [N*S, W] -> x[n*S + argmax(ids[n])] f32 [N, W] (open_clip 'argmax' text pooling)"""
    _need(ids, torch.int32, "ids")
    _need(x, torch.float32, "x")
    N, S = ids.shape
    W = x.shape[1]
    if out is None:
        out = torch.empty((N, W), dtype=torch.float32, device=x.device)
    _need(out, torch.float32, "out")
    _check(lib().bf_text_pool(_ptr(ids), c_int(N), c_int(S), _ptr(x), c_int(W), _ptr(out), _stream()),
           "bf_text_pool")
    return out


def l2_normalize_rows(x, out=None):
    """x f32 [R, W] -> x / ||x||_2 per row (out may be x)"""
    _need(x, torch.float32, "x")
    if out is None:
        out = torch.empty_like(x)
    _need(out, torch.float32, "out")
    _check(lib().bf_l2_normalize_rows(_ptr(x), c_int(x.shape[0]), c_int(x.shape[1]), _ptr(out), _stream()),
           "bf_l2_normalize_rows")
    return out


def ingest_rgbd(bgr, depth_u16, depth_scale, rot_k=0, rgb_out=None, depth_out=None, src_bgr=True):
    """decoded frames -> sample tensors (capture_stream.py:194-311): bgr u8 [F,Hc,Wc,3], depth
    int16/uint16 [F,Hd,Wd] (or None) -> rgb u8 [F,3,Ho,Wo] (RGB, cv2-resized to the depth size,
    rot90 k) and depth f32 [F,Ho,Wo] = depth / depth_scale (rot90 k)"""
    _need(bgr, torch.uint8, "bgr")
    if bgr.dim() == 3:
        bgr = bgr[None]
    F_, Hc, Wc, C = bgr.shape
    if C != 3:
        raise HipError("ingest_rgbd: BGR frames [F,H,W,3]")
    if depth_u16 is not None:
        if depth_u16.dtype not in (torch.uint16, torch.int16):
            raise HipError(f"depth: expected a 16-bit PNG map, got {depth_u16.dtype}")
        if depth_u16.dim() == 2:
            depth_u16 = depth_u16[None]
        if depth_u16.shape[0] != F_:
            raise HipError("ingest_rgbd: one depth map per frame")
        Hd, Wd = depth_u16.shape[1:]
    else:
        Hd, Wd = Hc, Wc
    k = rot_k % 4
    Ho, Wo = (Wd, Hd) if k % 2 else (Hd, Wd)
    if rgb_out is None:
        rgb_out = torch.empty((F_, 3, Ho, Wo), dtype=torch.uint8, device=bgr.device)
    _need(rgb_out, torch.uint8, "rgb_out")
    if depth_u16 is not None and depth_out is None:
        depth_out = torch.empty((F_, Ho, Wo), dtype=torch.float32, device=bgr.device)
    _check(lib().bf_ingest_rgbd(_ptr(bgr), c_int(Hc), c_int(Wc), _ptr(depth_u16), c_int(Hd), c_int(Wd),
                                c_int(F_), c_float(depth_scale), c_int(k), c_int(int(bool(src_bgr))), _ptr(rgb_out),
                                _ptr(depth_out) if depth_u16 is not None else None, _stream()),
           "bf_ingest_rgbd")
    return rgb_out, depth_out


PNG_STATUS = {1: "bad signature", 2: "bad IHDR", 4: "unsupported PNG kind", 8: "bad chunk list",
              16: "bad zlib / deflate stream", 32: "Adler-32 mismatch", 64: "bad row filter", 128: "size mismatch"}


def png_decode_u16(files, offsets, H, W, out=None, offsets_host=None, check=True, depth_scale=None, work=None):
    """cv2.imread(path, IMREAD_UNCHANGED) for F 16-bit greyscale PNGs (capture_stream.py:197/:405):
    files u8 [total] device bytes of the files back to back, offsets int64 [F+1] device (and the
    same offsets on the host, `offsets_host`, to size the launch) -> out u16 [F,H,W] and the int32
    status word per file.  depth_scale given: out f32 [F,H,W] = sample / depth_scale
    (capture_stream.py:203, bf_png_decode_depth).  check=True synchronises and raises on any file
    that did not decode."""
    _need(files, torch.uint8, "files")
    _need(offsets, torch.int64, "offsets")
    if offsets_host is None:
        offsets_host = offsets.cpu()
    oh = [int(v) for v in offsets_host]
    F_ = len(oh) - 1
    if F_ < 0 or offsets.numel() != F_ + 1:
        raise HipError("png_decode_u16: offsets [F+1]")
    total = oh[-1] if F_ >= 0 else 0
    if total > files.numel():
        raise HipError("png_decode_u16: offsets run past the file bytes")
    mx = max((oh[i + 1] - oh[i] for i in range(F_)), default=0)
    wb = png_workspace_bytes(F_, H, W, total)
    if work is None or work.numel() < wb:
        work = torch.empty(max(wb, 1), dtype=torch.uint8, device=files.device)
    dt = torch.uint16 if depth_scale is None else torch.float32
    if out is None:
        out = torch.empty((F_, H, W), dtype=dt, device=files.device)
    _need(out, dt, "out")
    if out.numel() != F_ * H * W:
        raise HipError("png_decode_u16: out [F,H,W]")
    status = torch.zeros(max(F_, 1), dtype=torch.int32, device=files.device)
    if depth_scale is None:
        rc = lib().bf_png_decode_u16(_ptr(files), _ptr(offsets), c_int(F_), c_int(H), c_int(W), ctypes.c_longlong(total),
                                     ctypes.c_longlong(mx), _ptr(out), _ptr(work), c_size_t(wb), _ptr(status),
                                     _stream())
    else:
        rc = lib().bf_png_decode_depth(_ptr(files), _ptr(offsets), c_int(F_), c_int(H), c_int(W),
                                       ctypes.c_longlong(total), ctypes.c_longlong(mx), c_float(depth_scale),
                                       _ptr(out), _ptr(work), c_size_t(wb), _ptr(status), _stream())
    _check(rc, "bf_png_decode")
    if check and F_:
        st = status[:F_].cpu()
        bad = torch.nonzero(st).flatten().tolist()
        if bad:
            f = bad[0]
            why = ", ".join(v for k, v in PNG_STATUS.items() if int(st[f]) & k)
            raise HipError(f"png_decode_u16: {len(bad)} of {F_} files did not decode (file {f}: {why})")
    return out, status[:F_]


def png_workspace_bytes(F, H, W, total_file_bytes):
    L = lib()
    L.bf_png_workspace_bytes.restype = c_size_t
    L.bf_png_workspace_bytes.argtypes = [c_int, c_int, c_int, ctypes.c_longlong]
    return int(L.bf_png_workspace_bytes(F, H, W, total_file_bytes))


JPEG_STATUS = {1: "bad / missing marker segment", 2: "unsupported JPEG kind (not baseline 1/3-component h2v2/h2v1/h1v1)",
               4: "size mismatch", 8: "corrupt entropy-coded data"}


def jpeg_decode_rgb(files, offsets, H, W, out=None, check=True, work=None):
    """cv2.imread(color_path) for F baseline JPEGs (capture_stream.py:194/:402), in RGB order (the
    cvtColor(BGR2RGB) of the streams folded in): files u8 [total] device bytes back to back, offsets
    int64 [F+1] device -> out u8 [F,H,W,3] and the int32 status word per file (BF_JPG_* bits).
    check=True synchronises and raises on any file that did not decode."""
    _need(files, torch.uint8, "files")
    _need(offsets, torch.int64, "offsets")
    F_ = offsets.numel() - 1
    if F_ < 0:
        raise HipError("jpeg_decode_rgb: offsets [F+1]")
    wb = jpeg_workspace_bytes(F_, H, W)
    if work is None or work.numel() < wb:
        work = torch.empty(max(wb, 1), dtype=torch.uint8, device=files.device)
    if out is None:
        out = torch.empty((F_, H, W, 3), dtype=torch.uint8, device=files.device)
    _need(out, torch.uint8, "out")
    if out.numel() != F_ * H * W * 3:
        raise HipError("jpeg_decode_rgb: out [F,H,W,3]")
    status = torch.zeros(max(F_, 1), dtype=torch.int32, device=files.device)
    _check(lib().bf_jpeg_decode_rgb(_ptr(files), _ptr(offsets), c_int(F_), c_int(H), c_int(W), _ptr(out), _ptr(work),
                                    c_size_t(wb), _ptr(status), _stream()), "bf_jpeg_decode_rgb")
    if check and F_:
        st = status[:F_].cpu()
        bad = torch.nonzero(st).flatten().tolist()
        if bad:
            f = bad[0]
            why = ", ".join(v for k, v in JPEG_STATUS.items() if int(st[f]) & k)
            raise HipError(f"jpeg_decode_rgb: {len(bad)} of {F_} files did not decode (file {f}: {why})")
    return out, status[:F_]


def jpeg_workspace_bytes(F, H, W):
    L = lib()
    L.bf_jpeg_workspace_bytes.restype = c_size_t
    L.bf_jpeg_workspace_bytes.argtypes = [c_int, c_int, c_int]
    return int(L.bf_jpeg_workspace_bytes(F, H, W))


def cv2_resize_u8(src, Wd, Hd, out=None):
    """cv2.resize(src, (Wd, Hd)) (u8 INTER_LINEAR) of u8 images [H,W], [H,W,cn] or [F,H,W,cn]"""
    _need(src, torch.uint8, "src")
    x = src
    if x.dim() == 2:
        x = x[None, :, :, None]
    elif x.dim() == 3:
        x = x[None]
    F_, Hs, Ws, cn = x.shape
    if out is None:
        out = torch.empty((F_, Hd, Wd, cn), dtype=torch.uint8, device=src.device)
    _check(lib().bf_cv2_resize_u8(_ptr(x), c_int(Hs), c_int(Ws), c_int(cn), c_int(Hd), c_int(Wd), c_int(F_),
                                  _ptr(out), _stream()), "bf_cv2_resize_u8")
    if src.dim() == 2:
        return out[0, :, :, 0]
    return out[0] if src.dim() == 3 else out

FP8 = torch.float8_e4m3fn      # OCP e4m3 (gfx950's fp8; not the MI300 fnuz variant)
FP8_MAX = 448.0
_FP8_OUT = {torch.float32: 0, torch.bfloat16: 1, FP8: 2}


def gemm_fp8(a, w, scale, bias=None, act=None, resid=None, out=None, out_dtype=torch.bfloat16,
             out_qscale=1.0, plan=None):
    """out = resid + act(scale * (a @ w.T) + bias); a fp8 e4m3 [M,K], w fp8 [N,K] (per-tensor
    scales folded into `scale`); out f32 / bf16 / fp8 (fp8: saturate(value * out_qscale))."""
    _need(a, FP8, "a")
    _need(w, FP8, "w")
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise HipError(f"gemm_fp8: a K={K} vs w K={w.shape[1]}")
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=a.device)
    if out.dtype not in _FP8_OUT:
        raise HipError("gemm_fp8 output must be f32, bf16 or fp8")
    if resid is not None:
        _need(resid, torch.float32, "resid")
    if bias is not None:
        _need(bias, torch.float32, "bias")
    if a.stride(1) != 1 or w.stride(1) != 1 or out.stride(1) != 1:
        raise HipError("gemm_fp8 operands need unit column stride")
    _check(lib().bf_gemm_fp8_plan(c_void_p(a.data_ptr()), c_int(a.stride(0)), c_void_p(w.data_ptr()),
                                  c_int(w.stride(0)), c_float(scale), _ptr(bias) if bias is not None else None,
                                  c_void_p(resid.data_ptr()) if resid is not None else None,
                                  c_int(resid.stride(0) if resid is not None else 0), c_void_p(out.data_ptr()),
                                  c_int(out.stride(0)), c_int(_FP8_OUT[out.dtype]), c_float(out_qscale),
                                  c_int(M), c_int(N), c_int(K), c_int(ACT[act]), _plan(plan), _stream()),
           "bf_gemm_fp8")
    return out


def layernorm_fp8(x, weight, bias, eps, qscale, out=None):
    """x f32 [M, C] -> fp8 e4m3 saturate(LayerNorm(x) * qscale)"""
    _need(x, torch.float32, "x")
    M, C = x.shape
    if out is None:
        out = torch.empty((M, C), dtype=FP8, device=x.device)
    _need(out, FP8, "out")
    if x.stride(1) != 1 or out.stride(1) != 1:
        raise HipError("layernorm_fp8: unit column stride")
    _check(lib().bf_layernorm_fp8(c_void_p(x.data_ptr()), c_int(x.stride(0)), _ptr(weight), _ptr(bias),
                                  c_float(eps), c_void_p(out.data_ptr()), c_int(out.stride(0)),
                                  c_float(qscale), c_int(M), c_int(C), _stream()), "bf_layernorm_fp8")
    return out


def _f3(vals):
    return (c_float * 3)(*[float(v) for v in vals])


def im2col_rgb8(img, pad, patch, mean, std, out=None, chw=False):
    """img u8 [B,H,W,3] (chw=True: [B,3,H,W]) -> bf16 [B*(pad/patch)^2, 3*patch*patch]"""
    _need(img, torch.uint8, "img")
    if chw:
        B, _, H, W = img.shape
    else:
        B, H, W, _ = img.shape
    n = B * (pad // patch) ** 2
    if out is None:
        out = torch.empty((n, 3 * patch * patch), dtype=torch.bfloat16, device=img.device)
    _check(lib().bf_im2col_rgb8_chw(_ptr(img), c_int(B), c_int(H), c_int(W), c_int(int(chw)),
                                    c_int(pad), c_int(patch), _f3(mean), _f3(std),
                                    c_void_p(out.data_ptr()), c_int(out.stride(0)), _stream()),
           "bf_im2col_rgb8_chw")
    return out


def im2col_f32(x, pad, patch, out=None):
    _need(x, torch.float32, "x")
    B, H, W = x.shape
    n = B * (pad // patch) ** 2
    if out is None:
        out = torch.empty((n, patch * patch), dtype=torch.bfloat16, device=x.device)
    _check(lib().bf_im2col_f32(_ptr(x), c_int(B), c_int(H), c_int(W), c_int(pad), c_int(patch),
                               c_void_p(out.data_ptr()), c_int(out.stride(0)), _stream()),
           "bf_im2col_f32")
    return out


def crop_resize_im2col(img, boxes, img_idx, size, patch, mean, std, kpad, out=None):
    """img u8 [F,H,W,3]; boxes i32 [N,4]; img_idx i32 [N] -> bf16 [N*(size/patch)^2, kpad]"""
    _need(img, torch.uint8, "img")
    F, H, W, _ = img.shape
    N = boxes.shape[0]
    if out is None:
        out = torch.empty((N * (size // patch) ** 2, kpad), dtype=torch.bfloat16,
                          device=img.device)
    _check(lib().bf_crop_resize_im2col(_ptr(img), c_int(H), c_int(W), _ptr(boxes),
                                       _ptr(img_idx) if img_idx is not None else None, c_int(N),
                                       c_int(size), c_int(patch), _f3(mean), _f3(std),
                                       c_void_p(out.data_ptr()), c_int(out.stride(0)), _stream()),
           "bf_crop_resize_im2col")
    return out


class KernelTimer:
    """HIP-event timing of the MFMA tower launches (bench.py's roofline objects): while active,
    every bf_gemm_bf16 and bf_attention_bf16 launch made from Python is bracketed by two events
    on the launch stream and recorded with its algorithmic FLOPs and bytes:
      gemm       2*M*N*K FLOPs; bytes A + W + out (+ the f32 residual read)
      attention  4*Sq*Sk*D FLOPs per (batch, head); bytes Q + K + V read + O written
    `summary(pred)` aggregates the records selected by pred(tags)."""

    def __init__(self):
        self.records = []      # (tags, flops, bytes, start event, end event)
        self.active = False

    def __enter__(self):
        global _TIMER
        import threading
        self.thread = threading.get_ident()     # records launches made from this thread only
        _TIMER = self
        self.active = True
        return self

    def __exit__(self, *exc):
        global _TIMER
        _TIMER = None
        self.active = False

    def record(self, tags, flops, nbytes, fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        self.records.append((tags, flops, nbytes, s, e))
        return r

    def summary(self, pred=lambda tags: True):
        torch.cuda.synchronize()
        sel = [r for r in self.records if pred(r[0])]
        if not sel:
            return dict(launches=0, flops=0.0, bytes=0.0, ms=0.0)
        ms = sum(s.elapsed_time(e) for _, _, _, s, e in sel)
        # work may be a callable resolved now (e.g. particle-views from the iteration counts a
        # fusion launch wrote)
        fl = sum(f() if callable(f) else f for _, f, _, _, _ in sel)
        nb = sum(b for _, _, b, _, _ in sel)
        return dict(launches=len(sel), flops=fl, bytes=nb, ms=ms, avg_us=1e3 * ms / len(sel),
                    tflops=fl / (ms * 1e-3) / 1e12, gbs=nb / (ms * 1e-3) / 1e9,
                    flops_per_launch=fl / len(sel), bytes_per_launch=nb / len(sel))


_TIMER = None


def _timer():
    """the active KernelTimer if it was entered on this thread (a fusion worker thread's
    launches are not recorded by the detect thread's timer)"""
    t = _TIMER
    if t is None:
        return None
    import threading
    return t if t.thread == threading.get_ident() else None


_gemm_untimed = gemm
_gemm_fp8_untimed = gemm_fp8
_attention_untimed = attention
_attention_fp8out_untimed = attention_fp8out


def gemm(a, w, bias=None, act=None, resid=None, resid_mod=0, out=None, out_dtype=torch.bfloat16,
         row_map=None, m=None, plan=None):
    t = _timer()
    if t is None:
        return _gemm_untimed(a, w, bias, act, resid, resid_mod, out, out_dtype, row_map, m, plan)
    M = a.shape[0] if m is None else m
    N, K = w.shape
    ob = (out.dtype if out is not None else out_dtype) == torch.bfloat16
    tags = dict(kind="gemm", act=ACT[act], out_bf16=ob, resid=resid is not None, M=M, N=N, K=K,
                large=bool(lib().bf_gemm_large_tiles(c_int(M), c_int(N), c_int(K))))
    nbytes = 2.0 * (M * K + N * K) + M * N * (2 if ob else 4)
    if resid is not None:
        nbytes += 4.0 * (M * N if not resid_mod else resid_mod * N)
    return t.record(tags, 2.0 * M * N * K, nbytes,
                    lambda: _gemm_untimed(a, w, bias, act, resid, resid_mod, out, out_dtype, row_map, m, plan))


def gemm_fp8(a, w, scale, bias=None, act=None, resid=None, out=None, out_dtype=torch.bfloat16,
             out_qscale=1.0, plan=None):
    t = _timer()
    if t is None:
        return _gemm_fp8_untimed(a, w, scale, bias, act, resid, out, out_dtype, out_qscale, plan)
    M, K = a.shape
    N = w.shape[0]
    od = out.dtype if out is not None else out_dtype
    tags = dict(kind="gemm_fp8", act=ACT[act], out=str(od), resid=resid is not None, M=M, N=N, K=K)
    nbytes = 1.0 * (M * K + N * K) + M * N * od.itemsize + (4.0 * M * N if resid is not None else 0.0)
    return t.record(tags, 2.0 * M * N * K, nbytes,
                    lambda: _gemm_fp8_untimed(a, w, scale, bias, act, resid, out, out_dtype, out_qscale, plan))


def attention(q, k, v, o, batch, heads, sq, sk, head_dim, scale, q_bs=None, k_bs=None, v_bs=None,
              o_bs=None, o_map=None, variant=0):
    t = _timer()
    if t is None:
        return _attention_untimed(q, k, v, o, batch, heads, sq, sk, head_dim, scale, q_bs, k_bs, v_bs,
                                  o_bs, o_map, variant)
    tags = dict(kind="attn", D=head_dim, sq=sq, sk=sk, batch=batch, heads=heads)
    bh = float(batch * heads)
    return t.record(tags, 4.0 * bh * sq * sk * head_dim, 2.0 * bh * head_dim * (2 * sq + 2 * sk),
                    lambda: _attention_untimed(q, k, v, o, batch, heads, sq, sk, head_dim, scale,
                                               q_bs, k_bs, v_bs, o_bs, o_map, variant))


def attention_fp8out(q, k, v, o, batch, heads, sq, sk, head_dim, scale, out_qscale, q_bs=None,
                     k_bs=None, v_bs=None, o_bs=None, variant=0):
    t = _timer()
    fn = lambda: _attention_fp8out_untimed(q, k, v, o, batch, heads, sq, sk, head_dim, scale, out_qscale,
                                           q_bs, k_bs, v_bs, o_bs, variant)
    if t is None:
        return fn()
    tags = dict(kind="attn", D=head_dim, sq=sq, sk=sk, batch=batch, heads=heads, fp8out=True)
    bh = float(batch * heads)
    return t.record(tags, 4.0 * bh * sq * sk * head_dim, bh * head_dim * (2 * sq + 4 * sk + sq), fn)


_depth_preprocess_untimed = depth_preprocess
_obb_iou_matrix_untimed = obb_iou_matrix
_nms_scan_untimed = nms_scan
_fusion_fit_untimed = fusion_fit


def obb_iou_matrix(corners):
    t = _timer()
    if t is None:
        return _obb_iou_matrix_untimed(corners)
    n = int(corners.shape[0])
    # work = box pairs (i < j) of the IoU matrix (gate + 25^3 grid count launches)
    return t.record(dict(kind="obb_iou", n=n), n * (n - 1) / 2.0, 96.0 * n + 8.0 * n * n,
                    lambda: _obb_iou_matrix_untimed(corners))


def nms_scan(iou, corners, scores, init_id, cam_poses, fl_items, fl_len, valid_num, cfg, out=None):
    t = _timer()
    fn = lambda: _nms_scan_untimed(iou, corners, scores, init_id, cam_poses, fl_items, fl_len, valid_num,
                                   cfg, out)
    if t is None:
        return fn()
    n = int(scores.shape[0])
    return t.record(dict(kind="nms_scan", n=n), float(n), 8.0 * n * n, fn)


def fusion_fit(view_off, n_views, view_box, view_R, view_score, view_pose, view_tc, pst, cfg,
               trace=False, max_views=None, packed_out=False, packed=None):
    t = _timer()
    fn = lambda: _fusion_fit_untimed(view_off, n_views, view_box, view_R, view_score, view_pose, view_tc,
                                     pst, cfg, trace, max_views, packed_out, packed)
    if t is None:
        return fn()
    res = []
    nj = int(view_off.shape[0])
    P = int(cfg.pst_size)
    # work = particle-view fitness evaluations: sum over jobs of views * particles * iterations
    # (the iteration counts are read when the summary is taken)
    work = lambda: float((res[0][1][nj:2 * nj].long() * n_views.long()).sum().item() * P if packed_out
                         else (res[0][2].long() * n_views.long()).sum().item() * P)
    t.record(dict(kind="fusion_fit", jobs=nj), work, 0.0, lambda: res.append(fn()))
    return res[0]


def depth_preprocess(depth, K=None, RT=None, max_depth=10.0, out=None, params=None, xyz=None, valid=None,
                     ws=None):
    t = _timer()
    if t is None:
        return _depth_preprocess_untimed(depth, K, RT, max_depth, out, params, xyz, valid, ws)
    b, h, w = depth.shape
    # outputs and workspace allocated before the start event: the events bracket the launches only
    out = torch.empty_like(depth) if out is None else out
    params = torch.empty((b, 2), dtype=torch.float32, device=depth.device) if params is None else params
    if K is not None:
        xyz = torch.empty((b, h, w, 3), dtype=torch.float32, device=depth.device) if xyz is None else xyz
        valid = torch.empty((b, h, w), dtype=torch.uint8, device=depth.device) if valid is None else valid
    if ws is None and not torch.cuda.is_current_stream_capturing():
        ws = depth_workspace(b, h, w, depth.device)
    fn = lambda: _depth_preprocess_untimed(depth, K, RT, max_depth, out, params, xyz, valid, ws)
    n = float(b * h * w)
    # algorithmic bytes: read the depth once, write the standardised map (+ xyz and
    # the valid mask when back-projecting)
    nbytes = 8.0 * n + (13.0 * n if K is not None else 0.0)
    tags = dict(kind="depth", backproject=K is not None, b=b, h=h, w=w)
    return t.record(tags, 0.0, nbytes, fn)


def depth_standardize(depth, out=None, params=None, ws=None):
    """depth f32[b,h,w] -> (standardised f32[b,h,w], params f32[b,2])"""
    return depth_preprocess(depth, out=out, params=params, ws=ws)


def new_depth_workspace(b, h, w, device):
    """a caller-owned zero-filled workspace for bf_depth_preprocess (one per concurrent user)"""
    size = int(lib().bf_depth_standardize_workspace_size(c_int(b), c_int(h), c_int(w)))
    return torch.zeros(max(size, 1), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------------------------------
# chip partitioning: CU-masked HIP streams (fusion on a few CUs, detection on the rest)
# ------------------------------------------------------------------------------------------
def cu_masked_stream(cus, device=None):
    """torch ExternalStream on a new HIP stream restricted to the CUs in `cus` (indices as the
    runtime enumerates them) via hipExtStreamCreateWithCUMask."""
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.cuda.current_device() if device is None else device
    n = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ctypes.c_uint32 * ((n + 31) // 32))()
    for c in cus:
        if not 0 <= c < n:
            raise HipError(f"CU index {c} outside 0..{n - 1}")
        words[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    with torch.cuda.device(dev):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), words)
    if rc != 0:
        raise HipError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    _MASKED_STREAMS.append((dev, s.value))
    return torch.cuda.ExternalStream(s.value, device=dev)


_MASKED_STREAMS = []


def _destroy_masked_streams():
    """destroy the CU-masked streams while the HIP runtime is still up (interpreter exit, before
    the runtime's own static teardown: left to that teardown, a profiler's finalisation crashed)"""
    hip = ctypes.CDLL("libamdhip64.so")
    while _MASKED_STREAMS:
        dev, h = _MASKED_STREAMS.pop()
        with torch.cuda.device(dev):
            hip.hipStreamSynchronize(ctypes.c_void_p(h))
            hip.hipStreamDestroy(ctypes.c_void_p(h))


# Objects that hold HIP resources past their last use: fusion worker threads (which may still launch
# on a CU-masked stream) and keyframe sequencers (device buffers, a stored stream).  At interpreter
# exit they are released in dependency order while the HIP runtime is still up: workers stopped,
# then sequencers destroyed, then the masked streams.
_LIVE_WORKERS = weakref.WeakSet()
_LIVE_SEQUENCERS = weakref.WeakSet()


def register_worker(w):
    """an object with stop(timeout) that runs HIP work on a thread (fusion_stage.AsyncFusion)"""
    _LIVE_WORKERS.add(w)


def _shutdown():
    stuck = False
    for w in list(_LIVE_WORKERS):
        try:
            stuck |= w.stop(timeout=30.0) is False
        except Exception:  # noqa: BLE001 - exit path: keep releasing the rest
            pass
    if stuck:
        # a worker thread is still launching on the sequencers / masked streams: releasing them
        # now would be a use-after-free under it, so process teardown reclaims them instead
        return
    for q in list(_LIVE_SEQUENCERS):
        try:
            q.close()
        except Exception:  # noqa: BLE001
            pass
    _destroy_masked_streams()


atexit.register(_shutdown)


def partition_streams(n_reserved, device=None, masked=False):
    """(detect_stream, fusion_stream) for a rank that also runs the fusion state machine.
    The persistent GEMMs are told to leave `n_reserved` CUs free (their grid is n_cu - n_reserved
    workgroups, one per CU), so the fusion kernels always find CUs while a GEMM runs; the fusion
    stream gets high priority for the CUs that free up in between.  masked=True additionally
    confines each stream to its CUs with hipExtStreamCreateWithCUMask."""
    dev = torch.cuda.current_device() if device is None else device
    det, fus = partition_cus(n_reserved, dev)
    set_cu_budget(len(det))
    if not masked:
        return torch.cuda.current_stream(dev), torch.cuda.Stream(device=dev, priority=-1)
    return cu_masked_stream(det, dev), cu_masked_stream(fus, dev)


XCDS = 8


def cu_placement(stream, n_wg=4096, spin=20000):
    """{(xcc, se, sh, cu)} of the CUs that n_wg probe workgroups ran on when launched on `stream`
    (bf_cu_probe): what a CU mask really does on this chip"""
    out = torch.zeros(2 * n_wg, dtype=torch.int32, device=torch.device("cuda", stream.device_index))
    _check(lib().bf_cu_probe(_ptr(out), c_int(n_wg), c_int(spin), c_void_p(stream.cuda_stream)), "bf_cu_probe")
    stream.synchronize()
    v = out.view(-1, 2).cpu().numpy()
    hw, xcc = v[:, 0], v[:, 1] & 0xF
    return {(int(x), int((h >> 13) & 7), int((h >> 12) & 1), int((h >> 8) & 0xF)) for h, x in zip(hw, xcc)}


def partition_cus(n_reserved, device=None, n_cu=None):
    """(detect CUs, fusion CUs) as CU-mask bit indices.  Mask bit i is CU i // 8 of XCD i % 8, and
    a mask that leaves an XCD without CUs is not applied at all (the stream then runs on every CU:
    measured with scripts/diag/cu_probe.py), so the fusion set takes the first n_reserved bits —
    n_reserved / 8 CUs on every XCD — and detection the rest."""
    if n_cu is None:
        dev = torch.cuda.current_device() if device is None else device
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    n = n_cu
    k = -(-max(1, n_reserved) // XCDS) * XCDS
    if k >= n:
        raise HipError(f"cannot reserve {n_reserved} of {n} CUs for the fusion stream")
    fus = list(range(k))
    det = list(range(k, n))
    return det, fus


# ------------------------------------------------------------------------------------------
# CuTR decoder: cross-attention position bias + clip + softmax
# ------------------------------------------------------------------------------------------
def cpb_mlp(ref, pos, axis, w1, b1, w2):
    """ref f32 [B,nq,4], pos f32 [n] -> f32 [B,nq,n,heads] (GlobalCrossAttention.rpe's MLP)"""
    ref = _need(ref.contiguous(), torch.float32, "ref")
    B, nq = ref.shape[0], ref.shape[1]
    heads, hidden = w2.shape
    out = torch.empty((B, nq, pos.shape[0], heads), dtype=torch.float32, device=ref.device)
    _check(lib().bf_cpb_mlp(_ptr(ref), c_int(B), c_int(nq), _ptr(pos.contiguous()), c_int(pos.shape[0]),
                            c_int(axis), _ptr(w1.contiguous()), _ptr(b1.contiguous()),
                            _ptr(w2.contiguous()), c_int(hidden), c_int(heads), _ptr(out), _stream()),
           "bf_cpb_mlp")
    return out


def xattn(q, k, v, rx, ry, hh, ww, q0, heads, scale, out=None):
    """fused global cross-attention (bf_xattn_f32): q f32 [B,Nq,C], k / v f32 [B,hh*ww,C] (any row
    stride, unit column stride), rx [B,Nq-q0,ww,heads], ry [B,Nq-q0,hh,heads] -> out f32 [B,Nq,C]"""
    for x, n in ((q, "q"), (k, "k"), (v, "v")):
        _need(x, torch.float32, n)
        if x.dim() != 3 or x.stride(2) != 1 or x.stride(0) != x.shape[1] * x.stride(1):
            raise HipError(f"xattn: {n} must be [B, rows, C] with unit column stride and packed batches")
    B, Nq, C = q.shape
    if C != heads * 32 or k.shape != (B, hh * ww, C) or v.shape != k.shape:
        raise HipError("xattn: head dim 32, k / v [B, hh*ww, C]")
    if out is None:
        out = torch.empty((B, Nq, C), dtype=torch.float32, device=q.device)
    if q0 < Nq:
        rx = _need(rx.contiguous(), torch.float32, "rx")
        ry = _need(ry.contiguous(), torch.float32, "ry")
    _check(lib().bf_xattn_f32(c_void_p(q.data_ptr()), c_int(q.stride(1)), c_void_p(k.data_ptr()),
                              c_int(k.stride(1)), c_void_p(v.data_ptr()), c_int(v.stride(1)),
                              _ptr(rx) if q0 < Nq else None, _ptr(ry) if q0 < Nq else None,
                              c_void_p(out.data_ptr()), c_int(out.stride(1)), c_int(B), c_int(heads),
                              c_int(Nq), c_int(q0), c_int(hh), c_int(ww), c_float(scale), _stream()),
           "bf_xattn_f32")
    return out


def rpe_softmax(attn, rx, ry, hh, ww, q0):
    """attn f32 [B,H,Nq,hh*ww] in place: + bias on rows q >= q0, clip, softmax"""
    _need(attn, torch.float32, "attn")
    B, H, Nq, N = attn.shape
    _check(lib().bf_rpe_softmax(_ptr(attn), c_int(B), c_int(H), c_int(Nq), c_int(q0), _ptr(rx),
                                _ptr(ry), c_int(hh), c_int(ww), _stream()), "bf_rpe_softmax")
    return attn


# ------------------------------------------------------------------------------------------
# CuTR decoder tail, f32 (bf_dec_native.hip + bf_self_attn_f32): thin pointer-level wrappers.
# Views with a row stride and unit column stride are accepted (the row stride is passed on).
# ------------------------------------------------------------------------------------------
def _rows(t, name, dtype=torch.float32):
    """(pointer, row stride) of a 2-D device view with unit column stride"""
    if t is None:
        return None, 0
    if not t.is_cuda:
        raise HipError("boxfusion_amd kernels need device tensors (no CPU fallback)")
    _need(t, dtype, name)
    if t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1):
        raise HipError(f"{name}: expected a 2-D view with unit column stride")
    return c_void_p(t.data_ptr()), t.stride(0)


def gemm_f32(a, w, bias=None, act=None, resid=None, out=None, a_map=None, c_map=None, m=None):
    """out[c_map[r]] = resid[c_map[r]] + act(a[a_map[r]] @ w.T + bias) for r < m (f32 MFMA);
    a_map / c_map int32 (< 0: zero row / dropped row); m defaults to len(a_map) or a.shape[0]"""
    N, K = w.shape
    M = m if m is not None else (a_map.shape[0] if a_map is not None else a.shape[0])
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    pa, lda = _rows(a, "a")
    pw, ldw = _rows(w, "w")
    pc, ldc = _rows(out, "out")
    pr, ldr = _rows(resid, "resid")
    for mp, n in ((a_map, "a_map"), (c_map, "c_map")):
        if mp is not None:
            _need(mp, torch.int32, n)
            if mp.shape[0] < M:
                raise HipError(f"gemm_f32: {n} shorter than M")
    if bias is not None:
        _need(bias, torch.float32, "bias")
    _check(lib().bf_gemm_f32(pa, c_int(lda), _ptr(a_map), pw, c_int(ldw), _ptr(bias), pr, c_int(ldr),
                             pc, c_int(ldc), _ptr(c_map), c_int(M), c_int(N), c_int(K), c_int(ACT[act]),
                             _stream()), "bf_gemm_f32")
    return out


def ln_rows(x, gamma, beta, eps, out=None, pos=None, out2=None, gelu=False):
    """out = LayerNorm(x rows) [GELU]; out2 = out + pos (optional).  C % 256 == 0, <= 1024"""
    M, C = x.shape
    if out is None:
        out = torch.empty((M, C), dtype=torch.float32, device=x.device)
    px, ldx = _rows(x, "x")
    po, ldo = _rows(out, "out")
    pp, ldp = _rows(pos, "pos")
    p2, ld2 = _rows(out2, "out2")
    _check(lib().bf_ln_rows_f32(px, c_int(ldx), _ptr(gamma), _ptr(beta), c_float(eps), po, c_int(ldo),
                                pp, c_int(ldp), p2, c_int(ld2), c_int(M), c_int(C), c_int(int(gelu)),
                                _stream()), "bf_ln_rows_f32")
    return out


def groupnorm_cl(x, frames, groups, gamma, beta, eps, out, pos=None, out2=None):
    """GroupNorm of a channel-last map x [frames*P, C] -> out (and out2 = out + pos)"""
    px, ldx = _rows(x, "x")
    po, ldo = _rows(out, "out")
    pp, ldp = _rows(pos, "pos")
    p2, ld2 = _rows(out2, "out2")
    P = x.shape[0] // frames
    _check(lib().bf_groupnorm_cl_f32(px, c_int(ldx), c_int(frames), c_int(P), c_int(x.shape[1]), c_int(groups),
                                     _ptr(gamma), _ptr(beta), c_float(eps), po, c_int(ldo), pp, c_int(ldp),
                                     p2, c_int(ld2), _stream()), "bf_groupnorm_cl_f32")
    return out


def s2d(x, frames, H, W, out=None):
    """space-to-depth rows (kernel-2 stride-2 conv operand) of a channel-last map [frames*H*W, C]"""
    C = x.shape[1]
    if out is None:
        out = torch.empty((frames * (H // 2) * (W // 2), 4 * C), dtype=torch.float32, device=x.device)
    px, ldx = _rows(x, "x")
    _check(lib().bf_s2d_f32(px, c_int(ldx), c_int(frames), c_int(H), c_int(W), c_int(C), _ptr(out), _stream()),
           "bf_s2d_f32")
    return out


HEAD_MODES = {"class": 0, "box2d": 1, "box3d": 2, "scale": 3}


def row_heads(x, in_fs, in_off, rows, nq, w, b, mode, out=None, prop=None, params=None, boxes=None,
              clamp_wh=(0.0, 0.0), max_ratio=0.0):
    """the predictors' output linears + transforms (bf_row_heads_f32; see bf_dec_native.hip)"""
    px, ldx = _rows(x, "x")
    po, ldo = _rows(out, "out")
    _check(lib().bf_row_heads_f32(px, c_int(ldx), c_int(in_fs), c_int(in_off), c_int(rows), c_int(nq),
                                  c_int(w.shape[1]), _ptr(w), _ptr(b), c_int(w.shape[0]), _ptr(prop),
                                  _ptr(params), po, c_int(ldo), _ptr(boxes), c_float(clamp_wh[0]),
                                  c_float(clamp_wh[1]), c_float(max_ratio), c_int(HEAD_MODES[mode]),
                                  _stream()), "bf_row_heads_f32")
    return out


def topk_rows(v, frames, n, k, ldv=1, idx=None, vals=None):
    """per-frame top-k of v[(f*n + i)*ldv] (descending, ties -> lower index): int32 idx [frames, k]"""
    if idx is None:
        idx = torch.empty((frames, k), dtype=torch.int32, device=v.device)
    _check(lib().bf_topk_rows_f32(c_void_p(v.data_ptr()), c_int(ldv), c_int(frames), c_int(n), c_int(k),
                                  _ptr(idx), _ptr(vals), _stream()), "bf_topk_rows_f32")
    return idx


def prop_select(boxes, frames, n, k, idx, ref, embs, max_e, qpos, qfs, qoff):
    """ref[f*k + j] = boxes[f*n + idx[f, j]]; qpos row f*qfs + qoff + j = the 4 box embeddings"""
    pq, ldq = _rows(qpos, "qpos")
    ex, ey, ew, eh = embs
    _check(lib().bf_prop_select_f32(_ptr(boxes), c_int(frames), c_int(n), c_int(k), _ptr(idx), _ptr(ref),
                                    _ptr(ex), _ptr(ey), _ptr(ew), _ptr(eh), c_int(ex.shape[1]),
                                    c_float(max_e), pq, c_int(ldq), c_int(qfs), c_int(qoff), _stream()),
           "bf_prop_select_f32")


def infer_select(logits, frames, nq, nc, boxes, b3info, desc, desc_fs, desc_off, Kinv, Tg, img_wh, k, outs):
    """inference_single_image for every frame (bf_infer_select_f32); outs = dict of output buffers
    scores [F,k], classes int64 [F,k], logits [F,k,nc], boxes [F,k,4], proj [F,k,2], b3 [F,k,6],
    R [F,k,3,3], desc [F,k,C]"""
    pd, ldd = _rows(desc, "desc")
    _check(lib().bf_infer_select_f32(_ptr(logits), c_int(frames), c_int(nq), c_int(nc), _ptr(boxes),
                                     _ptr(b3info), pd, c_int(ldd), c_int(desc_fs), c_int(desc_off),
                                     c_int(desc.shape[1]), _ptr(Kinv), _ptr(Tg), _ptr(img_wh), c_int(k),
                                     _ptr(outs["scores"]), _ptr(outs["classes"]), _ptr(outs["logits"]),
                                     _ptr(outs["boxes"]), _ptr(outs["proj"]), _ptr(outs["b3"]),
                                     _ptr(outs["R"]), _ptr(outs["desc"]), _stream()), "bf_infer_select_f32")


def ray_fourier(K3, W, H, feat, stride, scales, out):
    """CameraRayEmbedding's Fourier features of one camera into out [feat*feat, ld] (ld >= 3 * bands)"""
    K3 = np.asarray(K3, np.float32).reshape(3, 3)
    po, ld = _rows(out, "out")
    _check(lib().bf_ray_fourier_f32(c_float(K3[0, 0]), c_float(K3[1, 1]), c_float(K3[0, 2]), c_float(K3[1, 2]),
                                    c_int(W), c_int(H), c_int(feat), c_int(stride), _ptr(scales),
                                    c_int(scales.shape[0]), po, c_int(ld), _stream()), "bf_ray_fourier_f32")
    return out


def self_attn(q, k, v, out, frames, heads, n, q0, scale):
    """decoder self-attention with the metric / box block mask (bf_self_attn_f32); q / k / v / out
    [frames*n, heads*32] row views"""
    pq, ldq = _rows(q, "q")
    pk, ldk = _rows(k, "k")
    pv, ldv = _rows(v, "v")
    po, ldo = _rows(out, "out")
    _check(lib().bf_self_attn_f32(pq, c_int(ldq), pk, c_int(ldk), pv, c_int(ldv), po, c_int(ldo), c_int(frames),
                                  c_int(heads), c_int(n), c_int(q0), c_float(scale), _stream()), "bf_self_attn_f32")
    return out


def cpb_mlp_into(ref, pos, axis, w1, b1, w2, out):
    """cpb_mlp into a preallocated [B, nq, n, heads] buffer"""
    B, nq = ref.shape[0], ref.shape[1]
    heads, hidden = w2.shape
    _check(lib().bf_cpb_mlp(_ptr(ref), c_int(B), c_int(nq), _ptr(pos), c_int(pos.shape[0]), c_int(axis), _ptr(w1),
                            _ptr(b1), _ptr(w2), c_int(hidden), c_int(heads), _ptr(out), _stream()), "bf_cpb_mlp")
    return out
