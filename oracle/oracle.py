"""CPU ORACLE — test infrastructure only.

numpy/ctypes front end of ``libbf_oracle.so`` (plain-C restatement of the reference fusion path,
see bf_oracle.c for the file:line map) plus small numpy restatements of the per-frame host maths.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
module; the product package ``boxfusion_amd`` never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libbf_oracle.so")
        src = os.path.join(_HERE, "bf_oracle.c")
        if not os.path.exists(path) or (os.path.exists(src) and
                                         os.path.getmtime(src) > os.path.getmtime(path)):
            build()
        _LIB = ctypes.CDLL(path)
    return _LIB


def hull_overflow(reset=True):
    """(calls with > 36 intersection candidates, calls with an intersection hull > 8 points) since
    the last reset: the reference kernel's corners_i[36] / convex_inter[8] overflow there
    (box_fusion.py:378-384)"""
    out = (ctypes.c_long * 2)()
    lib().or_hull_overflow(out, ctypes.c_int(1 if reset else 0))
    return int(out[0]), int(out[1])


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


class NmsCfg(ctypes.Structure):
    _fields_ = [("iou_threshold", ctypes.c_double), ("translation_gap", ctypes.c_float),
                ("rotation_gap", ctypes.c_float), ("center_gap", ctypes.c_double),
                ("max_list", ctypes.c_int), ("list_capacity", ctypes.c_int)]


class CorrCfg(ctypes.Structure):
    _fields_ = [("small_size", ctypes.c_double), ("threshold", ctypes.c_double),
                ("translation_gap", ctypes.c_float), ("rotation_gap", ctypes.c_float),
                ("W", ctypes.c_float), ("H", ctypes.c_float),
                ("max_list", ctypes.c_int), ("list_capacity", ctypes.c_int)]


class FuseCfg(ctypes.Structure):
    _fields_ = [("iters", ctypes.c_int), ("pst_size", ctypes.c_int), ("max_accept", ctypes.c_int),
                ("legacy_promotion", ctypes.c_int),
                ("center_init", ctypes.c_double), ("shape_init", ctypes.c_double),
                ("center_coef", ctypes.c_double), ("shape_coef", ctypes.c_double),
                ("beta", ctypes.c_double), ("min_scale", ctypes.c_double),
                ("img_h", ctypes.c_float), ("img_w", ctypes.c_float),
                ("K", ctypes.c_float * 16)]


def fuse_cfg(cfg: dict, K4, H, W, legacy=True, pst_size=None) -> FuseCfg:
    ro = cfg["box_fusion"]["random_opt"]
    c = FuseCfg()
    c.iters = int(cfg["box_fusion"]["iters"])
    c.pst_size = int(pst_size if pst_size is not None else cfg["box_fusion"]["pst_size"])
    c.max_accept = 200
    c.legacy_promotion = 1 if legacy else 0
    c.center_init = float(ro["center_init_size"])
    c.shape_init = float(ro["shape_init_size"])
    c.center_coef = float(ro["center_scaling_coefficient"])
    c.shape_coef = float(ro["shape_scaling_coefficient"])
    c.beta = 0.9
    c.min_scale = 1e-3
    c.img_h = float(H)
    c.img_w = float(W)
    k = np.asarray(K4, dtype=np.float32).reshape(-1)
    for i in range(16):
        c.K[i] = float(k[i])
    return c


# ---------------------------------------------------------------------------------------------
# geometry / IoU
# ---------------------------------------------------------------------------------------------
def box_corners(xyzlhw, R):
    b = _f32(xyzlhw).reshape(-1, 6)
    r = _f32(R).reshape(-1, 9)
    out = np.zeros((b.shape[0], 8, 3), np.float32)
    lib().or_box_corners(_p(b), _p(r), ctypes.c_int(b.shape[0]), _p(out))
    return out


def obb_iou(c1, c2, with_counts=False):
    a = _f32(c1).reshape(8, 3)
    b = _f32(c2).reshape(8, 3)
    cnt = np.zeros(3, np.int64)
    f = lib().or_obb_iou
    f.restype = ctypes.c_double
    v = f(_p(a), _p(b), _p(cnt))
    return (v, cnt) if with_counts else v


def obb_iou_matrix(corners):
    c = _f32(corners).reshape(-1, 8, 3)
    n = c.shape[0]
    out = np.zeros((n, n), np.float64)
    lib().or_obb_iou_matrix(_p(c), ctypes.c_int(n), _p(out))
    return out


# ---------------------------------------------------------------------------------------------
# fusion lists <-> padded rows
# ---------------------------------------------------------------------------------------------
def pack_lists(lists, cap):
    n = len(lists)
    items = np.full((max(n, 1), cap), -1, np.int32)
    lens = np.zeros(max(n, 1), np.int32)
    for i, row in enumerate(lists):
        if len(row) > cap:
            raise ValueError("fusion list longer than capacity")
        items[i, :len(row)] = row
        lens[i] = len(row)
    return items, lens


def unpack_lists(items, lens, n):
    return [[int(v) for v in items[i, :lens[i]]] for i in range(n)]


def nms_scan(iou, corners, scores, init_id, cam_poses, fusion_list, valid_num, cfg: NmsCfg):
    n = len(scores)
    cap = cfg.list_capacity
    items, lens = pack_lists(fusion_list, cap)
    vn = _f32(valid_num).copy()
    keep = np.zeros(n + 1, np.int32)
    succ = np.zeros(n + 1, np.int32)
    ev = np.zeros((n + 1, 3), np.int32)
    nk = np.zeros(1, np.int32); ns = np.zeros(1, np.int32); ne = np.zeros(1, np.int32)
    iou = np.ascontiguousarray(iou, np.float64)
    st = lib().or_nms_scan(_p(iou), _p(_f32(corners)), _p(_f32(scores)), _p(_i32(init_id)),
                           _p(_f32(cam_poses)), ctypes.c_int(n), _p(items), _p(lens), _p(vn),
                           _p(keep), _p(nk), _p(succ), _p(ns), _p(ev), _p(ne),
                           ctypes.byref(cfg))
    return dict(keep=keep[:nk[0]].copy(), success=succ[:ns[0]].copy(), events=ev[:ne[0]].copy(),
                fusion_list=unpack_lists(items, lens, len(fusion_list)), valid_num=vn, status=st)


def corr_assoc(corners, dims, scores, boxes2d, init_id, cam_poses, cur_pose, K, n_glo, mask,
               success, fusion_list, valid_num, cfg: CorrCfg):
    n_all = len(scores)
    cap = cfg.list_capacity
    items, lens = pack_lists(fusion_list, cap)
    vn = _f32(valid_num).copy()
    mask = _i32(mask)
    n_success = len(success)
    success = _i32(success) if n_success else np.zeros(1, np.int32)
    keep = np.zeros(len(mask) + 1, np.int32)
    ev = np.zeros((n_all + 1, 3), np.int32)
    nk = np.zeros(1, np.int32); ne = np.zeros(1, np.int32)
    st = lib().or_corr_assoc(_p(_f32(corners)), _p(_f32(dims)), _p(_f32(scores)),
                             _p(_f32(boxes2d)), _p(_i32(init_id)), _p(_f32(cam_poses)),
                             _p(_f32(cur_pose)), _p(_f32(K)), ctypes.c_int(n_all),
                             ctypes.c_int(n_glo), _p(mask), ctypes.c_int(len(mask)), _p(success),
                             ctypes.c_int(n_success),
                             _p(items), _p(lens), _p(vn), _p(keep), _p(nk), _p(ev), _p(ne),
                             ctypes.byref(cfg))
    return dict(keep=keep[:nk[0]].copy(), events=ev[:ne[0]].copy(),
                fusion_list=unpack_lists(items, lens, len(fusion_list)), valid_num=vn, status=st)


def project_2d_box(corners, pose, K, W, H):
    """project_3d_to_2d_box for a set of boxes (f64), pose inverted like the device does."""
    c = _f32(corners).reshape(-1, 8, 3)
    pinv = np.linalg.inv(np.asarray(pose, np.float64)).astype(np.float32)
    out = np.zeros((c.shape[0], 4), np.float64)
    for i in range(c.shape[0]):
        lib().or_project_2d_box(_p(np.ascontiguousarray(c[i])), _p(pinv), _p(_f32(K)),
                                ctypes.c_double(W), ctypes.c_double(H), _p(out[i]))
    return out


# ---------------------------------------------------------------------------------------------
# fusion
# ---------------------------------------------------------------------------------------------
def fitness(box, R, poses, tc, pst, search_size, cfg: FuseCfg):
    nv = len(poses)
    out = np.zeros(pst.shape[0], np.float32)
    lib().or_fitness(_p(_f32(box)), _p(_f32(R)), ctypes.c_int(nv), _p(_f32(poses)), _p(_f32(tc)),
                     _p(_f32(pst)), ctypes.c_int(pst.shape[0]), _p(_f32(search_size)),
                     ctypes.byref(cfg), _p(out))
    return out


def fusion_fit(view_box, view_R, view_score, view_pose, view_tc, pst, cfg: FuseCfg, trace=False):
    nv = len(view_score)
    out = np.zeros(6, np.float32)
    it = np.zeros(1, np.int32)
    tr = np.zeros((cfg.iters, cfg.pst_size), np.float32) if trace else None
    upd = lib().or_fusion_fit(_p(_f32(view_box)), _p(_f32(view_R)), _p(_f32(view_score)),
                              _p(_f32(view_pose)), _p(_f32(view_tc)), ctypes.c_int(nv),
                              _p(_f32(pst)), ctypes.byref(cfg), _p(out), _p(it),
                              _p(tr) if trace else None)
    res = dict(box=out, updated=int(upd), iters=int(it[0]))
    if trace:
        res["trace"] = tr[:it[0]]
    return res


# ---------------------------------------------------------------------------------------------
# per-frame maths
# ---------------------------------------------------------------------------------------------
def depth_standardize(depth):
    d = _f32(depth)
    out = np.zeros_like(d)
    params = np.zeros(2, np.float32)
    lib().or_depth_standardize(_p(d), ctypes.c_int(d.size), _p(out), _p(params))
    return out, params


def backproject(depth, K, RT, max_depth=10.0):
    """tools/utils.py:245-287 in numpy float32."""
    d = _f32(depth)
    h, w = d.shape
    u, v = np.meshgrid(np.arange(w), np.arange(h), indexing="xy")
    K4 = np.eye(4, dtype=np.float32)
    K4[:3, :3] = K
    Ki = np.linalg.inv(K4.astype(np.float64)).astype(np.float32)
    uvd = np.stack([u * d, v * d, d, np.ones_like(d)], -1).reshape(-1, 4).astype(np.float32)
    cam = (Ki @ uvd.T)
    world = (np.asarray(RT, np.float32) @ cam).T[:, :3].reshape(h, w, 3)
    valid = d > 0
    if max_depth is not None and max_depth > 0:
        valid &= d < max_depth
    return world.astype(np.float32), valid


def cv2_resize_u8(src, Wd, Hd):
    """cv2.resize(src, (Wd, Hd)) for a u8 [H, W] or [H, W, cn] image (INTER_LINEAR), restated"""
    a = np.ascontiguousarray(src, dtype=np.uint8)
    cn = 1 if a.ndim == 2 else a.shape[2]
    out = np.empty((Hd, Wd) + (() if a.ndim == 2 else (cn,)), dtype=np.uint8)
    lib().or_cv2_resize_u8(_p(a), ctypes.c_int(a.shape[0]), ctypes.c_int(a.shape[1]), ctypes.c_int(cn),
                           _p(out), ctypes.c_int(Hd), ctypes.c_int(Wd))
    return out


def ingest_rgbd(bgr, depth_u16, depth_scale, rot_k):
    """capture_stream.py:194-311: BGR -> RGB, cv2.resize to the depth size, CHW, rot90; depth
    u16 -> f32 / scale, rot90 (numpy restatement over or_cv2_resize_u8)"""
    Hd, Wd = depth_u16.shape
    rgb = np.ascontiguousarray(bgr[..., ::-1])
    rgb = cv2_resize_u8(rgb, Wd, Hd)
    chw = np.moveaxis(rgb, -1, 0)
    d = depth_u16.astype(np.float32) / np.float32(depth_scale)
    return (np.ascontiguousarray(np.rot90(chw, rot_k, axes=(-2, -1))),
            np.ascontiguousarray(np.rot90(d, rot_k, axes=(-2, -1))))
