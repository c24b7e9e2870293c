"""Helpers to replay tests/golden/fusion_trace.npz (the reference's fusion chain, recorded by
tests/golden/make_golden.py) keyframe by keyframe against a backend (oracle or HIP)."""
from __future__ import annotations

import copy
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SCANNET_CFG = dict(
    dataset="scannet",
    data=dict(datadir="/synthetic/scannet", gap=1),
    cam=dict(H=480, W=640, fx=574.540771, fy=577.583740, cx=322.522827, cy=238.558853),
    detection=dict(score_thresh=0.5, uv_bound=True, uv_bound_value=0.9, floor_mask=True,
                   floor_ratio=15, scale_box=1.5),
    association=dict(small_threshold=0.1, rotation_gap=30, translation_gap=0.8),
    box_fusion=dict(use=True, iters=20, pst_path="pst_1024_0", pst_size=1024,
                    check_valid=False, nms_threshold=0.1, small_size=0.35,
                    random_opt=dict(center_init_size=0.1, center_scaling_coefficient=0.1,
                                    shape_init_size=0.5, shape_scaling_coefficient=0.5)),
)


SCANNET_K = np.array([[574.540771, 0.0, 322.522827], [0.0, 577.583740, 238.558853], [0, 0, 1]],
                     np.float32)

# the fusion-chain traces (make_golden.py): ScanNet scene traces, the CA-1M config trace (ca1m.yaml
# thresholds, 384 x 512 portrait) and the overrun-free face-on trace
TRACES = ["fusion_trace.npz", "fusion_trace_small.npz", "fusion_trace_ca1m.npz", "fusion_trace_faceon.npz"]


def trace_setup(t):
    """(cfg, K [3,3], H, W) the trace was generated with; traces without a recorded config ran
    with SCANNET_CFG on the 640 x 480 ScanNet camera"""
    if "cfg_json" not in t:
        return SCANNET_CFG, SCANNET_K, 480, 640
    cfg = json.loads(str(t["cfg_json"]))
    cfg["box_fusion"]["pst_path"] = "pst_1024_0"
    cfg["data"] = dict(gap=1)
    return cfg, np.asarray(t["K"], np.float32), int(t["H"]), int(t["W"])


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


def _lists(t, key, k):
    """fusion lists (list of lists) recorded under `key` at keyframe k."""
    nrows = t[key + "_nrows"]
    r0 = int(nrows[:k].sum())
    off = t[key + "_rowoff"]
    flat = t[key + "_flat"]
    return [[int(v) for v in flat[off[r]:off[r + 1]]] for r in range(r0, r0 + int(nrows[k]))]


def _rows(t, key, k):
    o = t[key + "_off"]
    return t[key][o[k]:o[k + 1]]


class Keyframe:
    """All inputs/outputs of one recorded keyframe (k >= 1)."""

    def __init__(self, t, k):
        self.k = k
        self.frame = int(t["frame"][k])
        self.pose = t["pose"][k]
        nd = t["n_det"]
        id0 = int(nd[:k].sum())
        self.new_ids = np.arange(id0, id0 + int(nd[k]), dtype=np.int64)
        n_pre = int(t["pre_n"][k])
        self.n_glo = n_pre
        pf_t, pf_R = t["pf_tensor"], t["pf_R"]
        self.tensor = np.concatenate([_rows(t, "pre_tensor", k), pf_t[self.new_ids]], 0)
        self.R = np.concatenate([_rows(t, "pre_R", k), pf_R[self.new_ids]], 0)
        det_s = t["det_scores"][id0:id0 + int(nd[k])]
        self.scores = np.concatenate([_rows(t, "pre_scores", k), det_s], 0).astype(np.float32)
        self.init_id = np.concatenate([_rows(t, "pre_init_id", k), self.new_ids]).astype(np.int64)
        self.valid_num = np.concatenate([_rows(t, "pre_valid_num", k),
                                         np.zeros(len(self.new_ids), np.float32)])
        det_b = t["det_pred_boxes"][id0:id0 + int(nd[k])]
        self.boxes2d = np.concatenate([_rows(t, "pre_boxes2d", k), det_b], 0).astype(np.float32)
        pre_fl = _lists(t, "pre_fl", k)
        self.fusion_list = pre_fl + [[int(i)] for i in self.new_ids]
        self.cam_poses = t["pf_pose"]
        # expected
        self.nms_keep = _rows(t, "nms_keep", k)
        self.nms_success = _rows(t, "nms_success", k)
        self.nms_valid_num = _rows(t, "nms_valid_num", k)
        self.nms_fl = _lists(t, "nms_fl", k)
        self.corr_keep = _rows(t, "corr_keep", k)
        self.corr_fl = _lists(t, "corr_fl", k)
        self.post_fl = _lists(t, "post_fl", k)
        self.post_tensor = _rows(t, "post_tensor", k)
        self.post_valid_num = _rows(t, "post_valid_num", k)
        self.fused = _lists(t, "fused", k)
        self.fused_before = _lists(t, "fused", k - 1)
        self.per_frame = dict(tensor=t["pf_tensor"], R=t["pf_R"], scores=t["pf_scores"],
                              pose=t["pf_pose"], proj=t["pf_proj"])

    @property
    def dims(self):
        return self.tensor[:, 3:6]

    def fusion_jobs(self):
        """Boxes BoxFusion.boxfusion would fuse after this keyframe's association, with the
        reference's skip rules (box_fusion.py:631-635); duplicates of an earlier job list in the
        same call are marked so the caller can apply them only if the first one did not update."""
        jobs = []
        fused = [list(f) for f in self.fused_before]
        for i, fl in enumerate(self.post_fl):
            if len(fl) < 3 or fl in fused:
                continue
            jobs.append((i, fl))
        return jobs


def keyframes(t):
    return [Keyframe(t, k) for k in range(1, len(t["frame"]))]


def replay(t, backend, fuse_legacy=False):
    """Replay every keyframe of trace `t` through `backend` and compare bit-for-bit with the
    reference's recorded outputs.  `backend` provides:
        corners(tensor, R) -> f32[n,8,3]
        iou_matrix(corners) -> f64[n,n]
        nms(iou, corners, scores, init_id, cam_poses, fusion_list, valid_num) -> dict
        corr(corners, dims, scores, boxes2d, init_id, cam_poses, pose, K, n_glo, keep, success,
             fusion_list, valid_num) -> dict
        fuse(list of (view_box, view_R, view_score, view_pose, view_tc)) -> list of (box, updated)
    A backend with hull_overflow() (True when a fitness evaluation since the last call had an
    intersection hull the reference kernel's fixed buffers cannot hold) is checked against the
    trace's per-keyframe record.  Keyframes before the first such evaluation are pinned to the
    reference outright (stats["reference_pinned"]); from there on the trace is the reference's
    control flow with the exact hull where its kernel overruns convex_inter[8] / corners_i[36]
    (box_fusion.py:378-384, undefined behaviour in the reference).
    Returns counters of the exercised paths."""
    _, K, _, _ = trace_setup(t)
    stats = dict(keyframes=0, suppressions=0, corr_changes=0, fused=0, reference_pinned=0,
                 hull_overflow_keyframes=0)
    over_seen = False
    if hasattr(backend, "hull_overflow"):
        backend.hull_overflow()
    for kf in keyframes(t):
        msg = f"keyframe {kf.k}"
        corners = backend.corners(kf.tensor, kf.R)
        iou = backend.iou_matrix(corners)
        r = backend.nms(iou, corners, kf.scores, kf.init_id, kf.cam_poses, kf.fusion_list,
                        kf.valid_num)
        np.testing.assert_array_equal(r["keep"], kf.nms_keep, err_msg=msg)
        np.testing.assert_array_equal(r["success"], kf.nms_success, err_msg=msg)
        assert r["fusion_list"] == kf.nms_fl, msg
        np.testing.assert_array_equal(r["valid_num"], kf.nms_valid_num, err_msg=msg)
        has_new = bool((r["keep"] >= kf.n_glo).any())
        keep, vn = r["keep"], r["valid_num"]
        if has_new:
            c = backend.corr(corners, kf.dims, kf.scores, kf.boxes2d, kf.init_id, kf.cam_poses,
                             kf.pose, K, kf.n_glo, r["keep"], r["success"], r["fusion_list"],
                             r["valid_num"])
            np.testing.assert_array_equal(c["keep"], kf.corr_keep, err_msg=msg)
            assert c["fusion_list"] == kf.corr_fl, msg
            keep, vn = c["keep"], c["valid_num"]
            stats["corr_changes"] += int(not np.array_equal(c["keep"], r["keep"]))
        np.testing.assert_array_equal(vn[keep], kf.post_valid_num, err_msg=msg)
        post = kf.tensor[keep].copy()
        if has_new:
            pf = kf.per_frame
            jobs = kf.fusion_jobs()
            views = []
            for _, fl in jobs:
                idx = np.asarray(fl)
                views.append((pf["tensor"][idx], pf["R"][idx], pf["scores"][idx], pf["pose"][idx],
                              pf["proj"][idx]))
            results = backend.fuse(views) if views else []
            done = []
            for (i, fl), (box, upd) in zip(jobs, results):
                if fl in done:
                    continue
                if upd:
                    post[i] = box
                    done.append(fl)
                    stats["fused"] += 1
        np.testing.assert_array_equal(post, kf.post_tensor, err_msg=msg)
        if not over_seen:
            stats["reference_pinned"] += 1
        if "hull_over" in t:
            want = bool(np.asarray(t["hull_over"][kf.k]).any())
            if hasattr(backend, "hull_overflow"):
                assert backend.hull_overflow() == want, msg + ": hull-overflow record"
            over_seen |= want
            stats["hull_overflow_keyframes"] += int(want)
        stats["keyframes"] += 1
        stats["suppressions"] += len(kf.nms_success)
    return stats
