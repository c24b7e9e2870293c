"""CPU restatement of the keyframe fusion chain of demo.py:200-305 over the oracle kernels.

TEST/BENCH INFRASTRUCTURE ONLY: used by tests/ as a checker and by bench.py's `cpu_baseline` leg
as the timed CPU path.  The product path (boxfusion_amd.pipeline) never imports it.

Per keyframe, in the reference's order:
  transform2world (boxes.py:825-833) -> project_3d_boxes (instances.py:333-369)
  -> first keyframe: initialise (demo.py:226-241)
  -> else: cat, nms_3d + record (instances.py:22-101, box_manager.py:40-88)
     -> new boxes kept: correspondence_association (instances.py:411-490), update, boxfusion
        (box_fusion.py:622-724);  none kept: all_pred_box[mask] (demo.py:300-304)
The kernels (obb_iou_matrix, nms_scan, corr_assoc, fusion_fit) are the C restatement pinned
bit-exact against the reference traces (tests/test_oracle_golden.py); transform2world and the
projection repeat the reference's own torch f32 CPU expressions.  The whole chain is pinned against
the recorded traces by tests/test_oracle_chain.py.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle as OR


def transform2world(xyzlhw, R, pose):
    """boxes.py:825-833, same torch f32 CPU expressions (bit-identical on CPU)."""
    t = torch.from_numpy(np.ascontiguousarray(xyzlhw, np.float32)).clone()
    Rt = torch.from_numpy(np.ascontiguousarray(R, np.float32))
    cp = torch.from_numpy(np.repeat(np.asarray(pose, np.float32)[None], len(t), 0))
    t[:, :3] = (cp[:, :3, :3] @ t[:, :3].unsqueeze(-1) + cp[:, :3, 3:]).squeeze(-1)
    return t.numpy(), (cp[:, :3, :3] @ Rt).numpy()


def project_3d_boxes(corners, poses, K, H, W):
    """instances.py:333-369, same torch f32 CPU expressions."""
    c = torch.from_numpy(np.ascontiguousarray(corners, np.float32))
    n = c.shape[0]
    homo = torch.cat([c, torch.ones((n, 8, 1))], dim=2)
    pinv = torch.linalg.inv(torch.from_numpy(np.ascontiguousarray(poses, np.float32)))
    cam = torch.einsum("nij,nkj->nki", pinv, homo)
    X, Y, Z = cam[..., 0], cam[..., 1], cam[..., 2]
    K = np.asarray(K, np.float32)
    u = torch.clamp(K[0, 0] * X / Z + K[0, 2], 0, W)
    v = torch.clamp(K[1, 1] * Y / Z + K[1, 2], 0, H)
    return torch.stack([u, v], dim=-1).numpy()


class OracleChain:
    def __init__(self, cfg, K3, H=480, W=640, pst=None, legacy=True):
        self.cfg, self.H, self.W = cfg, H, W
        self.K3 = np.asarray(K3, np.float32)
        K4 = np.eye(4, dtype=np.float32)
        K4[:3, :3] = self.K3
        bf, asc = cfg["box_fusion"], cfg["association"]
        self.fcfg = OR.fuse_cfg(cfg, K4, H, W, legacy=legacy)
        self.pst = pst
        cap = 64
        self.ncfg = OR.NmsCfg()
        self.ncfg.iou_threshold = bf["nms_threshold"]
        self.ncfg.translation_gap, self.ncfg.rotation_gap = asc["translation_gap"], asc["rotation_gap"]
        self.ncfg.center_gap, self.ncfg.max_list, self.ncfg.list_capacity = 0.5, 5, cap
        self.ccfg = OR.CorrCfg()
        self.ccfg.small_size, self.ccfg.threshold = bf["small_size"], asc["small_threshold"]
        self.ccfg.translation_gap, self.ccfg.rotation_gap = asc["translation_gap"], asc["rotation_gap"]
        self.ccfg.W, self.ccfg.H = float(W), float(H)
        self.ccfg.max_list, self.ccfg.list_capacity = 5, cap
        self.use_fusion = bf.get("use", True)
        self.g = None            # global boxes: dict of arrays (all_pred_box)
        self.pf = None           # per-frame boxes (per_frame_ins)
        self.fusion_list, self.already_fusion = [], []
        self.box_count = 0
        self.num_record, self.all_kf_pose = {}, {}

    @staticmethod
    def _cat(a, b):
        return {k: np.concatenate([a[k], b[k]], 0) for k in a}

    @staticmethod
    def _take(a, idx):
        return {k: v[idx] for k, v in a.items()}

    def keyframe(self, count, pose, det):
        """det: camera-frame detections {scores[n], pred_boxes[n,4], xyzlhw[n,6], R[n,3,3]}"""
        n = len(det["scores"])
        self.all_kf_pose[count] = pose
        if n == 0:
            self.num_record[count] = self.box_count
            return
        t, R = transform2world(det["xyzlhw"], det["R"], pose)
        poses = np.repeat(pose[None].astype(np.float32), n, 0)
        corners = OR.box_corners(t, R)
        pred = dict(tensor=t, R=R, scores=det["scores"].astype(np.float32),
                    boxes2d=det["pred_boxes"].astype(np.float32),
                    init_id=self.box_count + np.arange(n, dtype=np.int64),
                    valid_num=np.zeros(n, np.float32), pose=poses,
                    proj=project_3d_boxes(corners, poses, self.K3, self.H, self.W))
        self.box_count += n
        self.num_record[count] = self.box_count
        if self.g is None:
            self.g, self.pf = pred, pred
            self.fusion_list += [[i] for i in range(n)]
            return
        n_glo = len(self.g["scores"])
        self.fusion_list += [[len(self.pf["scores"]) + i] for i in range(n)]
        self.g = self._cat(self.g, pred)
        self.pf = self._cat(self.pf, pred)
        g = self.g
        corners = OR.box_corners(g["tensor"], g["R"])
        iou = OR.obb_iou_matrix(corners)
        r = OR.nms_scan(iou, corners, g["scores"], g["init_id"], self.pf["pose"], self.fusion_list,
                        g["valid_num"], self.ncfg)
        self.fusion_list = r["fusion_list"]
        g["valid_num"] = r["valid_num"]
        keep = r["keep"]
        if not (keep >= n_glo).any():
            self.g = self._take(g, keep)
            self.fusion_list = [self.fusion_list[i] for i in keep]
            return
        c = OR.corr_assoc(corners, g["tensor"][:, 3:6], g["scores"], g["boxes2d"], g["init_id"],
                          self.pf["pose"], pose, self.K3, n_glo, keep, r["success"],
                          self.fusion_list, g["valid_num"], self.ccfg)
        keep = c["keep"]
        g["valid_num"] = c["valid_num"]
        self.fusion_list = [c["fusion_list"][i] for i in keep]
        self.g = self._take(g, keep)
        if self.use_fusion:
            self._boxfusion()

    def _boxfusion(self):
        pf = self.pf
        for i, fl in enumerate(self.fusion_list):
            if len(fl) < 3 or fl in self.already_fusion:
                continue
            idx = np.asarray(fl)
            res = OR.fusion_fit(pf["tensor"][idx], pf["R"][idx], pf["scores"][idx], pf["pose"][idx],
                                pf["proj"][idx], self.pst, self.fcfg)
            if res["updated"]:
                self.g["tensor"][i] = res["box"]
                self.already_fusion.append(list(fl))
