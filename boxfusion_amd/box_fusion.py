"""Multi-view box fusion (reference: boxfusion/box_fusion.py).

`BoxFusion.boxfusion(all_pred_box, per_frame_box, box_manager)` keeps the reference's selection
rules (>= 3 views, list not already fused; box_fusion.py:631-635) and write-back semantics
(xyz + lhw refined, lhw >= 0.01, R unchanged; :716-724), but every box is refined by ONE call of
bf_fusion_fit with all iterations on the device (no per-iteration host round trip; the particle
evaluations of all boxes spread over the whole chip).
"""
from __future__ import annotations

import os
import warnings

import numpy as np
import torch

from boxfusion_amd import _lib

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def load_pst(path=None):
    """particle table [pst_size, 6] f32 (data/pst_1024_0.tiff in the reference)."""
    if path and path.endswith(".npy") and os.path.exists(path):
        return np.load(path).astype(np.float32)
    if path and os.path.exists(path) and path.endswith((".tif", ".tiff")):
        from PIL import Image
        return np.array(Image.open(path)).astype(np.float32)
    return np.load(os.path.join(DATA, "pst_1024_0.npy")).astype(np.float32)


_HULL_WARNED = [False]


def _warn_hull_once():
    if _HULL_WARNED[0]:
        return
    _HULL_WARNED[0] = True
    warnings.warn("BoxFusion.boxfusion: a particle's 2-D intersection hull has more than the 8 points "
                  "the reference kernel's convex_inter[8] holds (box_fusion.py:381; undefined "
                  "behaviour there); the exact hull was used.  BoxFusion.hull_overflow_calls counts "
                  "the calls; cfg box_fusion.strict_hull=True raises instead.", RuntimeWarning,
                  stacklevel=4)


class BoxFusion:
    def __init__(self, cfg, device="cuda", legacy_promotion=True):
        self.cfg = cfg
        self.PST = load_pst(cfg["box_fusion"].get("pst_path"))
        self.K = np.eye(4)
        cam = cfg.get("cam", {})
        basedir = str(cfg.get("data", {}).get("datadir", ""))
        if "scannet" in basedir.lower() or cfg.get("dataset") == "online" or \
                ("fx" in cam and not basedir):
            # box_fusion.py:36-42: the config's camera
            self.K[:3, :3] = [[cam["fx"], 0.0, cam["cx"]], [0.0, cam["fy"], cam["cy"]], [0, 0, 1]]
            self.H, self.W = cam["H"], cam["W"]
        else:
            # CA-1M (box_fusion.py:44-51): the sequence's K_depth.txt, H / W swapped (portrait);
            # demo.py:117 replaces both with the first frame's image K and size anyway
            kd = os.path.join(basedir, "K_depth.txt")
            if os.path.exists(kd):
                Kd = np.loadtxt(kd).reshape(3, 3)
                self.K[:3, :3] = [[Kd[0, 0], 0.0, Kd[0, 2]], [0.0, Kd[1, 1], Kd[1, 2]], [0, 0, 1]]
            elif "fx" not in cam:
                # the reference's np.loadtxt raises here; demo.py:117 would replace K before the
                # first fusion anyway, so warn (a run without update_intrinsics fuses with K = I)
                warnings.warn(f"BoxFusion: {kd} not found and cfg.cam has no fx: K stays identity "
                              "until update_intrinsics() (the reference raises here)", RuntimeWarning,
                              stacklevel=2)
            self.H, self.W = cam.get("W", 480), cam.get("H", 640)
        self.update_K_flag = False
        bf = cfg["box_fusion"]
        ro = bf["random_opt"]
        self.fusion_iters = int(bf["iters"])
        self.pst_size = int(bf["pst_size"])
        self.center_init_size = ro["center_init_size"]
        self.center_scaling_coefficient = ro["center_scaling_coefficient"]
        self.shape_init_size = ro["shape_init_size"]
        self.shape_scaling_coefficient = ro["shape_scaling_coefficient"]
        # numpy<2 value-based promotion (requirements.txt pins numpy 1.26.4) unless overridden
        self.legacy_promotion = bool(bf.get("legacy_promotion", legacy_promotion))
        self.device = torch.device(device)
        self._pst_dev = torch.from_numpy(self.PST[: self.pst_size]).to(self.device).contiguous()
        self.last_stats = {}
        self.updated_total = 0    # boxes updated over every call (resolved results)
        # BF_DEV_HULL_OVERFLOW policy: False = count + warn once (the exact hull is used),
        # True = raise (cfg box_fusion.strict_hull)
        self.strict_hull = bool(bf.get("strict_hull", False))
        self.hull_overflow_calls = 0    # boxfusion calls with >= 1 such evaluation
        self.fit_calls = 0              # boxfusion calls that refined >= 1 box

    def update_intrinsics(self, size, K):
        self.H = size[1]
        self.W = size[0]
        self.K[:3, :3] = K

    def fuse_cfg(self):
        c = _lib.FuseCfg()
        c.iters = self.fusion_iters
        c.pst_size = self.pst_size
        c.max_accept = 200
        c.legacy_promotion = 1 if self.legacy_promotion else 0
        c.center_init = float(self.center_init_size)
        c.shape_init = float(self.shape_init_size)
        c.center_coef = float(self.center_scaling_coefficient)
        c.shape_coef = float(self.shape_scaling_coefficient)
        c.beta = 0.9
        c.min_scale = 1e-3
        c.img_h, c.img_w = float(self.H), float(self.W)
        k = self.K.astype(np.float32).reshape(-1)
        for i in range(16):
            c.K[i] = float(k[i])
        return c

    def boxfusion(self, all_pred_box, per_frame_box, box_manager, beta=0.9, verbose=False,
                  defer=False):
        """box_fusion.py:622-724 on bf_fusion_fit.  defer=True (FusionStage) writes the fused boxes
        back on the device and leaves the host bookkeeping (fusion_flag, already_fusion, stats)
        to the box manager's next read of that state, so no synchronisation happens here."""
        box_manager.flush()
        jobs, seen = [], set()
        for i, fl in enumerate(box_manager.fusion_list[: len(all_pred_box)]):
            if len(fl) >= 3 and not box_manager.check_if_fusion(fl):
                key = tuple(fl)
                if key in seen:   # an identical list earlier in this call wins (its result is the same)
                    continue
                seen.add(key)
                jobs.append((i, fl))
        self.last_stats = dict(jobs=len(jobs), updated=0, views=sum(len(f) for _, f in jobs))
        if not jobs:
            return
        self.fit_calls += 1
        dev = self.device
        nj = len(jobs)
        nv = np.array([len(fl) for _, fl in jobs], np.int32)
        off = np.concatenate([[0], np.cumsum(nv)[:-1]]).astype(np.int32)
        rows = np.array([i for i, _ in jobs], np.int32)
        # one upload: view offsets, view counts, target rows, flattened view indices
        host = np.concatenate([off, nv, rows] + [np.asarray(fl, np.int32) for _, fl in jobs])
        idx = _lib.h2d(host, dev)
        flat = idx[3 * nj:]
        b3 = per_frame_box.pred_boxes_3d
        # updated flags, iteration counts and the status word of the whole call: one read-back
        # (the view gather's BF_DEV_INDEX_RANGE and the fit's flags land in the same word)
        packed = torch.zeros(2 * nj + 1, dtype=torch.int32, device=dev)
        # every view's box, rotation, score, pose and 2-D hull in one gather launch
        vb, vr, vs, vp, vt = _lib.rows_gather(
            [(b3.tensor.contiguous(), None), (b3.R.contiguous(), None),
             (per_frame_box.scores.to(dev, torch.float32).contiguous(), None),
             (per_frame_box.cam_pose.to(dev, torch.float32).contiguous(), None),
             (per_frame_box.projected_boxes.contiguous(), None)], flat, status=packed[2 * nj:])
        out_box, packed, _ = _lib.fusion_fit(idx[:nj], idx[nj:2 * nj], vb, vr, vs, vp, vt,
                                             self._pst_dev, self.fuse_cfg(),
                                             max_views=min(int(nv.max()), 32), packed_out=True,
                                             packed=packed)
        # write-back of the updated rows on the device (xyz + lhw; R unchanged, quirk 6)
        target = all_pred_box.pred_boxes_3d.tensor
        if target.is_contiguous():
            _lib.fusion_writeback(out_box, packed[:nj], idx[2 * nj:3 * nj], target)
        else:
            rows_dev = idx[2 * nj:3 * nj].long()
            target[rows_dev] = torch.where(packed[:nj, None] != 0, out_box,
                                           target.index_select(0, rows_dev))

        def resolve():
            h = packed.cpu().numpy()
            upd, iters, st = h[:nj], h[nj:2 * nj], int(h[2 * nj])
            if st & _lib.BF_DEV_VIEW_OVERFLOW:
                raise _lib.HipError("bf_fusion_fit: a fusion list has more views than the kernel holds")
            if st & _lib.BF_DEV_INDEX_RANGE:
                raise _lib.HipError("boxfusion: a fusion list names a per-frame box that does not exist")
            if st & _lib.BF_DEV_HULL_TRUNC:
                raise _lib.HipError("bf_fusion_fit: more 2-D intersection candidates than the kernel "
                                    "holds (BF_DEV_HULL_TRUNC): the IoU would not be exact")
            if st & _lib.BF_DEV_HULL_OVERFLOW:
                # an intersection polygon with more points than the reference kernel's fixed
                # buffers hold (convex_inter[8] / corners_i[36], box_fusion.py:378-384; two
                # overlapping projected hexagons can intersect in up to 12 points): the reference
                # writes past its stack arrays there (undefined behaviour), the kernel here keeps
                # 64 slots and returns the exact IoU.  Counted per call (hull_overflow_calls) and
                # warned once per process by default; strict_hull raises.
                self.hull_overflow_calls += 1
                if self.strict_hull:
                    raise _lib.HipError("bf_fusion_fit: hull capacity exceeded (BF_DEV_HULL_OVERFLOW): "
                                        "the reference kernel overruns its fixed buffers on this input")
                _warn_hull_once()
            n_upd = 0
            for j, (i, fl) in enumerate(jobs):
                if upd[j]:
                    n_upd += 1
                    box_manager.update_fusion_flag(i)
                    box_manager.add_fusion_ind(fl)
            self.last_stats["updated"] = n_upd
            self.last_stats["iters"] = int(iters.sum())
            self.updated_total += n_upd

        if defer:
            box_manager._pending = resolve
        else:
            resolve()
