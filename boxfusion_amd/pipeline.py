"""Per-frame detect + multi-view fusion, in demo.py `run()` order (demo.py:88-332), on the GPU.

    DetectStage  (independent per frame; batched B frames per call)
      a1  depth standardisation            bf_depth_standardize          preprocessor.py:97-129
      a13 depth back-projection            bf_backproject                 tools/utils.py:232-287
      a2-a9 CuTR RGB-D forward             CuTREngine (MFMA kernels)      cubify_transformer.py
      a10 detection filters                bf_detection_filter            demo.py:138-148
      a11 scale_boxes + crop + CLIP        CLIPEngine (fused crop/resize  tools/utils.py:355-495
          + text match                      im2col + MFMA ViT-H/14)       demo.py:162-171
    FusionStage  (serial over keyframes, fusion_stage.py)                demo.py:200-305

`Pipeline.run(stream)` drives both over a frame stream with the reference's keyframe rule
(`count % gap == 0`, plus the last-frame re-entry).  The detection batch is the unit that shards
across GPUs (bench.py); fusion consumes keyframes strictly in frame order.
"""
from __future__ import annotations

import inspect
import os

import numpy as np
import torch

from boxfusion_amd import _lib
from boxfusion_amd.box_manager import BoxManager
from boxfusion_amd.engine import CLIPEngine, CuTREngine
from boxfusion_amd.fusion_stage import FusionStage
from boxfusion_amd.instances import Instances3D
from boxfusion_amd.preprocessor import square_pad_size
from boxfusion_amd.sensor import camera_to_gravity
from boxfusion_amd.tools_utils import match_features

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")

# keys read by demo.py that only cubicle.yaml defines: documented defaults
DETECTION_DEFAULTS = dict(class_sim_thres=25.0, size_max_thres=None)
FUSION_DEFAULTS = dict(clip_sim_coeff=1.0)


def load_class_names():
    with open(os.path.join(DATA, "panoptic_categories_nomerge.txt")) as f:
        return [ln.strip() for ln in f if ln.strip()]


def load_class_features():
    return torch.from_numpy(np.load(os.path.join(DATA, "class_features.npy")).astype(np.float32))


def scale_boxes(boxes, H, W, scale=1.2):
    """tools/utils.py:355-381 on device (same f32 expression order)."""
    cx = (boxes[:, 0] + boxes[:, 2]) / 2
    cy = (boxes[:, 1] + boxes[:, 3]) / 2
    w = (boxes[:, 2] - boxes[:, 0]) * scale
    h = (boxes[:, 3] - boxes[:, 1]) * scale
    return torch.stack([torch.clamp(cx - w / 2, 0, W), torch.clamp(cy - h / 2, 0, H),
                        torch.clamp(cx + w / 2, 0, W), torch.clamp(cy + h / 2, 0, H)], 1)


def detection_mask(scores, proj_xy, box3d, cfg, H, W):
    """demo.py:138-148 filters for a [B,100] batch (score, uv bound, floor, large) in one
    bf_detection_filter launch.  The reference filters sequentially (each mask on the survivors
    of the previous one); the masks are per-instance, so their conjunction is the same set."""
    return _lib.detection_filter(scores, proj_xy, box3d, _lib.filter_cfg(cfg["detection"], W, H))


class DetectStage:
    """Everything demo.py does per frame before the fusion step, for a batch of B frames.

    crop_source: "filtered" (reference: CLIP on every instance surviving the filters),
    "top" (throughput runs with random weights: CLIP on the top `crops_per_frame` instances of
    every frame, so the CLIP tower does the work it would do on real detections) or "given"
    (CLIP on `crops_per_frame` caller-supplied boxes per frame, `crop_boxes` of __call__: the
    benchmark crops the seeded scene's detections, whose features then travel with them into
    fusion).

    The device work reads fixed input buffers (frames, depth, T_gravity, K, K^-1) and is free of
    host synchronisation; with `graph=True` it is captured once into a HIP graph and replayed
    (one launch per batch instead of ~2000).  "filtered" mode captures CuTR + filters and runs
    the variable-size CLIP step eagerly; "top" mode captures CLIP as well."""

    def __init__(self, cutr_model, clip_visual, cfg, batch, H=480, W=640, K3=None, text_features=None,
                 class_names=None, crops_per_frame=16, crop_source="filtered", backproject=True,
                 clip_capacity=256, device="cuda", graph=False, clip_fp8=False, depth_ratio=1):
        self.cfg = cfg
        self.dev = torch.device(device)
        self.B, self.H, self.W = batch, H, W
        self.r = int(depth_ratio)        # RGB:depth resolution ratio (CA-1M: 2 or 4)
        self.pad = square_pad_size(H, W)
        self.cutr = CuTREngine(cutr_model, batch, H, W, pad=self.pad, device=device, depth_ratio=self.r)
        self.clip = (CLIPEngine(clip_visual, clip_capacity, device=device, fp8=clip_fp8)
                     if clip_visual is not None else None)
        self.K3 = np.asarray(K3, np.float32)
        self.K_host = np.stack([self.K3] * batch)
        self.K_dev = torch.from_numpy(self.K_host).to(self.dev)
        self.Kinv_dev = torch.linalg.inv(self.K_dev)
        # the depth map's intrinsics (image K at 1/r, the synthetic CA-1M K_depth) for unproject
        Kd = self.K3.copy()
        Kd[:2] /= self.r
        self.Kd_dev = torch.from_numpy(np.stack([Kd] * batch)).to(self.dev)
        self.text = (text_features if text_features is not None else load_class_features()).to(self.dev).contiguous()
        names = class_names if class_names is not None else load_class_names()
        self.prompt = np.concatenate([np.asarray(names), np.full(1, "")])
        self.crops_per_frame = crops_per_frame
        self.crop_source = crop_source
        self.backproject = backproject
        det = dict(DETECTION_DEFAULTS, **cfg["detection"])
        self.sim_thres = float(det["class_sim_thres"])
        self.scale_box = float(det.get("scale_box", 1.2))
        self.coeff = float(dict(FUSION_DEFAULTS, **cfg["box_fusion"])["clip_sim_coeff"])
        # fixed input buffers (the graph reads these)
        self.in_rgb = torch.zeros((batch, H, W, 3), dtype=torch.uint8, device=self.dev)
        self.in_depth = torch.zeros((batch, H // self.r, W // self.r), dtype=torch.float32, device=self.dev)
        self.in_Tg = torch.zeros((batch, 3, 3), dtype=torch.float32, device=self.dev)
        self.in_pose = torch.zeros((batch, 4, 4), dtype=torch.float32, device=self.dev)
        # the depth kernels' workspace (zero-filled, left zeroed by every call; eager and graph
        # replays of this stage use it one at a time)
        self.ds_ws = _lib.new_depth_workspace(batch, H // self.r, W // self.r, self.dev)
        k = crops_per_frame
        self.top_b = torch.arange(batch, device=self.dev).repeat_interleave(k)
        self.top_b32 = self.top_b.to(torch.int32)
        self.top_i = torch.arange(k, device=self.dev).repeat(batch)
        # crop_source "given": the caller supplies k 2-D boxes (xyxy, image pixels) per frame
        self.in_crops = torch.zeros((batch * k, 4), dtype=torch.float32, device=self.dev)
        self.use_graph = graph
        self.graph = None
        self.out = {}
        self.last = {}

    def text_prompt(self, frames_u8, boxes, frame_idx):
        """tools/utils.py:478-495 + retriev :383-403 for crops of several frames at once.
        Returns (category index [N] into self.prompt, L2-normalised features [N,1024], max sims)."""
        feats = []
        cap = self.clip.N
        bi = scale_boxes(boxes, self.H, self.W, self.scale_box).to(torch.int32)
        for s in range(0, boxes.shape[0], cap):
            feats.append(self.clip(frames_u8, bi[s:s + cap].contiguous(), frame_idx[s:s + cap].contiguous()))
        f = torch.cat(feats, 0) if len(feats) > 1 else feats[0]
        # normalise, in-place text renorm every call (quirk 4), threshold column, argmax
        return match_features(f, self.text, self.sim_thres)

    def _device_forward(self):
        """host-sync-free device work on the input buffers -> self.out"""
        B, H, W = self.B, self.H, self.W
        if self.backproject:
            # depth standardisation + unproject of the same depth maps in one pass (demo.py:121-131)
            dstd, params, xyz, valid = _lib.depth_preprocess(self.in_depth, self.Kd_dev, self.in_pose, 10.0,
                                                             ws=self.ds_ws)
            self.out["xyz"] = [(xyz[b], valid[b]) for b in range(B)]
        else:
            dstd, params = _lib.depth_standardize(self.in_depth, ws=self.ds_ws)
        res = self.cutr(self.in_rgb, dstd, params, self.K_dev, self.in_Tg, [(H, W)] * B,
                        K_host=self.K_host, K_inv=self.Kinv_dev)
        scores = torch.stack([r.scores for r in res])
        proj = torch.stack([r.pred_proj_xy for r in res])
        box3d = torch.stack([r.pred_boxes_3d.tensor for r in res])
        self.out.update(res=res, keep=detection_mask(scores, proj, box3d, self.cfg, H, W),
                        boxes2d=torch.stack([r.pred_boxes for r in res]))
        if self.clip is not None and self.crop_source in ("top", "given"):
            bidx, iidx = self.top_b, self.top_i
            boxes = (self.in_crops if self.crop_source == "given"
                     else self.out["boxes2d"][bidx, iidx].contiguous())
            cat_idx, feats, sims = self.text_prompt(self.in_rgb, boxes, self.top_b32)
            self.out["clip"] = (bidx, iidx, cat_idx, feats, sims)

    def _run_device(self):
        if not self.use_graph:
            self._device_forward()
            return
        if self.graph is None:
            # warm up (kernel attributes, ray-embedding cache, allocator pools) on a side stream
            s = torch.cuda.Stream(device=self.dev)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._device_forward()
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            # thread-local capture: other threads (the fusion worker) keep running their own work
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self._device_forward()
        self.graph.replay()

    @torch.no_grad()
    def preprocess_frames(self, depth, poses):
        """demo.py:121-131 on frames that are not keyframes: depth standardisation (Preprocessor)
        and, with backproject, the unproject of the same depth (viz_on_gt_points, on by default)
        -- one bf_depth_preprocess pass over any number of frames.  Nothing reads the results
        back (in the reference they feed rerun only); they stay in self.last_frames."""
        n = depth.shape[0]
        self.last_frames = None          # release the previous call's outputs before allocating
        if self.backproject:
            RT = torch.from_numpy(np.ascontiguousarray(poses, np.float32)).to(self.dev, non_blocking=True)
            self.last_frames = _lib.depth_preprocess(depth, self.Kd_dev[:1].expand(n, 3, 3), RT, 10.0)
        else:
            self.last_frames = _lib.depth_standardize(depth)
        return self.last_frames

    @torch.no_grad()
    def __call__(self, rgb_u8, depth, poses, return_instances=True, crop_boxes=None):
        """rgb_u8 [B,H,W,3] u8, depth [B,H,W] f32 (device), poses [B,4,4] host -> list of B
        Instances3D (camera frame, filtered, with categories / features / CLIP-adjusted scores).
        With return_instances=False (throughput runs) nothing is read back: results stay in
        self.last (device tensors) and the call never waits for the device.
        crop_boxes: f32 device [B*crops_per_frame, 4] (crop_source "given")."""
        B, H, W = self.B, self.H, self.W
        assert rgb_u8.shape == (B, H, W, 3) and depth.shape == (B, H // self.r, W // self.r)
        self.in_rgb.copy_(rgb_u8, non_blocking=True)
        self.in_depth.copy_(depth, non_blocking=True)
        if self.crop_source == "given":
            if crop_boxes is None or tuple(crop_boxes.shape) != tuple(self.in_crops.shape):
                raise ValueError(f"crop_source='given' needs crop_boxes of shape {tuple(self.in_crops.shape)}")
            self.in_crops.copy_(crop_boxes, non_blocking=True)
        poses = np.asarray(poses, np.float32)
        self.in_Tg.copy_(torch.from_numpy(np.stack([camera_to_gravity(p) for p in poses])))
        self.in_pose.copy_(torch.from_numpy(poses))
        self._run_device()
        o = self.out
        self.last = dict(xyz=o.get("xyz"), keep=o["keep"], res=o["res"])
        if "clip" in o:
            self.last["clip"] = o["clip"]
        if not return_instances:
            return None
        res, keep = o["res"], o["keep"]
        out = [r[keep[b]] for b, r in enumerate(res)]
        if self.clip is None or self.crop_source in ("top", "given"):
            return out
        # reference mode: CLIP on every surviving instance (variable count, eager)
        bidx, iidx = keep.nonzero(as_tuple=True)
        if bidx.numel() == 0:
            return out
        cat_idx, feats, sims = self.text_prompt(self.in_rgb, o["boxes2d"][bidx, iidx].contiguous(),
                                                bidx.to(torch.int32))
        self.last["clip"] = (bidx, iidx, cat_idx, feats, sims)
        counts = keep.sum(1).tolist()
        ci = cat_idx.cpu().numpy()
        off = 0
        final = []
        for b, r in enumerate(out):
            n = counts[b]
            if n == 0:
                final.append(r)
                continue
            # scatter back per frame: categories, features, scores += coeff * sim / 100
            r.categories = self.prompt[ci[off:off + n]]
            r.features = feats[off:off + n]
            r.scores = r.scores + self.coeff * sims[off:off + n] / 100.0
            final.append(r[r.categories != ""])
            off += n
        return final


def scene_instances(det, device, H=480, W=640):
    """Instances3D from a synthetic-scene detection dict (boxfusion_amd.synthetic.Scene)."""
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    p = Instances3D((H, W))
    p.scores = torch.from_numpy(det["scores"]).to(device)
    p.pred_boxes = torch.from_numpy(det["pred_boxes"]).to(device)
    p.pred_boxes_3d = GeneralInstance3DBoxes(torch.from_numpy(det["xyzlhw"]).to(device),
                                             torch.from_numpy(det["R"]).to(device))
    p.pred_proj_xy = torch.from_numpy(det["proj_xy"]).to(device)
    return p


def _viz_images(viz, rgb, depth, j):
    """(image, depth) of frame j on the host for a FrameLogger that logs images (demo.py:180-190
    logs the RGB frame and the raw depth of every frame); (None, None) otherwise"""
    if not getattr(viz, "log_images", False) or rgb is None:
        return None, None
    return rgb[j].cpu().numpy(), depth[j].cpu().numpy()


class Pipeline:
    """demo.py run() over a stream of (rgb, depth, pose) frames: every frame goes through the
    per-frame preprocessing, keyframes (count % gap == 0) through CuTR + CLIP, and the fusion
    state machine in frame order."""

    def __init__(self, detect: DetectStage, fusion: FusionStage, gap):
        self.detect, self.fusion, self.gap = detect, fusion, gap

    def run(self, frames, n_frames, per_frame=True, frames_per_call=64, viz=None):
        """frames(ids) -> (rgb [b,H,W,3] u8 dev, depth [b,H,W] f32 dev, poses [b,4,4] host).
        A frames callable that takes a `need_rgb` keyword is called with need_rgb=False for the
        non-keyframes whose RGB nothing reads (their per-frame work uses depth and pose only) and
        may return None for rgb then.
        per_frame: the frames between keyframes get demo.py:121-131's per-frame work too
        (DetectStage.preprocess_frames, up to `frames_per_call` frames per call).
        viz: a visualize.FrameLogger -- demo.py's per-frame rerun calls (pose, pinhole, image,
        depth, trajectory) for every frame in frame order and the global boxes after each
        keyframe's fusion (host side, after the frame's GPU work; not used by the bench)."""
        B = self.detect.B
        kf = [i for i in range(n_frames) if i % self.gap == 0]
        try:
            lazy_rgb = "need_rgb" in inspect.signature(frames).parameters
        except (TypeError, ValueError):
            lazy_rgb = False
        nk_rgb = viz is not None and getattr(viz, "log_images", False)

        def nk_frames(ids_):
            return frames(ids_, need_rgb=nk_rgb) if lazy_rgb else frames(ids_)
        self.frames_preprocessed = 0
        for s in range(0, len(kf), B):
            ids = kf[s:s + B]
            nk_pose = {}           # non-keyframe poses of this batch, logged in frame order below
            if per_frame:
                nk = [i for i in range(ids[0], min(ids[-1] + self.gap, n_frames)) if i % self.gap != 0]
                for c in range(0, len(nk), frames_per_call):
                    _rgb, depth, poses = nk_frames(nk[c:c + frames_per_call])
                    self.detect.preprocess_frames(depth.contiguous(), poses)
                    self.frames_preprocessed += len(nk[c:c + frames_per_call])
                    if viz is not None:
                        for j, i in enumerate(nk[c:c + frames_per_call]):
                            nk_pose[i] = (np.asarray(poses[j]),) + _viz_images(viz, _rgb, depth, j)
            rgb, depth, poses = frames(ids)
            if len(ids) < B:   # ragged tail: pad the batch with the last frame, drop its results
                pad = B - len(ids)
                rgb = torch.cat([rgb, rgb[-1:].expand(pad, -1, -1, -1)])
                depth = torch.cat([depth, depth[-1:].expand(pad, -1, -1)])
                poses = np.concatenate([poses, np.repeat(poses[-1:], pad, 0)])
            preds = self.detect(rgb.contiguous(), depth.contiguous(), poses)
            for j, i in enumerate(ids):
                self.fusion.keyframe(i, poses[j], preds[j])
                if viz is not None:
                    # demo.py order: keyframe i's frame logs, its boxes after the fusion step, then
                    # the frames up to the next keyframe (the trajectory grows frame by frame)
                    viz.frame(i, poses[j], *_viz_images(viz, rgb, depth, j))
                    viz.boxes(self.fusion.all_pred_box, i)
                    for f in range(i + 1, min(i + self.gap, n_frames)):
                        if f in nk_pose:
                            viz.frame(f, *nk_pose[f])
        last = n_frames - 1
        if last % self.gap != 0:
            _, _, p = nk_frames([last])
            self.fusion.finish(last, p[0], False)
            if viz is not None:        # demo.py:330: the boxes after the last frame's block too
                viz.boxes(self.fusion.all_pred_box, last)
        return self.fusion
