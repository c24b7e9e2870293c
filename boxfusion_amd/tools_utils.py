"""The hot-path helpers of the reference's tools/utils.py with its signatures (drop-in for the
calls demo.py makes: `unproject`, `scale_boxes`, `text_prompt`):

  unproject(depth, K, RT, max_depth)          tools/utils.py:232-287  -> bf_backproject
  scale_boxes(boxes, H, W, scale)             tools/utils.py:355-381  (numpy, as the reference)
  text_prompt(boxes, class_prompt, text_features, image, clip_model, preprocess, sim_thres)
                                              tools/utils.py:478-495 (crop_image :405-476,
                                              retriev :383-403)

text_prompt's CLIP step runs on the MI355X when `clip_model` is a `CLIPCropModel` (the fused
crop + bilinear 224x224 + CLIP normalise + im2col kernel feeding the MFMA ViT-H/14 engine, boxes
cropped on the device straight from the frame).  Any other model is called like the reference
calls SAMCLIP: `clip_model.get_batch_images_clip_features(list of 224x224x3 uint8 crops)`, the
crops cut with the reference's integer box semantics and resized on the device.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from boxfusion_amd import _lib


def unproject(depth, K, RT, max_depth=10.0):
    """depth [H,W] f32, K [3,3], RT [4,4] camera->world (device tensors) -> (world xyz [H,W,3],
    valid [H,W] = depth > 0 (& depth < max_depth))"""
    dev = depth.device
    return _lib.backproject(depth.float().contiguous(), torch.as_tensor(K, dtype=torch.float32, device=dev),
                            torch.as_tensor(RT, dtype=torch.float32, device=dev), max_depth=max_depth)


def scale_boxes(boxes, H, W, scale=1.2):
    """scale xyxy boxes about their centres and clip to the image (numpy f32 like the reference)"""
    cx = (boxes[:, 0] + boxes[:, 2]) / 2
    cy = (boxes[:, 1] + boxes[:, 3]) / 2
    w = (boxes[:, 2] - boxes[:, 0]) * scale
    h = (boxes[:, 3] - boxes[:, 1]) * scale
    return np.stack([np.clip(cx - w / 2, 0, W), np.clip(cy - h / 2, 0, H),
                     np.clip(cx + w / 2, 0, W), np.clip(cy + h / 2, 0, H)], axis=1)


def crop_boxes_int(boxes):
    """segment_image's integer crop box (tools/utils.py:436-437): int() truncation of each
    coordinate; the crop is image[y1:y2, x1:x2] (empty when x2 <= x1 or y2 <= y1)"""
    b = np.asarray(boxes)
    return np.trunc(b).astype(np.int64)


def match_features(img_features, text_features, sim_thres):
    """retriev's normalisation + similarity (tools/utils.py:397-401) and text_prompt's threshold
    column + argmax (:486-493).  text_features is renormalised IN PLACE, as the reference does on
    every call.  Returns (class index [N] into class_prompt + [""], normalised
    image features [N, D], max similarity [N])."""
    f = img_features / img_features.norm(dim=-1, keepdim=True)
    text_features /= text_features.norm(dim=-1, keepdim=True)
    if f.is_cuda:
        # (100 f) @ text^T as the reference groups it, on the f32 MFMA GEMM (bf_gemm_f32)
        from boxfusion_amd import _lib
        a, t = (100.0 * f).contiguous(), text_features.contiguous()
        K = a.shape[-1]
        if K % 4 or a.data_ptr() % 16 or t.data_ptr() % 16:
            # bf_gemm_f32 wants 16-B aligned rows: zero-pad K to a multiple of 4 in fresh (aligned)
            # buffers -- the added products are exact zeros, so the sums are unchanged
            K4 = (K + 3) // 4 * 4
            a = torch.nn.functional.pad(a, (0, K4 - K))
            t = torch.nn.functional.pad(t, (0, K4 - K))
        probs = _lib.gemm_f32(a, t)
    else:
        probs = 100.0 * f @ text_features.T
    probs = torch.cat([probs, torch.full_like(probs, float(sim_thres))[..., :1]], dim=-1)
    mx, idx = torch.max(probs, dim=-1)
    return idx, f, mx


class CLIPCropModel:
    """text_prompt's CLIP model on the MI355X: a CLIPEngine (ViT-H/14 visual tower) fed by the
    fused device crop kernel.  `encode_boxes(frames_u8 [F,H,W,3] device, boxes_i32 [N,4],
    frame_idx_i32 [N]) -> image features [N, 1024]`."""

    def __init__(self, visual, max_crops=256, device="cuda"):
        from boxfusion_amd.engine import CLIPEngine
        self.engine = CLIPEngine(visual, max_crops, device=device)
        self.device = self.engine.dev

    @torch.no_grad()
    def encode_boxes(self, frames_u8, boxes_i32, frame_idx_i32):
        out = []
        cap = self.engine.N
        for s in range(0, boxes_i32.shape[0], cap):
            out.append(self.engine(frames_u8, boxes_i32[s:s + cap].contiguous(),
                                   frame_idx_i32[s:s + cap].contiguous()))
        return torch.cat(out) if len(out) > 1 else out[0]


def _crops_224(image_u8_dev, ib):
    """the reference's crops (image[y1:y2, x1:x2]) resized to 224x224 (bilinear, rounded to
    uint8; a zero image for an empty crop), on the device -> list of numpy [224,224,3] uint8"""
    out = []
    H, W = image_u8_dev.shape[:2]
    for x1, y1, x2, y2 in ib.tolist():
        x1, y1 = max(x1, 0), max(y1, 0)
        x2, y2 = min(x2, W), min(y2, H)
        if x2 <= x1 or y2 <= y1:
            out.append(np.zeros((224, 224, 3), np.uint8))
            continue
        c = image_u8_dev[y1:y2, x1:x2].permute(2, 0, 1)[None].float()
        r = F.interpolate(c, (224, 224), mode="bilinear", align_corners=False)
        out.append(r[0].permute(1, 2, 0).round().clamp(0, 255).to(torch.uint8).cpu().numpy())
    return out


@torch.no_grad()
def text_prompt(boxes, class_prompt, text_features, image, clip_model, preprocess, sim_thres=0.0):
    """tools/utils.py:478-495: CLIP features of the crops of `boxes` (numpy xyxy, already scaled)
    in `image` (HWC uint8, numpy or device tensor), matched against `text_features` ->
    (categories np.ndarray[str] ("" below sim_thres), image features [N, D], max values [N])"""
    dev = text_features.device
    ib = crop_boxes_int(boxes)
    if isinstance(clip_model, CLIPCropModel):
        frame = image if isinstance(image, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(image))
        frame = frame.to(clip_model.device)[None].contiguous()
        bi = torch.from_numpy(ib.astype(np.int32)).to(clip_model.device)
        feats = clip_model.encode_boxes(frame, bi, torch.zeros(len(ib), dtype=torch.int32, device=clip_model.device))
    else:
        frame = (image if isinstance(image, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(image)))
        if torch.cuda.is_available():
            frame = frame.cuda()
        feats, _ = clip_model.get_batch_images_clip_features(_crops_224(frame, ib))
    idx, f, mx = match_features(feats.to(dev, torch.float32), text_features, sim_thres)
    prompt = np.concatenate([np.asarray(class_prompt), np.full_like(np.asarray(class_prompt), "")[..., :1]], axis=-1)
    return prompt[idx.cpu().numpy()], f, mx
