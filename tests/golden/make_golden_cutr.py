"""Golden CuTR fixture: run the REFERENCE detector (boxfusion/cubify_transformer.py, vit.py,
preprocessor.py) on a synthetic 640x480 RGB-D frame with seeded synthetic weights (same rule as
boxfusion_amd/weights.py) and record inputs, backbone features and the final instances.

Stand-ins only for absent third-party modules: timm.layers.Mlp (fc1 -> GELU -> fc2, the pinned
timm 1.0.19 layout) plus the stubs of make_golden.py.  Run: python tests/golden/make_golden_cutr.py [case.npz ...]
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (installs the shared stubs, puts the reference on sys.path)

timm = types.ModuleType("timm")
timm_layers = types.ModuleType("timm.layers")


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU,
                 norm_layer=None, bias=True, drop=0.0, use_conv=False):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.drop1 = nn.Dropout(drop)
        self.norm = nn.Identity()
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x):
        return self.drop2(self.fc2(self.norm(self.drop1(self.act(self.fc1(x))))))


timm_layers.Mlp = Mlp
timm.layers = timm_layers
sys.modules["timm"] = timm
sys.modules["timm.layers"] = timm_layers

from boxfusion.measurement import ImageMeasurementInfo, DepthMeasurementInfo  # noqa: E402
from boxfusion.sensor import SensorArrayInfo, PosedSensorInfo  # noqa: E402
from boxfusion.orientation import ImageOrientation, rotate_tensor  # noqa: E402
from boxfusion.capture_stream import get_camera_to_gravity_transform  # noqa: E402
from boxfusion.preprocessor import Augmentor, Preprocessor  # noqa: E402
from boxfusion.cubify_transformer import make_cubify_transformer  # noqa: E402

from boxfusion_amd.synthetic import Scene, frame_rgbd, SCANNET_K  # noqa: E402
from boxfusion_amd.weights import seeded_state_dict  # noqa: E402


def make_sample(rgb, depth, K, pose, image_hw=None):
    """restates ScannetDataset.__iter__ (capture_stream.py:185-311) for one in-memory frame; a
    depth smaller than the image gets its own info size and K scaled to its resolution"""
    H, W = image_hw if image_hw is not None else depth.shape
    Hd, Wd = depth.shape
    Kd = np.asarray(K, np.float32).copy()
    Kd[:2] *= Wd / W
    wide = PosedSensorInfo()
    wide.image = ImageMeasurementInfo(size=(W, H), K=torch.tensor(K)[None])
    depth_info = DepthMeasurementInfo(size=(Wd, Hd), K=torch.tensor(Kd)[None])
    wide.depth = depth_info
    result = dict(wide=dict())
    result["wide"]["image"] = torch.tensor(np.moveaxis(rgb, -1, 0))[None]
    result["wide"]["depth"] = torch.tensor(depth)[None].float()
    RT = torch.from_numpy(pose.astype(np.float32).reshape(4, 4))
    wide.RT = RT[None]
    cur, tgt = wide.orientation, ImageOrientation.UPRIGHT
    T_gravity = get_camera_to_gravity_transform(wide.RT[-1], cur, target=tgt)
    wide = wide.orient(cur, tgt)
    result["wide"]["image"] = rotate_tensor(result["wide"]["image"], cur, target=tgt)
    result["wide"]["depth"] = rotate_tensor(result["wide"]["depth"], cur, target=tgt)
    wide.RT = torch.eye(4)[None]
    wide.T_gravity = T_gravity[None]
    gt = PosedSensorInfo()
    gt.RT = RT[None]
    gt.depth = depth_info
    si = SensorArrayInfo()
    si.wide = wide
    si.gt = gt
    result["meta"] = dict(video_id=0, timestamp=0)
    result["sensor_info"] = si
    return result, T_gravity, cur


FILTER_CFG = dict(  # demo.py:138-148 thresholds: scannet.yaml + cubicle.yaml's size_max_thres
    scannet=dict(score_thresh=0.5, uv_bound_value=0.9, floor_ratio=15, size_max_thres=0.5),
    ca1m=dict(score_thresh=0.4, uv_bound_value=0.9, floor_ratio=15, size_max_thres=0.5),
)


def filter_masks(pred, W, H, thr):
    """the reference's own BoxManager filters (box_manager.py:217-245) on all 100 instances, each
    mask separately, plus the sequential demo.py:138-148 survivor indices"""
    from boxfusion.box_manager import BoxManager
    cfg = dict(association=dict(rotation_gap=30, translation_gap=0.8), box_fusion=dict(small_size=0.35))
    bm = BoxManager(cfg)
    score = (pred.scores >= float(thr["score_thresh"])).numpy()
    uv = bm.check_uv_bounds(pred.pred_proj_xy, W, H, ratio=thr["uv_bound_value"]).numpy()
    floor = bm.check_floor_mask(pred.pred_boxes_3d.tensor, ratio=thr["floor_ratio"]).numpy()
    large = bm.check_large_mask(pred.pred_boxes_3d.tensor, thres=thr["size_max_thres"]).numpy()
    idx = np.arange(len(score))
    p = pred[pred.scores >= float(thr["score_thresh"])]
    idx = idx[score]
    m = bm.check_uv_bounds(p.pred_proj_xy, W, H, ratio=thr["uv_bound_value"])
    p, idx = p[m], idx[m.numpy()]
    m = bm.check_floor_mask(p.pred_boxes_3d.tensor, ratio=thr["floor_ratio"])
    p, idx = p[~m], idx[~m.numpy()]
    m = bm.check_large_mask(p.pred_boxes_3d.tensor, thres=thr["size_max_thres"])
    idx = idx[~m.numpy()]
    return dict(mask_score=score, mask_uv=uv, mask_floor=floor, mask_large=large,
                kept_sequential=idx.astype(np.int64))


def run_case(name, dim, frame, seed, H, W, ratio, K, thr, keep_features=False):
    """one frame through demo.py:129-136's exact sequence on the reference:
    augmentor.package -> move_input_to_current_device(., model.pixel_mean) -> preprocess -> model"""
    from boxfusion.preprocessor import move_input_to_current_device
    torch.set_num_threads(8)
    model = make_cubify_transformer(dimension=dim, depth_model=True).eval()
    model.load_state_dict(seeded_state_dict(model, seed))
    keys = np.array(sorted(f"{k}:{tuple(v.shape)}" for k, v in model.state_dict().items()))
    rgb, depth = frame_rgbd(frame, H, W)
    if ratio > 1:           # a lower-resolution depth sensor: every ratio-th pixel
        depth = np.ascontiguousarray(depth[::ratio, ::ratio])
    pose = Scene().pose(frame)
    sample, T_gravity, orient = make_sample(rgb, depth, K, pose, image_hw=(H, W))
    aug = Augmentor(("wide/image", "wide/depth"))
    pre = Preprocessor()
    packaged = pre.preprocess([move_input_to_current_device(aug.package(sample), model.pixel_mean)])
    sensor = packaged["wide"]
    with torch.no_grad():
        feats = model.backbone(sensor)[0].tensors
        pred = model(packaged)[0]
    out = dict(
        dim=np.int32(dim), frame=np.int32(frame), seed=np.int32(seed), H=np.int32(H), W=np.int32(W),
        ratio=np.int32(ratio), K=np.asarray(K, np.float32), keys=keys,
        orientation=np.int32(orient.value), T_gravity=T_gravity.numpy(),
        depth_params=np.asarray(sensor["depth"].info[0].parameters, np.float32).reshape(-1),
        image_sum=np.float64(sensor["image"].data.tensor.double().sum()),
        pad=np.int32(sensor["image"].data.tensor.shape[-1]),
        depth_pad=np.int32(sensor["depth"].data.tensor.shape[-1]),
        scores=pred.scores.numpy(), pred_classes=pred.pred_classes.numpy(),
        pred_boxes=pred.pred_boxes.numpy(), pred_logits=pred.pred_logits.numpy(),
        boxes3d=pred.pred_boxes_3d.tensor.numpy(), R=pred.pred_boxes_3d.R.numpy(),
        object_desc=pred.object_desc.numpy().astype(np.float16),
        pred_proj_xy=pred.pred_proj_xy.numpy())
    # the same frame with the proposal content embedding made uniform (weights.py
    # uniform_queries): the end-to-end GPU test compares these instances one by one
    model_u = make_cubify_transformer(dimension=dim, depth_model=True).eval()
    model_u.load_state_dict(seeded_state_dict(model_u, seed, uniform_queries=True))
    # the encoder's proposal logits (EncoderProposals.get_proposals, cubify_transformer.py:918-943):
    # query slot q of the decoder is the proposal of top-300 rank q, so an instance whose proposal
    # sits at the top-300 cut can trade places with the 301st under bf16 rounding
    from boxfusion.cubify_transformer import EncoderProposals
    seen = {}
    orig_gp, orig_inf = EncoderProposals.get_proposals, EncoderProposals.inference_single_image

    def get_proposals(self, *a, **k):
        enc, inst = orig_gp(self, *a, **k)
        seen["logits"] = enc[0].pred_logits[..., 0].detach().clone()
        return enc, inst

    def inference_single_image(self, output, image_size, topk):
        # the query slot of every instance (the reference takes rows topk_index // 2)
        idx = torch.topk(output.pred_logits.sigmoid().view(-1), topk)[1]
        seen["query"] = (idx // output.pred_logits.shape[-1]).clone()
        return orig_inf(self, output, image_size, topk)
    EncoderProposals.get_proposals = get_proposals
    EncoderProposals.inference_single_image = inference_single_image
    try:
        with torch.no_grad():
            pu = model_u(packaged)[0]
    finally:
        EncoderProposals.get_proposals = orig_gp
        EncoderProposals.inference_single_image = orig_inf
    enc_sorted = torch.sort(seen["logits"], descending=True)[0]
    out["uq_enc_logits_sorted"] = enc_sorted[:320].numpy()
    out["uq_query"] = seen["query"].numpy().astype(np.int32)
    out.update(uq_scores=pu.scores.numpy(), uq_pred_classes=pu.pred_classes.numpy(),
               uq_pred_boxes=pu.pred_boxes.numpy(), uq_pred_logits=pu.pred_logits.numpy(),
               uq_boxes3d=pu.pred_boxes_3d.tensor.numpy(), uq_R=pu.pred_boxes_3d.R.numpy(),
               uq_object_desc=pu.object_desc.numpy().astype(np.float16),
               uq_pred_proj_xy=pu.pred_proj_xy.numpy())
    if keep_features:
        out["features"] = feats.numpy()          # f32: the GPU test feeds them to the decoder
    out["depth_sum"] = np.float64(sensor["depth"].data.tensor.double().sum())
    out.update(filter_masks(pred, W, H, thr))
    # random weights put every score / size on one side of the config thresholds: a second set of
    # thresholds at the medians of this prediction splits each mask (recorded with the masks)
    dims = pred.pred_boxes_3d.tensor[:, 3:]
    med = dict(score_thresh=float(pred.scores.median()), uv_bound_value=thr["uv_bound_value"],
               floor_ratio=float((dims.amax(1) / dims.amin(1)).median()),
               size_max_thres=float(dims.amax(1).median()))
    out.update({k + "_med": v for k, v in filter_masks(pred, W, H, med).items()})
    out["thr"] = np.array([thr[k] for k in ("score_thresh", "uv_bound_value", "floor_ratio", "size_max_thres")])
    out["thr_med"] = np.array([med[k] for k in ("score_thresh", "uv_bound_value", "floor_ratio", "size_max_thres")])
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(name, {k: getattr(v, "shape", v) for k, v in out.items() if k != "keys"})


CA1M_K = np.array([[360.0, 0.0, 191.5], [0.0, 360.0, 255.5], [0.0, 0.0, 1.0]], np.float32)


CASES = {
    # ScanNet-shaped frame (640x480, depth at image resolution): the synthetic stream's camera
    "cutr_vit_t.npz": (192, 7, 0, 480, 640, 1, SCANNET_K, "scannet"),
    # CA-1M-shaped portrait frame (384 wide x 512 tall, ca1m.yaml cam) with a half-resolution depth
    "cutr_ca1m_r2.npz": (192, 11, 1, 512, 384, 2, CA1M_K, "ca1m"),
    # quarter-resolution depth at 640x480
    "cutr_r4.npz": (192, 3, 2, 480, 640, 4, SCANNET_K, "scannet"),
    # configs[1] as CA1MDataset streams it: depth resized to the image (capture_stream.py:445-459),
    # i.e. RGB:depth ratio 1 on the 512 x 384 portrait frame
    "cutr_ca1m_r1.npz": (192, 13, 3, 512, 384, 1, CA1M_K, "ca1m"),
    # the bench's width: ViT-B (dim 768, 12 x 64 heads, MLP 3072; cubify_transformer.py:1232-1240)
    "cutr_vitb.npz": (768, 5, 4, 480, 640, 1, SCANNET_K, "scannet"),
}


def main(names=None):
    for name in (names or CASES):
        dim, frame, seed, H, W, ratio, K, thr = CASES[name]
        run_case(name, dim, frame, seed, H, W, ratio, K, FILTER_CFG[thr], keep_features=True)


if __name__ == "__main__":
    main(sys.argv[1:])
