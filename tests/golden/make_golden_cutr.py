"""Golden CuTR fixture: run the REFERENCE detector (boxfusion/cubify_transformer.py, vit.py,
preprocessor.py) on a synthetic 640x480 RGB-D frame with seeded synthetic weights (same rule as
boxfusion_amd/weights.py) and record inputs, backbone features and the final instances.

Stand-ins only for absent third-party modules: timm.layers.Mlp (fc1 -> GELU -> fc2, the pinned
timm 1.0.19 layout) plus the stubs of make_golden.py.  Run: python tests/golden/make_golden_cutr.py
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


def make_sample(rgb, depth, K, pose):
    """restates ScannetDataset.__iter__ (capture_stream.py:185-311) for one in-memory frame"""
    H, W = depth.shape
    wide = PosedSensorInfo()
    wide.image = ImageMeasurementInfo(size=(W, H), K=torch.tensor(K)[None])
    depth_info = DepthMeasurementInfo(size=(W, H), K=torch.tensor(K)[None])
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


def main(dim=192, frame=7, seed=0):
    torch.set_num_threads(8)
    model = make_cubify_transformer(dimension=dim, depth_model=True).eval()
    sd = seeded_state_dict(model, seed)
    model.load_state_dict(sd)
    keys = np.array(sorted(f"{k}:{tuple(v.shape)}" for k, v in model.state_dict().items()))
    rgb, depth = frame_rgbd(frame)
    pose = Scene().pose(frame)
    sample, T_gravity, orient = make_sample(rgb, depth, SCANNET_K, pose)
    aug = Augmentor(("wide/image", "wide/depth"))
    pre = Preprocessor()
    packaged = pre.preprocess([aug.package(sample)])
    sensor = packaged["wide"]
    with torch.no_grad():
        feats = model.backbone(sensor)[0].tensors
        pred = model(packaged)[0]
    out = dict(
        dim=np.int32(dim), frame=np.int32(frame), seed=np.int32(seed), keys=keys,
        orientation=np.int32(orient.value), T_gravity=T_gravity.numpy(),
        image=sensor["image"].data.tensor.numpy().astype(np.float16),
        depth=sensor["depth"].data.tensor.numpy(),
        depth_params=np.asarray(sensor["depth"].info[0].parameters, np.float32).reshape(-1),
        features=feats.numpy().astype(np.float16),
        scores=pred.scores.numpy(), pred_classes=pred.pred_classes.numpy(),
        pred_boxes=pred.pred_boxes.numpy(), pred_logits=pred.pred_logits.numpy(),
        boxes3d=pred.pred_boxes_3d.tensor.numpy(), R=pred.pred_boxes_3d.R.numpy(),
        object_desc=pred.object_desc.numpy().astype(np.float16),
        pred_proj_xy=pred.pred_proj_xy.numpy())
    # the full-size depth/image arrays are regenerable from (frame); keep the fixture small
    del out["image"], out["depth"]
    out["depth_sum"] = np.float64(sensor["depth"].data.tensor.double().sum())
    np.savez_compressed(os.path.join(HERE, "cutr_vit_t.npz"), **out)
    print("cutr golden written", {k: getattr(v, "shape", v) for k, v in out.items() if k != "keys"})


if __name__ == "__main__":
    main()
