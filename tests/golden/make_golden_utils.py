"""Golden fixture for the per-frame helpers of tools/utils.py, run on the REFERENCE module:
  * unproject (tools/utils.py:232-287) on a seeded 120x160 depth map, K and pose;
  * scale_boxes (:355-381) + text_prompt (:478-495) with the reference's crop_image / retriev,
    a stand-in CLIP model returning fixed seeded features (SAMCLIP is absent from the reference),
    the real 473-class text features and class list.  crop_image is wrapped to record the size of
    every crop it returns (which pins the integer crop boxes); the cv2.resize stand-in returns a
    224x224 zero image (the stand-in model ignores pixels).
Only absent third-party modules are replaced (rerun, open3d, cv2, torchvision).
Run:  python tests/golden/make_golden_utils.py  ->  tests/golden/utils.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden_results  # noqa: E402,F401  (installs the stand-ins, imports tools.utils)
from tools import utils as U  # noqa: E402

REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from boxfusion_amd.synthetic import SCANNET_K, Scene, frame_rgbd  # noqa: E402

CROP_SHAPES = []
_crop_image = U.crop_image


def crop_image(boxes, rgb):
    """the reference's crop_image, recording (height, width) of every crop it returns"""
    b, crops = _crop_image(boxes, rgb)
    CROP_SHAPES.extend((c.height, c.width) for c in crops)
    return b, crops


def resize(img, size, *a, **k):
    return np.zeros((size[1], size[0], 3), np.uint8)


U.crop_image = crop_image
U.cv2.resize = resize


class StubCLIP:
    """get_batch_images_clip_features(images) -> (features [N,1024] f32, outliers): fixed seeded
    features, scaled so some crops clear the similarity threshold"""

    def __init__(self, feats):
        self.feats = feats

    def get_batch_images_clip_features(self, images):
        assert len(images) == len(self.feats)
        return torch.from_numpy(self.feats.copy()), None


def main():
    rng = np.random.default_rng(5)
    # ---- unproject ----------------------------------------------------------------------------
    _, depth = frame_rgbd(4, 120, 160)
    depth[rng.uniform(0, 1, depth.shape) < 0.03] = 12.0          # beyond max_depth
    K = SCANNET_K.copy() / 4.0
    K[2, 2] = 1.0
    RT = Scene().pose(4)
    xyz, valid = U.unproject(torch.from_numpy(depth), torch.from_numpy(K), torch.from_numpy(RT), max_depth=10.0)
    # ---- scale_boxes + text_prompt ------------------------------------------------------------
    rgb, _ = frame_rgbd(9)
    n = 24
    x1 = rng.uniform(-20, 600, n)
    y1 = rng.uniform(-20, 440, n)
    boxes = np.stack([x1, y1, x1 + rng.uniform(0, 160, n), y1 + rng.uniform(0, 120, n)], 1).astype(np.float32)
    boxes[3] = [100.0, 100.0, 100.0, 150.0]                      # zero width: an empty crop
    boxes[5] = [630.0, 470.0, 700.0, 520.0]                      # clipped at the image corner
    scaled = U.scale_boxes(boxes, 480, 640, scale=1.5)
    text = torch.from_numpy(np.load(os.path.join(REPO, "boxfusion_amd", "data", "class_features.npy")).astype(np.float32))
    names = np.genfromtxt(os.path.join(REPO, "boxfusion_amd", "data", "panoptic_categories_nomerge.txt"),
                          delimiter="\n", dtype=str)
    # features near random text rows for half the crops (similarity above the threshold), noise for the rest
    pick = rng.integers(0, len(text), n)
    feats = rng.normal(0, 1, (n, 1024)).astype(np.float32)
    feats[::2] = text.numpy()[pick[::2]] * 30.0 + feats[::2] * 0.4
    text_in = text.clone() * 1.7                                   # not unit-norm: the in-place renorm matters
    cats, img_f, maxv = U.text_prompt(scaled, names, text_in, rgb, StubCLIP(feats), None, 25.0)
    cat_idx = np.array([np.where(np.append(names, "") == c)[0][0] for c in cats])
    out = dict(depth=depth, K=K, RT=RT, xyz=xyz.numpy(), valid=valid.numpy(),
               rgb_frame=np.int32(9), boxes=boxes, scaled=scaled, crop_hw=np.array(CROP_SHAPES),
               feats=feats, text_scale=np.float32(1.7), sim_thres=np.float32(25.0),
               cat_idx=cat_idx, img_features=img_f.numpy(), max_values=maxv.numpy(),
               text_after=text_in.numpy()[:4])
    np.savez_compressed(os.path.join(HERE, "utils.npz"), **out)
    print("utils golden:", {k: getattr(v, "shape", v) for k, v in out.items()}, "matched",
          int((cat_idx < len(names)).sum()))


if __name__ == "__main__":
    main()
