"""The CuTR restatement (boxfusion_amd.cubify_transformer / vit / pos) reproduces the REFERENCE
detector on the golden frame: same state-dict keys and shapes, same backbone features and same
top-100 instances (fp32 on CPU; fixture from tests/golden/make_golden_cutr.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import oracle as OR
from tests import trace_util as TU


@pytest.fixture(scope="module")
def golden():
    return TU.load("cutr_vit_t.npz")


def cpu_frame_batch(frame, pad=640):
    from boxfusion_amd.cubify_transformer import FrameBatch
    from boxfusion_amd.sensor import camera_to_gravity
    from boxfusion_amd.synthetic import Scene, frame_rgbd, SCANNET_K
    rgb, depth = frame_rgbd(frame)
    # preprocessor.py:142 casts pixel_mean/std to the uint8 image dtype: (123, 116, 103)/(58, 57, 57)
    from boxfusion_amd.preprocessor import PIXEL_MEAN_U8, PIXEL_STD_U8
    mean = torch.tensor(PIXEL_MEAN_U8).view(3, 1, 1)
    std = torch.tensor(PIXEL_STD_U8).view(3, 1, 1)
    img = (torch.from_numpy(np.moveaxis(rgb, -1, 0)).float() - mean) / std
    img = F.pad(img, (0, pad - img.shape[2], 0, pad - img.shape[1]))[None]
    d, params = OR.depth_standardize(depth)
    d = F.pad(torch.from_numpy(d), (0, pad - d.shape[1], 0, pad - d.shape[0]))[None]
    return FrameBatch(image=img, depth=d, depth_params=torch.from_numpy(params)[None],
                      K=torch.from_numpy(SCANNET_K)[None],
                      T_gravity=torch.from_numpy(camera_to_gravity(Scene().pose(frame)))[None],
                      image_sizes=[(480, 640)]), params


@pytest.fixture(scope="module")
def model(golden):
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.weights import init_seeded
    torch.manual_seed(0)
    m = make_cubify_transformer(int(golden["dim"]), depth_model=True).eval()
    return init_seeded(m, int(golden["seed"]))


def test_state_dict_keys_match_reference(model, golden):
    keys = sorted(f"{k}:{tuple(v.shape)}" for k, v in model.state_dict().items())
    assert keys == sorted(golden["keys"].tolist())


def test_forward_matches_reference(model, golden):
    torch.set_num_threads(8)
    batch, params = cpu_frame_batch(int(golden["frame"]))
    np.testing.assert_allclose(params, golden["depth_params"], rtol=2e-6)
    np.testing.assert_allclose(batch.depth.double().sum().item(), golden["depth_sum"], rtol=1e-6)
    np.testing.assert_allclose(batch.T_gravity[0].numpy(), golden["T_gravity"], atol=1e-6)
    with torch.no_grad():
        feat = model.backbone.backbone.forward_tensors(batch.image, batch.depth)
        ref = torch.from_numpy(golden["features"].astype(np.float32))
        assert ((feat - ref).norm() / ref.norm()).item() < 2e-3
        r = model(batch)[0]
    np.testing.assert_allclose(r.scores.numpy(), golden["scores"], rtol=1e-4, atol=1e-6)
    # compare instances whose score is separated from its neighbours (stable top-k order)
    s = golden["scores"]
    gap = np.minimum(np.abs(np.diff(s, prepend=np.inf)), np.abs(np.diff(s, append=-np.inf)))
    ok = gap > 1e-5
    assert ok.sum() > 50
    np.testing.assert_array_equal(r.pred_classes.numpy()[ok], golden["pred_classes"][ok])
    np.testing.assert_allclose(r.pred_boxes.numpy()[ok], golden["pred_boxes"][ok], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(r.pred_boxes_3d.tensor.numpy()[ok], golden["boxes3d"][ok], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(r.pred_boxes_3d.R.numpy()[ok], golden["R"][ok], atol=1e-5)
    np.testing.assert_allclose(r.pred_proj_xy.numpy()[ok], golden["pred_proj_xy"][ok], rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(r.object_desc.numpy()[ok], golden["object_desc"][ok].astype(np.float32),
                               rtol=2e-3, atol=2e-3)
