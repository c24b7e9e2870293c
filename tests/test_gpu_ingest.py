"""GPU frame ingestion and the cv2-exact resize (bf_ingest.hip, bf_cv2.h) against the oracle's
OpenCV restatement (oracle/bf_oracle.c or_cv2_resize_u8; itself pinned by cv2 known answers in
tests/test_oracle_cv2.py): bit-exact u8 for the resize, the ingested RGB frame and every rotation;
the depth map bit-exact f32 (u16 / scale in IEEE f32 division).  The CLIP crop kernel uses the
same resize: its bf16 im2col rows are compared with the oracle-resized crops normalised in f32
(equal up to one bf16 rounding step)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    _lib.lib()
    return _lib


@pytest.mark.parametrize("Hs,Ws,cn,Hd,Wd", [(968, 1296, 3, 480, 640), (130, 90, 3, 224, 224), (5, 300, 3, 224, 224),
                                            (17, 23, 1, 31, 7), (100, 7, 1, 13, 301), (33, 65, 4, 20, 11),
                                            (64, 96, 3, 32, 48), (224, 224, 3, 224, 224), (1, 2, 1, 1, 4)])
def test_cv2_resize_bit_exact(L, Hs, Ws, cn, Hd, Wd):
    rng = np.random.default_rng(Hs + Ws + cn)
    img = rng.integers(0, 256, (2, Hs, Ws, cn), dtype=np.uint8)
    got = L.cv2_resize_u8(torch.from_numpy(img).cuda(), Wd, Hd).cpu().numpy()
    for f in range(2):
        ref = O.cv2_resize_u8(img[f] if cn > 1 else img[f, ..., 0], Wd, Hd)
        assert np.array_equal(got[f].reshape(ref.shape), ref), f


@pytest.mark.parametrize("rot_k", [0, 1, 2, 3])
def test_ingest_rgbd_vs_oracle(L, rot_k):
    rng = np.random.default_rng(rot_k)
    F = 2
    bgr = rng.integers(0, 256, (F, 968, 1296, 3), dtype=np.uint8)
    dep = rng.integers(0, 65535, (F, 480, 640), dtype=np.uint16)
    dep[:, :10] = 0
    rgb, d = L.ingest_rgbd(torch.from_numpy(bgr).cuda(), torch.from_numpy(dep.view(np.int16)).cuda(), 1000.0, rot_k)
    rgb, d = rgb.cpu().numpy(), d.cpu().numpy()
    for f in range(F):
        r_ref, d_ref = O.ingest_rgbd(bgr[f], dep[f], 1000.0, rot_k)
        assert np.array_equal(rgb[f], r_ref)
        assert np.array_equal(d[f], d_ref)
    # RGB order input (PIL decode) gives the same frame as its BGR twin
    rgb2, _ = L.ingest_rgbd(torch.from_numpy(np.ascontiguousarray(bgr[..., ::-1])).cuda(), None, 1.0, rot_k,
                            src_bgr=False)
    assert rgb2.shape[-2:] == (968, 1296) if rot_k % 2 == 0 else (1296, 968)


def test_make_sample_decoded(L):
    from boxfusion_amd.capture_stream import make_sample_decoded
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    rng = np.random.default_rng(9)
    bgr = torch.from_numpy(rng.integers(0, 256, (968, 1296, 3), dtype=np.uint8)).cuda()
    dep = torch.from_numpy(rng.integers(0, 5000, (480, 640), dtype=np.uint16).view(np.int16)).cuda()
    s = make_sample_decoded(bgr, dep, 1000.0, SCANNET_K, Scene().pose(3))
    assert s["wide"]["image"].shape == (1, 3, 480, 640) and s["wide"]["image"].dtype == torch.uint8
    assert s["wide"]["depth"].shape == (1, 480, 640)
    assert s["sensor_info"].wide.image.size == (640, 480)


def test_crop_resize_im2col_cv2(L):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (2, 480, 640, 3), dtype=np.uint8)
    boxes = np.array([[10, 20, 200, 150], [0, 0, 640, 480], [300, 300, 301, 310], [5, 5, 5, 40],
                      [100, 50, 324, 274], [600, 400, 640, 480]], np.int32)
    idx = np.array([0, 1, 1, 0, 1, 0], np.int32)
    mean = np.array([0.48145466, 0.4578275, 0.40821073], np.float32)
    std = np.array([0.26862954, 0.26130258, 0.27577711], np.float32)
    out = L.crop_resize_im2col(torch.from_numpy(img).cuda(), torch.from_numpy(boxes).cuda(),
                               torch.from_numpy(idx).cuda(), 224, 14, mean.tolist(), std.tolist(), 640)
    out = out.float().cpu()
    assert torch.all(out[:, 588:] == 0)
    for n in range(len(boxes)):
        x1, y1, x2, y2 = boxes[n]
        crop = img[idx[n], y1:y2, x1:x2]
        r = O.cv2_resize_u8(crop, 224, 224) if crop.size else np.zeros((224, 224, 3), np.uint8)
        x = (torch.from_numpy(r).float().permute(2, 0, 1) / 255 - torch.from_numpy(mean).view(3, 1, 1)) \
            / torch.from_numpy(std).view(3, 1, 1)
        ref = torch.nn.functional.unfold(x[None], 14, stride=14).transpose(1, 2).reshape(-1, 588)
        got = out[n * 256:(n + 1) * 256, :588]
        refb = ref.bfloat16().float()
        ulp = refb.abs().clamp_min(1e-3) * 2.0 ** -7
        assert ((got - refb).abs() <= ulp + 1e-6).all(), n
        assert (got == refb).float().mean().item() > 0.99, n
