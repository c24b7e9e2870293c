"""The oracle's restatement of cv2.resize (u8 INTER_LINEAR, OpenCV 4.x fixed point) — the checker
for bf_cv2.h (frame ingestion, CLIP crops).  OpenCV is absent here, so it is pinned by known
answers of cv2 itself (the widely reproduced 2x2 -> 4x4 upscale of [[10,20],[30,40]] and the
[0,255] -> 4 row), by the identity / exact-2x-downscale cases (cv2's INTER_AREA equivalence:
(a+b+c+d+2)>>2), and by a float bilinear with half-pixel centres, which it matches within one
level.  Parity with cv2 on arbitrary shapes is otherwise UNPINNED."""
import numpy as np
import pytest

from oracle import oracle as O


def test_known_answers():
    a = np.array([[10, 20], [30, 40]], np.uint8)
    assert O.cv2_resize_u8(a, 4, 4).tolist() == [[10, 13, 18, 20], [15, 18, 23, 25], [25, 28, 33, 35],
                                                 [30, 33, 38, 40]]
    assert O.cv2_resize_u8(np.array([[0, 255]], np.uint8), 4, 1).tolist() == [[0, 64, 191, 255]]


def test_identity_and_exact_half():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    assert np.array_equal(O.cv2_resize_u8(img, 53, 37), img)
    img = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8).astype(np.int32)
    half = O.cv2_resize_u8(img.astype(np.uint8), 48, 32).astype(np.int32)
    area = (img[0::2, 0::2] + img[0::2, 1::2] + img[1::2, 0::2] + img[1::2, 1::2] + 2) >> 2
    assert np.array_equal(half, area)


def _bilinear(img, Wd, Hd):
    Hs, Ws = img.shape[:2]
    x = np.clip((np.arange(Wd) + 0.5) * Ws / Wd - 0.5, 0, None)
    y = np.clip((np.arange(Hd) + 0.5) * Hs / Hd - 0.5, 0, None)
    x0 = np.minimum(np.floor(x).astype(int), Ws - 1)
    y0 = np.minimum(np.floor(y).astype(int), Hs - 1)
    x1, y1 = np.minimum(x0 + 1, Ws - 1), np.minimum(y0 + 1, Hs - 1)
    fx, fy = (x - x0)[None, :, None], (y - y0)[:, None, None]
    f = img.astype(np.float64)
    top = f[y0][:, x0] * (1 - fx) + f[y0][:, x1] * fx
    bot = f[y1][:, x0] * (1 - fx) + f[y1][:, x1] * fx
    return top * (1 - fy) + bot * fy


@pytest.mark.parametrize("Hs,Ws,Hd,Wd", [(968, 1296, 480, 640), (130, 90, 224, 224), (5, 300, 224, 224),
                                         (480, 640, 192, 256), (17, 23, 31, 7)])
def test_vs_float_bilinear(Hs, Ws, Hd, Wd):
    rng = np.random.default_rng(Hs * Ws)
    img = rng.integers(0, 256, (Hs, Ws, 3), dtype=np.uint8)
    out = O.cv2_resize_u8(img, Wd, Hd).astype(np.float64)
    ref = _bilinear(img, Wd, Hd)
    assert np.abs(out - ref).max() <= 1.0 + 1e-9
    assert np.abs(out - ref).mean() < 0.5


def test_ingest_restatement():
    rng = np.random.default_rng(5)
    bgr = rng.integers(0, 256, (96, 128, 3), dtype=np.uint8)
    dep = rng.integers(0, 65535, (48, 64), dtype=np.uint16)
    rgb, d = O.ingest_rgbd(bgr, dep, 1000.0, 1)
    assert rgb.shape == (3, 64, 48) and d.shape == (64, 48) and d.dtype == np.float32
    assert np.array_equal(np.rot90(d, -1), dep.astype(np.float32) / np.float32(1000.0))
    assert np.array_equal(np.rot90(rgb, -1, axes=(-2, -1))[0], O.cv2_resize_u8(bgr[..., 2].copy(), 64, 48))
