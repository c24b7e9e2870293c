"""GPU colour-JPEG decode (bf_jpeg.hip) bit-exact against PIL (libjpeg-turbo's default decompression,
the library behind the reference's cv2.imread(color_path), capture_stream.py:194/:402) and the
oracle restatement (oracle/jpeg.py): the committed fixtures (4:2:0 / 4:2:2 / 4:4:4, qualities 5-100,
optimised tables, restart markers, greyscale, sizes off the MCU grid), ScanNet-size 1296 x 968
frames in one batch, mixed kinds in one launch, and corrupt / unsupported files each flagged with
its own status bit while the good files of the batch stay exact."""
import io
import os

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import jpeg as J

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(__file__), "golden", "jpeg_fixtures.npz")


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    _lib.lib()
    return _lib


def fixtures():
    z = np.load(FIX)
    n = sum(1 for k in z.files if k.startswith("jpg_"))
    return [(str(z[f"name_{i}"]), z[f"jpg_{i}"].tobytes(), z[f"img_{i}"]) for i in range(n)]


def decode(L, blobs, H, W, check=True):
    from boxfusion_amd.capture_stream import upload_files
    files, offs, _ = upload_files(blobs, "cuda")
    out, st = L.jpeg_decode_rgb(files, offs, H, W, check=check)
    torch.cuda.synchronize()
    return out.cpu().numpy(), st.cpu().numpy()


def pil(jpg):
    return np.asarray(Image.open(io.BytesIO(jpg)).convert("RGB"))


def scene(H, W, seed):
    from tests.golden.make_jpeg_fixtures import scene as sc
    return sc(H, W, seed)


def jpeg(img, **kw):
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("name,jpg,img", fixtures(), ids=lambda v: v if isinstance(v, str) else "")
def test_fixture_bit_exact(L, name, jpg, img):
    H, W = img.shape[:2]
    got, st = decode(L, [jpg], H, W)
    assert st.tolist() == [0]
    np.testing.assert_array_equal(got[0], img, err_msg=name)


def test_fixture_batch_mixed_kinds(L):
    """every 48 x 64 fixture (sampling, quality, restart, greyscale mixed) in one launch"""
    fx = [(n, p, i) for n, p, i in fixtures() if i.shape[:2] == (48, 64)]
    assert len(fx) >= 12
    got, st = decode(L, [p for _, p, _ in fx], 48, 64)
    assert not st.any()
    for k, (n, _, img) in enumerate(fx):
        np.testing.assert_array_equal(got[k], img, err_msg=n)


def test_scannet_size_frames(L):
    """1296 x 968 colour frames (ScanNet's colour resolution) at the qualities / sampling a capture
    writer uses, one launch; PIL equality on every pixel"""
    from boxfusion_amd.synthetic import frame_rgbd
    specs = [dict(quality=90), dict(quality=75), dict(quality=95, subsampling=0), dict(quality=85, subsampling=1),
             dict(quality=90, restart_marker_rows=2), dict(quality=60, optimize=True)]
    blobs = []
    for k, sp in enumerate(specs):
        rgb = frame_rgbd(k * 9, 484, 648)[0]
        img = np.asarray(Image.fromarray(rgb).resize((1296, 968), Image.BILINEAR))
        blobs.append(jpeg(img, **sp))
    got, st = decode(L, blobs, 968, 1296)
    assert not st.any()
    for k, b in enumerate(blobs):
        np.testing.assert_array_equal(got[k], pil(b), err_msg=str(specs[k]))


def test_oracle_agrees(L):
    img = scene(40, 72, 11)
    for sp in (dict(quality=70), dict(quality=70, subsampling=1, restart_marker_blocks=5)):
        b = jpeg(img, **sp)
        got, _ = decode(L, [b], 40, 72)
        np.testing.assert_array_equal(got[0], J.decode_rgb(b))


def _entropy_start(jpg):
    i = 2
    while True:
        m, ln = jpg[i + 1], int.from_bytes(jpg[i + 2:i + 4], "big")
        if m == 0xDA:
            return i + 2 + ln
        i += 2 + ln


def test_corrupt_and_unsupported_flagged_good_exact(L):
    img = scene(48, 64, 3)
    good = jpeg(img, quality=80)
    s = _entropy_start(good)
    garbage = bytearray(good)
    garbage[s:s + 40] = b"\xff\x00" * 20                  # all-ones bits: no valid Huffman code
    prog = jpeg(img, quality=80, progressive=True)
    cases = [("good", good, 0),
             ("no_soi", b"\x00" + good[1:], 1),
             ("truncated_header", good[:s - 20], 1),
             ("progressive", prog, 2),
             ("size", jpeg(scene(40, 64, 3), quality=80), 4),
             ("bad_huffman", bytes(garbage), 8),
             ("good_rst", jpeg(img, quality=80, restart_marker_blocks=2), 0)]
    got, st = decode(L, [c[1] for c in cases], 48, 64, check=False)
    for k, (name, b, bit) in enumerate(cases):
        if bit == 0:
            assert st[k] == 0, name
            np.testing.assert_array_equal(got[k], pil(b), err_msg=name)
        else:
            assert st[k] & bit, (name, st[k])
    with pytest.raises(L.HipError, match="did not decode"):
        decode(L, [good, cases[1][1]], 48, 64, check=True)


def test_truncated_scan_grey_tail(L):
    """a file cut inside its scan (no EOI): libjpeg's stdio source (cv2.imread) feeds zero bits
    past the end and leaves every MCU after the first one that needed them zero, i.e. grey 128.
    PIL's suspending source stops instead, so the tail is pinned to jdhuff.c's rule, the head to
    the full file's PIL decode"""
    img = scene(96, 64, 5)
    good = jpeg(img, quality=80)
    cut = good[:_entropy_start(good) + 700]
    got, st = decode(L, [cut], 96, 64, check=False)
    assert st[0] == 0
    full = pil(good)
    r0 = next(r for r in range(96) if not np.array_equal(got[0, r], full[r]))    # first row off
    assert r0 >= 15, "the MCU rows before the cut decode as in the full file"
    band = (r0 + 1) // 16                       # the MCU row holding the cut (r0 may be its context row)
    grey = (band + 1) * 16 + 1                  # below it: zero blocks, and chroma context from them
    assert grey < 96
    np.testing.assert_array_equal(got[0, grey:], 128)


def test_decoded_frame_stream_gpu_colour_equals_host(L, tmp_path):
    """DecodedFrameStream with color_decode="gpu" (bf_jpeg_decode_rgb, batches of 3) gives the same
    samples as the host PIL decode: the image after bf_ingest_rgbd's resize / rotation, bit for bit"""
    from boxfusion_amd.capture_stream import DecodedFrameStream
    from boxfusion_amd.synthetic import SCANNET_K, frame_rgbd
    cps, dps = [], []
    for f in range(5):
        rgb, d = frame_rgbd(f, 480, 640)
        big = np.asarray(Image.fromarray(rgb).resize((1296, 968), Image.BILINEAR))
        cp, dp = tmp_path / f"{f}.jpg", tmp_path / f"{f}.png"
        Image.fromarray(big).save(cp, quality=90)
        Image.fromarray(np.clip(d * 1000.0, 0, 65535).astype(np.uint16)).save(dp)
        cps.append(str(cp))
        dps.append(str(dp))
    up = np.eye(4, dtype=np.float32)
    up[1:3, :3] = [[0, 0, 1], [0, -1, 0]]
    poses = [up] * 5
    host = list(DecodedFrameStream(cps, dps, poses, SCANNET_K, 1000.0, device="cuda", batch=3))
    gpu = list(DecodedFrameStream(cps, dps, poses, SCANNET_K, 1000.0, device="cuda", batch=3, color_decode="gpu"))
    assert len(host) == len(gpu) == 5
    for a, b in zip(host, gpu):
        torch.testing.assert_close(a["wide"]["image"].cpu(), b["wide"]["image"].cpu(), rtol=0, atol=0)
        torch.testing.assert_close(a["wide"]["depth"].cpu(), b["wide"]["depth"].cpu(), rtol=0, atol=0)
