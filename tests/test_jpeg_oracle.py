"""The colour-JPEG oracle (oracle/jpeg.py) against PIL's decoder (libjpeg-turbo, the library behind
the reference's cv2.imread(color_path), capture_stream.py:194/:402) on the committed fixtures
(tests/golden/jpeg_fixtures.npz, made by tests/golden/make_jpeg_fixtures.py), and the kinds the
GPU decode refuses."""
import io
import os

import numpy as np
import pytest
from PIL import Image

from oracle import jpeg as J

FIX = os.path.join(os.path.dirname(__file__), "golden", "jpeg_fixtures.npz")


def fixtures():
    z = np.load(FIX)
    n = sum(1 for k in z.files if k.startswith("jpg_"))
    return [(str(z[f"name_{i}"]), z[f"jpg_{i}"].tobytes(), z[f"img_{i}"]) for i in range(n)]


@pytest.mark.parametrize("name,jpg,img", fixtures(), ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_matches_pil_fixture(name, jpg, img):
    got = J.decode_rgb(jpg)
    assert got.dtype == np.uint8 and got.shape == img.shape
    np.testing.assert_array_equal(got, img, err_msg=name)
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(jpg)).convert("RGB")), img, err_msg=name)


def test_fixtures_cover_sampling_restarts_and_grey():
    kinds, dri, ncomp = set(), set(), set()
    for _, jpg, _ in fixtures():
        j = J.parse(jpg)
        comps = j["frame"][2]
        ncomp.add(len(comps))
        if len(comps) == 3:
            kinds.add((comps[0][1], comps[0][2]))
        dri.add(bool(j["dri"]))
    assert kinds == {(1, 1), (2, 1), (2, 2)}
    assert dri == {False, True} and ncomp == {1, 3}


def test_progressive_is_refused():
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, format="JPEG", progressive=True)
    with pytest.raises(J.JpegError):
        J.decode_rgb(b.getvalue())


def test_jpeg_size_reads_the_frame_header():
    from boxfusion_amd.capture_stream import jpeg_size
    for _, jpg, img in fixtures():
        assert jpeg_size(jpg) == (img.shape[1], img.shape[0])
    with pytest.raises(ValueError):
        jpeg_size(b"\x89PNG\r\n\x1a\n")
