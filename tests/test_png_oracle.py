"""The depth-PNG oracle (oracle/png.py) against PIL's decoder on the committed fixtures
(tests/golden/png_fixtures.npz, made by tests/golden/make_png_fixtures.py), and the encoder that
the GPU tests use to force every filter / block kind round-trips through PIL."""
import io
import os
import zlib

import numpy as np
import pytest
from PIL import Image

from oracle import png as P

FIX = os.path.join(os.path.dirname(__file__), "golden", "png_fixtures.npz")


def fixtures():
    z = np.load(FIX)
    n = sum(1 for k in z.files if k.startswith("png_"))
    return [(str(z[f"name_{i}"]), z[f"png_{i}"].tobytes(), z[f"img_{i}"]) for i in range(n)]


@pytest.mark.parametrize("name,png,img", fixtures(), ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_matches_pil_fixture(name, png, img):
    got = P.decode_u16(png)
    assert got.dtype == np.uint16 and got.shape == img.shape
    np.testing.assert_array_equal(got, img, err_msg=name)
    # the fixture is still what PIL decodes here
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(png))), img, err_msg=name)


def test_fixtures_cover_every_filter_and_block_kind():
    seen_f, seen_b = set(), set()
    for _, png, img in fixtures():
        raw = zlib.decompress(b"".join(d for t, d in P.chunks(png) if t == b"IDAT"))
        H, W = img.shape
        seen_f |= {raw[r * (2 * W + 1)] for r in range(H)}
        z = b"".join(d for t, d in P.chunks(png) if t == b"IDAT")
        seen_b.add((z[2] >> 1) & 3)          # the first block's BTYPE
    assert seen_f == {0, 1, 2, 3, 4}
    assert {0, 1, 2} <= seen_b


@pytest.mark.parametrize("ft", [0, 1, 2, 3, 4, None])
def test_encoder_round_trip_through_pil(ft):
    rng = np.random.default_rng(7)
    img = rng.integers(0, 65536, (9, 13)).astype(np.uint16)
    flt = list(rng.integers(0, 5, 9)) if ft is None else ft
    png = P.encode_u16(img, filters=flt, idat_size=5)
    np.testing.assert_array_equal(np.asarray(Image.open(io.BytesIO(png))), img)
    np.testing.assert_array_equal(P.decode_u16(png), img)
