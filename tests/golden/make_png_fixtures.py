"""Generate tests/golden/png_fixtures.npz: small 16-bit greyscale PNG files and their decoded
samples as PIL (libpng-equivalent, the library stand-in for the reference's cv2.imread(...,
IMREAD_UNCHANGED), capture_stream.py:197/:405) returns them.  Run: python tests/golden/make_png_fixtures.py

The files cover what a depth PNG writer can emit: PIL's own encoder (adaptive row filters) at
compress levels 0 / 1 / 6 / 9, and oracle/png.py's encoder with every row filter forced (None,
Sub, Up, Average, Paeth, a per-row mix), stored / fixed-Huffman / Huffman-only / RLE / default
deflate blocks, IDAT split into 1-byte, 7-byte and single chunks, ancillary chunks before the
data, and odd sizes (1 x 1, 1 x 37, 29 x 3).  Data only: key png_<i> (u8 file bytes), img_<i> (u16
[H, W] expected), name_<i>.
"""
from __future__ import annotations

import io
import os
import sys
import zlib

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.png import encode_u16  # noqa: E402


def depth_like(H, W, seed):
    """a depth map in mm: planes and a box, zero holes, sensor noise"""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W]
    d = 1500 + 3.0 * y + 1.5 * x
    d[H // 4:H // 2, W // 3:2 * W // 3] = 900 + 0.5 * x[H // 4:H // 2, W // 3:2 * W // 3]
    d += rng.normal(0, 4, (H, W))
    d[rng.random((H, W)) < 0.05] = 0
    d[:max(1, H // 8), :max(1, W // 6)] = 0
    return np.clip(d, 0, 65535).astype(np.uint16)


def pil_png(img, **kw):
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="PNG", **kw)
    return b.getvalue()


def cases():
    out = []
    base = depth_like(48, 64, 0)
    for lvl in (0, 1, 6, 9):
        out.append((f"pil_level{lvl}", pil_png(base, compress_level=lvl)))
    rng = np.random.default_rng(1)
    for ft in range(5):
        out.append((f"filter{ft}", encode_u16(base, filters=ft)))
    mix = list(rng.integers(0, 5, 48))
    out.append(("filter_mix", encode_u16(base, filters=mix)))
    out.append(("stored", encode_u16(base, filters=mix, level=0)))
    out.append(("fixed", encode_u16(base, filters=mix, strategy=zlib.Z_FIXED)))
    out.append(("huffman_only", encode_u16(base, filters=mix, strategy=zlib.Z_HUFFMAN_ONLY)))
    out.append(("rle", encode_u16(base, filters=mix, strategy=zlib.Z_RLE)))
    out.append(("idat1", encode_u16(base, filters=mix, idat_size=1)))
    out.append(("idat7_level9", encode_u16(base, filters=mix, level=9, idat_size=7)))
    out.append(("ancillary", encode_u16(base, filters=mix, extra_chunks=[(b"tEXt", b"Software\x00test"),
                                                                          (b"gAMA", b"\x00\x00\xb1\x8f")])))
    full = rng.integers(0, 65536, (40, 33)).astype(np.uint16)       # incompressible: long codes, stored
    out.append(("noise_mix", encode_u16(full, filters=list(rng.integers(0, 5, 40)))))
    out.append(("noise_pil", pil_png(full)))
    out.append(("zeros", encode_u16(np.zeros((30, 50), np.uint16), filters=2)))
    out.append(("one_pixel", encode_u16(np.array([[513]], np.uint16), filters=4)))
    out.append(("row37", encode_u16(depth_like(1, 37, 2), filters=1)))
    out.append(("col3", encode_u16(depth_like(29, 3, 3), filters=list(rng.integers(0, 5, 29)))))
    return out


def main():
    arrs = {}
    for i, (name, png) in enumerate(cases()):
        img = np.asarray(Image.open(io.BytesIO(png)))
        assert img.dtype == np.uint16, (name, img.dtype)
        arrs[f"png_{i}"] = np.frombuffer(png, np.uint8)
        arrs[f"img_{i}"] = img
        arrs[f"name_{i}"] = np.array(name)
    path = os.path.join(HERE, "png_fixtures.npz")
    np.savez_compressed(path, **arrs)
    print(path, len(arrs) // 3, "files")


if __name__ == "__main__":
    main()
