"""Generate tests/golden/jpeg_fixtures.npz: small baseline JPEG files and the RGB samples PIL's
decoder (libjpeg-turbo with its default islow IDCT and fancy upsampling -- the library the
reference's cv2.imread(color_path), capture_stream.py:194/:402, runs) returns for them.
Run: python tests/golden/make_jpeg_fixtures.py

The files cover what a colour-frame writer can emit: 4:2:0 / 4:2:2 / 4:4:4 chroma, qualities 5 /
50 / 75 / 95 / 100, optimised Huffman tables, restart markers (every block, every 3 MCUs, every MCU
row; fill bytes before them and before a stuffed FF), greyscale, and sizes that are not multiples of the MCU (1 x 1, 17 x 9, 37 x 53, 8 x 23,
33 x 71).  Data only: key jpg_<i> (u8 file bytes), img_<i> (u8 [H, W, 3] RGB expected), name_<i>.
"""
from __future__ import annotations

import io
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))


def scene(H, W, seed):
    """a colour frame: gradients, a saturated box, texture and noise"""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    r = 40 + 180 * x / max(W - 1, 1)
    g = 60 + 150 * y / max(H - 1, 1)
    b = 128 + 100 * np.sin(x / 3.0) * np.cos(y / 5.0)
    img = np.stack([r, g, b], -1)
    img[H // 4:H // 2 + 1, W // 3:2 * W // 3 + 1] = (250, 20, 30)
    img += rng.normal(0, 12, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def pil_jpeg(img, **kw):
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", **kw)
    return b.getvalue()


def with_fill_bytes(jpg):
    """the same file with fill bytes (FF FF) before each RSTn marker and before one stuffed FF 00"""
    i = 2
    while True:
        m, ln = jpg[i + 1], int.from_bytes(jpg[i + 2:i + 4], "big")
        if m == 0xDA:
            e = i + 2 + ln
            break
        i += 2 + ln
    out, k, stuffed = bytearray(jpg[:e]), e, False
    while k < len(jpg):
        if jpg[k] == 0xFF and k + 1 < len(jpg) and (0xD0 <= jpg[k + 1] <= 0xD7 or (jpg[k + 1] == 0 and not stuffed)):
            stuffed |= jpg[k + 1] == 0
            out += b"\xff\xff\xff" + bytes([jpg[k + 1]])
            k += 2
            continue
        out.append(jpg[k])
        k += 1
    return bytes(out)


def cases():
    base = scene(48, 64, 0)
    out = []
    for ss, tag in ((2, "420"), (1, "422"), (0, "444")):
        for q in (50, 95):
            out.append((f"s{tag}_q{q}", pil_jpeg(base, quality=q, subsampling=ss)))
    out.append(("s420_q5", pil_jpeg(base, quality=5)))
    out.append(("s420_q100", pil_jpeg(base, quality=100)))
    out.append(("s444_q100", pil_jpeg(base, quality=100, subsampling=0)))
    out.append(("s420_optimize", pil_jpeg(base, quality=75, optimize=True)))
    out.append(("s420_rst_block1", pil_jpeg(base, quality=75, restart_marker_blocks=1)))
    out.append(("s422_rst_block3", pil_jpeg(base, quality=75, subsampling=1, restart_marker_blocks=3)))
    out.append(("s444_rst_row", pil_jpeg(base, quality=75, subsampling=0, restart_marker_rows=1)))
    out.append(("grey_q75", pil_jpeg(np.asarray(Image.fromarray(base).convert("L")), quality=75)))
    out.append(("grey_rst", pil_jpeg(np.asarray(Image.fromarray(scene(37, 53, 4)).convert("L")), quality=60,
                                      restart_marker_blocks=2)))
    for (H, W), ss in (((1, 1), 2), ((17, 9), 2), ((37, 53), 2), ((8, 23), 1), ((33, 71), 0), ((24, 40), 2)):
        out.append((f"odd{H}x{W}_s{ss}", pil_jpeg(scene(H, W, H * W), quality=85, subsampling=ss)))
    out.append(("s420_rst_fill", with_fill_bytes(pil_jpeg(base, quality=75, restart_marker_blocks=2))))
    flat = np.full((16, 24, 3), (12, 200, 99), np.uint8)          # DC-only blocks, long EOB runs
    out.append(("flat", pil_jpeg(flat, quality=90)))
    sat = np.zeros((16, 16, 3), np.uint8)
    sat[::2, ::2] = 255                                           # high-frequency, range-limit clamps
    out.append(("checker_q100", pil_jpeg(sat, quality=100, subsampling=0)))
    return out


def main():
    arrs = {}
    for i, (name, jpg) in enumerate(cases()):
        img = np.asarray(Image.open(io.BytesIO(jpg)).convert("RGB"))
        arrs[f"jpg_{i}"] = np.frombuffer(jpg, np.uint8)
        arrs[f"img_{i}"] = img
        arrs[f"name_{i}"] = np.array(name)
    path = os.path.join(HERE, "jpeg_fixtures.npz")
    np.savez_compressed(path, **arrs)
    print(path, len(arrs) // 3, "files", sum(a.nbytes for k, a in arrs.items() if k.startswith("jpg_")), "bytes")


if __name__ == "__main__":
    main()
