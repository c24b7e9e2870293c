"""Frame preprocessing (reference: boxfusion/preprocessor.py) on the GPU.

Reference semantics reproduced:
  * RGB: (x - pixel_mean) / pixel_std where `pixel_mean.to(measurement.data)` casts the constants
    to the image's uint8 dtype first (preprocessor.py:142), i.e. (123, 116, 103) / (58, 57, 57);
  * depth: trimmed standardisation (preprocessor.py:97-129) -> bf_depth_standardize;
  * zero padding to the smallest square in [256..1024] >= the longest edge, /32 (:146-200,
    imagelist.py:55-115); both fused into the patch-embedding im2col of the engine.
"""
from __future__ import annotations

PIXEL_MEAN = (123.675, 116.28, 103.53)
PIXEL_STD = (58.395, 57.12, 57.375)
PIXEL_MEAN_U8 = tuple(float(int(v)) for v in PIXEL_MEAN)   # uint8 cast of the constants
PIXEL_STD_U8 = tuple(float(int(v)) for v in PIXEL_STD)
SQUARE_PAD = (256, 384, 512, 640, 768, 896, 1024)
SIZE_DIVISIBILITY = 32


def square_pad_size(h, w, square_pad=SQUARE_PAD, div=SIZE_DIVISIBILITY):
    longest = max(h, w)
    s = int(min(s for s in square_pad if s >= longest))
    return (s + div - 1) // div * div
