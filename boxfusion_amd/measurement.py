"""Per-measurement camera info (reference: boxfusion/measurement.py:10-151).

`ImageMeasurementInfo(size=(w, h), K=[N,3,3])`, `DepthMeasurementInfo` and the whitened depth info
that `Preprocessor.normalize` produces (depth standardisation parameters [N, 2] = (trunc_mean,
trunc_std), read by the CuTR decoder as its metric z / dims scale, cubify_transformer.py:568-586).
Host-side containers only: a few 3x3 matrices per frame.
"""
from __future__ import annotations

from typing import Any

import numpy as np
import torch

from boxfusion_amd.sensor import ImageOrientation, rotate_K


class BaseMeasurementInfo:
    def __init__(self, meta=None, **kwargs):
        self.meta = meta

    @property
    def ts(self):
        return getattr(self.meta, "ts", None) if self.meta is not None else None


class MeasurementInfo(BaseMeasurementInfo):
    pass


class ImageMeasurementInfo(MeasurementInfo):
    """size = (width, height); K = [N, 3, 3] pixel intrinsics (normalised intrinsics rejected,
    measurement.py:37-39)"""

    def __init__(self, size, K, meta=None, original_size=None):
        super().__init__(meta=meta)
        if isinstance(size, torch.Tensor):
            size = (int(size[0].item()), int(size[1].item()))
        self.size = tuple(size)
        self.original_size = original_size or self.size
        K = torch.as_tensor(K)
        if ((K[..., 2] >= 0) & (K[..., 2] < 1)).all():
            raise ValueError("Normalized intrinsics are not supported")
        self.K = K.float()

    @property
    def device(self):
        return self.K.device

    def _get_fields(self):
        return dict(size=torch.tensor(self.size), K=self.K)

    def __len__(self):
        return len(self.K)

    def _like(self, size, K, **kw):
        return type(self)(size, K, meta=self.meta, original_size=kw.pop("original_size", self.original_size), **kw)

    def __getitem__(self, item):
        return self._like(self.size, self.K[item])

    def to(self, *args: Any, **kwargs: Any):
        return self._like(self.size, self.K.to(*args, **kwargs))

    @classmethod
    def cat(cls, info_list):
        return type(info_list[0])(size=info_list[0].size, K=torch.cat([i.K for i in info_list]))

    @staticmethod
    def _oriented_size(current, target, size):
        if target != ImageOrientation.UPRIGHT and current != ImageOrientation.UPRIGHT:
            raise NotImplementedError
        same = {(ImageOrientation.UPRIGHT, ImageOrientation.UPRIGHT),
                (ImageOrientation.UPSIDE_DOWN, ImageOrientation.UPRIGHT),
                (ImageOrientation.UPRIGHT, ImageOrientation.UPSIDE_DOWN),
                (ImageOrientation.LEFT, ImageOrientation.RIGHT),
                (ImageOrientation.RIGHT, ImageOrientation.LEFT)}
        return tuple(size) if (current, target) in same else (size[1], size[0])

    def orient(self, current, target):
        return self._like(self._oriented_size(current, target, self.size),
                          rotate_K(self.K, current, self.size, target),
                          original_size=self._oriented_size(current, target, self.original_size))

    def rescale(self, factor):
        K = self.K.clone()
        K[..., :2, :] = K[..., :2, :] * factor
        return self._like((int(self.size[0] * factor), int(self.size[1] * factor)), K)

    def resize(self, new_size):
        if isinstance(new_size, float):
            return self.rescale(new_size)
        ws, hs = new_size[0] / self.size[0], new_size[1] / self.size[1]
        if not np.isclose(hs, ws, atol=0.025):
            print(f"Rescaling from {self.size} to {new_size}. This does not seem uniform but may be "
                  "due to discretization error.")
        out = self.rescale(hs)
        out.size = tuple(new_size)
        return out


class DepthMeasurementInfo(ImageMeasurementInfo):
    def normalize(self, parameters):
        return WhitenedDepthMeasurementInfo(size=self.size, K=self.K, meta=self.meta,
                                            parameters=parameters, original_size=self.original_size)


class WhitenedDepthMeasurementInfo(DepthMeasurementInfo):
    def __init__(self, size, K, meta=None, parameters=None, original_size=None):
        super().__init__(size, K, meta=meta, original_size=original_size)
        self.parameters = parameters          # [N, 2] (trunc_mean, trunc_std)

    def _like(self, size, K, **kw):
        return WhitenedDepthMeasurementInfo(size, K, meta=self.meta, parameters=self.parameters,
                                            original_size=kw.pop("original_size", self.original_size))

    def _get_fields(self):
        return dict(size=torch.tensor(self.size), K=self.K, parameters=self.parameters)

    def to(self, *args: Any, **kwargs: Any):
        p = self.parameters.to(*args, **kwargs) if isinstance(self.parameters, torch.Tensor) else self.parameters
        return WhitenedDepthMeasurementInfo(self.size, self.K.to(*args, **kwargs), meta=self.meta,
                                            parameters=p, original_size=self.original_size)
