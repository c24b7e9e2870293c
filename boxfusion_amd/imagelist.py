"""Padded image batch (reference: boxfusion/imagelist.py, Detectron2's ImageList).

`ImageList.from_tensors` pads to the square size the preprocessor picks (imagelist.py:55-115) —
but lazily: the MI355X engine never needs the padded tensor (its im2col kernels read the square
virtually, zero rows / columns past the frame), so the padded copy is only built when someone
reads `.tensor`.  `.raw` is the unpadded batch [N, ..., h, w] and `.padded_hw` the padded size.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F


class ImageList:
    def __init__(self, tensor: Optional[torch.Tensor], image_sizes: List[Tuple[int, int]],
                 raw: Optional[torch.Tensor] = None, padded_hw: Optional[Tuple[int, int]] = None,
                 materialize: Optional[Callable[[], torch.Tensor]] = None):
        self._tensor = tensor
        self.image_sizes = image_sizes
        self.raw = raw
        self.padded_hw = padded_hw if padded_hw is not None else (
            tuple(tensor.shape[-2:]) if tensor is not None else None)
        self._materialize = materialize
        self._transform = None

    @property
    def tensor(self) -> torch.Tensor:
        if self._tensor is None:
            self._tensor = self._materialize()
        return self._tensor

    @tensor.setter
    def tensor(self, t):
        self._tensor = t

    def __len__(self) -> int:
        return len(self.image_sizes)

    def __getitem__(self, idx) -> torch.Tensor:
        h, w = self.image_sizes[idx]
        return self.tensor[idx, ..., :h, :w]

    def to(self, *args: Any, **kwargs: Any) -> "ImageList":
        raw = self.raw.to(*args, **kwargs) if self.raw is not None else None
        if self._tensor is not None:
            return ImageList(self._tensor.to(*args, **kwargs), self.image_sizes, raw, self.padded_hw)
        return ImageList.lazy(raw, self.image_sizes, self.padded_hw, self._transform)

    @property
    def device(self):
        return (self._tensor if self._tensor is not None else self.raw).device

    @staticmethod
    def padded_size(image_sizes, size_divisibility=0, padding_constraints: Optional[Dict[str, int]] = None):
        H = max(h for h, _ in image_sizes)
        W = max(w for _, w in image_sizes)
        if padding_constraints is not None:
            sq = padding_constraints.get("square_size", 0)
            if sq > 0:
                H = W = sq
            size_divisibility = padding_constraints.get("size_divisibility", size_divisibility)
        if size_divisibility > 1:
            s = size_divisibility
            H, W = (H + s - 1) // s * s, (W + s - 1) // s * s
        return H, W

    @staticmethod
    def lazy(raw, image_sizes, padded_hw, transform=None, pad_value=0.0):
        """raw [N, ..., h, w] (one size for the batch) + an optional elementwise transform applied
        before padding (the preprocessor's pending RGB normalisation)"""
        def build():
            x = transform(raw) if transform is not None else raw
            h, w = x.shape[-2:]
            return F.pad(x, [0, padded_hw[1] - w, 0, padded_hw[0] - h], value=pad_value).contiguous()
        il = ImageList(None, image_sizes, raw=raw, padded_hw=padded_hw, materialize=build)
        il._transform = transform
        return il

    @staticmethod
    def from_tensors(tensors: List[torch.Tensor], size_divisibility: int = 0, pad_value: float = 0.0,
                     padding_constraints: Optional[Dict[str, int]] = None,
                     transform=None) -> "ImageList":
        assert len(tensors) > 0 and isinstance(tensors, (tuple, list))
        for t in tensors:
            assert isinstance(t, torch.Tensor), type(t)
            assert t.shape[:-2] == tensors[0].shape[:-2], t.shape
        sizes = [(int(t.shape[-2]), int(t.shape[-1])) for t in tensors]
        if len(set(sizes)) != 1:
            raise NotImplementedError("frames of one batch must share their size")
        hw = ImageList.padded_size(sizes, size_divisibility, padding_constraints)
        raw = torch.stack(tensors) if len(tensors) > 1 else tensors[0][None]
        return ImageList.lazy(raw, sizes, hw, transform, pad_value)
