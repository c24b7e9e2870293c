"""Frame packaging and preprocessing (reference: boxfusion/preprocessor.py:1-217), drop-in for
demo.py:129-131:

    packaged = augmentor.package(sample)
    packaged = move_input_to_current_device(packaged, device)
    packaged = preprocessor.preprocess([packaged])
    pred_instances = model(packaged)[0]

Reference semantics, and where they run here:
  * RGB: (x - pixel_mean) / pixel_std with `pixel_mean.to(measurement.data)` (preprocessor.py:142).
    In demo.py's order the frame was already turned into float32 by move_input_to_current_device
    (Measurement.to(model.pixel_mean)), so the constants are (123.675, 116.28, 103.53) /
    (58.395, 57.12, 57.375); a frame preprocessed while still uint8 gets them cast to uint8,
    (123, 116, 103) / (58, 57, 57), exactly as in the reference.  The normalisation is recorded,
    not applied: the engine fuses it into the patch-embedding im2col (bf_im2col_rgb8_chw), and
    `ImageList.tensor` builds the normalised padded batch only if something reads it;
  * depth: trimmed standardisation (preprocessor.py:97-129) -> bf_depth_standardize (radix
    select on the device instead of a CPU sort of every pixel);
  * zero padding to the smallest square in [256..1024] >= the longest edge, /32; depth at
    square // round(rgb_w / depth_w), ratio in {1, 2, 4} (:146-200, imagelist.py:55-115) --
    virtual (the im2col kernels read past the frame as zeros).
There is no CPU path: preprocessing tensors that are not on the HIP device raises.
"""
from __future__ import annotations

import copy
import os
from typing import Dict, List

import torch

from boxfusion_amd.batching import (BatchedPosedDepth, BatchedPosedImage, Measurement, PosedDepth,
                                    PosedImage)
from boxfusion_amd.measurement import DepthMeasurementInfo, ImageMeasurementInfo

PIXEL_MEAN = (123.675, 116.28, 103.53)
PIXEL_STD = (58.395, 57.12, 57.375)
PIXEL_MEAN_U8 = tuple(float(int(v)) for v in PIXEL_MEAN)   # uint8 cast of the constants
PIXEL_STD_U8 = tuple(float(int(v)) for v in PIXEL_STD)
SQUARE_PAD = (256, 384, 512, 640, 768, 896, 1024)
SIZE_DIVISIBILITY = 32
IGNORE_KEYS = ["sensor_info", "__key__", "gt", "video_info", "meta"]


def square_pad_size(h, w, square_pad=SQUARE_PAD, div=SIZE_DIVISIBILITY):
    longest = max(h, w)
    s = int(min(s for s in square_pad if s >= longest))
    return (s + div - 1) // div * div


def rgb_to_depth_ratio(rgb_size, depth_size):
    """preprocessor.py:159-164 (sizes are (w, h))"""
    r = round(rgb_size[0] / depth_size[0])
    if r not in (1, 2, 4):
        raise ValueError(f"Unsupported rgb -> depth ratio: {r}")
    return r


def _move(x, t):
    if isinstance(x, (list, tuple)):
        return [_move(x_, t) for x_ in x]
    if isinstance(x, Measurement) and isinstance(t, torch.Tensor) and x.data.dtype == torch.uint8 \
            and t.is_floating_point():
        # the reference's Measurement.to(pixel_mean) turns a uint8 frame into float32 (Tensor.to of
        # a tensor takes its dtype), so demo.py normalises with the float constants.  The frame
        # stays uint8 here (exact in f32; the patch-embedding kernel converts it) and is marked.
        m = type(x)(x.data.to(t.device), x.info.to(t.device), x.sensor.to(t.device))
        m._as_float = True
        return m
    try:
        return x.to(t)
    except Exception:  # noqa: BLE001 - the reference's move_device_like fallback
        return x.to(t.device)


def move_input_to_current_device(batched_input, t):
    """preprocessor.py:34-36 (demo.py:130 passes model.pixel_mean): every measurement moved to
    `t`'s device and, as in the reference, to its dtype -- a uint8 frame only virtually (above)."""
    return {name: {n_: _move(m, t) for n_, m in s.items()} for name, s in batched_input.items()}


class Augmentor:
    """preprocessor.py:40-82: sample dict -> {sensor: {measurement: PosedImage | PosedDepth}}
    (last frame of each measurement, its info and a copy of the sensor info)."""

    def __init__(self, measurement_keys=None):
        self.measurement_keys = measurement_keys

    def package(self, sample) -> Dict[str, Dict[str, Measurement]]:
        result = {}
        for sensor_name, sensor_data in sample.items():
            if sensor_name in IGNORE_KEYS or not isinstance(sensor_data, dict):
                continue
            sensor_info = copy.deepcopy(getattr(sample["sensor_info"], sensor_name))
            out = {}
            for name, meas in sensor_data.items():
                key = os.path.join(sensor_name, name)
                if self.measurement_keys is not None and key not in self.measurement_keys:
                    if sensor_info.has(name):
                        sensor_info.remove(name)
                    continue
                info = getattr(sensor_info, name)
                if _is_depth_info(info):
                    out[name] = PosedDepth(meas[-1], info, sensor_info)
                elif _is_image_info(info):
                    out[name] = PosedImage(meas[-1], info, sensor_info)
            if out:
                result[sensor_name] = out
        return result


def _is_depth_info(info):
    # the reference's own info classes (a sample from its capture stream) or this package's
    return isinstance(info, DepthMeasurementInfo) or type(info).__name__ in (
        "DepthMeasurementInfo", "WhitenedDepthMeasurementInfo")


def _is_image_info(info):
    return isinstance(info, ImageMeasurementInfo) or type(info).__name__ == "ImageMeasurementInfo"


def _whiten(info, parameters):
    if hasattr(info, "normalize"):
        return info.normalize(parameters)
    from boxfusion_amd.measurement import WhitenedDepthMeasurementInfo
    return WhitenedDepthMeasurementInfo(info.size, info.K, meta=getattr(info, "meta", None),
                                        parameters=parameters,
                                        original_size=getattr(info, "original_size", None))


def _is_posed_depth(m):
    return isinstance(m, PosedDepth) or (isinstance(m, Measurement) and _is_depth_info(m.info))


def _is_posed_image(m):
    return isinstance(m, PosedImage) or (isinstance(m, Measurement) and _is_image_info(m.info)
                                         and not _is_depth_info(m.info))


class Preprocessor:
    def __init__(self, square_pad=list(SQUARE_PAD), size_divisibility=SIZE_DIVISIBILITY,
                 pixel_mean=list(PIXEL_MEAN), pixel_std=list(PIXEL_STD), device=None):
        self.square_pad = square_pad
        self.size_divisibility = size_divisibility
        self.pixel_mean = torch.tensor(pixel_mean).view(-1, 1, 1)
        self.pixel_std = torch.tensor(pixel_std).view(-1, 1, 1)
        self.device = device

    @staticmethod
    def standardize_depth_map(img, trunc_value=0.1):
        """preprocessor.py:97-129 on the device: img [H, W] (or [N, H, W]) f32 ->
        (standardised, [mean, std]) via bf_depth_standardize"""
        if trunc_value != 0.1:
            raise NotImplementedError("bf_depth_standardize trims 10 % per side (the reference default)")
        from boxfusion_amd import _lib
        x = img if img.dim() == 3 else img[None]
        out, params = _lib.depth_standardize(x.float().contiguous())
        return (out if img.dim() == 3 else out[0]), (params if img.dim() == 3 else params[0])

    def normalize(self, batched_input):
        """in place, like the reference (preprocessor.py:131-144)"""
        for sensor in batched_input.values():
            for name, m in sensor.items():
                if name == "features":
                    continue
                if _is_posed_depth(m):
                    m.data, scaling = self.standardize_depth_map(m.data)
                    m.info = _whiten(m.info, scaling[None])
                elif _is_posed_image(m):
                    if m.data.dtype != torch.uint8:
                        raise NotImplementedError("the MI355X patch embedding takes uint8 frames")
                    # `pixel_mean.to(measurement.data)`: float constants for a frame the reference
                    # holds as float32 (moved by move_input_to_current_device), constants cast to
                    # uint8 -- (123, 116, 103) / (58, 57, 57) -- for a frame still uint8
                    if getattr(m, "_as_float", False):
                        m._normalize = (self.pixel_mean.float(), self.pixel_std.float())
                    else:
                        m._normalize = (self.pixel_mean.to(torch.uint8).float(),
                                        self.pixel_std.to(torch.uint8).float())
        return batched_input

    def batch(self, batched_inputs: List[Dict]) -> Dict:
        result = {}
        for sensor_name in batched_inputs[0].keys():
            out = {}
            names = list(batched_inputs[0][sensor_name].keys())
            # images first: the depth's square follows the image's (preprocessor.py:157-158)
            names.sort(key=lambda n: 0 if _is_posed_image(batched_inputs[0][sensor_name][n]) else 1)
            square, rgb_size = None, None
            for name in names:
                ms = [bi[sensor_name][name] for bi in batched_inputs]
                if name == "features":
                    out["features"] = ms[0]
                    continue
                if _is_posed_image(ms[0]):
                    rgb_size = ms[0].info.size
                    square = self.square_pad
                    if isinstance(square, (list, tuple)):
                        longest = max(max(m.info.size) for m in ms)
                        square = int(min(s for s in square if s >= longest))
                    mean, std = getattr(ms[0], "_normalize", (None, None))
                    tf = (lambda x, mean=mean, std=std: (x.float() - mean.to(x.device)) / std.to(x.device)) \
                        if mean is not None else None
                    b = Measurement.batch(ms, transform=tf, size_divisibility=self.size_divisibility,
                                          padding_constraints={"size_divisibility": self.size_divisibility,
                                                               "square_size": square})
                    b.normalize_consts = (tuple(mean.view(-1).tolist()), tuple(std.view(-1).tolist())) \
                        if mean is not None else None
                elif _is_posed_depth(ms[0]):
                    if square is None:
                        raise ValueError("the image must be batched before the depth")
                    r = rgb_to_depth_ratio(rgb_size, ms[0].info.size)
                    b = Measurement.batch(ms, size_divisibility=self.size_divisibility,
                                          padding_constraints={"size_divisibility": self.size_divisibility,
                                                               "square_size": square // r})
                    b.rgb_to_depth_ratio = r
                else:
                    continue
                out[name] = b
            result[sensor_name] = out
        return result

    def __call__(self, batches):
        for batch in batches:
            if isinstance(batch, tuple):
                input_, gt_ = batch
                if self.device is not None:
                    input_ = move_input_to_current_device(input_, self.device)
                yield self.preprocess([input_]), gt_
            else:
                yield self.preprocess(batch)

    def preprocess(self, batched_inputs: List[Dict]) -> Dict:
        return self.batch([self.normalize(bi) for bi in batched_inputs])
