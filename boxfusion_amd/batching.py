"""Measurement containers (reference: boxfusion/batching.py:26-90).

`PosedImage` / `PosedDepth` = (data, info, sensor) of one frame as `Augmentor.package` builds them;
`BatchedPosedImage` / `BatchedPosedDepth` = (ImageList, [info], [sensor]) after
`Preprocessor.batch`.  The reference tells them apart through typing generics' `__orig_class__`;
here they are plain subclasses.
"""
from __future__ import annotations

from typing import Any, Dict, List

from boxfusion_amd.imagelist import ImageList
from boxfusion_amd.measurement import DepthMeasurementInfo, ImageMeasurementInfo


class Measurement:
    def __init__(self, data, info, sensor):
        self.data = data
        self.info = info
        self.sensor = sensor

    @classmethod
    def batch(cls, args: List["Measurement"], transform=None, **kwargs) -> "BatchedMeasurement":
        il = ImageList.from_tensors([a.data for a in args], transform=transform, **kwargs)
        kind = BatchedPosedDepth if isinstance(args[0].info, DepthMeasurementInfo) else (
            BatchedPosedImage if isinstance(args[0].info, ImageMeasurementInfo) else None)
        if kind is None:
            raise NotImplementedError
        return kind(il, [a.info for a in args], [a.sensor for a in args])

    def to(self, *args: Any, **kwargs: Any) -> "Measurement":
        return type(self)(self.data.to(*args, **kwargs), self.info.to(*args, **kwargs),
                          self.sensor.to(*args, **kwargs))


class PosedImage(Measurement):
    pass


class PosedDepth(Measurement):
    pass


class BatchedMeasurement:
    def __init__(self, data, info: List, sensor: List):
        self.data = data
        self.info = info
        self.sensor = sensor

    def __getitem__(self, index):
        return type(self)(data=self.data if isinstance(self.data, ImageList) else self.data[index],
                          info=self.info[index], sensor=self.sensor[index])


class BatchedPosedImage(BatchedMeasurement):
    pass


class BatchedPosedDepth(BatchedMeasurement):
    pass


Sensors = Dict[str, Dict[str, Measurement]]
BatchedSensors = Dict[str, Dict[str, BatchedMeasurement]]
