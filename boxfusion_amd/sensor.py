"""Per-frame camera bookkeeping on the host (tiny 3x3/4x4 maths, once per frame):
orientation detection (orientation.py:43-57) and the camera->gravity rotation T_gravity
(capture_stream.py:62-82) that CuTR applies to its yaw-only box poses."""
from __future__ import annotations

from enum import Enum

import numpy as np
from scipy.spatial.transform import Rotation


class ImageOrientation(Enum):
    UPRIGHT = 0
    LEFT = 1
    UPSIDE_DOWN = 2
    RIGHT = 3
    ORIGINAL = 4


_ROT_Z_ANGLE = {
    (ImageOrientation.UPRIGHT, ImageOrientation.UPRIGHT): 0.0,
    (ImageOrientation.LEFT, ImageOrientation.UPRIGHT): np.pi / 2,
    (ImageOrientation.UPSIDE_DOWN, ImageOrientation.UPRIGHT): np.pi,
    (ImageOrientation.RIGHT, ImageOrientation.UPRIGHT): -np.pi / 2,
}


def get_orientation(pose):
    """argmax of the camera axes' world-z components against the 4 canonical rolls"""
    z = np.asarray(pose, np.float32)[2, :3]
    cand = np.array([[0.0, -1.0, 0.0], [-1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [1.0, 0.0, 0.0]],
                    np.float32)
    return ImageOrientation(int(np.argmax(cand @ z)))


def camera_to_gravity(pose, current=ImageOrientation.UPRIGHT):
    """T_gravity (3x3, f32) for a camera->world pose with z-up world."""
    P = np.asarray(pose, np.float64).copy()
    Rz = np.eye(4)
    Rz[:3, :3] = Rotation.from_euler("z", _ROT_Z_ANGLE[(current, ImageOrientation.UPRIGHT)]).as_matrix()
    P = P @ np.linalg.inv(Rz)
    R = P[:3, :3]
    # world-space basis of the reference's unit "fake box" (x, -z, y), seen from the camera
    basis = R.T @ np.array([[1.0, 0.0, 0.0], [0.0, 0.0, -1.0], [0.0, 1.0, 0.0]]).T
    basis = basis / np.linalg.norm(basis, axis=0, keepdims=True)
    ang = Rotation.from_matrix(basis).as_euler("yxz")[1:]
    return Rotation.from_euler("xz", ang).as_matrix().astype(np.float32)


def rotate_K(K, current, image_size, target=ImageOrientation.UPRIGHT):
    """intrinsics [N,3,3] after rotating the image from `current` to `target` orientation
    (orientation.py:59-86): a quarter turn swaps the focal lengths and principal-point axes, a
    half turn mirrors the principal point (image_size = (w, h))"""
    K = K.clone()
    key = (current, target)
    if key == (ImageOrientation.UPRIGHT, ImageOrientation.UPRIGHT):
        return K
    quarter = {(ImageOrientation.LEFT, ImageOrientation.UPRIGHT), (ImageOrientation.UPRIGHT, ImageOrientation.RIGHT),
               (ImageOrientation.RIGHT, ImageOrientation.UPRIGHT), (ImageOrientation.UPRIGHT, ImageOrientation.LEFT)}
    half = {(ImageOrientation.UPSIDE_DOWN, ImageOrientation.UPRIGHT),
            (ImageOrientation.UPRIGHT, ImageOrientation.UPSIDE_DOWN)}
    if key in quarter:
        out = K.clone()
        out[:, 0, 0], out[:, 0, 1], out[:, 0, 2] = K[:, 1, 1], K[:, 0, 1], K[:, 1, 2]
        out[:, 1, 0], out[:, 1, 1], out[:, 1, 2] = K[:, 1, 0], K[:, 0, 0], K[:, 0, 2]
        return out
    if key in half:
        K[:, 0, 2] = image_size[0] - K[:, 0, 2]
        K[:, 1, 2] = image_size[1] - K[:, 1, 2]
        return K
    raise ValueError("unknown orientation")


class SensorInfo:
    """named per-sensor measurement infos (sensor.py:13-156): image / depth infos, RT poses,
    T_gravity; attribute access, has / remove / get, to()"""

    def __init__(self, **kwargs):
        object.__setattr__(self, "_measurements", {})
        object.__setattr__(self, "_other", {})
        for k, v in kwargs.items():
            self.set(k, v)

    def __setattr__(self, name, val):
        if name.startswith("_"):
            self._other[name] = val
        else:
            self.set(name, val)

    def __getattr__(self, name):
        if name.startswith("_"):
            other = object.__getattribute__(self, "_other")
            if name in other:
                return other[name]
            raise AttributeError(name)
        m = object.__getattribute__(self, "_measurements")
        if name not in m:
            raise AttributeError(f"Cannot find field '{name}' in the given measurements!")
        return m[name]

    def set(self, name, value):
        self._measurements[name] = value

    def has(self, name):
        return name in self._measurements

    def remove(self, name):
        del self._measurements[name]

    def get(self, name):
        return self._measurements[name]

    def __len__(self):
        for v in self._measurements.values():
            return len(v)
        return 0

    def get_measurements(self):
        from boxfusion_amd.measurement import MeasurementInfo
        return {k: m for k, m in self._measurements.items() if isinstance(m, MeasurementInfo)}

    def to(self, *args, **kwargs):
        ret = type(self)()
        for k, v in self._measurements.items():
            ret.set(k, v.to(*args, **kwargs) if hasattr(v, "to") else v)
        for k, v in self._other.items():
            ret._other[k] = v
        return ret


class PosedSensorInfo(SensorInfo):
    @property
    def orientation(self):
        if "_orientation" in self._other:
            return self._other["_orientation"]
        RT = self.RT
        votes = [get_orientation(np.asarray(p.detach().cpu() if hasattr(p, "detach") else p)).value
                 for p in RT]
        return ImageOrientation(int(np.bincount(votes).argmax()))


class SensorArrayInfo:
    """named sensors of one sample (sensor.py:231-293), e.g. `wide` and `gt`"""

    def __init__(self, **kwargs):
        object.__setattr__(self, "_sensors", {})
        for k, v in kwargs.items():
            self.set(k, v)

    def __setattr__(self, name, val):
        if name.startswith("_"):
            object.__setattr__(self, name, val)
        else:
            self.set(name, val)

    def __getattr__(self, name):
        s = object.__getattribute__(self, "_sensors")
        if name.startswith("_") or name not in s:
            raise AttributeError(f"Cannot find field '{name}' in the given sensors!")
        return s[name]

    def set(self, name, value):
        self._sensors[name] = value

    def has(self, name):
        return name in self._sensors

    def remove(self, name):
        del self._sensors[name]

    def get(self, name):
        return self._sensors[name]

    def to(self, *args, **kwargs):
        ret = type(self)()
        for k, v in self._sensors.items():
            ret.set(k, v.to(*args, **kwargs) if hasattr(v, "to") else v)
        return ret
