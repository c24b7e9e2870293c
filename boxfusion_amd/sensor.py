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
