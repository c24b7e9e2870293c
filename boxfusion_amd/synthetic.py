"""Synthetic RGB-D stream and seeded 3-D scene.

The reference runs on CA-1M / ScanNet captures (boxfusion/capture_stream.py), which are not
available offline.  This module produces the stream the benchmark and the parity fixtures use:

* frames: 640x480 uint8 RGB (seed 1234 + frame), float32 depth U[0.5, 4.5] m with 5 % zeros,
  ScanNet intrinsics (config/scannet.yaml:9-16);
* poses: camera->world, z-up world, camera y pointing down (ImageOrientation.UPRIGHT,
  orientation.py:43-57), circular trajectory of radius 3.5 m at 1.5 m height;
* detections: a seeded world of oriented objects observed with noise, in the layout CuTR emits
  (cubify_transformer.py:945-978): scores, xyxy 2-D boxes, camera-frame xyz + lhw + R, projected
  centres.  These feed the fusion chain so that NMS / association / fusion see realistic work even
  though the detector runs with random weights.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

SCANNET_K = np.array([[574.540771, 0.0, 322.522827],
                      [0.0, 577.583740, 238.558853],
                      [0.0, 0.0, 1.0]], dtype=np.float32)
W, H = 640, 480


def look_at_pose(pos, target):
    """camera->world pose (OpenCV camera: x right, y down, z forward) looking at target, z-up."""
    z = np.asarray(target, np.float64) - np.asarray(pos, np.float64)
    z /= np.linalg.norm(z)
    up = np.array([0.0, 0.0, 1.0])
    x = np.cross(z, up)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    P = np.eye(4)
    P[:3, 0], P[:3, 1], P[:3, 2], P[:3, 3] = x, y, z, pos
    return P.astype(np.float32)


def trajectory_pose(frame, period=1000, radius=3.5, height=1.5):
    th = 2.0 * np.pi * (frame % period) / period
    pos = np.array([radius * np.cos(th), radius * np.sin(th), height])
    return look_at_pose(pos, [0.0, 0.0, 0.6])


def rot_z(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float64)


# box-local (l, h, w) axes -> world (x, -z, y): gravity-aligned, h along gravity
_A = np.array([[1, 0, 0], [0, 0, 1], [0, -1, 0]], np.float64)


def box_corners_np(xyzlhw, R):
    """boxes.py:725-778 layout (v0..v7) in float64 for scene bookkeeping."""
    l, h, w = xyzlhw[3], xyzlhw[4], xyzlhw[5]
    sx = np.array([-1, 1, 1, -1, -1, 1, 1, -1]) * l / 2
    sy = np.array([-1, -1, 1, 1, -1, -1, 1, 1]) * h / 2
    sz = np.array([-1, -1, -1, -1, 1, 1, 1, 1]) * w / 2
    v = np.stack([sx, sy, sz], 0)
    return (R @ v).T + xyzlhw[:3]


@dataclass
class Scene:
    seed: int = 0
    n_objects: int = 30
    period: int = 1000
    dup_prob: float = 0.15
    drop_prob: float = 0.1
    noise: float = 1.0           # detection noise multiplier (centre sigma = 2 cm * noise)
    dim_lo: float = 0.15
    dim_hi: float = 1.0
    objects: np.ndarray = field(default=None, repr=False)  # [n,7] xyz lhw yaw

    def __post_init__(self):
        rng = np.random.default_rng(self.seed)
        r = 2.2 * np.sqrt(rng.uniform(0, 1, self.n_objects))
        a = rng.uniform(-np.pi, np.pi, self.n_objects)
        dims = rng.uniform(self.dim_lo, self.dim_hi, (self.n_objects, 3))
        z = dims[:, 1] / 2 + rng.uniform(0, 0.6, self.n_objects)
        yaw = rng.uniform(-np.pi, np.pi, self.n_objects)
        self.objects = np.column_stack([r * np.cos(a), r * np.sin(a), z, dims, yaw])

    def pose(self, frame):
        return trajectory_pose(frame, self.period)

    def detections(self, frame, K=SCANNET_K, size=(W, H)):
        """Detections of keyframe `frame` in CuTR's output layout (camera frame); size = (W, H) of
        the image the 2-D boxes live in."""
        W, H = size
        rng = np.random.default_rng(10_000 + self.seed * 7919 + frame)
        P = self.pose(frame).astype(np.float64)
        Rc, tc = P[:3, :3], P[:3, 3]
        out = dict(scores=[], pred_boxes=[], xyzlhw=[], R=[], proj_xy=[])

        def emit(c_world, dims, yaw, score, noise):
            xyz_c = Rc.T @ (c_world - tc) + rng.normal(0, 0.02 * noise, 3)
            if xyz_c[2] < 0.3 or xyz_c[2] > 6.0:
                return
            d = dims * (1.0 + rng.normal(0, 0.05 * noise, 3))
            d = np.maximum(d, 0.05)
            Rw = rot_z(yaw + rng.normal(0, 0.05 * noise)) @ _A
            Rcam = Rc.T @ Rw
            u = K[0, 0] * xyz_c[0] / xyz_c[2] + K[0, 2]
            v = K[1, 1] * xyz_c[1] / xyz_c[2] + K[1, 2]
            if not (0 <= u < W and 0 <= v < H):
                return
            cc = box_corners_np(np.concatenate([xyz_c, d]), Rcam)
            zc = np.maximum(cc[:, 2], 1e-3)
            uu = np.clip(K[0, 0] * cc[:, 0] / zc + K[0, 2], 0, W)
            vv = np.clip(K[1, 1] * cc[:, 1] / zc + K[1, 2], 0, H)
            out["scores"].append(score)
            out["pred_boxes"].append([uu.min(), vv.min(), uu.max(), vv.max()])
            out["xyzlhw"].append(np.concatenate([xyz_c, d]))
            out["R"].append(Rcam)
            out["proj_xy"].append([u, v])

        for o in self.objects:
            if rng.uniform() < self.drop_prob:
                continue
            s = rng.uniform(0.4, 0.95)
            emit(o[:3], o[3:6], o[6], s, self.noise)
            if rng.uniform() < self.dup_prob:
                emit(o[:3], o[3:6], o[6], s * rng.uniform(0.6, 0.99), 2.0 * self.noise)
        n = len(out["scores"])
        return dict(
            scores=np.asarray(out["scores"], np.float32).reshape(n),
            pred_boxes=np.asarray(out["pred_boxes"], np.float32).reshape(n, 4),
            xyzlhw=np.asarray(out["xyzlhw"], np.float32).reshape(n, 6),
            R=np.asarray(out["R"], np.float32).reshape(n, 3, 3),
            proj_xy=np.asarray(out["proj_xy"], np.float32).reshape(n, 2),
        )


def frame_rgbd(frame, h=H, w=W):
    """Seeded synthetic RGB-D frame: uint8 [h,w,3], float32 depth [h,w] (5 % zeros)."""
    rng = np.random.default_rng(1234 + frame)
    rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    depth = rng.uniform(0.5, 4.5, (h, w)).astype(np.float32)
    depth[rng.uniform(0, 1, (h, w)) < 0.05] = 0.0
    return rgb, depth
