"""Run visualisation: what demo.py logs to rerun, kept off the hot path.

The reference logs, per frame, the camera pose / pinhole, the RGB image, the depth image, the
back-projected GT points, the trajectory, and after every keyframe the global boxes
(`tools/utils.py:37-96 visualize_online_boxes`, demo.py:35-65 blueprint, demo.py:93-197 the log
calls); `boxes3d_to_ply` (`tools/utils.py:99-141`) writes the boxes as a coloured triangle mesh
through open3d.

Here `Recording` takes the same `log(entity_path, archetype)` calls.  It forwards them to rerun
when the `rerun` package is importable (it is not in this image) and otherwise keeps them as
plain records -- entity path, time, archetype name, arrays -- that `save()` writes as JSON lines
(image pixels as their shape and a checksum, or as .npy files with `keep_images=True`).  The PLY
writer needs no open3d (binary little-endian PLY: float64 vertices, uchar RGB, int32 triangles --
the fields open3d writes).  Nothing here runs in the timed bench.
"""
from __future__ import annotations

import json
import os
import zlib

import numpy as np

try:                                  # the real viewer when present (never in this image)
    import rerun as _rr               # noqa: F401
except ImportError:                   # pragma: no cover - depends on the image
    _rr = None


def random_color_v2(value, maximum=255):
    """boxfusion/color.py random_color_v2: the jet colormap at `value` in [0, 1] (RGB in [0, 1];
    `maximum` is unused there too)"""
    import matplotlib
    rgba = matplotlib.colormaps["jet"](value)
    return np.array(rgba[:3])


def _quat_xyzw(R):
    """rotation matrices [n,3,3] -> quaternions [n,4] (x, y, z, w), scipy's from_matrix().as_quat()"""
    from scipy.spatial.transform import Rotation
    R = np.asarray(R, dtype=np.float64).reshape(-1, 3, 3)
    return Rotation.from_matrix(R).as_quat() if len(R) else np.zeros((0, 4))


# --- archetypes: the fields demo.py passes; plain data -----------------------------------------
class Archetype(dict):
    kind = "Archetype"

    def __init__(self, **fields):
        super().__init__(**fields)


def _arch(name):
    return type(name, (Archetype,), {"kind": name})


Transform3D = _arch("Transform3D")          # translation, quaternion_xyzw
Pinhole = _arch("Pinhole")                  # image_from_camera [3,3], resolution [W,H]
Image = _arch("Image")                      # image [H,W,3] u8
DepthImage = _arch("DepthImage")            # image [H,W] f32
Points3D = _arch("Points3D")                # positions [n,3], colors [n,3]
LineStrips3D = _arch("LineStrips3D")        # strips: list of [n,3], colors
Boxes3D = _arch("Boxes3D")                  # centers, sizes, quaternions_xyzw, colors, labels, show_labels


class Recording:
    """rerun.new_recording + rerun.set_time_seconds + rerun.log, as records (or forwarded)"""

    def __init__(self, application_id="boxfusion", keep_images=False, forward=True):
        self.application_id = str(application_id)
        self.keep_images = keep_images
        self.records = []
        self.time = None
        self._rr = _rr if forward else None
        if self._rr is not None:
            self._rr.init(self.application_id, spawn=False)

    def set_time_seconds(self, timeline, seconds):
        self.time = (timeline, float(seconds))
        if self._rr is not None:
            self._rr.set_time_seconds(timeline, seconds)

    def log(self, path, arch):
        self.records.append((path, self.time, arch.kind, arch))
        if self._rr is not None:
            self._rr.log(path, _to_rerun(self._rr, arch))

    def entities(self):
        return sorted({p for p, _, _, _ in self.records})

    def last(self, path, kind=None):
        for p, _, k, a in reversed(self.records):
            if p == path and (kind is None or k == kind):
                return a
        return None

    def save(self, path):
        """JSON lines: {"path", "time", "kind", fields...}; images as shape + adler32 unless
        keep_images (then an .npy beside the file)"""
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            for i, (p, t, k, a) in enumerate(self.records):
                rec = {"path": p, "time": t, "kind": k}
                for key, v in a.items():
                    if k in ("Image", "DepthImage") and key == "image":
                        arr = np.ascontiguousarray(v)
                        rec["shape"] = list(arr.shape)
                        rec["adler32"] = zlib.adler32(arr.tobytes())
                        if self.keep_images:
                            fn = f"{os.path.splitext(path)[0]}_{i:06d}.npy"
                            np.save(fn, arr)
                            rec["file"] = os.path.basename(fn)
                    elif isinstance(v, np.ndarray):
                        rec[key] = v.tolist()
                    elif isinstance(v, (list, tuple)):
                        rec[key] = [x.tolist() if isinstance(x, np.ndarray) else x for x in v]
                    else:
                        rec[key] = v
                f.write(json.dumps(rec) + "\n")


def _to_rerun(rr, a):               # pragma: no cover - rerun is not installed here
    k = a.kind
    if k == "Transform3D":
        return rr.Transform3D(translation=a["translation"], rotation=rr.Quaternion(xyzw=a["quaternion_xyzw"]))
    if k == "Pinhole":
        return rr.Pinhole(image_from_camera=a["image_from_camera"], resolution=a["resolution"])
    if k == "Image":
        return rr.Image(a["image"])
    if k == "DepthImage":
        return rr.DepthImage(a["image"])
    if k == "Points3D":
        return rr.Points3D(positions=a["positions"], colors=a["colors"])
    if k == "LineStrips3D":
        return rr.LineStrips3D(a["strips"], colors=a["colors"])
    return rr.Boxes3D(centers=a["centers"], sizes=a["sizes"],
                      quaternions=[rr.Quaternion(xyzw=q) for q in a["quaternions_xyzw"]],
                      colors=a["colors"], labels=a["labels"], show_labels=a["show_labels"])


def visualize_online_boxes(instances, prefix, recording, boxes_3d_name="gt_boxes_3d",
                           log_instances_name="instances", count=0, save=False, show_class=False,
                           show_label=True, out_dir="./result"):
    """tools/utils.py:37-96: one Boxes3D per call at {prefix}/{log_instances_name} -- gravity
    centres, dims, the box rotations as quaternions, jet colours by index, labels = indices or
    categories; `save` also writes {out_dir}/box_{count}.ply"""
    boxes = getattr(instances, boxes_3d_name)
    n = len(boxes)
    colors = [random_color_v2(i / n) for i in range(n)]
    quats = _quat_xyzw(boxes.R.detach().cpu().numpy()) if n else np.zeros((0, 4))
    centers = boxes.gravity_center.detach().cpu().numpy()
    sizes = boxes.dims.detach().cpu().numpy()
    if not show_class:
        ids = np.arange(n).astype(str)
    else:
        ids = np.asarray(instances.categories)
    arch = Boxes3D(centers=centers, sizes=sizes, quaternions_xyzw=quats,
                   colors=np.asarray(colors).reshape(-1, 3), labels=[str(x) for x in ids],
                   show_labels=bool(show_label))
    recording.log(f"{prefix}/{log_instances_name}", arch)
    if save:
        boxes3d_to_ply(sizes, centers, colors, quats, os.path.join(out_dir, f"box_{count}.ply"))
    return arch


_FACES = np.array([[0, 1, 2], [0, 2, 3], [4, 5, 6], [4, 6, 7], [0, 1, 5], [0, 5, 4],
                   [1, 2, 6], [1, 6, 5], [2, 3, 7], [2, 7, 6], [3, 0, 4], [3, 4, 7]], dtype=np.int32)
_UNIT = np.array([[-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1],
                  [-1, -1, 1], [1, -1, 1], [1, 1, 1], [-1, 1, 1]], dtype=np.float64)


def box_mesh(sizes, centers, quaternions):
    """the vertices [8n,3] and triangles [12n,3] of tools/utils.py:99-141"""
    from scipy.spatial.transform import Rotation
    sizes = np.asarray(sizes, np.float64).reshape(-1, 3)
    centers = np.asarray(centers, np.float64).reshape(-1, 3)
    verts, faces = [], []
    for i in range(len(centers)):
        rot = Rotation.from_quat(np.asarray(quaternions[i], np.float64)).as_matrix()
        verts.append((_UNIT * (sizes[i] / 2)) @ rot.T + centers[i])
        faces.append(_FACES + 8 * i)
    if not verts:
        return np.zeros((0, 3)), np.zeros((0, 3), np.int32)
    return np.vstack(verts), np.vstack(faces)


def boxes3d_to_ply(sizes, centers, colors, quaternions, output_path):
    """tools/utils.py:99-141 without open3d: a binary little-endian PLY triangle mesh, eight
    vertices per box in the box's colour"""
    verts, faces = box_mesh(sizes, centers, quaternions)
    cols = np.repeat(np.clip(np.rint(np.asarray(colors, np.float64).reshape(-1, 3) * 255.0), 0, 255)
                     .astype(np.uint8), 8, axis=0)
    os.makedirs(os.path.dirname(os.path.abspath(output_path)), exist_ok=True)
    vdt = np.dtype([("x", "<f8"), ("y", "<f8"), ("z", "<f8"), ("red", "u1"), ("green", "u1"), ("blue", "u1")])
    v = np.empty(len(verts), vdt)
    v["x"], v["y"], v["z"] = verts[:, 0], verts[:, 1], verts[:, 2]
    v["red"], v["green"], v["blue"] = cols[:, 0], cols[:, 1], cols[:, 2]
    fdt = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
    f = np.empty(len(faces), fdt)
    f["n"] = 3
    f["i"] = faces
    header = ("ply\nformat binary_little_endian 1.0\n"
              f"element vertex {len(v)}\nproperty double x\nproperty double y\nproperty double z\n"
              "property uchar red\nproperty uchar green\nproperty uchar blue\n"
              f"element face {len(f)}\nproperty list uchar int vertex_indices\nend_header\n")
    with open(output_path, "wb") as fh:
        fh.write(header.encode("ascii"))
        fh.write(v.tobytes())
        fh.write(f.tobytes())


def read_ply_mesh(path):
    """the vertices, colours and triangles of a PLY written by boxes3d_to_ply"""
    with open(path, "rb") as fh:
        data = fh.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    head = data[:end].decode("ascii").split("\n")
    nv = int([h for h in head if h.startswith("element vertex")][0].split()[-1])
    nf = int([h for h in head if h.startswith("element face")][0].split()[-1])
    vdt = np.dtype([("x", "<f8"), ("y", "<f8"), ("z", "<f8"), ("red", "u1"), ("green", "u1"), ("blue", "u1")])
    fdt = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
    v = np.frombuffer(data, vdt, nv, end)
    f = np.frombuffer(data, fdt, nf, end + nv * vdt.itemsize)
    return (np.stack([v["x"], v["y"], v["z"]], 1), np.stack([v["red"], v["green"], v["blue"]], 1),
            f["i"].copy())


class FrameLogger:
    """demo.py:93-197's per-frame log calls in the reference's order: set_time, camera pose +
    pinhole on /world/image and /device/wide/image, the RGB image, the depth image and its
    pinhole, the back-projected points, the trajectory, and after a keyframe's fusion the global
    boxes under /device/wide/pred_instances"""

    def __init__(self, recording, K_image, image_size, K_depth=None, depth_size=None, fps=30.0,
                 trajectory=True, show_class=False, show_label=True, log_images=True, save_ply=False,
                 out_dir="./result", depth_invalid_nan=False):
        self.rec = recording
        self.K_image, self.image_size = np.asarray(K_image, np.float64), list(image_size)
        self.K_depth = None if K_depth is None else np.asarray(K_depth, np.float64)
        self.depth_size = None if depth_size is None else list(depth_size)
        self.fps = fps
        self.trajectory = trajectory
        self.show_class, self.show_label = show_class, show_label
        self.log_images, self.save_ply, self.out_dir = log_images, save_ply, out_dir
        # depth_invalid_nan: the logged depth with its <= 0 pixels as NaN -- what demo.py:190 logs
        # on a --device cpu run, where Preprocessor.standardize_depth_map's in-place NaN fill
        # (preprocessor.py:102) reaches the sample's own depth tensor (on a GPU run the .cpu()
        # copy keeps the logged depth raw)
        self.depth_invalid_nan = depth_invalid_nan
        self.traj_xyz = []

    def frame(self, count, RT, image=None, depth=None, xyzrgb=None, timestamp=None):
        r = self.rec
        RT = np.asarray(RT, np.float64)
        r.set_time_seconds("pts", count / self.fps if timestamp is None else timestamp)
        pose = Transform3D(translation=RT[:3, 3], quaternion_xyzw=_quat_xyzw(RT[None, :3, :3])[0])
        cam = Pinhole(image_from_camera=self.K_image, resolution=self.image_size)
        r.log("/world/image", pose)
        r.log("/world/image", cam)
        r.log("/device/wide/image", pose)
        if self.log_images and image is not None:
            r.log("/device/wide/image", Image(image=np.asarray(image)))
        r.log("/device/wide/image", cam)
        self.traj_xyz.append(RT[:3, 3].copy())
        if depth is not None and self.log_images and self.K_depth is not None:
            depth = np.asarray(depth)
            if self.depth_invalid_nan:
                depth = np.where(depth <= 0, np.float32(np.nan), depth).astype(depth.dtype)
            r.log("/device/wide/depth", DepthImage(image=depth))
            r.log("/device/wide/depth", Pinhole(image_from_camera=self.K_depth, resolution=self.depth_size))
        if xyzrgb is not None:
            xyzrgb = np.asarray(xyzrgb)
            r.log("/world/xyz", Points3D(positions=xyzrgb[..., :3], colors=xyzrgb[..., 3:]))
        if self.trajectory:
            # demo.py:108 logs the trajectory up to (not including) the current count
            r.log("/world/trajectory", LineStrips3D(strips=[np.array(self.traj_xyz)[:count]],
                                                    colors=[84, 255, 159]))

    def boxes(self, all_pred_box, count):
        if all_pred_box is None or len(all_pred_box) == 0:
            return None
        return visualize_online_boxes(all_pred_box, "/device/wide", self.rec, boxes_3d_name="pred_boxes_3d",
                                      log_instances_name="pred_instances", count=count,
                                      save=self.save_ply, show_class=self.show_class,
                                      show_label=self.show_label, out_dir=self.out_dir)
