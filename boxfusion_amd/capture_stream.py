"""Frame packaging of the reference's capture streams (capture_stream.py:185-311 ScanNet,
:381-529 CA-1M) for frames already in memory, and a synthetic stream in that format.

`make_sample(rgb, depth, K, pose)` builds the sample dict demo.py iterates over: the CHW uint8
image and the depth map under sample["wide"], a SensorArrayInfo with the `wide` sensor (image /
depth infos, T_gravity = camera -> gravity rotation, RT = identity) and the `gt` sensor (the
camera -> world pose), the frame rotated to the upright orientation first (torch.rot90 on
whatever device the frame is on).  `make_sample_decoded` / `DecodedFrameStream` take decoded
colour + 16-bit depth frames and run the rest of the streams' per-frame work on the GPU
(bf_ingest_rgbd: cvtColor, cv2.resize, depth scaling, rotation); the 16-bit depth PNGs
(bf_png_decode_u16) and the baseline colour JPEGs (bf_jpeg_decode_rgb) are decoded on the GPU too,
or on host threads (PIL) when configured so.
"""
from __future__ import annotations

import numpy as np
import torch

from boxfusion_amd.measurement import DepthMeasurementInfo, ImageMeasurementInfo
from boxfusion_amd.sensor import (ImageOrientation, PosedSensorInfo, SensorArrayInfo, camera_to_gravity,
                                  get_orientation)

# image quarter turns to the upright orientation (orientation.py:29-40 ROT_K)
ROT_K = {ImageOrientation.UPRIGHT: 0, ImageOrientation.LEFT: -1, ImageOrientation.UPSIDE_DOWN: 2,
         ImageOrientation.RIGHT: 1}
# camera roll about its optical axis undone by the rotation (orientation.py:17-27 ROT_Z)
ROT_Z_ANGLE = {ImageOrientation.UPRIGHT: 0.0, ImageOrientation.LEFT: np.pi / 2,
               ImageOrientation.UPSIDE_DOWN: np.pi, ImageOrientation.RIGHT: -np.pi / 2}


def _rot_z4(angle):
    c, s = np.cos(angle), np.sin(angle)
    m = np.eye(4, dtype=np.float32)
    m[:2, :2] = [[c, -s], [s, c]]
    return m


def make_sample(rgb, depth, K, pose, depth_K=None, video_id=0, index=0):
    """rgb [H,W,3] uint8 (numpy or tensor), depth [Hd,Wd] f32 metres, K [3,3] image intrinsics
    (depth_K: the depth map's, default K scaled to its width), pose [4,4] camera -> world"""
    rgb_t = rgb if isinstance(rgb, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(rgb))
    dep_t = depth if isinstance(depth, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(depth))
    H, W = rgb_t.shape[:2]
    Hd, Wd = dep_t.shape[-2:]
    K = np.asarray(K, np.float32)
    if depth_K is None:
        depth_K = K.copy()
        depth_K[:2] *= Wd / W
    wide = PosedSensorInfo()
    wide.image = ImageMeasurementInfo(size=(W, H), K=torch.from_numpy(K)[None])
    depth_info = DepthMeasurementInfo(size=(Wd, Hd), K=torch.from_numpy(np.asarray(depth_K, np.float32))[None])
    wide.depth = depth_info
    pose = np.asarray(pose, np.float32)
    cur = get_orientation(pose)
    T_gravity = torch.from_numpy(camera_to_gravity(pose, cur))
    image = rgb_t.permute(2, 0, 1)[None]
    dep = dep_t.float()[None]
    k = ROT_K[cur]
    if k:
        image = torch.rot90(image, k, dims=(-2, -1))
        dep = torch.rot90(dep, k, dims=(-2, -1))
    up = PosedSensorInfo()
    up.image = wide.image.orient(cur, ImageOrientation.UPRIGHT)
    up.depth = wide.depth.orient(cur, ImageOrientation.UPRIGHT)
    up.RT = torch.eye(4)[None]            # "no need for pose anymore" (capture_stream.py:296)
    up.T_gravity = T_gravity[None]
    gt = PosedSensorInfo()
    gt.RT = torch.from_numpy(pose)[None]
    gt.depth = depth_info
    si = SensorArrayInfo()
    si.wide = up
    si.gt = gt
    return {"wide": {"image": image.contiguous(), "depth": dep.contiguous()},
            "meta": dict(video_id=video_id, timestamp=index), "sensor_info": si}


def make_sample_decoded(bgr, depth_u16, depth_scale, K, pose, video_id=0, index=0, src_bgr=True):
    """the reference streams' per-frame work after decode (capture_stream.py:194-311 ScanNet,
    :402-529 CA-1M) on the GPU: `bgr` u8 [Hc,Wc,3] as cv2.imread returns it (src_bgr=False: RGB,
    as PIL decodes), `depth_u16` [Hd,Wd] the 16-bit PNG depth, both device tensors.  One
    bf_ingest_rgbd launch does cvtColor, cv2.resize(color, (Wd, Hd)), astype(f32) / depth_scale,
    moveaxis and the rotation to the upright orientation; the sensor infos follow make_sample.
    K: the cfg intrinsics at the depth resolution (the reference uses one K for image and depth)."""
    from boxfusion_amd import _lib
    pose = np.asarray(pose, np.float32)
    cur = get_orientation(pose)
    rgb, dep = _lib.ingest_rgbd(bgr, depth_u16, depth_scale, ROT_K[cur], src_bgr=src_bgr)
    Hd, Wd = depth_u16.shape[-2:]
    K = np.asarray(K, np.float32)
    wide = PosedSensorInfo()
    wide.image = ImageMeasurementInfo(size=(Wd, Hd), K=torch.from_numpy(K)[None])
    depth_info = DepthMeasurementInfo(size=(Wd, Hd), K=torch.from_numpy(K.copy())[None])
    wide.depth = depth_info
    up = PosedSensorInfo()
    up.image = wide.image.orient(cur, ImageOrientation.UPRIGHT)
    up.depth = wide.depth.orient(cur, ImageOrientation.UPRIGHT)
    up.RT = torch.eye(4)[None]
    up.T_gravity = torch.from_numpy(camera_to_gravity(pose, cur))[None]
    gt = PosedSensorInfo()
    gt.RT = torch.from_numpy(pose)[None]
    gt.depth = depth_info
    si = SensorArrayInfo()
    si.wide = up
    si.gt = gt
    return {"wide": {"image": rgb, "depth": dep},
            "meta": dict(video_id=video_id, timestamp=index), "sensor_info": si}


def upload_files(blobs, device="cuda"):
    """file bytes -> (device u8 [total] of the files back to back, device int64 offsets [F+1],
    host offsets): one pinned staging copy and one host-to-device transfer per batch"""
    offs = np.zeros(len(blobs) + 1, np.int64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    host = torch.empty(max(int(offs[-1]), 1), dtype=torch.uint8).pin_memory()
    hv = host.numpy()
    for b, o in zip(blobs, offs[:-1]):
        hv[o:o + len(b)] = np.frombuffer(b, np.uint8)
    dev = host.to(device, non_blocking=True)
    return dev, torch.from_numpy(offs).to(device, non_blocking=True), offs


def decode_depth_pngs(blobs, H, W, device="cuda"):
    """cv2.imread(p, IMREAD_UNCHANGED) (capture_stream.py:197/:405) for a batch of 16-bit depth
    PNG files (their bytes), decoded on the GPU (bf_png_decode_u16) -> u16 [F, H, W] on device;
    raises if any file does not decode"""
    from boxfusion_amd import _lib
    files, offs, offs_h = upload_files(blobs, device)
    out, _ = _lib.png_decode_u16(files, offs, H, W, offsets_host=offs_h)
    return out


def decode_color_jpegs(blobs, H, W, device="cuda"):
    """cv2.imread(color_path) + cvtColor(BGR2RGB) (capture_stream.py:194/:402) for a batch of
    baseline JPEG files (their bytes), decoded on the GPU (bf_jpeg_decode_rgb) -> u8 [F, H, W, 3]
    RGB on device; raises if any file does not decode"""
    from boxfusion_amd import _lib
    files, offs, _ = upload_files(blobs, device)
    out, _ = _lib.jpeg_decode_rgb(files, offs, H, W)
    return out


def jpeg_size(blob):
    """(W, H) from a JPEG's SOFn frame header (file bytes); ValueError if there is none"""
    if blob[:2] != b"\xff\xd8":
        raise ValueError("not a JPEG")
    i = 2
    while i + 4 <= len(blob):
        if blob[i] != 0xFF:
            raise ValueError("JPEG marker expected")
        m = blob[i + 1]
        if m == 0xFF:
            i += 1
            continue
        ln = int.from_bytes(blob[i + 2:i + 4], "big")
        if 0xC0 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            return int.from_bytes(blob[i + 7:i + 9], "big"), int.from_bytes(blob[i + 5:i + 7], "big")
        i += 2 + ln
    raise ValueError("JPEG without a frame header")


class DecodedFrameStream:
    """a ScanNet / CA-1M style frame directory as demo.py's dataset: colour JPEG / PNG and 16-bit
    depth PNG paths plus camera -> world poses.  Depth PNGs are decoded on the GPU
    (bf_png_decode_u16, `batch` files per launch) or on host threads; colour images on the host
    (PIL: cv2 is absent here) or, baseline JPEGs, on the GPU (bf_jpeg_decode_rgb).  Everything
    after decode runs in bf_ingest_rgbd on `device`."""

    def __init__(self, color_paths, depth_paths, poses, K, depth_scale, device="cuda", video_id=0, batch=16,
                 depth_decode="gpu", host_threads=16, color_decode="host"):
        """depth_decode "gpu": bf_png_decode_u16 on `batch` files per launch; "host": PIL on
        `host_threads` threads (the faster choice when a GPU's share of host cores decodes more
        files per second than the GPU path, DESIGN.md §4 "Depth PNG decode").  color_decode "gpu":
        bf_jpeg_decode_rgb on `batch` baseline JPEGs per launch (a file of another kind raises);
        "host": PIL, one file at a time"""
        if not (len(color_paths) == len(depth_paths) == len(poses)):
            raise ValueError("one colour image, depth map and pose per frame")
        if depth_decode not in ("gpu", "host"):
            raise ValueError("depth_decode: 'gpu' or 'host'")
        if color_decode not in ("gpu", "host"):
            raise ValueError("color_decode: 'gpu' or 'host'")
        self.color, self.depth, self.poses = list(color_paths), list(depth_paths), list(poses)
        self.K, self.scale, self.dev, self.video_id = np.asarray(K, np.float32), float(depth_scale), device, video_id
        self.batch = max(1, int(batch))
        self.depth_decode, self.host_threads = depth_decode, max(1, int(host_threads))
        self.color_decode = color_decode

    def __len__(self):
        return len(self.color)

    def _depth_size(self, path):
        with open(path, "rb") as fh:
            head = fh.read(24)
        if head[:8] != b"\x89PNG\r\n\x1a\n" or head[12:16] != b"IHDR":
            raise ValueError(f"{path}: not a PNG")
        return int.from_bytes(head[20:24], "big"), int.from_bytes(head[16:20], "big")

    def __iter__(self):
        from PIL import Image
        for b0 in range(0, len(self), self.batch):
            idx = range(b0, min(len(self), b0 + self.batch))
            H, W = self._depth_size(self.depth[b0])
            if self.depth_decode == "gpu":
                blobs = []
                for i in idx:
                    with open(self.depth[i], "rb") as fh:
                        blobs.append(fh.read())
                deps = decode_depth_pngs(blobs, H, W, self.dev)
            else:
                from concurrent.futures import ThreadPoolExecutor
                with ThreadPoolExecutor(self.host_threads) as ex:
                    arrs = list(ex.map(lambda i: np.asarray(Image.open(self.depth[i])).astype(np.uint16), idx))
                deps = torch.from_numpy(np.stack(arrs).view(np.int16)).to(self.dev).view(torch.uint16)
            cols = None
            if self.color_decode == "gpu":
                blobs = []
                for i in idx:
                    with open(self.color[i], "rb") as fh:
                        blobs.append(fh.read())
                Wc, Hc = jpeg_size(blobs[0])
                cols = decode_color_jpegs(blobs, Hc, Wc, self.dev)
            for j, i in enumerate(idx):
                if cols is not None:
                    rgb_t = cols[j]
                else:
                    rgb = np.array(Image.open(self.color[i]).convert("RGB"))     # (a writable copy)
                    rgb_t = torch.from_numpy(rgb).to(self.dev, non_blocking=True)
                yield make_sample_decoded(rgb_t, deps[j].view(torch.int16), self.scale, self.K, self.poses[i],
                                          video_id=self.video_id, index=i, src_bgr=False)


class SyntheticDataset:
    """the seeded synthetic RGB-D stream (boxfusion_amd.synthetic) as demo.py's dataset:
    iterable of samples, len() frames"""

    def __init__(self, n_frames=1000, H=480, W=640, K=None, depth_ratio=1, scene=None):
        from boxfusion_amd.synthetic import SCANNET_K, Scene
        self.n, self.H, self.W, self.r = n_frames, H, W, depth_ratio
        self.K = np.asarray(SCANNET_K if K is None else K, np.float32)
        self.scene = scene if scene is not None else Scene()

    def __len__(self):
        return self.n

    def frame(self, i):
        from boxfusion_amd.synthetic import frame_rgbd
        rgb, depth = frame_rgbd(i, self.H, self.W)
        if self.r > 1:
            depth = np.ascontiguousarray(depth[::self.r, ::self.r])
        return rgb, depth, self.scene.pose(i)

    def __iter__(self):
        for i in range(self.n):
            rgb, depth, pose = self.frame(i)
            yield make_sample(rgb, depth, self.K, pose, index=i)
