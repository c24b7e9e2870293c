#!/usr/bin/env python3
"""Throughput benchmark: RGB-D frames/s of per-frame detect + multi-view 3D box fusion.

Workload (BASELINE.json configs[2]): synthetic 640x480 RGB-D stream, batch 8 frames
per step per GPU, every frame a keyframe (gap=1, the per-frame-detect roofline run):
  per frame  depth standardisation + back-projection, CuTR RGB-D ViT-B (dim 768) forward,
             detection filters, CLIP ViT-H/14 on the 16 highest-scoring detections of the frame
             (16 crops/frame), text match against the 473-class vocabulary;
  per step   all-gather (RCCL) of every rank's per-frame records (detections + camera pose) and
             CLIP rows (features, best similarity, class) -> rank 0 runs the fusion state machine
             (NMS + association + box fusion) over all gathered frames in global frame order; the
             CLIP features ride on the detections through fusion (demo.py:167-171) and the
             similarity raises their scores by clip_sim_coeff*sim/100.
Weights are random (no checkpoint offline); the detections come from the seeded 30-object scene
generator (boxfusion_amd/synthetic.py), since random-weight CuTR boxes are noise.  With random
CLIP weights every crop would fall below class_sim_thres, so the "" category filter of
demo.py:171 is not applied (the match itself runs).
Inputs (frames, scene detections) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W]
With --gpus N > 1 and no torch.distributed environment the script starts
`python -m torch.distributed.run --nproc-per-node N` on itself as a child process (before anything
touches the GPU) and exits with its status; under torch.distributed.run each rank checks
WORLD_SIZE == N.  `--cpu-rehearsal` runs the same launch / sharding / all-gather / max-over-ranks
control flow on CPU with gloo and no kernels (a test harness, not a measurement).
"""
from __future__ import annotations

import argparse
import copy
import json
import gc
import os
import re
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md), no sparsity
PEAK_HBM_GBS = 8000.0
PEAK_FP8_TFLOPS = 5000.0    # dense fp8 (block-scaled MFMA) peak, no sparsity

CFG = dict(
    dataset="scannet",
    data=dict(gap=1),
    cam=dict(H=480, W=640, fx=574.540771, fy=577.583740, cx=322.522827, cy=238.558853),
    detection=dict(score_thresh=0.5, uv_bound=True, uv_bound_value=0.9, floor_mask=True,
                   floor_ratio=15, scale_box=1.5, class_sim_thres=25.0),
    association=dict(small_threshold=0.1, rotation_gap=30, translation_gap=0.8),
    box_fusion=dict(use=True, iters=20, pst_size=1024, check_valid=False, nms_threshold=0.1,
                    small_size=0.35, clip_sim_coeff=1.0,
                    random_opt=dict(center_init_size=0.1, center_scaling_coefficient=0.1,
                                    shape_init_size=0.5, shape_scaling_coefficient=0.5)),
)
# the stream's frame geometry (set by --dataset): image H x W, depth at 1/r, intrinsics K
CA1M_K = np.array([[360.0, 0.0, 191.5], [0.0, 360.0, 255.5], [0.0, 0.0, 1.0]], np.float32)
FRAME = dict(H=480, W=640, r=1, K=None)
REC_ROWS, REC_W = 64, 22     # per-frame detection record: rows x (score, xyxy, xyzlhw, R, proj_xy)
REC_HEAD = 17                # record head: detection count, camera pose (4x4)
CLIP_W = 1026                # per-crop CLIP row: feature[1024], best similarity, class index


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=125, help="timed steps (125 x 8 = 1000 frames)")
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--dim", type=int, default=768, help="CuTR ViT width (768 = ViT-B)")
    p.add_argument("--clip-layers", type=int, default=32)
    p.add_argument("--crops", type=int, default=16)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--breakdown", action="store_true",
                   help="synchronous fusion, sync between stages, report ms/step of each")
    p.add_argument("--eager", action="store_true", help="no HIP graph for the detect stage")
    p.add_argument("--roofline-steps", type=int, default=2)
    p.add_argument("--roofline-keyframes", type=int, default=24,
                   help="keyframes of the post-timing fusion re-run (pairs/s, particle-views/s)")
    p.add_argument("--fusion-cus", type=int, default=-1,
                   help="CUs reserved for the fusion stream (-1: 32 on rank 0 when N > 1, else 0)")
    p.add_argument("--sim-ranks", type=int, default=1,
                   help="stress test at N=1: rank 0 also fuses the frames of R virtual ranks per step")
    p.add_argument("--mask-cus", type=int, default=-1,
                   help="1: confine detection and fusion streams to disjoint CU sets (CU-masked "
                        "streams) when CUs are reserved for fusion; -1: on when fusing for N > 1")
    p.add_argument("--sync-fusion", action="store_true",
                   help="run the fusion state machine inline instead of on the worker stream")
    p.add_argument("--cpu-detect-frames", type=int, default=2,
                   help="frames of the CPU detect sample (0: no cpu_baseline, for A/B runs)")
    p.add_argument("--inflight", type=int, default=-1,
                   help="detect steps in flight per GPU: independent batches replayed on this many "
                        "streams (each its own DetectStage buffers / graph), so one batch's CLIP "
                        "phases overlap the next batch's CuTR phases (default 2; with 32 CUs "
                        "reserved for rank 0's fusion at N > 1 the two detect streams run on the "
                        "other 224)")
    p.add_argument("--cpu-fusion-frames", type=int, default=24)
    p.add_argument("--clip-fp8", action="store_true",
                   help="configs[4]: CLIP ViT-H qkv / fc1 / fc2 as fp8 e4m3 GEMMs (static per-tensor "
                        "scales calibrated on the first batch)")
    p.add_argument("--vocab", type=int, default=0,
                   help="text-match vocabulary rows (0 = the 473-class table; configs[4]: 200)")
    p.add_argument("--scene-objects", type=int, default=30,
                   help="objects in the seeded synthetic scene (150: global box sets past the "
                        "one-wave NMS scan's 96, so the 256-thread scan runs)")
    p.add_argument("--gap", type=int, default=1,
                   help="keyframe gap (demo.py:134 `count %% gap == 0`): every step covers batch*gap "
                        "frames per GPU; the non-keyframes get demo.py's per-frame preprocessing "
                        "(depth standardisation), the keyframes detect + CLIP + fusion.  Default "
                        "steps at gap > 1: the 1000-frame stream")
    p.add_argument("--rank0-batch", type=int, default=-1,
                   help="frames rank 0 detects per step when it also fuses other ranks' frames (N > 1 or "
                        "--sim-ranks): the fusion owner's share of detection is lowered so its serial "
                        "fusion keeps pace; the other ranks detect --batch; -1: auto")
    p.add_argument("--switch-interval", type=float, default=-1.0,
                   help="Python thread switch interval in ms for the host threads (detect launcher vs "
                        "the fusion worker); <0: the interpreter default")
    p.add_argument("--dataset", choices=("scannet", "ca1m"), default="scannet",
                   help="ca1m: BASELINE configs[1]'s stream as CA1MDataset delivers it -- 384x512 portrait "
                        "frames with the depth resized to the image (RGB:depth ratio 1, "
                        "capture_stream.py:445-459), ca1m.yaml thresholds and gap 20")
    p.add_argument("--depth-ratio", type=int, default=1, choices=(1, 2, 4),
                   help="RGB:depth resolution ratio of the stream (--dataset ca1m: 2 / 4 = a lower-"
                        "resolution depth sensor through the CuTR depth grid; not what CA1MDataset streams)")
    p.add_argument("--png-depth", action="store_true",
                   help="every frame's depth arrives as a 16-bit PNG file (bytes resident in HBM) and is "
                        "decoded on the GPU inside the timed region (bf_png_decode_depth: cv2.imread "
                        "IMREAD_UNCHANGED + astype(f32) / depth_scale, capture_stream.py:197-203); the "
                        "line gains a `decode` object: the GPU PNG and colour-JPEG decode rates with the "
                        "host PIL rates beside them")
    p.add_argument("--decode", action="store_true",
                   help="--png-depth, and every keyframe's colour image arrives as a 1296x968 baseline JPEG "
                        "decoded on the GPU ahead of its detect (bf_jpeg_decode_rgb + cv2.resize, "
                        "capture_stream.py:194-199)")
    p.add_argument("--jpeg-ahead", type=int, default=6,
                   help="--decode: steps per colour-JPEG decode launch (one group, decoded a group ahead of its detects) "
                        "")
    p.add_argument("--cpu-rehearsal", action="store_true",
                   help="CPU/gloo rehearsal of the N-rank control flow (no kernels; test harness)")
    a = p.parse_args(argv)
    a.png_depth = a.png_depth or a.decode
    return a


def launch_ranks(argv, n):
    """--gpus N > 1 without a torch.distributed environment: run this script under
    torch.distributed.run as a child process (one rank per GPU, rendezvous on 127.0.0.1) and
    return its exit status.  Nothing here touches the GPU (no exec from a GPU-initialised
    process)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=env).returncode


# ------------------------------------------------------------------------------------------------
def gen_frames(frame_ids, dev):
    """seeded synthetic RGB-D frames generated on the device (seed 1234 + frame)."""
    n = len(frame_ids)
    H, W, r = FRAME["H"], FRAME["W"], FRAME["r"]
    rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device=dev)
    depth = torch.empty((n, H // r, W // r), dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for j, f in enumerate(frame_ids):
        g.manual_seed(1234 + int(f))
        rgb[j].random_(0, 256, generator=g)
        depth[j].uniform_(0.5, 4.5, generator=g)
        depth[j].masked_fill_(torch.rand(depth.shape[1:], device=dev, generator=g) < 0.05, 0.0)
    return rgb, depth


def sorted_dets(d):
    """a frame's detections in descending score order, the order CuTR emits them
    (cubify_transformer.py:945-978: top-k over the sigmoid scores)"""
    o = np.argsort(-d["scores"], kind="stable")
    return {k: v[o] for k, v in d.items()}


def pack_records(dets, poses):
    """scene detections + camera poses of a batch of frames -> f32 [b, REC_HEAD + REC_ROWS*REC_W]
    records: (count, pose 4x4, rows in descending score order).  The pose and count travel with
    the detections, so the exchange is one device all-gather (no host-object collective, which
    would synchronise the detect stream every step)."""
    out = np.zeros((len(dets), REC_HEAD + REC_ROWS * REC_W), np.float32)
    for j, d in enumerate(dets):
        d = sorted_dets(d)
        n = min(len(d["scores"]), REC_ROWS)
        rows = np.concatenate([d["scores"][:n, None], d["pred_boxes"][:n], d["xyzlhw"][:n],
                               d["R"][:n].reshape(n, 9), d["proj_xy"][:n]], 1)
        out[j, 0] = n
        out[j, 1:REC_HEAD] = np.asarray(poses[j], np.float32).reshape(-1)
        out[j, REC_HEAD:REC_HEAD + n * REC_W] = rows.reshape(-1)
    return out


def crop_boxes(dets, crops):
    """f32 [b*crops, 4]: the 2-D boxes of each frame's `crops` highest-scoring detections (the
    CLIP inputs; a frame with fewer repeats its last box, an empty frame gets zero-size boxes)"""
    out = np.zeros((len(dets), crops, 4), np.float32)
    for j, d in enumerate(dets):
        b = sorted_dets(d)["pred_boxes"][:crops]
        if len(b):
            out[j, :len(b)] = b
            out[j, len(b):] = b[-1]
    return out.reshape(-1, 4)


def clip_rows(feats, sims, cat_idx):
    """per-crop CLIP rows [n, CLIP_W] = feature, best similarity (x100 scale), class index"""
    return torch.cat([feats, sims[:, None].to(feats.dtype), cat_idx[:, None].to(feats.dtype)], 1)


def record_meta(recs):
    """(poses [k,4,4], counts [k]) on the host from gathered records (one device read)"""
    h = recs[:, :REC_HEAD].cpu().numpy() if hasattr(recs, "cpu") else np.asarray(recs)[:, :REC_HEAD]
    return h[:, 1:REC_HEAD].reshape(-1, 4, 4).copy(), h[:, 0].astype(np.int64)


def unpack_record(rec, dev, n=None):
    """record -> Instances3D; `n` (detections in the record) from the host when known, so the
    fusion worker does not read the device to learn it"""
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    from boxfusion_amd.instances import Instances3D
    if n is None:
        n = int(rec[0].item())
    rows = rec[REC_HEAD:REC_HEAD + n * REC_W].view(n, REC_W)
    p = Instances3D((FRAME["H"], FRAME["W"]))
    p.scores = rows[:, 0].contiguous()
    p.pred_boxes = rows[:, 1:5].contiguous()
    p.pred_boxes_3d = GeneralInstance3DBoxes(rows[:, 5:11], rows[:, 11:20].reshape(n, 3, 3))
    p.pred_proj_xy = rows[:, 20:22].contiguous()
    return p


def record_rows(cnts, crops):
    """host index maps of a step's keyframes: detection row j*REC_ROWS + r, and its CLIP row
    j*crops + r (r < crops) or the zero row (len(cnts)*crops) for detections without a crop"""
    cnts = np.asarray(cnts, np.int64)
    if not cnts.sum():
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    idx = np.concatenate([j * REC_ROWS + np.arange(c) for j, c in enumerate(cnts)])
    zero = len(cnts) * crops
    cidx = np.concatenate([np.where(np.arange(c) < crops, j * crops + np.arange(c), zero)
                           for j, c in enumerate(cnts)])
    return idx, cidx


def unpack_records(recs, cnts, dev, clip=None, crops=16, clip_coeff=1.0):
    """records [nkf, REC_HEAD + REC_ROWS*REC_W] of several keyframes -> ONE Instances3D holding every
    keyframe's detections in order (keyframe j: cnts[j] rows).  clip [nkf*crops, CLIP_W]: the
    CLIP rows of the keyframes' crops; detection r < crops of keyframe j gets feature row
    j*crops + r and score += clip_coeff * sim / 100 (demo.py:167-170), the others zeros."""
    from boxfusion_amd import _lib
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    from boxfusion_amd.instances import Instances3D
    idx, cidx = record_rows(cnts, crops)
    rows = recs[:, REC_HEAD:REC_HEAD + REC_ROWS * REC_W].reshape(-1, REC_W).index_select(
        0, _lib.h2d(idx, dev))
    p = Instances3D((FRAME["H"], FRAME["W"]))
    p.scores = rows[:, 0].contiguous()
    p.pred_boxes = rows[:, 1:5].contiguous()
    p.pred_boxes_3d = GeneralInstance3DBoxes._views(rows[:, 5:11].contiguous(),
                                                     rows[:, 11:20].reshape(-1, 3, 3).contiguous())
    p.pred_proj_xy = rows[:, 20:22].contiguous()
    if clip is not None:
        cz = torch.cat([clip, clip.new_zeros((1, clip.shape[1]))])
        crow = cz.index_select(0, _lib.h2d(cidx, dev))
        p.features = crow[:, :1024].contiguous()
        p.scores = p.scores + clip_coeff * crow[:, 1024] / 100.0
    return p


def gather_step(recs, clip, dist, world, force=False):
    """Exchange of one step: every rank's per-frame records [b, R] (detections, count and camera
    pose) and CLIP rows [b*crops, CLIP_W] are all-gathered with all_gather_into_tensor (RCCL over
    xGMI on the GPU; gloo on CPU tensors in the rehearsal and the tests: the same call sequence)
    so that the fusion owner sees the step's frames in global frame order (rank-major = frame
    order, since rank r holds frames step*b*world + r*b ... + b-1).  On the GPU both collectives
    are asynchronous device operations: nothing here waits for the detect stream.  force: run
    the collectives at world 1 too (the one-GPU RCCL test)."""
    if dist is None or (world == 1 and not force):
        return recs, clip
    if recs.is_cuda and dist.get_backend() == "gloo":     # BF_BENCH_REHEARSE=1 (one-GPU rehearsal)
        g_rec, g_clip = gather_step(recs.cpu(), clip.cpu(), dist, world)
        return g_rec.to(recs.device), g_clip.to(clip.device)
    g_rec = recs.new_empty((world * recs.shape[0],) + tuple(recs.shape[1:]))
    dist.all_gather_into_tensor(g_rec, recs.contiguous())
    g_clip = clip.new_empty((world * clip.shape[0],) + tuple(clip.shape[1:]))
    dist.all_gather_into_tensor(g_clip, clip.contiguous())
    return g_rec, g_clip


def rank_frames(step, rank, B, B0, per_step, G=1):
    """frame ids a rank detects in a step: rank 0 the step's first B0 frames, rank r >= 1 the B
    frames after B0 + (r - 1) B (per_step = B0 + (N - 1) B); gap G: every G-th frame"""
    first = step * per_step + (0 if rank == 0 else B0 + (rank - 1) * B)
    return [(first + j) * G for j in range(B0 if rank == 0 else B)]


def exchange_step(recs, clip, dist, N, B, B0, crops, rank):
    """gather_step with rank 0's smaller share: its chunk is padded to B frames (all_gather needs
    equal chunks) and the padding is dropped from the gathered tensors on rank 0, so the fusion
    owner sees the step's frames in global order"""
    if N > 1 and recs.shape[0] < B:
        pad = B - recs.shape[0]
        recs = torch.cat([recs, recs.new_zeros((pad,) + tuple(recs.shape[1:]))])
        clip = torch.cat([clip, clip.new_zeros((pad * crops,) + tuple(clip.shape[1:]))])
    g_rec, g_clip = gather_step(recs, clip, dist, N)
    if N > 1 and B0 < B and rank == 0:
        g_rec = torch.cat([g_rec[:B0], g_rec[B:]])
        g_clip = torch.cat([g_clip[:B0 * crops], g_clip[B * crops:]])
    return g_rec, g_clip


# ------------------------------------------------------------------------------------------------
def cpu_baseline(cutr, clip_vis, args, scene):
    """The parity-checked CPU restatement timed on this host on the bench's own frame geometry
    (FRAME: 640x480 ScanNet, or the CA-1M 384x512 portrait stream at its RGB:depth ratio) and CFG:
      per frame  depth standardisation + back-projection (oracle C), RGB normalise + pad
      keyframe   fp32 torch-CPU CuTR + CLIP on `crops` scene-detection crops (cpu_detect_frames
                 frames timed) + the oracle fusion chain (oracle/chain.py)
    Rates: every frame a keyframe (gap 1) and the stream's keyframe rule (gap 25 for ScanNet,
    ca1m.yaml's 20 for CA-1M; fusion chain timed on keyframes 0, g, 2g, ...); `value` is the rate
    at the bench's own --gap."""
    from oracle.chain import OracleChain
    from boxfusion_amd.box_fusion import load_pst
    from boxfusion_amd.cubify_transformer import FrameBatch
    from boxfusion_amd.preprocessor import PIXEL_MEAN, PIXEL_STD, square_pad_size
    from boxfusion_amd.sensor import camera_to_gravity
    from boxfusion_amd.synthetic import SCANNET_K, frame_rgbd
    from boxfusion_amd.clip import CLIP_MEAN, CLIP_STD
    from oracle import oracle as OR
    import torch.nn.functional as F
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    H, W, r = FRAME["H"], FRAME["W"], FRAME["r"]
    K = SCANNET_K if FRAME["K"] is None else FRAME["K"]
    Kd = K.copy()
    Kd[:2] /= r
    pad = square_pad_size(H, W)
    cm = copy.deepcopy(cutr).float().cpu().eval()
    vm = copy.deepcopy(clip_vis).float().cpu().eval()
    nf = args.cpu_detect_frames
    sb = CFG["detection"]["scale_box"]
    t_pre = t_model = 0.0
    with torch.no_grad():
        for f in range(nf):
            rgb, depth = frame_rgbd(f, H, W)
            depth = np.ascontiguousarray(depth[::r, ::r])
            t0 = time.perf_counter()
            mean = torch.tensor(PIXEL_MEAN).view(3, 1, 1)
            std = torch.tensor(PIXEL_STD).view(3, 1, 1)
            img = (torch.from_numpy(np.moveaxis(rgb, -1, 0)).float() - mean) / std
            img = F.pad(img, (0, pad - W, 0, pad - H))[None]
            d, params = OR.depth_standardize(depth)
            OR.backproject(depth, Kd, scene.pose(f))
            d = F.pad(torch.from_numpy(d), (0, pad // r - d.shape[1], 0, pad // r - d.shape[0]))[None]
            t1 = time.perf_counter()
            batch = FrameBatch(image=img, depth=d, depth_params=torch.from_numpy(params)[None],
                               K=torch.from_numpy(K)[None],
                               T_gravity=torch.from_numpy(camera_to_gravity(scene.pose(f)))[None],
                               image_sizes=[(H, W)])
            cm(batch)
            crops = []
            for x1, y1, x2, y2 in crop_boxes([scene.detections(f, K, (W, H))], args.crops):
                cx, cy, w, h = (x1 + x2) / 2, (y1 + y2) / 2, (x2 - x1) * sb, (y2 - y1) * sb
                x1, x2 = int(np.clip(cx - w / 2, 0, W)), int(np.clip(cx + w / 2, 0, W))
                y1, y2 = int(np.clip(cy - h / 2, 0, H)), int(np.clip(cy + h / 2, 0, H))
                c = torch.from_numpy(rgb[y1:y2, x1:x2]).permute(2, 0, 1).float()[None]
                c = F.interpolate(c, (224, 224), mode="bilinear", align_corners=False) if c.numel() \
                    else torch.zeros((1, 3, 224, 224))
                crops.append(c)
            x = torch.cat(crops) / 255.0
            x = (x - torch.tensor(CLIP_MEAN).view(1, 3, 1, 1)) / torch.tensor(CLIP_STD).view(1, 3, 1, 1)
            vm(x)
            t_pre += t1 - t0
            t_model += time.perf_counter() - t1
    t_pre, t_model = t_pre / nf, t_model / nf
    g_ref = 20 if CFG["dataset"] == "CA1M" else 25
    fuse = {}
    for gap in sorted({1, g_ref, max(1, args.gap)}):
        ch = OracleChain(CFG, K, H=H, W=W, pst=load_pst(), legacy=True)
        t0 = time.perf_counter()
        for k in range(args.cpu_fusion_frames):
            f = k * gap
            ch.keyframe(f, scene.pose(f), scene.detections(f, K, (W, H)))
        fuse[gap] = (time.perf_counter() - t0) / args.cpu_fusion_frames
    rate = lambda g: g / (g * t_pre + t_model + fuse[g])
    out = {"value": rate(max(1, args.gap)), "unit": "frames/s", "cores": cores, "kind": "port",
           "gap": max(1, args.gap), "gap1_value": rate(1), f"gap{g_ref}_value": rate(g_ref),
           "sample": (f"{nf} frame(s) of fp32 torch-CPU CuTR ViT-{ {768: 'B', 384: 'S', 192: 'T'}.get(args.dim, args.dim)} "
                      f"on {W}x{H} RGB (depth 1/{r}) + {args.crops} CLIP ViT-H/14 crops ({t_model:.2f} "
                      f"s/keyframe), per-frame depth standardisation + back-projection + normalise "
                      f"({1e3 * t_pre:.1f} ms/frame), oracle fusion chain over {args.cpu_fusion_frames} "
                      f"keyframes ({', '.join(f'{1e3 * v:.1f} ms/keyframe at gap {g}' for g, v in fuse.items())}); "
                      f"value = the bench's gap {max(1, args.gap)} (keyframe every gap-th frame)")}
    return out


# PMC record keys of the bench line's roofline objects: group names of scripts/profile_round.sh,
# or "sum:<regex>" over the kernel names of one multi-launch call (every one must match a kernel
# of the newest committed profiles/r*_pmc.json: tests/test_bench_pmc.py)
PMC_KEYS = {
    "gemm": "k_gemm256p",
    "resid_gemm": "k_gemm256p<false, 0>",
    "gelu_gemm": "k_gemm256p<true, 1>",
    "fp8_gemm": "k_gemm256p_fp8",
    "attention": "k_attn",
    "attention_clip": "k_attn_clip",
    "attention_cutr": "k_attn_cutr",
    # bf_depth_preprocess at a keyframe batch: the three histogram passes + the normalise pass
    "depth_small": r"sum:k_ds_(hist[123]<\d+, true>|norm<\d+>)",
}


def load_pmc_traffic(kernel):
    """HBM-side bytes per launch of `kernel` from the committed PMC passes (profiles/*_pmc.json,
    newest round); counters cannot be read from inside the run."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    for fn in reversed(files):      # newest round first; a key may live in a workload's own file
        with open(fn) as f:
            full = json.load(f)
        if kernel.startswith("sum:"):
            # a multi-launch call: the per-launch bytes of every kernel name matching the regex,
            # summed (each runs once per call)
            sel = [v for n, v in full.get("kernels", {}).items()
                   if re.search(kernel[4:], n) and "bytes_per_launch" in v]
            d = ({"bytes_per_launch": sum(v["bytes_per_launch"] for v in sel), "kernels": len(sel)}
                 if sel else None)
        else:
            d = full.get(kernel)
        if d:
            d = dict(d)
            d["source"] = (os.path.relpath(fn, ROOT) + " (2 x FETCH_SIZE + WRITE_SIZE per launch, "
                           "separate --pmc passes)")
            return d
    return {}


def roofline_obj(ks, kernel, bound, pmc_key=None, peak_tflops=PEAK_BF16_TFLOPS):
    """roofline object of a KernelTimer summary: achieved = algorithmic FLOPs (or bytes) per launch
    / average launch time (HIP events on the launch stream)"""
    pmc = load_pmc_traffic(pmc_key or kernel) if ks["launches"] else {}
    if bound == "hbm":
        achieved, peak, unit = ks.get("gbs", 0.0), PEAK_HBM_GBS, "GB/s"
    else:
        achieved, peak, unit = ks.get("tflops", 0.0), peak_tflops, "TFLOP/s"
    return {"bound": bound, "kernel": kernel, "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak, "traffic": pmc.get("bytes_per_launch"),
            "traffic_source": pmc.get("source"), "launches": ks["launches"],
            "avg_us": ks.get("avg_us", 0.0), "flops_per_launch": ks.get("flops_per_launch", 0.0),
            "algorithmic_bytes_per_launch": ks.get("bytes_per_launch", 0.0)}


def auto_rank0_batch(B, ranks):
    """rank 0's detection share when it also fuses `ranks` ranks' frames.  Measured on one MI355X
    with --sim-ranks 8, all arms on one box (scripts/sim8_ab.sh, profiles/r05_bench_sim8.json,
    DESIGN.md §8): N = 1 step 54.7 ms; rank 0 with its 32 reserved CUs on 7 frames 51.3 ms (the
    other ranks set the step: 63/64 = 0.984 of the ideal, worker busy 16.2 ms per step); without
    the reservation on 8 frames 56.0 ms (0.977, worker 36.7 ms); reservation + 8 frames 57.2 ms
    (0.956).  7 frames with the reservation is kept: it is the fastest arm, and the reserved CUs
    keep the worker's own time small where scenes are heavier (150 objects: ~33 ms of fusion
    kernels per 64 keyframes on an idle chip), which it would otherwise spend queued behind the
    persistent GEMMs that hold every CU."""
    if ranks >= 8:
        return max(1, B - 1)
    return B


def png_pool(n, H, W, level=6):
    """n distinct 16-bit depth PNGs (mm) of the synthetic scene's frames as PIL writes them
    (adaptive row filters, zlib level 6), the kind of file a ScanNet / CA-1M depth directory holds"""
    import io
    from PIL import Image
    from boxfusion_amd.synthetic import frame_rgbd
    out = []
    for f in range(n):
        d = np.clip(frame_rgbd(f * 5, H, W)[1] * 1000.0, 0, 65535).astype(np.uint16)
        b = io.BytesIO()
        Image.fromarray(d).save(b, format="PNG", compress_level=level)
        out.append(b.getvalue())
    return out


def host_png_rate(pool, threads, seconds=3.0):
    """PIL decode of the pool on `threads` host threads for ~`seconds` (frames/s): the host decode
    wall a CPU loader would hit (PIL releases the GIL inside the zlib / unfilter code)"""
    import io
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image

    def dec(b):
        return np.asarray(Image.open(io.BytesIO(b)))
    rep = pool * max(1, -(-4 * threads // len(pool)))
    n = 0
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(dec, pool))
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            list(ex.map(dec, rep))
            n += len(rep)
        return n / (time.perf_counter() - t0)


def keyframe_jpeg():
    """a ScanNet-sized colour JPEG (1296 x 968, quality 90, 4:2:0: the synthetic scene frame upsampled)"""
    import io
    from PIL import Image
    from boxfusion_amd.synthetic import frame_rgbd
    img = Image.fromarray(frame_rgbd(3, 480, 640)[0]).resize((1296, 968), Image.BILINEAR)
    b = io.BytesIO()
    img.save(b, format="JPEG", quality=90)
    return b.getvalue()


def jpeg_pool(n, H=968, W=1296, quality=90):
    """n distinct colour JPEGs of the synthetic scene's frames upsampled to ScanNet's colour size
    (PIL, quality 90, 4:2:0): the kind of file a ScanNet colour directory holds"""
    import io
    from PIL import Image
    from boxfusion_amd.synthetic import frame_rgbd
    out = []
    for f in range(n):
        img = Image.fromarray(frame_rgbd(f * 5, 480, 640)[0]).resize((W, H), Image.BILINEAR)
        b = io.BytesIO()
        img.save(b, format="JPEG", quality=quality)
        out.append(b.getvalue())
    return out


def gpu_jpeg_rate(n=1024, reps=3):
    """bf_jpeg_decode_rgb over n copies of the keyframe JPEG resident in HBM (one wave per file: n =
    1024 puts one on every SIMD), frames/s from HIP events (min of reps), and the batch size"""
    from boxfusion_amd import _lib
    from boxfusion_amd.capture_stream import upload_files
    blob = keyframe_jpeg()
    files, offs, _ = upload_files([blob] * n, "cuda")
    out = torch.empty((n, 968, 1296, 3), dtype=torch.uint8, device="cuda")
    work = torch.empty(_lib.jpeg_workspace_bytes(n, 968, 1296), dtype=torch.uint8, device="cuda")
    _lib.jpeg_decode_rgb(files, offs, 968, 1296, out=out, work=work)
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.jpeg_decode_rgb(files, offs, 968, 1296, out=out, work=work, check=False)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del out, work, files
    return n / (best * 1e-3), n


def host_jpeg_rate(threads, seconds=2.0):
    """PIL decode of the keyframe JPEG on `threads` host threads (frames/s) -- the colour half of
    cv2.imread (capture_stream.py:194): only keyframes need their colour image"""
    from concurrent.futures import ThreadPoolExecutor
    from PIL import Image
    import io
    blob = keyframe_jpeg()

    def dec(_):
        return np.asarray(Image.open(io.BytesIO(blob)).convert("RGB"))
    n = 0
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(dec, range(threads)))
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            list(ex.map(dec, range(4 * threads)))
            n += 4 * threads
        return n / (time.perf_counter() - t0), len(blob)


def emit(line):
    print(json.dumps(line), flush=True)


def base_line(args, N, frames, dt, per_step, n_inflight):
    if getattr(args, "clip_fp8", False):
        line = base_line_bf16(args, N, frames, dt, per_step, n_inflight)
        line["dtype"] = "bf16 + fp8 e4m3 (CLIP ViT-H qkv / fc1 / fc2)"
        line["config"]["workload"] = (
            f"configs[4]: synthetic 640x480 RGB-D (ScanNetV2 scene0000_00 absent offline), batch "
            f"{args.batch}/step/GPU, gap=1, CuTR ViT-B RGB-D bf16 + CLIP ViT-H/14 fp8 x{args.crops} "
            f"crops/frame + {args.vocab or 473}-class text match + fusion")
        return line
    return base_line_bf16(args, N, frames, dt, per_step, n_inflight)


def base_line_bf16(args, N, frames, dt, per_step, n_inflight):
    return {
        "metric": "RGB-D frames/sec (whole node) on 640x480 stream",
        "value": frames / dt, "unit": "frames/s", "n_gpus": N, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic 640x480 RGB-D stream (seeded), random-init weights, seeded scene detections",
        "config": {"workload": f"configs[2]: synthetic 640x480 RGB-D, batch {args.batch}/step/GPU, gap=1, "
                               f"CuTR ViT-{ {768: 'B', 384: 'S', 192: 'T'}.get(args.dim, args.dim)} "
                               f"RGB-D + CLIP ViT-H/14 x{args.crops} crops/frame + fusion",
                   "frames": frames, "global_batch": per_step, "parallelism": f"dp{N}",
                   "inflight_batches_per_gpu": n_inflight},
    }


# ------------------------------------------------------------------------------------------------
def rehearse_cpu(args, dist, world, rank):
    """--cpu-rehearsal: the N-rank control flow of main() on CPU tensors with gloo and no
    kernels -- frame sharding, per-step records and CLIP rows, gather_step's all_gather_into_tensor
    sequence, the fusion owner's global frame order check, barrier + max-over-ranks timing and
    rank 0's JSON line.  CLIP rows are rank/frame-coded stand-ins (no CLIP runs)."""
    from boxfusion_amd.synthetic import Scene
    scene = Scene(seed=0, n_objects=args.scene_objects)
    B, N = args.batch, world
    B0 = min(B, args.rank0_batch if args.rank0_batch > 0 else auto_rank0_batch(B, N)) if N > 1 else B
    Bm = B0 if rank == 0 else B
    per_step = B * N - (B - B0)
    total = args.warmup + args.steps

    def my_frames(step):
        return rank_frames(step, rank, B, B0, per_step)

    mine = [f for s_ in range(total) for f in my_frames(s_)]
    dets = [scene.detections(f) for f in mine]
    rec_all = torch.from_numpy(pack_records(dets, [scene.pose(f) for f in mine]))
    ok = True
    fused_frames = 0
    t0 = None
    for s_ in range(total):
        if s_ == args.warmup:            # barrier, then time exactly the --steps steps
            if dist is not None:
                dist.barrier()
            t0 = time.perf_counter()
        sl = slice(s_ * Bm, s_ * Bm + Bm)
        fr = torch.tensor(mine[sl], dtype=torch.float32)
        clip = fr.repeat_interleave(args.crops)[:, None].expand(-1, CLIP_W).contiguous()
        g_rec, g_clip = exchange_step(rec_all[sl], clip, dist, N, B, B0, args.crops, rank)
        if rank == 0:
            want = [s_ * per_step + j for j in range(per_step)]
            g_pose, g_cnt = record_meta(g_rec)
            ok &= bool(np.array_equal(g_pose, np.stack([scene.pose(f) for f in want]).astype(np.float32)))
            ok &= bool(np.array_equal(g_cnt, [min(len(scene.detections(f)["scores"]), REC_ROWS) for f in want]))
            ok &= bool(torch.equal(g_clip[:, 0], torch.tensor(want, dtype=torch.float32).repeat_interleave(args.crops)))
            idx, cidx = record_rows(g_cnt, args.crops)
            ok &= len(idx) == int(g_cnt.sum()) and int(cidx.max(initial=0)) <= per_step * args.crops
            fused_frames += len(want)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank == 0:
        line = base_line(args, N, per_step * args.steps, dt, per_step, 1)
        if B0 < B:
            line["config"]["rank0_batch"] = B0
        line.update(data="cpu rehearsal of the N-rank control flow (no kernels; not a measurement)",
                    rehearsal={"frame_order_ok": bool(ok), "frames_received": fused_frames})
        emit(line)


# ------------------------------------------------------------------------------------------------
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.dataset == "ca1m":
        # ca1m.yaml (config/ca1m.yaml): cam 384 x 512 (portrait after BoxFusion's H/W swap), gap 20,
        # score 0.4, small_threshold 0.2, small_size 0.5; CA1MDataset resizes the depth to the image
        # (ratio 1); the synthetic CA-1M frame geometry of the CuTR goldens
        FRAME.update(H=512, W=384, r=args.depth_ratio, K=CA1M_K)
        CFG.update(dataset="CA1M", cam=dict(H=384, W=512, png_depth_scale=1000.0))
        CFG["detection"].update(score_thresh=0.4)
        CFG["association"].update(small_threshold=0.2)
        CFG["box_fusion"].update(small_size=0.5)
        if "--gap" not in " ".join(argv):
            args.gap = 20
    if args.gap > 1 and "--steps" not in " ".join(argv):
        args.steps = max(1, -(-1000 // (args.batch * args.gap * args.gpus)))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(argv, args.gpus)
    if args.breakdown:
        args.sync_fusion = True
    if args.switch_interval > 0:
        sys.setswitchinterval(args.switch_interval * 1e-3)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    if args.cpu_rehearsal:
        dist = None
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        rehearse_cpu(args, dist, world, rank)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return 0
    # BF_BENCH_REHEARSE=1: every rank on cuda:0 with gloo collectives -- a one-GPU rehearsal of the
    # N>1 control flow (sharding, exchange, rank-0 fusion, max-over-ranks timing); not a measurement
    rehearse = os.environ.get("BF_BENCH_REHEARSE", "0") == "1"
    if rehearse:
        local = 0
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from boxfusion_amd import _lib
    _lib.lib()                                         # fail loudly without the HIP library
    from boxfusion_amd.clip import VisionTransformer
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.fusion_stage import AsyncFusion, FusionStage
    from boxfusion_amd.pipeline import DetectStage
    from boxfusion_amd.synthetic import SCANNET_K, Scene

    torch.manual_seed(0)
    with torch.device(dev):
        cutr = make_cubify_transformer(args.dim, True).eval()
        clip_vis = VisionTransformer(224, 14, 1280, args.clip_layers, 16, 1024).eval()
    B = args.batch
    R_fuse = world if world > 1 else max(1, args.sim_ranks)      # ranks whose frames rank 0 fuses
    B0 = args.rank0_batch if args.rank0_batch > 0 else auto_rank0_batch(B, R_fuse)
    B0 = min(B, B0) if R_fuse > 1 else B
    Bm = B0 if rank == 0 else B                                  # this rank's frames per step
    n_inflight = args.inflight if args.inflight > 0 else 2
    from boxfusion_amd.pipeline import load_class_features, load_class_names
    text, names = load_class_features(), load_class_names()
    if args.vocab:
        # configs[4]'s 200-class vocabulary: the ScanNet200 names / CLIP text features are not in
        # the reference; the first `vocab` rows of its 473-class table stand in (same match kernel
        # path, vocabulary-sized)
        text, names = text[:args.vocab].clone(), names[:args.vocab]
    Kf = SCANNET_K if FRAME["K"] is None else FRAME["K"]
    FH, FW = FRAME["H"], FRAME["W"]
    detects = [DetectStage(cutr, clip_vis, CFG, Bm, FH, FW, Kf, text_features=text.clone(),
                           class_names=names, crops_per_frame=args.crops,
                           crop_source="given", backproject=True, clip_capacity=Bm * args.crops,
                           device=dev, graph=not args.eager, clip_fp8=args.clip_fp8,
                           depth_ratio=FRAME["r"])
               for _ in range(n_inflight)]
    detect = detects[0]
    scene = Scene(seed=0, n_objects=args.scene_objects)
    N = world
    per_step = B * N - (B - B0)          # frames per step (all ranks; rank 0 detects B0)
    total_steps = args.warmup + args.steps
    coeff = CFG["box_fusion"]["clip_sim_coeff"]

    G = max(1, args.gap)
    CFG["data"]["gap"] = G

    def my_frames(step):
        """this rank's keyframes of a step (frame ids; gap G: every G-th frame of the stream)"""
        return rank_frames(step, rank, B, B0, per_step, G)

    # ---- inputs resident in HBM before timing -----------------------------------------------
    all_mine = [f for s in range(total_steps) for f in my_frames(s)]
    rgb_all, depth_all = gen_frames(all_mine, dev)
    nk_depth = None
    if G > 1:
        # the rank's non-keyframes of every step: depth maps only (demo.py:129-131 standardises
        # every frame's depth; nothing else runs on a non-keyframe)
        gnk = torch.Generator(device=dev)
        gnk.manual_seed(4321 + rank)
        nk_depth = torch.empty((total_steps, (G - 1) * Bm, FH // FRAME["r"], FW // FRAME["r"]),
                               dtype=torch.float32, device=dev)
        nk_depth.uniform_(0.5, 4.5, generator=gnk)
        nk_depth.masked_fill_(torch.rand(nk_depth.shape, device=dev, generator=gnk) < 0.05, 0.0)
        # their camera poses and the depth intrinsics: demo.py:121-127 back-projects every
        # frame's depth too (viz_on_gt_points defaults to True)
        nk_ids = [[kf + o for kf in my_frames(s_) for o in range(1, G)] for s_ in range(total_steps)]
        nk_RT = torch.from_numpy(np.stack([np.stack([scene.pose(f) for f in ids]) for ids in nk_ids])
                                 .astype(np.float32)).to(dev)
        nk_K = detect.Kd_dev[:1].expand((G - 1) * Bm, 3, 3).contiguous()
        # one workspace per in-flight detect stream (the steps on two streams overlap)
        nk_ws = [_lib.new_depth_workspace((G - 1) * Bm, FH // FRAME["r"], FW // FRAME["r"], dev)
                 for _ in range(n_inflight)]
    png_in = None
    if args.png_depth:
        # every frame's depth file of every step (keyframes first, then the non-keyframes in
        # stream order), bytes resident in HBM before timing; decoded per step in the timed region
        from boxfusion_amd.capture_stream import upload_files
        Hd_, Wd_ = FH // FRAME["r"], FW // FRAME["r"]
        pool = png_pool(16, Hd_, Wd_)
        png_in = {"pool": pool, "steps": {}, "H": Hd_, "W": Wd_}

        def step_ids(s_):
            kf = my_frames(s_)
            return list(kf) + [f + o for f in kf for o in range(1, G)]
        # --decode: the files go in groups of D steps, decoded a group ahead (below); one step's
        # files stay for the decode-alone measurement
        for s_ in ([args.warmup] if args.decode else range(total_steps)):
            png_in["steps"][s_] = upload_files([pool[f % len(pool)] for f in step_ids(s_)], dev)
        nfile = G * Bm
        tot = max(int(o[2][-1]) for o in png_in["steps"].values())
        png_in["work"] = [torch.empty(_lib.png_workspace_bytes(nfile, Hd_, Wd_, tot), dtype=torch.uint8, device=dev)
                          for _ in range(n_inflight)]
        png_in["out"] = [torch.empty((nfile, Hd_, Wd_), dtype=torch.float32, device=dev) for _ in range(n_inflight)]
        png_in["bytes_per_frame"] = float(np.mean([len(pool[f % len(pool)]) for f in range(nfile)]))
        if args.decode:
            D = max(1, args.jpeg_ahead)
            png_in["groups"] = [upload_files([pool[f % len(pool)] for s_ in range(g * D, (g + 1) * D)
                                              for f in step_ids(s_)], dev)
                                for g in range(-(-total_steps // D) + 1)]
            gt = max(int(o[2][-1]) for o in png_in["groups"])
            png_in["gwork"] = [torch.empty(_lib.png_workspace_bytes(D * nfile, Hd_, Wd_, gt), dtype=torch.uint8,
                                           device=dev) for _ in range(2)]
            png_in["gout"] = [torch.empty((D * nfile, Hd_, Wd_), dtype=torch.float32, device=dev) for _ in range(2)]
    jpg_in = None
    if args.decode:
        # every keyframe's colour image as a ScanNet-size 1296 x 968 baseline JPEG (bytes resident in
        # HBM), decoded on the GPU ahead of its detect on one decode stream, then cv2.resize to the
        # frame size (capture_stream.py:194-199).  A launch's latency is one wave's Huffman walk over a
        # whole file (~130 ms) whatever the batch, so the files of D = `jpeg_ahead` steps go in one
        # launch: group g + 1 is issued at group g's first step (double-buffered slots), and the timed
        # region carries one group's decode per D steps.  (One stream per step instead oversubscribes
        # the 4 hardware queues: a long decode then blocks detect launches sharing its queue.)
        from boxfusion_amd.capture_stream import upload_files
        D = max(1, args.jpeg_ahead)
        ngroups = -(-total_steps // D) + 1
        cpool = jpeg_pool(16)
        nf = D * Bm
        jpg_in = {"D": D, "H": 968, "W": 1296, "ready": {}, "used": {},
                  "groups": [upload_files([cpool[f % len(cpool)] for s_ in range(g * D, (g + 1) * D)
                                           for f in my_frames(s_)], dev) for g in range(ngroups)],
                  "work": [torch.empty(_lib.jpeg_workspace_bytes(nf, 968, 1296), dtype=torch.uint8, device=dev)
                           for _ in range(2)],
                  "full": [torch.empty((nf, 968, 1296, 3), dtype=torch.uint8, device=dev) for _ in range(2)],
                  "rgb": [torch.empty((nf, FH, FW, 3), dtype=torch.uint8, device=dev) for _ in range(2)],
                  "stream": torch.cuda.Stream(device=dev, priority=-1),
                  "bytes_per_frame": float(np.mean([len(b) for b in cpool]))}

    def jpeg_issue(g):
        """group g's depth PNGs and keyframe JPEGs (steps g*D .. g*D + D - 1) -> f32 depth and RGB at the
        frame size on the decode stream, into slot g % 2 once the last step of group g - 2 has read
        its inputs"""
        st = jpg_in["stream"]
        with torch.cuda.stream(st):
            prev = jpg_in["used"].pop(g - 2, None)
            if prev is not None:
                st.wait_event(prev)
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            if png_in is not None and "groups" in png_in:     # the group's depth files
                files, offs, offs_h = png_in["groups"][g]
                _lib.png_decode_u16(files, offs, png_in["H"], png_in["W"], out=png_in["gout"][g % 2],
                                    offsets_host=offs_h, depth_scale=CFG["cam"].get("png_depth_scale", 1000.0),
                                    work=png_in["gwork"][g % 2], check=False)
            files, offs, _ = jpg_in["groups"][g]
            _lib.jpeg_decode_rgb(files, offs, jpg_in["H"], jpg_in["W"], out=jpg_in["full"][g % 2],
                                 work=jpg_in["work"][g % 2], check=False)
            _lib.cv2_resize_u8(jpg_in["full"][g % 2], FW, FH, out=jpg_in["rgb"][g % 2])
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(st)
            jpg_in["ready"][g] = ev
            jpg_in.setdefault("spans", []).append((e0, ev))

    poses_all = np.stack([scene.pose(f) for f in all_mine]).astype(np.float32)
    dets_mine = [scene.detections(f, Kf, (FW, FH)) for f in all_mine]
    rec_all = torch.from_numpy(pack_records(dets_mine, poses_all)).to(dev)
    crops_all = torch.from_numpy(crop_boxes(dets_mine, args.crops)).to(dev)
    if args.clip_fp8:
        # static fp8 activation scales: calibrated once (bf16 forward of this rank's first batch
        # of crops, untimed) and shared by every in-flight detect stage
        from boxfusion_amd.pipeline import scale_boxes
        bi = scale_boxes(crops_all[:Bm * args.crops], FH, FW, detect.scale_box).to(torch.int32)
        scales = detect.clip.calibrate(rgb_all[:Bm], bi.contiguous(), detect.top_b32)
        for d in detects[1:]:
            d.clip.act_scales = scales
    sim = None
    if args.sim_ranks > 1 and world == 1:
        # what rank 0 of an R-GPU run fuses: R*B frames per step (stress test, not the metric)
        R = args.sim_ranks
        sim = {"rec": [], "per_step": B * R - (B - B0)}
        for s_ in range(total_steps):
            fr = [s_ * sim["per_step"] + j for j in range(sim["per_step"])]
            rh = pack_records([scene.detections(f, Kf, (FW, FH)) for f in fr], [scene.pose(f) for f in fr])
            sim["rec"].append(torch.from_numpy(rh).to(dev))
    torch.cuda.synchronize()

    brk = dict(detect=0.0, fusion=0.0)

    def run_steps(s0, s1, fusion, timer=None):
        for s in range(s0, s1):
            o = s * Bm
            sl = slice(o, o + Bm)
            tb = time.perf_counter()
            k = s % n_inflight
            st_ctx = torch.cuda.stream(det_streams[k])
            st_ctx.__enter__()      # this step's detect, gather and fusion hand-off on its stream
            det = detects[k]
            kf_depth = depth_all[sl]
            kf_rgb = rgb_all[sl]
            if jpg_in is not None:            # --decode: colour + depth decoded one group ahead; at a
                g, j = divmod(s, jpg_in["D"])  # group's first step, issue the next group's decode
                torch.cuda.current_stream().wait_event(jpg_in["ready"][g])
                if j == 0:                    # (after the wait: a wait issued behind a new decode
                    jpeg_issue(g + 1)         # launch on that stream would wait for it too)
                kf_rgb = jpg_in["rgb"][g % 2][j * Bm:(j + 1) * Bm]
                dec = png_in["gout"][g % 2][j * G * Bm:(j + 1) * G * Bm]
                kf_depth = dec[:Bm]
            elif png_in is not None:          # the step's depth files -> f32 depth (GPU decode, in stream)
                files, offs, offs_h = png_in["steps"][s]
                dec = png_in["out"][k]
                _lib.png_decode_u16(files, offs, png_in["H"], png_in["W"], out=dec, offsets_host=offs_h,
                                    depth_scale=CFG["cam"].get("png_depth_scale", 1000.0), work=png_in["work"][k], check=False)
                kf_depth = dec[:Bm]
            if nk_depth is not None:          # the step's non-keyframes: per-frame work only
                _lib.depth_preprocess(dec[Bm:] if png_in is not None else nk_depth[s], nk_K, nk_RT[s], 10.0,
                                      ws=nk_ws[k])
            det(kf_rgb, kf_depth, poses_all[sl], return_instances=False,
                crop_boxes=crops_all[s * Bm * args.crops:(s + 1) * Bm * args.crops])
            if jpg_in is not None and j == jpg_in["D"] - 1:   # the group's slot is free after this copy
                evu = torch.cuda.Event()
                evu.record()
                jpg_in["used"][g] = evu
            if args.breakdown:
                torch.cuda.synchronize()
                brk["detect"] += time.perf_counter() - tb
                tb = time.perf_counter()
            bidx, iidx, cat_idx, feats, sims = det.last["clip"]
            clip = clip_rows(feats, sims, cat_idx)
            g_rec, g_clip = exchange_step(rec_all[sl], clip, dist, N, B, B0, args.crops, rank)
            if sim is not None:       # --sim-ranks: rank 0 fuses the frames of R virtual ranks
                g_rec = sim["rec"][s]
                reps = -(-sim["per_step"] // Bm)
                g_clip = g_clip.repeat(reps, 1)[:sim["per_step"] * args.crops]
            if rank == 0:
                base = s * (per_step if sim is None else sim["per_step"])
                counts = [(base + j - s0 * (g_rec.shape[0])) * G for j in range(g_rec.shape[0])]
                if args.sync_fusion:
                    g_pose, g_cnt = record_meta(g_rec)
                    fusion.keyframes(counts, g_pose, unpack_records(g_rec, g_cnt, dev, g_clip,
                                                                    args.crops, coeff), g_cnt)
                else:
                    # hand the step's frames to the fusion worker (side stream), keep detecting
                    ev = torch.cuda.Event()
                    ev.record()
                    g_rec.record_stream(fusion.stream)
                    g_clip.record_stream(fusion.stream)

                    # the whole step's keyframes as one job: geometry batched, association serial
                    def job(st, r=g_rec, c_=g_clip, k_=counts):
                        tj = time.perf_counter()
                        p, c = record_meta(r)       # on the worker's stream, after the gather
                        u = unpack_records(r, c, dev, c_, args.crops, coeff)
                        if os.environ.get("BF_FSEQ_PROFILE"):
                            print(f"job: meta + unpack {1e3 * (time.perf_counter() - tj):.2f} ms",
                                  file=sys.stderr, flush=True)
                        st.keyframes(k_, p, u, c)
                    fusion.submit_call(job, ev)
            st_ctx.__exit__(None, None, None)
            if args.breakdown:
                torch.cuda.synchronize()
                brk["fusion"] += time.perf_counter() - tb

    # ---- warmup (own fusion state), then the timed stream from frame 0 ----------------------
    # rank 0 owns the serial fusion state machine; when it fuses more frames than it detects
    # (N > 1), 32 CUs (4 per XCD) are reserved for it so the persistent GEMMs cannot starve it
    fusion_cus = args.fusion_cus
    if fusion_cus < 0:
        fusion_cus = 32 if rank == 0 and (world > 1 or args.sim_ranks > 1) else 0
    masked = args.mask_cus if args.mask_cus >= 0 else int(fusion_cus > 0)
    det_stream, fus_stream = (_lib.partition_streams(fusion_cus, local, masked=bool(masked)) if fusion_cus > 0
                              else (torch.cuda.current_stream(), None))
    torch.cuda.synchronize()
    torch.cuda.set_stream(det_stream)          # detection (graph replays, gathers) on its CUs
    if masked and fusion_cus > 0:   # every detect stream on the detection CUs
        det_cus, _ = _lib.partition_cus(fusion_cus, local)
        det_streams = [det_stream] + [_lib.cu_masked_stream(det_cus, local) for _ in range(n_inflight - 1)]
    else:
        det_streams = [det_stream] + [torch.cuda.Stream(device=dev) for _ in range(n_inflight - 1)]
    if jpg_in is not None and masked and fusion_cus > 0:
        # --decode with reserved CUs: the colour decode runs on them, out of the detect kernels' way
        jpg_in["stream"] = _lib.cu_masked_stream(_lib.partition_cus(fusion_cus, local)[1], local)

    # capture every DetectStage's graph before the fusion worker exists: a capture must not see
    # another thread's synchronising calls
    for k, d in enumerate(detects):
        with torch.cuda.stream(det_streams[k]):
            d(rgb_all[:Bm], depth_all[:Bm], poses_all[:Bm], return_instances=False,
              crop_boxes=crops_all[:Bm * args.crops])
    torch.cuda.synchronize()

    def make_fusion():
        st = FusionStage(CFG, Kf, H=FH, W=FW, device=dev)
        return st if args.sync_fusion else AsyncFusion(st, stream=fus_stream)

    if jpg_in is not None:                     # the first group's colour decode, before the warmup
        jpeg_issue(0)
    wf = make_fusion()
    run_steps(0, args.warmup, wf)
    if not args.sync_fusion:
        wf.join()
    # the warm-up sequencer's device / pinned staging buffers go back to their pools, so the timed
    # sequencer's first keyframes reuse them instead of allocating under the detect load
    del wf
    gc.collect()
    torch.cuda.synchronize()
    fusion = make_fusion()
    brk.update(detect=0.0, fusion=0.0)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    timer = _lib.KernelTimer()
    owner = None
    t0 = time.perf_counter()
    with timer:       # records every eager GEMM / attention launch (graph replays launch none from Python)
        run_steps(args.warmup, total_steps, fusion)
        if not args.sync_fusion:
            worker = fusion
            fusion = fusion.join()
            owner = (worker.busy_s, fusion.stats["keyframes"])
            if rank == 0:
                print(f"fusion worker busy {1e3 * worker.busy_s / args.steps:.1f} ms/step "
                      f"({fusion.stats['keyframes']} keyframes)", file=sys.stderr, flush=True)
        if rank == 0 and G > 1:
            # demo.py:200: the stream's last frame is not a keyframe -> the stale re-fusion of the
            # previous keyframe's instances with the last pose
            last = per_step * args.steps * G - 1
            fusion.finish(last, scene.pose(total_steps * per_step * G - 1), False)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cpu" if rehearse else dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    source = "timed region"
    timed_records = timer      # the non-keyframe depth batches were launched eagerly in the timed region
    if not any(r[0]["kind"] in ("gemm", "gemm_fp8") for r in timer.records):
        # graph mode: time the same kernels launched eagerly on the same inputs, right after the
        # timed region (HIP events on the launch stream, every GEMM / attention launch of the steps)
        detect.use_graph = False
        timer = _lib.KernelTimer()
        with timer:
            for s in range(args.warmup, min(total_steps, args.warmup + args.roofline_steps)):
                sl = slice(s * Bm, s * Bm + Bm)
                detect(rgb_all[sl], depth_all[sl], poses_all[sl], return_instances=False,
                       crop_boxes=crops_all[s * Bm * args.crops:(s + 1) * Bm * args.crops])
        torch.cuda.synchronize()
        detect.use_graph = not args.eager
        source = f"eager re-run of {args.roofline_steps} timed steps"
    frames = per_step * args.steps * G
    fus_timer = None
    if rank == 0:
        # the fusion kernels (pairs/s of the 3-D IoU matrix, particle-views/s of the
        # box-fusion fitness) on their own after the timed region: a fresh fusion state machine
        # over the stream's first keyframes, synchronous, HIP events around every launch
        from boxfusion_amd.pipeline import scene_instances
        fst = FusionStage(CFG, Kf, H=FH, W=FW, device=dev, native=False)   # Python-driven: per-kernel timers
        fus_timer = _lib.KernelTimer()
        with fus_timer:
            for k in range(args.roofline_keyframes):
                f = k * G
                fst.keyframe(f, scene.pose(f), scene_instances(scene.detections(f, Kf, (FW, FH)), dev, FH, FW))
            fst.boxes()
        torch.cuda.synchronize()

    if rank == 0:
        big = lambda t: t["kind"] == "gemm" and t["large"]
        r_all = roofline_obj(timer.summary(big), "every bf16 linear launch of CLIP ViT-H and CuTR (qkv, "
                             "proj/fc2 + f32 residual, fc1 + GELU): the hand-written k_gemm256q / "
                             "k_gemm256p, tile height per shape", "mfma", pmc_key=PMC_KEYS["gemm"])
        r_all["traffic_note"] = ("PMC bytes per launch averaged over the GEMM family's kernels in "
                                 "the PMC run: k_gemm256p / k_gemm256q")
        comps = {
            "resid_gemm": roofline_obj(timer.summary(lambda t: big(t) and t["resid"]),
                                       "proj / fc2 + f32 residual (k_gemm256q at tile heights below 256 "
                                       "rows, k_gemm256p at 256)", "mfma",
                                       pmc_key=PMC_KEYS["resid_gemm"]),
            "gelu_gemm": roofline_obj(timer.summary(lambda t: big(t) and t["act"] == 1),
                                      "k_gemm256q<true, 1> (fc1 + GELU)", "mfma",
                                      pmc_key=PMC_KEYS["gelu_gemm"]),
            "attention": roofline_obj(timer.summary(lambda t: t["kind"] == "attn"),
                                      "k_attn_* (every ViT attention launch: CuTR window + global, "
                                      "CLIP)", "mfma", pmc_key=PMC_KEYS["attention"]),
            "attention_clip": roofline_obj(timer.summary(lambda t: t["kind"] == "attn" and t["D"] == 80),
                                           "CLIP ViT-H/14 attention (S=257, D=80)", "mfma",
                                           pmc_key=PMC_KEYS["attention_clip"]),
            "attention_cutr": roofline_obj(timer.summary(lambda t: t["kind"] == "attn" and t["D"] != 80),
                                           "CuTR attention (512-key joint windows, 1600-token global)",
                                           "mfma", pmc_key=PMC_KEYS["attention_cutr"]),
        }
        for v in comps.values():
            v["measured"] = source
        dks = (timed_records.summary(lambda t: t["kind"] == "depth" and t["b"] > Bm) if G > 1
               else timer.summary(lambda t: t["kind"] == "depth"))
        if dks["launches"]:
            # small batches run the four-launch form (k_ds_hist1..3 with the selects folded in +
            # k_ds_norm: the PMC passes' eager 8-frame call); large ones have no PMC record
            dfr = (G - 1) * Bm if G > 1 else Bm
            npx = (FRAME["H"] // FRAME["r"]) * (FRAME["W"] // FRAME["r"])
            small = dfr * -(-npx // 8192) < 4096
            comps["depth_preprocess"] = roofline_obj(
                dks, "bf_depth_preprocess (a1 + a13: trimmed depth standardisation + back-projection, "
                     "3-level radix select over the whole chip)", "hbm",
                pmc_key=PMC_KEYS["depth_small"] if small else "k_ds")
            comps["depth_preprocess"]["measured"] = (source if G == 1 else
                                                     "timed region (non-keyframe batches)")
            comps["depth_preprocess"]["frames_per_launch"] = (G - 1) * Bm if G > 1 else Bm
            # the same call replayed from a HIP graph: its launches (four for small batches, seven
            # for large ones) back to back, no host gaps between them (the eager events above
            # include them)
            dsrc = nk_depth[args.warmup] if G > 1 else depth_all[args.warmup * Bm:(args.warmup + 1) * Bm]
            nfr = dsrc.shape[0]
            dK = nk_K if G > 1 else detect.Kd_dev[:1].expand(nfr, 3, 3).contiguous()
            dRT = nk_RT[args.warmup] if G > 1 else torch.from_numpy(
                poses_all[args.warmup * Bm:(args.warmup + 1) * Bm]).to(dev)
            gst = torch.cuda.Stream(dev)
            gst.wait_stream(torch.cuda.current_stream(dev))
            g_ws = _lib.new_depth_workspace(*dsrc.shape, dev)       # the graph's own workspace
            with torch.cuda.stream(gst):
                _lib.depth_preprocess(dsrc, dK, dRT, 10.0, ws=g_ws)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=gst):
                    _lib.depth_preprocess(dsrc, dK, dRT, 10.0, ws=g_ws)
                for _ in range(3):
                    graph.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(gst)
                for _ in range(20):
                    graph.replay()
                e1.record(gst)
            torch.cuda.synchronize()
            g_us = 1e3 * e0.elapsed_time(e1) / 20
            g_bytes = dks["bytes_per_launch"] * nfr / comps["depth_preprocess"]["frames_per_launch"]
            comps["depth_preprocess"]["graph_replay"] = {
                "frames": nfr, "avg_us": g_us, "achieved_gbs": g_bytes / (g_us * 1e-6) / 1e9,
                "frac": g_bytes / (g_us * 1e-6) / 1e9 / PEAK_HBM_GBS,
                "note": "one bf_depth_preprocess call captured in a HIP graph, 20 replays timed with HIP events"}
        if fus_timer is not None:
            for kind, unit, name in (("obb_iou", "pairs/s", "bf_obb_iou_matrix (k_obb_gate + k_obb_grid): "
                                      "box pairs of the 3-D IoU matrix"),
                                     ("nms_scan", "boxes/s", "bf_nms_scan (greedy scan + record)"),
                                     ("fusion_fit", "particle-views/s", "bf_fusion_fit (k_fuse_terms + "
                                      "k_fuse_step): particle x view fitness evaluations, all iterations")):
                ks = fus_timer.summary(lambda t, k_=kind: t["kind"] == k_)
                if ks["launches"]:
                    comps[kind] = {"bound": "latency / VALU", "kernel": name, "unit": unit,
                                   "achieved": ks["flops"] / (ks["ms"] * 1e-3), "launches": ks["launches"],
                                   "avg_us": ks["avg_us"], "work_per_launch": ks["flops_per_launch"],
                                   "measured": f"fusion re-run over {args.roofline_keyframes} keyframes"}
        r_all["measured"] = source
        line = base_line(args, N, frames, dt, per_step * G, n_inflight)
        if B0 < B:
            line["config"]["rank0_batch"] = B0
        if args.dataset == "ca1m":
            r_ = FRAME["r"]
            line["metric"] = ("RGB-D frames/sec (whole node) on 384x512 portrait stream, depth at the image size"
                              if r_ == 1 else
                              f"RGB-D frames/sec (whole node) on 384x512 portrait stream, depth at 1/{r_} resolution")
            line["data"] = ("synthetic CA-1M-shaped RGB-D stream (seeded; CA-1M data absent offline), random-init "
                            "weights, seeded scene detections")
            line["config"]["workload"] = line["config"]["workload"].replace(
                "configs[2]: synthetic 640x480 RGB-D", "configs[1]: CA-1M-shaped 384x512 portrait RGB-D, "
                f"depth {384 // r_}x{512 // r_} (RGB:depth {r_}{', as CA1MDataset streams it' if r_ == 1 else ''}), "
                "ca1m.yaml thresholds")
            line["config"]["depth_ratio"] = r_
        if G > 1:
            line["config"]["workload"] = line["config"]["workload"].replace(
                "gap=1", f"gap={G} (demo.py keyframe rule: {B} keyframes + {(G - 1) * B} non-keyframe "
                         f"depth standardisations per step per GPU)")
            line["config"]["keyframes"] = per_step * args.steps
        line["config"].update(scene_objects=args.scene_objects, fused_boxes=fusion.stats["fused"],
                              global_boxes=len(fusion.all_pred_box) if fusion.all_pred_box is not None else 0)
        # box-fusion calls with a particle whose 2-D intersection hull exceeds the reference
        # kernel's convex_inter[8] (box_fusion.py:381: undefined behaviour there; exact hull here)
        line["hull_overflow"] = {"calls": fusion.fuser.hull_overflow_calls,
                                 "fusion_calls": fusion.fuser.fit_calls}
        if owner is not None and owner[1] > 0:
            # the fusion owner's worker thread (SURVEY §8e's serial term): time it spent fusing,
            # host and device waits included, beside the detect streams
            line["fusion_owner"] = {"busy_ms_per_step": 1e3 * owner[0] / args.steps,
                                    "keyframes": owner[1],
                                    "ms_per_keyframe": 1e3 * owner[0] / owner[1]}
        if args.clip_fp8:
            f8 = roofline_obj(timer.summary(lambda t: t["kind"] == "gemm_fp8"),
                              "k_gemm256p<*, *, fp8> (CLIP qkv, fc1 + GELU -> fp8, fc2 + f32 residual; "
                              "block-scaled fp8 MFMA)", "mfma", pmc_key=PMC_KEYS["fp8_gemm"],
                              peak_tflops=PEAK_FP8_TFLOPS)
            f8["measured"] = source
            comps["fp8_gemm"] = f8
        # the headline is the figure north_star names: "fraction of the ViT-attention MFMA
        # roofline" (every CLIP + CuTR attention launch); the GEMM family -- most of the GPU time --
        # is roofline_components.gemm
        comps["gemm"] = r_all
        head = dict(comps["attention"])
        head["note"] = ("north_star's ViT-attention MFMA roofline: algorithmic 4*Sq*Sk*D FLOPs of every "
                        "CLIP ViT-H/14 and CuTR attention launch / their HIP-event time / the 2.5 PF dense "
                        "bf16 peak; the GEMM family is roofline_components.gemm")
        line["roofline"] = head
        line["roofline_components"] = comps
        if png_in is not None:
            # the GPU decode alone: one step's files (keyframes + non-keyframes), HIP events, after
            # the timed region; and PIL on 16 host threads over the same files
            files, offs, offs_h = png_in["steps"][args.warmup]
            dec, wk = png_in["out"][0], png_in["work"][0]
            nfile = len(offs_h) - 1
            for _ in range(2):
                _lib.png_decode_u16(files, offs, png_in["H"], png_in["W"], out=dec, offsets_host=offs_h,
                                    depth_scale=1000.0, work=wk, check=False)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                _lib.png_decode_u16(files, offs, png_in["H"], png_in["W"], out=dec, offsets_host=offs_h,
                                    depth_scale=1000.0, work=wk, check=False)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 5
            _, st = _lib.png_decode_u16(files, offs, png_in["H"], png_in["W"], out=dec, offsets_host=offs_h,
                                        depth_scale=1000.0, work=wk, check=True)
            thr = min(16, os.cpu_count() or 1)
            line["decode"] = {
                "kernel": "bf_png_decode_depth (k_png_parse + k_png_gather + k_png_inflate + k_png_unfilter)",
                "files_per_step": nfile, "bytes_per_file": png_in["bytes_per_frame"],
                "gpu_ms_per_step": ms, "gpu_frames_per_s": nfile / (ms * 1e-3),
                "host_pil_frames_per_s": host_png_rate(png_in["pool"], thr), "host_threads": thr,
                "host_jpeg_keyframes_per_s": None, "jpeg_bytes": None,
                "note": ("depth files: the synthetic scene's 640x480 depth in mm written by PIL (adaptive "
                         "filters, zlib level 6); gpu = one step's files decoded alone (HIP events, mean of "
                         "5); host = PIL on the pool over ~3 s")}
            jr, jb = host_jpeg_rate(thr)
            gj, gn = gpu_jpeg_rate()
            line["decode"].update(host_jpeg_keyframes_per_s=jr, jpeg_bytes=jb,
                                  gpu_jpeg_keyframes_per_s=gj, gpu_jpeg_batch=gn,
                                  jpeg_kernel="bf_jpeg_decode_rgb (k_jpeg_parse + k_jpeg_entropy + k_jpeg_idct "
                                              "+ k_jpeg_color), bit-exact to libjpeg's defaults",
                                  keyframes_per_s_needed=line["value"] / G)
            line["config"]["depth_input"] = ("16-bit PNG bytes in HBM, decoded on the GPU in the timed region" +
                                             (f" (one group of {args.jpeg_ahead} steps ahead on a decode stream)"
                                              if args.decode else " (in the step's stream)"))
            if jpg_in is not None:
                spans = [a.elapsed_time(b) for a, b in jpg_in["spans"][1:]]
                line["decode"]["gpu_jpeg_group_ms"] = {"files": jpg_in["D"] * Bm, "mean": float(np.mean(spans)),
                                                      "max": float(np.max(spans))} if spans else None
                line["config"]["color_input"] = (f"1296x968 baseline JPEG bytes in HBM (q90 4:2:0, "
                                                 f"{jpg_in['bytes_per_frame'] / 1e3:.0f} KB), decoded on the GPU "
                                                 f"one group of {jpg_in['D']} steps ahead on a decode stream "
                                                 f"(bf_jpeg_decode_rgb + bf_cv2_resize_u8 to {FW}x{FH}) inside the "
                                                 f"timed region")
        if args.breakdown:
            line["breakdown_ms_per_step"] = {k: 1e3 * v / args.steps for k, v in brk.items()}
        if not args.no_cpu_baseline and N == 1:   # rank 0 at N=1 only
            line["cpu_baseline"] = (cpu_baseline(cutr, clip_vis, args, scene) if args.cpu_detect_frames > 0 else None)
        emit(line)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
