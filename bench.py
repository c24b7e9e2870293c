#!/usr/bin/env python3
"""Throughput benchmark: RGB-D frames/s of per-frame detect + multi-view 3D box fusion.

Workload (BASELINE.json configs[2]): synthetic 640x480 RGB-D stream, batch 8 frames
per step per GPU, every frame a keyframe (gap=1, the per-frame-detect roofline run):
  per frame  depth standardisation + back-projection, CuTR RGB-D ViT-B (dim 768) forward,
             detection filters, CLIP ViT-H/14 on the top-16 boxes (16 crops/frame), text match
             against the 473-class vocabulary;
  per step   all-gather (RCCL) of every rank's per-frame records (scene detections + CLIP
             features) -> rank 0 runs the fusion state machine (NMS + association + box fusion)
             over all gathered frames in global frame order.
Weights are random (no checkpoint offline); the detections feeding fusion come from the seeded
30-object scene generator (boxfusion_amd/synthetic.py), since random-weight CuTR boxes are noise.
Inputs (frames, scene detections) are resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W]      (N>1 under torch.distributed.run)
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md), no sparsity
PEAK_HBM_GBS = 8000.0

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
REC_ROWS, REC_W = 64, 22     # per-frame detection record: rows x (score, xyxy, xyzlhw, R, proj_xy)
REC_HEAD = 17                # record head: detection count, camera pose (4x4)


def parse():
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
    p.add_argument("--fusion-cus", type=int, default=-1,
                   help="CUs reserved for the fusion stream (-1: 32 on rank 0 when N > 1, else 0)")
    p.add_argument("--sim-ranks", type=int, default=1,
                   help="stress test at N=1: rank 0 also fuses the frames of R virtual ranks per step")
    p.add_argument("--mask-cus", type=int, default=-1,
                   help="1: confine detection and fusion streams to disjoint CU sets (CU-masked "
                        "streams) when CUs are reserved for fusion; -1: on when fusing for N > 1")
    p.add_argument("--sync-fusion", action="store_true",
                   help="run the fusion state machine inline instead of on the worker stream")
    p.add_argument("--cpu-detect-frames", type=int, default=1)
    p.add_argument("--inflight", type=int, default=-1,
                   help="detect steps in flight per GPU: independent batches replayed on this many "
                        "streams (each its own DetectStage buffers / graph), so one batch's CLIP "
                        "phases overlap the next batch's CuTR phases (default 2; with 32 CUs "
                        "reserved for rank 0's fusion at N > 1 the two detect streams run on the "
                        "other 224)")
    p.add_argument("--cpu-fusion-frames", type=int, default=24)
    return p.parse_args()


# ------------------------------------------------------------------------------------------------
def gen_frames(frame_ids, dev):
    """seeded synthetic RGB-D frames generated on the device (seed 1234 + frame)."""
    n = len(frame_ids)
    rgb = torch.empty((n, 480, 640, 3), dtype=torch.uint8, device=dev)
    depth = torch.empty((n, 480, 640), dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for j, f in enumerate(frame_ids):
        g.manual_seed(1234 + int(f))
        rgb[j].random_(0, 256, generator=g)
        depth[j].uniform_(0.5, 4.5, generator=g)
        depth[j].masked_fill_(torch.rand((480, 640), device=dev, generator=g) < 0.05, 0.0)
    return rgb, depth


def pack_records(dets, poses):
    """scene detections + camera poses of a batch of frames -> f32 [b, REC_HEAD + REC_ROWS*REC_W]
    records: (count, pose 4x4, rows).  The pose and count travel with the detections, so the
    exchange is one device all-gather (no host-object collective, which would synchronise the
    detect stream every step)."""
    out = np.zeros((len(dets), REC_HEAD + REC_ROWS * REC_W), np.float32)
    for j, d in enumerate(dets):
        n = min(len(d["scores"]), REC_ROWS)
        rows = np.concatenate([d["scores"][:n, None], d["pred_boxes"][:n], d["xyzlhw"][:n],
                               d["R"][:n].reshape(n, 9), d["proj_xy"][:n]], 1)
        out[j, 0] = n
        out[j, 1:REC_HEAD] = np.asarray(poses[j], np.float32).reshape(-1)
        out[j, REC_HEAD:REC_HEAD + n * REC_W] = rows.reshape(-1)
    return out


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
    p = Instances3D((480, 640))
    p.scores = rows[:, 0].contiguous()
    p.pred_boxes = rows[:, 1:5].contiguous()
    p.pred_boxes_3d = GeneralInstance3DBoxes(rows[:, 5:11], rows[:, 11:20].reshape(n, 3, 3))
    p.pred_proj_xy = rows[:, 20:22].contiguous()
    return p


def unpack_records(recs, cnts, dev):
    """records [nkf, REC_HEAD + REC_ROWS*REC_W] of several keyframes -> ONE Instances3D holding every
    keyframe's detections in order (keyframe j: cnts[j] rows), five gathers in total"""
    from boxfusion_amd import _lib
    from boxfusion_amd.boxes import GeneralInstance3DBoxes
    from boxfusion_amd.instances import Instances3D
    cnts = np.asarray(cnts, np.int64)
    idx = np.concatenate([j * REC_ROWS + np.arange(c) for j, c in enumerate(cnts)]) if cnts.sum() else \
        np.zeros(0, np.int64)
    rows = recs[:, REC_HEAD:REC_HEAD + REC_ROWS * REC_W].reshape(-1, REC_W).index_select(
        0, _lib.h2d(idx, dev))
    p = Instances3D((480, 640))
    p.scores = rows[:, 0].contiguous()
    p.pred_boxes = rows[:, 1:5].contiguous()
    p.pred_boxes_3d = GeneralInstance3DBoxes._views(rows[:, 5:11].contiguous(),
                                                     rows[:, 11:20].reshape(-1, 3, 3).contiguous())
    p.pred_proj_xy = rows[:, 20:22].contiguous()
    return p


def gather_step(recs, feats, dist, world):
    """Exchange of one step: every rank's per-frame records [b, R] (detections, count and camera
    pose) and CLIP features [n_crops, 1024] are all-gathered (RCCL over xGMI on the GPU; gloo in
    the CPU tests) so that the fusion owner sees the step's frames in global frame order
    (rank-major = frame order, since rank r holds frames step*b*world + r*b ... + b-1).  Both
    collectives are asynchronous device operations: nothing here waits for the detect stream."""
    if dist is None or world == 1:
        return recs, feats
    if recs.is_cuda and dist.get_backend() == "gloo":     # BF_BENCH_REHEARSE=1 (one-GPU rehearsal)
        g_rec, g_feat = gather_step(recs.cpu(), feats.cpu(), dist, world)
        return g_rec.to(recs.device), g_feat.to(feats.device)
    if recs.is_cuda:
        g_rec = torch.empty((world * recs.shape[0],) + recs.shape[1:], dtype=recs.dtype, device=recs.device)
        dist.all_gather_into_tensor(g_rec, recs.contiguous())
        g_feat = torch.empty((world * feats.shape[0],) + feats.shape[1:], dtype=feats.dtype,
                             device=feats.device)
        dist.all_gather_into_tensor(g_feat, feats.contiguous())
    else:
        parts = [torch.empty_like(recs) for _ in range(world)]
        dist.all_gather(parts, recs.contiguous())
        g_rec = torch.cat(parts)
        fparts = [torch.empty_like(feats) for _ in range(world)]
        dist.all_gather(fparts, feats.contiguous())
        g_feat = torch.cat(fparts)
    return g_rec, g_feat


# ------------------------------------------------------------------------------------------------
def cpu_baseline(cutr, clip_vis, args, scene):
    """The parity-checked CPU restatement timed on this host: fp32 torch-CPU CuTR + CLIP on
    `cpu_detect_frames` frames (16 crops each) and the oracle fusion chain (C restatement,
    oracle/chain.py) over the first `cpu_fusion_frames` frames of the stream."""
    from oracle.chain import OracleChain
    from boxfusion_amd.box_fusion import load_pst
    from boxfusion_amd.cubify_transformer import FrameBatch
    from boxfusion_amd.preprocessor import PIXEL_MEAN_U8, PIXEL_STD_U8
    from boxfusion_amd.sensor import camera_to_gravity
    from boxfusion_amd.synthetic import SCANNET_K, frame_rgbd
    from boxfusion_amd.clip import CLIP_MEAN, CLIP_STD
    from oracle import oracle as OR
    import torch.nn.functional as F
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    cm = copy.deepcopy(cutr).float().cpu().eval()
    vm = copy.deepcopy(clip_vis).float().cpu().eval()
    nf = args.cpu_detect_frames
    t0 = time.perf_counter()
    with torch.no_grad():
        for f in range(nf):
            rgb, depth = frame_rgbd(f)
            mean = torch.tensor(PIXEL_MEAN_U8).view(3, 1, 1)
            std = torch.tensor(PIXEL_STD_U8).view(3, 1, 1)
            img = (torch.from_numpy(np.moveaxis(rgb, -1, 0)).float() - mean) / std
            img = F.pad(img, (0, 0, 0, 160))[None]
            d, params = OR.depth_standardize(depth)
            OR.backproject(depth, SCANNET_K, scene.pose(f))
            d = F.pad(torch.from_numpy(d), (0, 0, 0, 160))[None]
            batch = FrameBatch(image=img, depth=d, depth_params=torch.from_numpy(params)[None],
                               K=torch.from_numpy(SCANNET_K)[None],
                               T_gravity=torch.from_numpy(camera_to_gravity(scene.pose(f)))[None],
                               image_sizes=[(480, 640)])
            r = cm(batch)[0]
            boxes = r.pred_boxes[: args.crops].numpy().astype(np.int64)
            crops = []
            for x1, y1, x2, y2 in boxes:
                c = torch.from_numpy(rgb[y1:y2, x1:x2]).permute(2, 0, 1).float()[None]
                c = F.interpolate(c, (224, 224), mode="bilinear", align_corners=False) if c.numel() \
                    else torch.zeros((1, 3, 224, 224))
                crops.append(c)
            x = torch.cat(crops) / 255.0
            x = (x - torch.tensor(CLIP_MEAN).view(1, 3, 1, 1)) / torch.tensor(CLIP_STD).view(1, 3, 1, 1)
            vm(x)
    t_det = (time.perf_counter() - t0) / nf
    ch = OracleChain(CFG, SCANNET_K, pst=load_pst(), legacy=True)
    t0 = time.perf_counter()
    for f in range(args.cpu_fusion_frames):
        ch.keyframe(f, scene.pose(f), scene.detections(f))
    t_fuse = (time.perf_counter() - t0) / args.cpu_fusion_frames
    return {"value": 1.0 / (t_det + t_fuse), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": (f"{nf} frame(s) of fp32 torch-CPU CuTR ViT-B + {args.crops} CLIP ViT-H/14 "
                       f"crops ({t_det:.2f} s/frame) + oracle fusion chain over frames "
                       f"0..{args.cpu_fusion_frames - 1} ({1e3 * t_fuse:.1f} ms/frame)")}


def load_pmc_traffic():
    """HBM-side bytes per launch of the roofline kernel from the committed PMC passes
    (profiles/*_pmc_gelu_gemm.json, newest round); counters cannot be read from inside the run."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_gelu_gemm.json")))
    if not files:
        return {}
    with open(files[-1]) as f:
        d = json.load(f)
    d["source"] = os.path.relpath(files[-1], ROOT) + " (FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes)"
    return d


# ------------------------------------------------------------------------------------------------
def main():
    args = parse()
    if args.breakdown:
        args.sync_fusion = True
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
    n_inflight = args.inflight if args.inflight > 0 else 2
    detects = [DetectStage(cutr, clip_vis, CFG, B, 480, 640, SCANNET_K, crops_per_frame=args.crops,
                           crop_source="top", backproject=True, clip_capacity=B * args.crops,
                           device=dev, graph=not args.eager) for _ in range(n_inflight)]
    detect = detects[0]
    scene = Scene(seed=0)
    N = world
    per_step = B * N
    total_steps = args.warmup + args.steps

    def my_frames(step):
        return [step * per_step + rank * B + j for j in range(B)]

    # ---- inputs resident in HBM before timing -----------------------------------------------
    all_mine = [f for s in range(total_steps) for f in my_frames(s)]
    rgb_all, depth_all = gen_frames(all_mine, dev)
    poses_all = np.stack([scene.pose(f) for f in all_mine]).astype(np.float32)
    rec_host = pack_records([scene.detections(f) for f in all_mine], poses_all)
    rec_all = torch.from_numpy(rec_host).to(dev)
    sim = None
    if args.sim_ranks > 1 and world == 1:
        # what rank 0 of an R-GPU run fuses: R*B frames per step (stress test, not the metric)
        R = args.sim_ranks
        sim = {"rec": []}
        for s_ in range(total_steps):
            fr = [s_ * B * R + j for j in range(B * R)]
            rh = pack_records([scene.detections(f) for f in fr], [scene.pose(f) for f in fr])
            sim["rec"].append(torch.from_numpy(rh).to(dev))
    torch.cuda.synchronize()

    brk = dict(detect=0.0, fusion=0.0)

    def run_steps(s0, s1, fusion, timer=None):
        for s in range(s0, s1):
            o = s * B
            sl = slice(o, o + B)
            tb = time.perf_counter()
            k = s % n_inflight
            st_ctx = torch.cuda.stream(det_streams[k])
            st_ctx.__enter__()      # this step's detect, gather and fusion hand-off on its stream
            det = detects[k]
            det(rgb_all[sl], depth_all[sl], poses_all[sl], return_instances=False)
            if args.breakdown:
                torch.cuda.synchronize()
                brk["detect"] += time.perf_counter() - tb
                tb = time.perf_counter()
            bidx, iidx, cat_idx, feats, sims = det.last["clip"]
            recs = rec_all[sl]
            g_rec, g_feat = gather_step(recs, feats, dist, N)
            if sim is not None:       # --sim-ranks: rank 0 fuses the frames of R virtual ranks
                g_rec = sim["rec"][s]
            if rank == 0:
                base = s * (per_step if sim is None else B * args.sim_ranks)
                if args.sync_fusion:
                    g_pose, g_cnt = record_meta(g_rec)
                    for j in range(g_rec.shape[0]):
                        fusion.keyframe(base + j - s0 * (g_rec.shape[0]), g_pose[j],
                                        unpack_record(g_rec[j], dev, int(g_cnt[j])))
                else:
                    # hand the step's frames to the fusion worker (side stream), keep detecting
                    ev = torch.cuda.Event()
                    ev.record()
                    g_rec.record_stream(fusion.stream)
                    counts = [base + j - s0 * (g_rec.shape[0]) for j in range(g_rec.shape[0])]
                    # the whole step's keyframes as one job: geometry batched, association serial
                    def job(st, r=g_rec, k=counts):
                        p, c = record_meta(r)       # on the worker's stream, after the gather
                        st.keyframes(k, p, unpack_records(r, c, dev), c)
                    fusion.submit_call(job, ev)
            st_ctx.__exit__(None, None, None)
            if args.breakdown:
                torch.cuda.synchronize()
                brk["fusion"] += time.perf_counter() - tb

    # ---- warmup (own fusion state), then the timed stream from frame 0 ----------------------
    # rank 0 owns the serial fusion state machine; when it fuses more frames than it detects
    # (N > 1), a few CUs are reserved for it so the persistent GEMMs cannot starve it
    fusion_cus = args.fusion_cus
    if fusion_cus < 0:
        fusion_cus = 32 if rank == 0 and (world > 1 or args.sim_ranks > 1) else 0
    masked = args.mask_cus if args.mask_cus >= 0 else int(fusion_cus > 0)
    det_stream, fus_stream = (_lib.partition_streams(fusion_cus, local, masked=bool(masked)) if fusion_cus > 0
                              else (torch.cuda.current_stream(), None))
    torch.cuda.synchronize()
    torch.cuda.set_stream(det_stream)          # detection (graph replays, gathers) on its CUs
    if masked and fusion_cus > 0:   # every detect stream on the detection CUs
        det_streams = [det_stream] + [_lib.partition_streams(fusion_cus, local, masked=True)[0]
                                      for _ in range(n_inflight - 1)]
    else:
        det_streams = [det_stream] + [torch.cuda.Stream(device=dev) for _ in range(n_inflight - 1)]

    # capture every DetectStage's graph before the fusion worker exists: a capture must not see
    # another thread's synchronising calls
    for k, d in enumerate(detects):
        with torch.cuda.stream(det_streams[k]):
            d(rgb_all[:B], depth_all[:B], poses_all[:B], return_instances=False)
    torch.cuda.synchronize()

    def make_fusion():
        st = FusionStage(CFG, SCANNET_K, device=dev)
        return st if args.sync_fusion else AsyncFusion(st, stream=fus_stream)

    wf = make_fusion()
    run_steps(0, args.warmup, wf)
    if not args.sync_fusion:
        wf.join()
    fusion = make_fusion()
    brk.update(detect=0.0, fusion=0.0)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    timer = _lib.KernelTimer(out_bf16=True, act="gelu", large_tiles=True)
    t0 = time.perf_counter()
    with timer:       # records every eager GELU-GEMM launch (graph replays launch none from Python)
        run_steps(args.warmup, total_steps, fusion)
        if not args.sync_fusion:
            worker = fusion
            fusion = fusion.join()
            if rank == 0:
                print(f"fusion worker busy {1e3 * worker.busy_s / args.steps:.1f} ms/step "
                      f"({fusion.stats['keyframes']} keyframes)", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cpu" if rehearse else dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ks = timer.summary()
    if ks["launches"] == 0:
        # graph mode: time the same kernel launched eagerly on the same inputs, right after the
        # timed region (HIP events on the launch stream, every GELU-GEMM launch of the steps)
        detect.use_graph = False
        timer = _lib.KernelTimer(out_bf16=True, act="gelu", large_tiles=True)
        with timer:
            for s in range(args.warmup, min(total_steps, args.warmup + args.roofline_steps)):
                sl = slice(s * B, s * B + B)
                detect(rgb_all[sl], depth_all[sl], poses_all[sl], return_instances=False)
        torch.cuda.synchronize()
        detect.use_graph = not args.eager
        ks = timer.summary()
        ks["source"] = f"eager re-run of {args.roofline_steps} timed steps"
    else:
        ks["source"] = "timed region"
    frames = per_step * args.steps

    if rank == 0:
        achieved = ks["tflops"] if ks["launches"] else 0.0
        pmc = load_pmc_traffic()
        line = {
            "metric": "RGB-D frames/sec (whole node) on 640x480 stream",
            "value": frames / dt, "unit": "frames/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic 640x480 RGB-D stream (seeded), random-init weights, seeded scene detections",
            "config": {"workload": f"configs[2]: synthetic 640x480 RGB-D, batch {B}/step/GPU, gap=1, "
                                   f"CuTR ViT-{ {768: 'B', 384: 'S', 192: 'T'}.get(args.dim, args.dim)} "
                                   f"RGB-D + CLIP ViT-H/14 x{args.crops} crops/frame + fusion",
                       "frames": frames, "global_batch": per_step, "parallelism": f"dp{N}",
                       "inflight_batches_per_gpu": n_inflight,
                       "fused_boxes": fusion.stats["fused"],
                       "global_boxes": len(fusion.all_pred_box) if fusion.all_pred_box is not None else 0},
            "roofline": {"bound": "mfma", "kernel": "k_gemm256p<true,1> (persistent bf16 GEMM + bias + GELU: MLP up-projections of CLIP ViT-H and CuTR window blocks)",
                         "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_BF16_TFLOPS, "traffic": pmc.get("bytes_per_launch"),
                         "traffic_source": pmc.get("source"),
                         "launches": ks["launches"], "avg_us": ks.get("avg_us", 0.0),
                         "flops_per_launch": ks["flops"] / max(ks["launches"], 1),
                         "measured": ks["source"]},
        }
        if args.breakdown:
            line["breakdown_ms_per_step"] = {k: 1e3 * v / args.steps for k, v in brk.items()}
        if not args.no_cpu_baseline and N == 1:      # rank 0 at N=1 only (a reported baseline)
            line["cpu_baseline"] = cpu_baseline(cutr, clip_vis, args, scene)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
