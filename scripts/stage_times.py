"""Probe: GPU time of each stage of one bench-shaped detect step (batch 8, 640x480, CuTR ViT-B
RGB-D + 16 CLIP ViT-H/14 crops per frame), every stage captured in its own HIP graph and replayed
alone on one stream, so launch overhead is excluded and nothing overlaps.

    PYTHONPATH=. python scripts/stage_times.py [reps]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from boxfusion_amd import _lib  # noqa: E402
from boxfusion_amd.clip import VisionTransformer  # noqa: E402
from boxfusion_amd.cubify_transformer import FrameBatch, make_cubify_transformer  # noqa: E402
from boxfusion_amd.pipeline import DetectStage  # noqa: E402
from boxfusion_amd.synthetic import SCANNET_K, Scene  # noqa: E402


def gtime(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    only = sys.argv[2] if len(sys.argv) > 2 else None      # time one stage (for a kernel trace)
    dev = torch.device("cuda")
    _lib.lib()
    torch.manual_seed(0)
    with torch.device(dev):
        cutr = make_cubify_transformer(768, True).eval()
        vis = VisionTransformer(224, 14, 1280, 32, 16, 1024).eval()
    B, H, W = 8, 480, 640
    det = DetectStage(cutr, vis, bench.CFG, B, H, W, SCANNET_K, crops_per_frame=16,
                      crop_source="top", clip_capacity=B * 16, device=dev)
    rgb, depth = bench.gen_frames(list(range(B)), dev)
    poses = np.stack([Scene(seed=0).pose(f) for f in range(B)])
    det(rgb, depth, poses, return_instances=False)
    torch.cuda.synchronize()
    eng = det.cutr
    t = {}

    def st(fn, reps):
        return gtime(fn, reps) if only is None else 0.0

    t["depth_standardize"] = st(lambda: _lib.depth_standardize(det.in_depth), reps)
    t["backproject_x8"] = st(lambda: [_lib.backproject(det.in_depth[b], det.K_dev[b], det.in_pose[b])
                                         for b in range(B)], reps)
    dstd, params = _lib.depth_standardize(det.in_depth)
    t["cutr_backbone"] = st(lambda: eng.backbone(det.in_rgb, dstd), reps)
    feat = eng.backbone(det.in_rgb, dstd).clone()
    pos = eng.positions(det.K_host, [(H, W)] * B)
    batch = FrameBatch(image=None, depth=dstd, depth_params=params, K=det.K_dev, T_gravity=det.in_Tg,
                       image_sizes=[(H, W)] * B, pad=eng.P, K_inv=det.Kinv_dev)
    dec = lambda: eng.model.decode(feat, batch, pos=pos)
    t["cutr_decode_torch"] = st(dec, reps) if only != "decode_torch" else gtime(dec, reps)
    if eng.decoder is not None:
        rows = feat.permute(0, 2, 3, 1).reshape(B * eng.T, eng.C).contiguous()
        npos = eng.decoder.positions(det.K_host, [(W, H)] * B)
        ndec = lambda: eng.decoder(rows, npos, params, det.Kinv_dev, det.in_Tg, [(H, W)] * B, (eng.P, eng.P))
        t["cutr_decode"] = st(ndec, reps) if only != "decode" else gtime(ndec, reps)
    boxes = det.out["boxes2d"][det.top_b, det.top_i].contiguous()
    t["clip_text_prompt_128"] = st(lambda: det.text_prompt(det.in_rgb, boxes, det.top_b32), reps)
    t["detect_step_total"] = st(lambda: det._device_forward(), reps)
    out = {k: round(v, 3) for k, v in t.items()}
    out["sum_of_stages"] = round(sum(v for k, v in t.items() if k != "detect_step_total"), 3)
    print(json.dumps({"stage_ms": out}))


if __name__ == "__main__":
    main()
