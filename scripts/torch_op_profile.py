"""Per-op device time of one eager detect step (bench workload, batch 8), torch.profiler.

Lists the torch / hipBLASLt ops (everything that is not one of our k_* kernels) by self device
time with input shapes and the Python line that issued them, to find what to fuse next.
  python scripts/torch_op_profile.py [--dim 768] [--batch 8]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--clip-layers", type=int, default=32)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    from bench import CFG, gen_frames
    from boxfusion_amd.clip import VisionTransformer
    from boxfusion_amd.cubify_transformer import make_cubify_transformer
    from boxfusion_amd.pipeline import DetectStage
    from boxfusion_amd.synthetic import SCANNET_K, Scene
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    with torch.device(dev):
        cutr = make_cubify_transformer(a.dim, True).eval()
        vis = VisionTransformer(224, 14, 1280, a.clip_layers, 16, 1024).eval()
    B = a.batch
    det = DetectStage(cutr, vis, CFG, B, 480, 640, SCANNET_K, crops_per_frame=16, crop_source="top",
                      backproject=True, clip_capacity=B * 16, device=dev, graph=False)
    scene = Scene(seed=0)
    rgb, depth = gen_frames(list(range(B)), dev)
    import numpy as np
    poses = np.stack([scene.pose(f) for f in range(B)]).astype(np.float32)
    for _ in range(3):
        det(rgb, depth, poses, return_instances=False)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        det(rgb, depth, poses, return_instances=False)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True, group_by_stack_n=4)
    rows = [e for e in ka if e.self_device_time_total > 0]
    rows.sort(key=lambda e: -e.self_device_time_total)
    tot = sum(e.self_device_time_total for e in rows)
    print(f"total self device time {tot / 1e3:.2f} ms")
    for e in rows[: a.top]:
        stack = " | ".join(s for s in (e.stack or []) if "boxfusion_amd" in s or "bench" in s)[:300]
        print(f"{e.self_device_time_total / 1e3:7.3f} ms {e.count:4d}x {e.key[:40]:40s} "
              f"{str(e.input_shapes)[:120]}  @ {stack}")


if __name__ == "__main__":
    main()
