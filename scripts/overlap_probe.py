"""Probe: throughput of the detect step (CuTR ViT-B + 16 CLIP crops/frame, batch 8) with one
stream vs two independent DetectStage graphs replayed concurrently on two streams.  If two
concurrent replays finish faster than two sequential ones, overlapping CLIP(step s) with
CuTR(step s+1) is worth building."""
import os
import sys
import time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from boxfusion_amd import _lib
from boxfusion_amd.clip import VisionTransformer
from boxfusion_amd.cubify_transformer import make_cubify_transformer
from boxfusion_amd.pipeline import DetectStage
from boxfusion_amd.synthetic import SCANNET_K, Scene

dev = torch.device("cuda")
_lib.lib()
torch.manual_seed(0)
with torch.device(dev):
    cutr = make_cubify_transformer(768, True).eval()
    vis = VisionTransformer(224, 14, 1280, 32, 16, 1024).eval()
scene = Scene(seed=0)
B = 8
dets = [DetectStage(cutr, vis, bench.CFG, B, 480, 640, SCANNET_K, crops_per_frame=16,
                    crop_source="top", clip_capacity=B * 16, device=dev, graph=True) for _ in range(2)]
rgb, depth = bench.gen_frames(list(range(B)), dev)
poses = [scene.pose(f) for f in range(B)]
for d in dets:
    for _ in range(2):
        d(rgb, depth, poses, return_instances=False)
torch.cuda.synchronize()
streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
N = 20
# sequential: 2N replays on one stream
t0 = time.perf_counter()
for i in range(2 * N):
    dets[i % 2](rgb, depth, poses, return_instances=False)
torch.cuda.synchronize()
t_seq = time.perf_counter() - t0
# concurrent: N replays on each of two streams
t0 = time.perf_counter()
for i in range(N):
    for k in range(2):
        with torch.cuda.stream(streams[k]):
            dets[k](rgb, depth, poses, return_instances=False)
torch.cuda.synchronize()
t_con = time.perf_counter() - t0
print(f"sequential {1e3 * t_seq / (2 * N):.2f} ms/step, two streams {1e3 * t_con / (2 * N):.2f} ms/step "
      f"-> {t_seq / t_con:.3f}x", flush=True)
