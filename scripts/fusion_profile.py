"""Fusion chain cost per keyframe (gap=1 scene stream, GPU otherwise idle): wall time of each
phase of FusionStage.keyframe, synchronised."""
import os
import sys
import time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from boxfusion_amd.fusion_stage import FusionStage
from boxfusion_amd.pipeline import scene_instances
from boxfusion_amd.synthetic import SCANNET_K, Scene
from boxfusion_amd import instances as I, box_fusion as BF

dev = torch.device("cuda")
acc = {}


def timed(name, fn):
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
        return r
    return w


I.Instances3D.spatial_association = staticmethod(timed("spatial", I.Instances3D.spatial_association))
I.Instances3D.correspondence_association = staticmethod(timed("corr", I.Instances3D.correspondence_association))
BF.BoxFusion.boxfusion = timed("boxfusion", BF.BoxFusion.boxfusion)
scene = Scene(seed=0)
dets = [scene_instances(scene.detections(f), dev) for f in range(80)]
st = FusionStage(bench.CFG, SCANNET_K, device=dev)
for f in range(16):   # warm up
    st.keyframe(f, scene.pose(f), dets[f])
acc.clear()
st = FusionStage(bench.CFG, SCANNET_K, device=dev)
dets = [scene_instances(scene.detections(f), dev) for f in range(80)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for f in range(80):
    st.keyframe(f, scene.pose(f), dets[f])
torch.cuda.synchronize()
tot = time.perf_counter() - t0
print(f"fusion chain: {1e3 * tot / 80:.3f} ms/keyframe over 80 keyframes; "
      + ", ".join(f"{k} {1e3 * v / 80:.3f}" for k, v in acc.items()), flush=True)
print("stats", st.stats, "global boxes", len(st.all_pred_box))
