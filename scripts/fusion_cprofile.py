"""cProfile of the fusion chain (host side) over 60 gap=1 keyframes."""
import cProfile
import os
import pstats
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
from boxfusion_amd.fusion_stage import FusionStage
from boxfusion_amd.pipeline import scene_instances
from boxfusion_amd.synthetic import SCANNET_K, Scene
dev = torch.device("cuda")
scene = Scene(seed=0)
st = FusionStage(bench.CFG, SCANNET_K, device=dev)
for f in range(10):
    st.keyframe(f, scene.pose(f), scene_instances(scene.detections(f), dev))
st = FusionStage(bench.CFG, SCANNET_K, device=dev)
dets = [scene_instances(scene.detections(f), dev) for f in range(60)]
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for f in range(60):
    st.keyframe(f, scene.pose(f), dets[f])
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
pstats.Stats(pr).sort_stats("cumtime").print_stats(45)
pstats.Stats(pr).print_callers("index_select")
pstats.Stats(pr).print_callers("'cpu'")
