"""Diagnostic: capture the detect stage into a HIP graph (small models) and report the first op
that breaks capture, with its Python stack."""
import os
import sys
import traceback
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd.clip import VisionTransformer
from boxfusion_amd.cubify_transformer import make_cubify_transformer
from boxfusion_amd.pipeline import DetectStage
from boxfusion_amd.synthetic import SCANNET_K, Scene
from tests.trace_util import SCANNET_CFG
dev = torch.device("cuda")
torch.manual_seed(0)
with torch.device(dev):
    cutr = make_cubify_transformer(192, True).eval()
    vis = VisionTransformer(224, 14, 1280, 2, 16, 1024).eval()
d = DetectStage(cutr, vis, SCANNET_CFG, 2, 480, 640, SCANNET_K, crop_source="top", crops_per_frame=4,
                clip_capacity=8, device=dev, graph=True)
rgb = torch.randint(0, 255, (2, 480, 640, 3), dtype=torch.uint8, device=dev)
depth = torch.rand((2, 480, 640), device=dev) * 4
try:
    d(rgb, depth, np.stack([Scene().pose(f) for f in range(2)]), return_instances=False)
    torch.cuda.synchronize()
    print("capture OK")
except Exception:
    traceback.print_exc()
    sys.exit(1)
