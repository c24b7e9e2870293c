"""Kernel-by-kernel view of one eager detect step (batch 8): run under
`rocprofv3 --kernel-trace --output-format csv` and summarise with --summarise <kernel_trace.csv>.
Marks the CuTR decode phase with two tiny marker kernels (torch.zeros on a 7-element tensor)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if len(sys.argv) > 2 and sys.argv[1] == "--summarise":
    import csv
    import collections
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    # last detect step: between the last two "marker" pairs
    agg = collections.OrderedDict()
    t_first = int(rows[0]["Start_Timestamp"])
    for r in rows[-int(sys.argv[3]) if len(sys.argv) > 3 else 0:]:
        n = r["Kernel_Name"]
        key = n.split("(")[0][:70] + (" .. " + n[-70:] if "at::native" in n else "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c, t = agg.get(key, (0, 0.0))
        agg[key] = (c + 1, t + d)
    tot = sum(t for _, t in agg.values())
    print(f"total {tot:.1f} us")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{c:5d} {t:9.1f} us  {k}")
    sys.exit(0)

import torch
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
B = 8
det = DetectStage(cutr, vis, bench.CFG, B, 480, 640, SCANNET_K, crops_per_frame=16, crop_source="top",
                  clip_capacity=B * 16, device=dev, graph=False)
scene = Scene(seed=0)
rgb, depth = bench.gen_frames(list(range(B)), dev)
poses = [scene.pose(f) for f in range(B)]
for _ in range(3):
    det(rgb, depth, poses, return_instances=False)
torch.cuda.synchronize()
print("done", flush=True)
