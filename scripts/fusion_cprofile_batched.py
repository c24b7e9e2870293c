"""cProfile of the batched fusion path rank 0 runs at N=8 (bench.py: records of 64 keyframes per
step -> FusionStage.keyframes), host side, GPU otherwise idle.  Prints ms per keyframe and the
top functions."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from boxfusion_amd.fusion_stage import FusionStage  # noqa: E402
from boxfusion_amd.synthetic import SCANNET_K, Scene  # noqa: E402

dev = torch.device("cuda")
scene = Scene(seed=0)
PER = 64
steps = 6
recs = []
for s in range(steps + 1):
    fr = list(range(s * PER, (s + 1) * PER))
    recs.append(torch.from_numpy(bench.pack_records([scene.detections(f) for f in fr],
                                                    [scene.pose(f) for f in fr])).to(dev))


def run(st, r, base):
    p, c = bench.record_meta(r)
    st.keyframes([base + j for j in range(r.shape[0])], p, bench.unpack_records(r, c, dev), c)


st = FusionStage(bench.CFG, SCANNET_K, device=dev)
run(st, recs[0], 0)
torch.cuda.synchronize()
st = FusionStage(bench.CFG, SCANNET_K, device=dev)
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for s in range(steps):
    run(st, recs[s], s * PER)
torch.cuda.synchronize()
pr.disable()
dt = time.perf_counter() - t0
print(f"{1e3 * dt / (steps * PER):.3f} ms/keyframe (under cProfile)")
t0 = time.perf_counter()
st2 = FusionStage(bench.CFG, SCANNET_K, device=dev)
for s in range(steps):
    run(st2, recs[s], s * PER)
torch.cuda.synchronize()
print(f"{1e3 * (time.perf_counter() - t0) / (steps * PER):.3f} ms/keyframe (plain)")
ps = pstats.Stats(pr)
ps.sort_stats("tottime").print_stats(25)
ps.sort_stats("cumulative").print_stats(40)
