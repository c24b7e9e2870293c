"""bf_depth_standardize timing on the path's shapes (8 and 192 frames of 480x640, 192x256)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

for b, h, w in [(8, 480, 640), (192, 480, 640), (8, 256, 192)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    d = torch.rand((b, h, w), device="cuda", generator=g) * 4 + 0.5
    d[torch.rand((b, h, w), device="cuda", generator=g) < 0.05] = 0
    for _ in range(3):
        _lib.depth_standardize(d)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        _lib.depth_standardize(d)
    e.record()
    torch.cuda.synchronize()
    print(f"{b}x{h}x{w}: {s.elapsed_time(e) / 10 * 1e3:8.1f} us", flush=True)
