"""bf_nms_scan cost split: n boxes with no overlap (the greedy loop alone: n steps of compaction),
pairwise duplicates (n/2 suppressions through record()), and everything overlapping one box (n-1
suppressions in one step), timed with HIP events, lists of length 1, identity poses."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from boxfusion_amd import _lib  # noqa: E402

dev = torch.device("cuda")
cfg = _lib.NmsCfg()
cfg.iou_threshold, cfg.translation_gap, cfg.rotation_gap, cfg.center_gap = 0.1, 0.3, 20.0, 0.5
cfg.max_list, cfg.list_capacity = 5, 64


def run(iou, n, reps=50):
    corners = torch.rand((n, 8, 3), device=dev)
    scores = torch.linspace(1, 0.1, n, device=dev)
    init_id = torch.arange(n, dtype=torch.int32, device=dev)
    poses = torch.eye(4, device=dev).repeat(n, 1, 1).contiguous()
    times = []
    for r in range(reps + 3):
        items = torch.full((n, 64), -1, dtype=torch.int32, device=dev)
        items[:, 0] = torch.arange(n, dtype=torch.int32, device=dev)
        lens = torch.ones(n, dtype=torch.int32, device=dev)
        vn = torch.zeros(n, device=dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = _lib.nms_scan(iou, corners, scores, init_id, poses, items, lens, vn, cfg)
        e.record()
        torch.cuda.synchronize()
        if r >= 3:
            times.append(s.elapsed_time(e) * 1e3)
    c = out[3].cpu().tolist()
    return np.median(times), c


for n in (16, 40, 80):
    eye = torch.eye(n, dtype=torch.float64, device=dev)
    pairs = eye.clone()
    for i in range(0, n - 1, 2):
        pairs[i, i + 1] = pairs[i + 1, i] = 0.5
    allov = torch.full((n, n), 0.5, dtype=torch.float64, device=dev)
    for name, m in (("no overlap", eye), ("pairs", pairs), ("all overlap", allov)):
        t, c = run(m.contiguous(), n)
        print(f"n={n:3d} {name:12s}: {t:6.1f} us  (keep {c[0]}, success {c[1]}, events {c[2]})", flush=True)
