"""Attention microbenchmark on the path's shapes (TFLOP/s of 4*Sq*Sk*D per head)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

SHAPES = [("clip", 128, 16, 257, 80), ("cutr_win", 72, 12, 512, 64), ("cutr_glob", 8, 12, 1600, 64)]
dev = torch.device("cuda")
for name, B, H, S, D in SHAPES:
    qkv = torch.randn(B * S, 3 * H * D, device=dev).bfloat16()
    o = torch.empty(B * S, H * D, device=dev, dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    f = lambda: _lib.attention(q, k, v, o, B, H, S, S, D, D ** -0.5)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    fl = 4.0 * B * H * S * S * D
    qq = q.view(B, S, H, D).transpose(1, 2)
    kk = k.view(B, S, H, D).transpose(1, 2)
    vv = v.view(B, S, H, D).transpose(1, 2)
    t = lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv)
    for _ in range(3):
        t()
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        t()
    e.record()
    torch.cuda.synchronize()
    mt = s.elapsed_time(e) / 20
    print(f"{name:10s} B={B} H={H} S={S} D={D}: ours {ms*1e3:8.1f} us {fl/ms/1e9:7.1f} TF/s | torch sdpa {mt*1e3:8.1f} us {fl/mt/1e9:7.1f} TF/s", flush=True)
