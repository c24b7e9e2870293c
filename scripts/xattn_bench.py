"""Microbenchmark of the decoder's fused RPE cross-attention (bf_xattn_f32) at the decoder shape
(8 frames x 302 queries x 8 heads x 32 dims over a 40x40 memory)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

dev = torch.device("cuda")
B, Nq, q0, H, hh, ww = 8, 302, 2, 8, 40, 40
C = H * 32
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, Nq, C, device=dev, generator=g)
k = torch.randn(B, hh * ww, C, device=dev, generator=g)
v = torch.randn(B, hh * ww, C, device=dev, generator=g)
rx = torch.randn(B, Nq - q0, ww, H, device=dev, generator=g)
ry = torch.randn(B, Nq - q0, hh, H, device=dev, generator=g)
out = _lib.xattn(q, k, v, rx, ry, hh, ww, q0, H, 32 ** -0.5)
for _ in range(3):
    _lib.xattn(q, k, v, rx, ry, hh, ww, q0, H, 32 ** -0.5, out=out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    _lib.xattn(q, k, v, rx, ry, hh, ww, q0, H, 32 ** -0.5, out=out)
e1.record()
torch.cuda.synchronize()
print(f"xattn: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us"
      f"  checksum {out.double().sum().item():.6f}", flush=True)
