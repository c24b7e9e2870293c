"""Per-tile fixed cost of bf_gemm_bf16: time vs K at fixed M, N (linear fit a + b*K)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib
dev = torch.device("cuda")
M, N = 32896, 3840
for act, ob in ((None, True), ("gelu", True), (None, False)):
    for K in (64, 128, 256, 640, 1280, 2560):
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        out = torch.empty((M, N), device=dev, dtype=torch.bfloat16 if ob else torch.float32)
        f = lambda: _lib.gemm(a, w, None, act=act, out=out)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        print(f"act={act} bf16={ob} K={K:5d}: {ms*1e3:8.1f} us  {2*M*N*K/ms/1e9:7.1f} TF/s", flush=True)
