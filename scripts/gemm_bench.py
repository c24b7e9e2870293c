"""GEMM microbenchmark: bf_gemm_bf16 vs torch (hipBLASLt) on the path's shapes (TFLOP/s)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

SHAPES = [  # (name, M, N, K, act, out_bf16)
    ("clip_fc1", 32896, 5120, 1280, "gelu", True),
    ("clip_fc2", 32896, 1280, 5120, None, False),
    ("clip_qkv", 32896, 3840, 1280, None, True),
    ("clip_proj", 32896, 1280, 1280, None, False),
    ("cutr_qkv_win", 36864, 2304, 768, None, True),
    ("cutr_fc1", 25600, 3072, 768, "gelu", True),
    ("cutr_fc2", 25600, 768, 3072, None, False),
    ("sq4096", 4096, 4096, 4096, None, True),
]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = torch.device("cuda")
for name, M, N, K, act, ob in SHAPES:
    a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
    bias = torch.zeros(N, device=dev)
    out = torch.empty((M, N), device=dev, dtype=torch.bfloat16 if ob else torch.float32)
    ms = bench(lambda: _lib.gemm(a, w, bias, act=act, out=out))
    ref = a[:512].float() @ w.float().T
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    err = ((out[:512].float() - ref).norm() / ref.norm()).item()
    ms_t = bench(lambda: torch.nn.functional.linear(a, w))
    fl = 2.0 * M * N * K
    print(f"{name:14s} M={M:6d} N={N:5d} K={K:5d}  ours {ms*1e3:8.1f} us {fl/ms/1e9:7.1f} TF/s   "
          f"torch {ms_t*1e3:8.1f} us {fl/ms_t/1e9:7.1f} TF/s  err {err:.1e}", flush=True)
