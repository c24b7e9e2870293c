"""The fp8 CLIP engine's four GEMMs (engine.py:390-412) as it calls them -- qkv fp8 -> bf16, proj fp8 ->
f32 + resid (in place), fc1 fp8 -> GELU -> fp8, fc2 fp8 -> f32 + resid -- at CLIP's 128-crop shape,
beside the same shapes without the residual / with a bf16 output, and under GEMM variant 6 (the
overlapped-epilogue kernel for every eligible shape).  TF/s against the 5 PF fp8 dense peak."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

M = 32896
L = _lib.lib()
F8 = _lib.FP8


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def mk(r, c):
    return (torch.randn(r, c, device="cuda") * 0.5).to(F8)


cases = []
for name, N, K in (("qkv", 3840, 1280), ("proj", 1280, 1280), ("fc1", 5120, 1280), ("fc2", 1280, 5120)):
    a, w = mk(M, K), mk(N, K)
    bias = torch.randn(N, device="cuda")
    X = torch.randn(M, N, device="cuda")
    ob = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    o8 = torch.empty(M, N, device="cuda", dtype=F8)
    of = torch.empty(M, N, device="cuda")
    sc = 1.0 / math.sqrt(K)
    if name == "qkv":
        forms = {"engine(bf16 out)": lambda: _lib.gemm_fp8(a, w, sc, bias=bias, out=ob)}
    elif name == "fc1":
        forms = {"engine(gelu fp8 out)": lambda: _lib.gemm_fp8(a, w, sc, bias=bias, act="gelu", out=o8, out_qscale=4.0),
                 "gelu bf16 out": lambda: _lib.gemm_fp8(a, w, sc, bias=bias, act="gelu", out=ob)}
    else:
        forms = {"engine(f32 + resid)": lambda: _lib.gemm_fp8(a, w, sc, bias=bias, resid=X, out=X),
                 "f32 no resid": lambda: _lib.gemm_fp8(a, w, sc, bias=bias, out=of),
                 "bf16 out": lambda: _lib.gemm_fp8(a, w, sc, bias=bias, out=ob)}
    fl = 2.0 * M * N * K
    for v in (5, 6):
        _lib.set_knobs(variant=v)
        for k, f in forms.items():
            ts = sorted(bench(f) for _ in range(3))
            print(f"{name:5s} variant {v} {k:22s} {ts[1]:7.1f} us {fl / ts[1] / 1e6:6.0f} TF  frac {fl / ts[1] / 1e6 / 5000:.3f}",
                  flush=True)
    _lib.set_knobs(variant=5)
