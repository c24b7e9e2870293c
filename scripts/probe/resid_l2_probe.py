"""Is the f32-residual GEMM's extra time the residual's HBM fetch or the kernel's wait structure?
C f32 = resid + A W^T + b with C separate from resid: resid rows from HBM (ldr = N) against every row
aliased to one L2-resident row (ldr = 0; same instructions and counted waits), and no residual."""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

SHAPES = [("clip_proj", 32896, 1280, 1280), ("clip_fc2", 32896, 1280, 5120), ("cutr_g_proj", 12800, 768, 768),
          ("cutr_w_fc2", 25600, 768, 3072)]
L = _lib.lib()
vp = ctypes.c_void_p


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


for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    bias = torch.randn(N, device="cuda")
    x = torch.randn(M, N, device="cuda")
    y = torch.empty(M, N, device="cuda")
    st = vp(torch.cuda.current_stream().cuda_stream)
    g = lambda r, ldr: L.bf_gemm_bf16(vp(a.data_ptr()), K, vp(w.data_ptr()), K, vp(bias.data_ptr()),
                                      vp(r.data_ptr()) if r is not None else None, ldr, 0, vp(y.data_ptr()), N, 0,
                                      None, M, N, K, 0, st)
    fns = {"resid_hbm": lambda: g(x, N), "resid_l2": lambda: g(x, 0), "inplace": lambda: L.bf_gemm_bf16(
        vp(a.data_ptr()), K, vp(w.data_ptr()), K, vp(bias.data_ptr()), vp(x.data_ptr()), N, 0, vp(x.data_ptr()), N, 0,
        None, M, N, K, 0, st), "no_resid": lambda: g(None, 0)}
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            res[k].append(bench(f))
    print(f"{name:12s} " + " | ".join(f"{k} {sorted(v)[1]:6.1f}" for k, v in res.items()), flush=True)
