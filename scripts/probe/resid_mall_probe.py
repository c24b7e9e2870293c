"""Would a residual already in the Infinity Cache (256 MB MALL) help the f32-residual GEMMs?  Each
timed GEMM (C = X + A W^T + b, in place) runs right after either a full read of X (X warm in the
MALL) or a read of an unrelated 1 GB buffer (MALL flushed); only the GEMM is timed (events)."""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

SHAPES = [("clip_proj", 32896, 1280, 1280), ("clip_fc2", 32896, 1280, 5120), ("cutr_g_proj", 12800, 768, 768),
          ("cutr_g_fc2", 12800, 768, 3072), ("cutr_w_proj", 25600, 768, 768), ("cutr_w_fc2", 25600, 768, 3072)]
L = _lib.lib()
vp = ctypes.c_void_p
flush = torch.empty(256 * 1024 * 1024, device="cuda")          # 1 GB
sink = torch.empty(1, device="cuda")


def timed(pre, fn, iters=10):
    ts = []
    for i in range(iters + 2):
        pre()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    bias = torch.randn(N, device="cuda")
    x = torch.randn(M, N, device="cuda")
    st = vp(torch.cuda.current_stream().cuda_stream)
    g = lambda: L.bf_gemm_bf16(vp(a.data_ptr()), K, vp(w.data_ptr()), K, vp(bias.data_ptr()), vp(x.data_ptr()), N, 0,
                               vp(x.data_ptr()), N, 0, None, M, N, K, 0, st)
    warm = lambda: torch.sum(x.view(-1), 0, out=sink.view(()))
    cold = lambda: torch.sum(flush, 0, out=sink.view(()))
    both = lambda: (cold(), warm())
    r = {"cold": [], "x_warm": [], "x_warm_after_flush": []}
    for _ in range(3):
        r["cold"].append(timed(cold, g))
        r["x_warm"].append(timed(warm, g))
        r["x_warm_after_flush"].append(timed(both, g))
    print(f"{name:12s} X {M * N * 4 / 1e6:5.0f} MB | " + " | ".join(f"{k} {sorted(v)[1]:6.1f}" for k, v in r.items()),
          flush=True)
