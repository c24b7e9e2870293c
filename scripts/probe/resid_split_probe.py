"""Where does the f32-residual GEMM's extra time go?  The path's residual shapes through bf_gemm_bf16:
C f32 = A W^T + b against C f32 = resid + A W^T + b (in place), the latter at the start-skew settings
given as arguments (units,groups; needs a build exporting bf_gemm_set_skew -- the round-5 experiment,
not kept: profiles/r05_resid_skew_probe.log)."""
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
# start-skew settings (units of ~512 cycles, groups) for the residual form
SKEWS = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(0, 4)]
if not hasattr(L, "bf_gemm_set_skew"):
    SKEWS = [(0, 4)]
    L.bf_gemm_set_skew = lambda u, g: None
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
    yb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    st = vp(torch.cuda.current_stream().cuda_stream)
    g = lambda r, c, ob: L.bf_gemm_bf16(vp(a.data_ptr()), K, vp(w.data_ptr()), K, vp(bias.data_ptr()),
                                        vp(r.data_ptr()) if r is not None else None, N, 0, vp(c.data_ptr()), N, ob,
                                        None, M, N, K, 0, st)
    fns = {"f32": lambda: g(None, y, 0)}
    for sk in SKEWS:
        def f(sk=sk):
            L.bf_gemm_set_skew(sk[0], sk[1])
            return g(x, x, 0)
        fns[f"resid_s{sk[0]}g{sk[1]}"] = f
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            res[k].append(bench(f))
    fl = 2.0 * M * N * K
    print(f"{name:12s} " + " | ".join(f"{k} {sorted(v)[1]:6.1f}" for k, v in res.items()), flush=True)
    L.bf_gemm_set_skew(0, 4)
