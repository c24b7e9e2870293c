"""Probe: one-wave-per-SIMD 256x256 GEMM (4 waves x 128x128 accumulators held in AGPRs through
"+a"-constrained inline-asm MFMAs) against the shipped bf_gemm_bf16 on the path's shapes (bf16 out)."""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

SHAPES = [("clip_qkv", 32896, 3840, 1280), ("clip_fc2", 32896, 1280, 5120), ("clip_fc1", 32896, 5120, 1280),
          ("clip_proj", 32896, 1280, 1280), ("cutr_w_fc2", 25600, 768, 3072), ("sq4096", 4096, 4096, 4096),
          ("sq8192", 8192, 8192, 8192)]


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


L = _lib.lib()
VARIANTS = sys.argv[1:] or ["na32"]
PS = {v: ctypes.CDLL(os.path.join(ROOT, f"boxfusion_amd/_build/probe/gemm4w_{v}.so")) for v in VARIANTS}
vp = ctypes.c_void_p
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    o1 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)
    st = vp(torch.cuda.current_stream().cuda_stream)
    prod = lambda: L.bf_gemm_bf16(vp(a.data_ptr()), K, vp(w.data_ptr()), K, None, None, 0, 0, vp(o1.data_ptr()), N, 1,
                                  None, M, N, K, 0, st)
    fns = {"prod": prod}
    prod()
    same = []
    for v, P in PS.items():
        fns[v] = (lambda P=P: P.gemm4w_launch(vp(a.data_ptr()), K, vp(w.data_ptr()), K, vp(o2.data_ptr()), N, M, N, K, st))
        o2.zero_()
        assert fns[v]() == 0
        torch.cuda.synchronize()
        same.append(f"{v}={'eq' if torch.equal(o1, o2) else 'DIFF'}")
    res = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            res[k].append(bench(f))
    fl = 2.0 * M * N * K
    print(f"{name:11s} {' '.join(same)} | " + " | ".join(
        f"{t} {sorted(v)[1]:7.1f} us {fl / sorted(v)[1] / 1e6:5.0f} TF" for t, v in res.items()), flush=True)
