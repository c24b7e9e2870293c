"""Split-K tail of the residual GEMMs (bf_gemm_bf16_ws) against the balanced unsplit grid, same
operands, interleaved.  python scripts/gemm_splitk_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


dev = torch.device("cuda")
ws = _lib.new_gemm_workspace(dev)
L = _lib.lib()
for (M, N, K, name) in [(32896, 1280, 1280, "CLIP out_proj"), (32896, 1280, 5120, "CLIP c_proj"),
                        (12800, 768, 3072, "CuTR fc2"), (12800, 768, 768, "CuTR proj")]:
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
    b = torch.randn(N, device=dev)
    x = torch.randn(M, N, device=dev)
    res = {}
    for rep in range(2):
        for mode in (0, 1, 2):
            L.bf_gemm_set_splitk(mode)
            t = timeit(lambda: _lib.gemm(a, w, b, resid=x, out=x, ws=ws))
            res.setdefault(mode, []).append(t)
    L.bf_gemm_set_splitk(1)
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    fl = 2.0 * M * N * K
    print(f"{name:14s} M={M} N={N} K={K} tiles={tiles}: " + "  ".join(
        f"splitk={m} {min(v):7.1f} us ({fl / min(v) / 1e6:6.1f} TF/s)" for m, v in res.items()), flush=True)
