"""128x128 vs 256x256 kernel on the CuTR / CLIP shapes (_lib.set_knobs(kernel=1 / -1))."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from boxfusion_amd import _lib
from gemm_bench_shapes import SHAPES
from gemm_bench import bench  # noqa: F401  (re-used timing helper)

L = _lib.lib()
dev = torch.device("cuda")
extra = [("cutr_proj", 25600, 768, 768, None, False, True), ("cutr_qkv_glb", 25600, 2304, 768, None, True, False),
         ("cutr_g_qkv", 12800, 2304, 768, None, True, False), ("cutr_g_proj", 12800, 768, 768, None, False, True),
         ("cutr_g_fc1", 12800, 3072, 768, "gelu", True, False), ("cutr_g_fc2", 12800, 768, 3072, None, False, True)]
for name, M, N, K, act, ob, use_resid in SHAPES + extra:
    if not name.startswith(("cutr", "clip")):
        continue
    a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
    bias = torch.rand(N, device=dev)
    out = torch.empty((M, N), device=dev, dtype=torch.bfloat16 if ob else torch.float32)
    resid = torch.rand((M, N), device=dev) if use_resid else None
    res = []
    for f in (1, -1, 0):
        _lib.set_knobs(kernel=f)
        t = min(bench(lambda: _lib.gemm(a, w, bias, act=act, resid=resid, out=out)) for _ in range(3))
        res.append(f"{ {1: 'small', -1: 'large', 0: 'auto'}[f]} {t * 1e3:6.1f} us {2 * M * N * K / t / 1e9:5.0f} TF")
    _lib.set_knobs(kernel=0)
    print(f"{name:14s} M={M} N={N} K={K} | " + " | ".join(res), flush=True)
