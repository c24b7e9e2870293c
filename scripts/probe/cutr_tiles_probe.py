"""CuTR's K = 768 GEMMs: the per-shape tile height (auto) against forced 256 / 160 rows and the 128x128
kernel (_lib.set_knobs(kernel=...)), in rotating order (auto measured last in odd rounds)."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

SHAPES = [("cutr_g_qkv", 12800, 2304, 768, None), ("cutr_g_fc1", 12800, 3072, 768, "gelu"),
          ("cutr_w_fc1", 25600, 3072, 768, "gelu"), ("cutr_w_qkv", 36864, 2304, 768, None)]
L = _lib.lib()


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
    return s.elapsed_time(e) / iters * 1e3


for name, M, N, K, act in SHAPES:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    bias = torch.randn(N, device="cuda")
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fn = lambda: _lib.gemm(a, w, bias, act=act, out=out)
    modes = {"auto": (0, 0), "256": (256, 0), "160": (160, 0), "128x128": (0, 1)}
    res = {k: [] for k in modes}
    keys = list(modes)
    for rnd in range(4):
        for k in (keys if rnd % 2 == 0 else keys[::-1]):
            _lib.set_knobs(tile_rows=modes[k][0])
            _lib.set_knobs(kernel=modes[k][1])
            res[k].append(bench(fn))
    _lib.set_knobs(tile_rows=0)
    _lib.set_knobs(kernel=0)
    ref = (a.float() @ w.float().T)
    print(f"{name:11s} " + " | ".join(f"{k} {sorted(v)[1]:6.1f} ({min(v):.1f}-{max(v):.1f})" for k, v in res.items()), flush=True)
