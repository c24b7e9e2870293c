"""CLIP attention time vs number of workgroup rounds (B crops x 16 heads, 1 WG per (crop, head),
one WG per CU): slope = per-round cost, intercept = launch + ramp; and the same with the key loop
skipped (BF_ATTN_PROBE) to split load / compute."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

L = _lib.lib()
H, S, D = 16, 257, 80


def timeit(f, iters=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for var in [int(v) for v in sys.argv[1:]] or [6]:
    _lib.set_knobs(attn_variant=var)
    for B in (16, 32, 64, 128, 256):
        qkv = torch.randn(B * S, 3 * H * D, device="cuda").bfloat16()
        o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
        t = timeit(lambda: _lib.attention(q, k, v, o, B, H, S, S, D, D ** -0.5))
        print(f"v{var} B={B:4d} pairs={B * H:5d} rounds={B * H / 256:5.1f}: {t:7.1f} us  {t / (B * H / 256):6.2f} us/round",
              flush=True)
