"""One attention shape, one kernel variant, a few launches (for rocprofv3 --pmc passes).
usage: attn_one.py B H S D variant [iters]"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib
B, H, S, D, var = (int(x) for x in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
_lib.set_knobs(attn_variant=var)
qkv = torch.randn(B * S, 3 * H * D, device="cuda").bfloat16()
o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
for _ in range(iters):
    _lib.attention(q, k, v, o, B, H, S, S, D, D ** -0.5)
torch.cuda.synchronize()
print("done")
