"""Run one GEMM shape with one variant a few times (for rocprofv3 --pmc passes).
usage: gemm_one.py name variant[:group_m] [iters]"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from boxfusion_amd import _lib
from gemm_bench_shapes import SHAPES

name, v = sys.argv[1], sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
_, M, N, K, act, ob, use_resid = [s for s in SHAPES if s[0] == name][0]
L = _lib.lib()
vv, _, gm = v.partition(":")
_lib.set_knobs(variant=int(vv))
_lib.set_knobs(group_m=int(gm or 4))
dev = torch.device("cuda")
a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
bias = torch.rand(N, device=dev)
out = torch.empty((M, N), device=dev, dtype=torch.bfloat16 if ob else torch.float32)
resid = torch.rand((M, N), device=dev) if use_resid else None
for _ in range(iters):
    _lib.gemm(a, w, bias, act=act, resid=resid, out=out)
torch.cuda.synchronize()
print("done", name, v)
