"""Microbenchmark of the decoder bias kernels (bf_cpb_mlp, bf_rpe_softmax) at decoder shapes."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

dev = torch.device("cuda")
B, nq, n, hidden, heads = 8, 300, 40, 512, 8
ref = torch.rand(B, nq, 4, device=dev) * 640
pos = torch.linspace(0.5, n - 0.5, n, device=dev) * 16
w1, b1, w2 = (torch.randn(hidden, 2, device=dev), torch.randn(hidden, device=dev),
              torch.randn(heads, hidden, device=dev))
attn = torch.randn(B, heads, nq + 2, n * n, device=dev)
rx = _lib.cpb_mlp(ref, pos, 0, w1, b1, w2)
for name, fn in [("cpb_mlp", lambda: _lib.cpb_mlp(ref, pos, 0, w1, b1, w2)),
                 ("rpe_softmax", lambda: _lib.rpe_softmax(attn, rx, rx, n, n, 2))]:
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)
