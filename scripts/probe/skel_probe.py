"""Skeleton probe (scripts/probe/skel.hip): TF/s of the 8-wave MFMA + barrier skeleton per section size."""
import ctypes
import os
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = ctypes.CDLL(os.path.join(ROOT, "boxfusion_amd/_build/probe/skel.so"))
out = torch.empty(256 * 512, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
ITERS = 400
for rnd, seed in ((0, 0.001), (1, 0.001), (2, -1.0), (3, -1.0), (4, 0.001)):
    for v in (0, 64, 32, 16, 8):
        f = lambda: P.skel_launch(v, ctypes.c_void_p(out.data_ptr()), 256, ITERS, ctypes.c_float(seed), st)
        assert f() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 5 * 1e3
        flops = 256 * 8 * ITERS * 64 * (16 * 16 * 32 * 2)
        print(f"round {rnd} {'random' if seed < 0 else 'smooth'} section {v if v else 'no barriers':>11}: {us:8.1f} us  {flops / us / 1e6:7.0f} TF/s", flush=True)
