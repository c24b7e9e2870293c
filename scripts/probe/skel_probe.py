"""Skeleton probe (scripts/probe/skel.hip): TF/s and in-kernel clock of the 8-wave MFMA + barrier
skeleton per section size, on 16x16x32 and on 32x32x16 MFMAs (variants 1xx)."""
import ctypes
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = ctypes.CDLL(os.path.join(ROOT, "boxfusion_amd/_build/probe/skel.so"))
out = torch.empty(256 * 512, device="cuda")
stamps = torch.zeros(256 * 2, device="cuda", dtype=torch.int64)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
ITERS = 400
for rnd, seed in ((0, 0.001), (1, -1.0), (2, -1.0), (3, 0.001)):
    for v in (0, 64, 16, 100, 164, 116):
        f = lambda: P.skel_launch(v, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stamps.data_ptr()), 256, ITERS,
                                  ctypes.c_float(seed), st)
        for _ in range(20):      # ~0.1 s of the same variant before timing
            f()
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
        d = stamps.view(256, 2).cpu().numpy().astype(np.float64)
        mhz = np.median(d[:, 0] / d[:, 1] * 100.0)
        sec = v % 100 if v % 100 else "no barriers"
        print(f"round {rnd} {'random' if seed < 0 else 'smooth'} {'32x32x16' if v >= 100 else '16x16x32'} section {sec:>11}: "
              f"{us:8.1f} us  {flops / us / 1e6:7.0f} TF/s  clock {mhz:5.0f} MHz", flush=True)
