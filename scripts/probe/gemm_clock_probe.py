"""In-kernel clock of k_gemm256q per GEMM form (diagnostic build with GEMM_STAMP=1: per-workgroup
s_memtime / s_memrealtime at entry and exit; clock = d(memtime) / d(realtime) x 100 MHz, the
guide's method).  Each form runs back to back for ~1.5 s before the stamps of its last launch are
read.  Stamp build (here, before the GPU call; same recipe as scripts/gemm_abl_probe.sh):
  cd boxfusion_amd && mkdir -p _build/variant &&
  hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c csrc/bf_gemm.hip -o _build/variant/bf_gemm_stamp.o -DGEMM_STAMP=1 &&
  hipcc --offload-arch=gfx950 -shared -fPIC -o _build/variant/lib_stamp.so $(ls _build/*.o | grep -v /bf_gemm.o) _build/variant/bf_gemm_stamp.o
usage: BF_LIB_PATH=boxfusion_amd/_build/variant/lib_stamp.so python scripts/probe/gemm_clock_probe.py"""
import ctypes
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from boxfusion_amd import _lib  # noqa: E402

L = _lib.lib()
vp = ctypes.c_void_p
st = vp(torch.cuda.current_stream().cuda_stream)
buf = (ctypes.c_ulonglong * (4096 * 4))()
for name, M, N, K in (("clip_proj", 32896, 1280, 1280), ("clip_fc2", 32896, 1280, 5120), ("clip_qkv", 32896, 3840, 1280)):
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    bias = torch.randn(N, device="cuda")
    x = torch.randn(M, N, device="cuda")
    y = torch.empty(M, N, device="cuda")
    yb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    g = lambda r, c, ob: L.bf_gemm_bf16(vp(a.data_ptr()), K, vp(w.data_ptr()), K, vp(bias.data_ptr()),
                                        vp(r.data_ptr()) if r is not None else None, N, 0, vp(c.data_ptr()), N, ob,
                                        None, M, N, K, 0, st)
    forms = {"bf16 out": lambda: g(None, yb, 1)}
    if N == 1280:
        forms = {"f32 + resid": lambda: g(x, x, 0), "f32 out": lambda: g(None, y, 0), **forms}
    for k, f in forms.items():
        f()
        torch.cuda.synchronize()
        t0, n = time.time(), 0
        while time.time() - t0 < 1.5:
            for _ in range(10):
                f()
            torch.cuda.synchronize()
            n += 10
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3
        assert L.bf_gemm_read_stamps(buf, 4096) == 0
        v = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).astype(np.float64)
        v = v[(v[:, 1] > v[:, 0]) & (v[:, 3] > v[:, 2])]
        clk = (v[:, 1] - v[:, 0]) / (v[:, 3] - v[:, 2]) * 100.0        # MHz
        print(f"{name:10s} {k:12s} {us:7.1f} us  clock median {np.median(clk):6.0f} MHz "
              f"(p10 {np.percentile(clk, 10):6.0f}, p90 {np.percentile(clk, 90):6.0f}, {len(clk)} WGs, {n} warm launches)",
              flush=True)
        buf = (ctypes.c_ulonglong * (4096 * 4))()
        ctypes.memset(buf, 0, ctypes.sizeof(buf))
