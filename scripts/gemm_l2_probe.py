"""Is the persistent GEMM's K loop bound by operand-fetch latency?  Times bf_gemm_bf16 on the path's
shapes with real operands and with every A row (lda = 0) and / or every W row (ldw = 0) aliased to
one row, so the aliased operand is L2-resident after the first K-tile; the MFMA work is identical."""
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib  # noqa: E402

SHAPES = [("clip_qkv", 32896, 3840, 1280, 1), ("clip_fc2", 32896, 1280, 5120, 0),
          ("clip_fc1", 32896, 5120, 1280, 1), ("clip_proj", 32896, 1280, 1280, 0),
          ("cutr_w_fc2", 25600, 768, 3072, 0), ("cutr_g_fc2", 12800, 768, 3072, 0), ("sq4096", 4096, 4096, 4096, 1)]


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


L = _lib.lib()
for name, M, N, K, ob in SHAPES:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if ob else torch.float32)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run(lda, ldw):
        return lambda: L.bf_gemm_bf16(ctypes.c_void_p(a.data_ptr()), lda, ctypes.c_void_p(w.data_ptr()), ldw,
                                      None, None, 0, 0, ctypes.c_void_p(out.data_ptr()), N, ob, None, M, N, K, 0, st)
    res = {}
    for rnd in range(3):
        for tag, lda, ldw in (("real", K, K), ("both_l2", 0, 0)):
            res.setdefault(tag, []).append(bench(run(lda, ldw)))
    fl = 2.0 * M * N * K
    print(f"{name:11s} " + " | ".join(f"{t} {sorted(v)[1]:7.1f} us {fl / sorted(v)[1] / 1e6:5.0f} TF"
                                       for t, v in res.items()), flush=True)
