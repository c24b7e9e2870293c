"""Residual GEMM epilogue A/B: accumulators initialised from the residual tile (default path) vs
residual loaded in the epilogue (forced with resid_mod = M + 1, same rows), vs no residual."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib

dev = torch.device("cuda")


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


for name, M, N, K in [("clip_proj", 32896, 1280, 1280), ("clip_fc2", 32896, 1280, 5120),
                      ("cutr_fc2", 25600, 768, 3072), ("cutr_proj_g", 12800, 768, 768)]:
    a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
    b = torch.rand(N, device=dev)
    r = torch.rand((M, N), device=dev)
    o1, o2 = torch.empty_like(r), torch.empty_like(r)
    _lib.gemm(a, w, b, resid=r, out=o1)
    _lib.gemm(a, w, b, resid=r, resid_mod=M + 1, out=o2)
    torch.cuda.synchronize()
    same = torch.equal(o1, o2)
    t = {}
    for rnd in range(3):
        for k, fn in [("acc_init", lambda: _lib.gemm(a, w, b, resid=r, out=o1)),
                      ("epi_load", lambda: _lib.gemm(a, w, b, resid=r, resid_mod=M + 1, out=o2)),
                      ("nores", lambda: _lib.gemm(a, w, b, out=o1))]:
            t.setdefault(k, []).append(bench(fn))
    fl = 2.0 * M * N * K
    print(f"{name:12s} " + " ".join(f"{k} {sorted(v)[1]:7.1f} us ({fl / sorted(v)[1] / 1e6:5.0f} TF)"
                                     for k, v in t.items()) + f" identical={same}", flush=True)
