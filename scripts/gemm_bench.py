"""GEMM microbenchmark: bf_gemm_bf16 variants vs torch (hipBLASLt) on the path's shapes (TFLOP/s).

Variants (bf_gemm_set_variant) are timed interleaved in one process, several rounds, median kept.
usage: gemm_bench.py [variant[:group_m] ...]   (default: 0:1 1:4)
"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from boxfusion_amd import _lib

from gemm_bench_shapes import SHAPES  # noqa: E402


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
    return s.elapsed_time(e) / iters


def main():
    pass


args = sys.argv[1:] if __name__ == "__main__" else ["--only=__none__"]
only = None
if args and args[0].startswith("--only="):
    only = args[0][7:].split(",")
    args = args[1:]
variants = args or ["0:1", "1:4"]
L = _lib.lib()
dev = torch.device("cuda")
for name, M, N, K, act, ob, use_resid in SHAPES:
    if only and name not in only:
        continue
    a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
    bias = torch.rand(N, device=dev)
    out = torch.empty((M, N), device=dev, dtype=torch.bfloat16 if ob else torch.float32)
    resid = torch.rand((M, N), device=dev) if use_resid else None
    ref = a[:512].float() @ w.float().T + bias
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    if use_resid:
        ref = ref + resid[:512]
    times = {v: [] for v in variants}
    errs = {}
    for rnd in range(3):
        for v in variants:
            vv, _, gm = v.partition(":")
            _lib.set_knobs(variant=int(vv))
            _lib.set_knobs(group_m=int(gm or 4))
            times[v].append(bench(lambda: _lib.gemm(a, w, bias, act=act, resid=resid, out=out)))
            if rnd == 0:
                out.zero_()
                _lib.gemm(a, w, bias, act=act, resid=resid, out=out)
                torch.cuda.synchronize()
                errs[v] = ((out[:512].float() - ref).norm() / ref.norm()).item()
                # last rows too (partial tiles)
                r2 = a[-300:].float() @ w.float().T + bias
                if act == "gelu":
                    r2 = torch.nn.functional.gelu(r2)
                if use_resid:
                    r2 = r2 + resid[-300:]
                errs[v] = max(errs[v], ((out[-300:].float() - r2).norm() / r2.norm()).item())
    ms_t = bench(lambda: torch.nn.functional.linear(a, w))
    fl = 2.0 * M * N * K
    msg = f"{name:15s} M={M:6d} N={N:5d} K={K:5d} "
    for v in variants:
        ms = sorted(times[v])[1]
        msg += f"| {v} {ms*1e3:6.1f} us {fl/ms/1e9:5.0f} TF {errs[v]:.0e} "
    msg += f"| torch {ms_t*1e3:7.1f} us {fl/ms_t/1e9:6.0f} TF"
    print(msg, flush=True)
