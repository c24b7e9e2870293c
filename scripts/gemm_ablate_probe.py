"""Per-tile cost split of the persistent GEMM on the CLIP shapes: full kernel, no global stores
(bf_gemm_set_variant 4), no epilogue at all (variant 3), and the K=1280 vs K=5120 K-loop rate.
python scripts/gemm_ablate_probe.py"""
import torch

from boxfusion_amd import _lib


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


dev = torch.device("cuda")
L = _lib.lib()
M = 32896
for name, N, K, act in [("qkv", 3840, 1280, None), ("fc1", 5120, 1280, "gelu"), ("fc2nores", 1280, 5120, None),
                        ("k640", 3840, 640, None), ("k2560", 3840, 2560, None)]:
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
    b = torch.randn(N, device=dev)
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    msg = f"{name:8s} N={N} K={K} tiles={tiles}:"
    for var, lab in [(1, "full"), (4, "nostore"), (3, "noepi")]:
        _lib.set_knobs(variant=var)
        t = timeit(lambda: _lib.gemm(a, w, b, act=act, out=o))
        rounds = (tiles + 255) // 256
        msg += f" {lab} {t:7.1f} us ({t / rounds:5.1f} us/round)"
    _lib.set_knobs(variant=1)
    print(msg, flush=True)
