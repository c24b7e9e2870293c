"""How much does the round quantisation cost the N=1280 residual GEMMs?  Time per 256x256 tile at
M giving 510 / 645 / 765 tiles (2 / 2.52 / 2.99 rounds on 256 CUs).  python scripts/gemm_tail_probe.py"""
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
for K in (1280, 5120):
    for M in (26112, 32896, 39168):
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(1280, K, device=dev) * 0.03).bfloat16()
        b = torch.randn(1280, device=dev)
        x = torch.randn(M, 1280, device=dev)
        tiles = ((M + 255) // 256) * 5
        for bal in (1, 0):
            _lib.set_knobs(balanced={1: 0, 0: 1, 2: 2}[bal])
            t = timeit(lambda: _lib.gemm(a, w, b, resid=x, out=x))
            print(f"K={K} M={M} tiles={tiles} balanced={bal}: {t:7.1f} us  {t / tiles * 256:6.1f} us per 256 tiles "
                  f"{2 * M * 1280 * K / t / 1e6:7.1f} TF/s", flush=True)
        _lib.set_knobs(balanced={1: 0, 0: 1, 2: 2}[1])
