"""CLIP ViT-H GEMMs and the whole crop tower: bf16 vs fp8 (one MI355X), each GEMM under the GEMM
variants given (default: 1 = k_gemm256p, 5 = k_gemm256q for bf16 / fp8 outputs).
python scripts/fp8_bench.py [variant ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from boxfusion_amd import _lib


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


VARIANTS = [int(v) for v in sys.argv[1:]] or [1, 5]


def main():
    dev = torch.device("cuda")
    M = 128 * 257
    for name, N, K, act, ob, res in [("qkv", 3840, 1280, None, "bf16", False), ("fc1", 5120, 1280, "gelu", "fp8", False),
                                     ("fc2", 1280, 5120, None, "f32", True)]:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.05
        b = torch.randn(N, device=dev)
        x = torch.randn(M, N, device=dev)
        fl = 2.0 * M * N * K
        a16, w16 = a.bfloat16(), w.bfloat16()
        o16 = torch.empty(M, N, device=dev, dtype=torch.float32 if res else torch.bfloat16)
        a8, w8 = a.to(_lib.FP8), (w * 20).to(_lib.FP8)
        od = {"bf16": torch.bfloat16, "fp8": _lib.FP8, "f32": torch.float32}[ob]
        o8 = torch.empty(M, N, device=dev, dtype=od)
        msg = f"{name:4s} M={M} N={N} K={K}:"
        for var in VARIANTS:
            _lib.set_knobs(variant=var)
            t16 = timeit(lambda: _lib.gemm(a16, w16, b, act=act, resid=x if res else None, out=x if res else o16))
            t8 = timeit(lambda: _lib.gemm_fp8(a8, w8, 0.05, bias=b, act=act, resid=x if res else None,
                                              out=x if res else o8, out_qscale=0.1))
            msg += (f" | v{var} bf16 {t16:7.1f} us {fl / t16 / 1e6:7.1f} TF/s, "
                    f"fp8 {t8:7.1f} us {fl / t8 / 1e6:7.1f} TF/s ({t16 / t8:.2f}x)")
        _lib.set_knobs(variant=5)
        print(msg, flush=True)
    from boxfusion_amd.clip import VisionTransformer
    from boxfusion_amd.engine import CLIPEngine
    from boxfusion_amd.weights import init_seeded
    vis = init_seeded(VisionTransformer(224, 14, 1280, 32, 16, 1024).eval(), seed=3).to(dev)
    g = torch.Generator(device="cuda").manual_seed(5)
    frames = torch.randint(0, 256, (8, 480, 640, 3), device=dev, dtype=torch.uint8, generator=g)
    n = 128
    x1 = torch.randint(0, 400, (n,), device=dev, generator=g)
    y1 = torch.randint(0, 300, (n,), device=dev, generator=g)
    boxes = torch.stack([x1, y1, x1 + 100, y1 + 90], 1).to(torch.int32)
    idx = (torch.arange(n, device=dev) % 8).to(torch.int32)
    res = {}
    for fp8 in (False, True):
        eng = CLIPEngine(vis, n, fp8=fp8)
        eng(frames, boxes, idx)
        res[fp8] = timeit(lambda: eng(frames, boxes, idx), n=5)
    print(f"CLIP ViT-H/14 x {n} crops: bf16 {res[False] / 1e3:.2f} ms, fp8 {res[True] / 1e3:.2f} ms "
          f"({res[False] / res[True]:.2f}x); {n * 334.6e9 / (res[True] * 1e-6) / 1e12:.0f} TF/s effective fp8",
          flush=True)


if __name__ == "__main__":
    main()
