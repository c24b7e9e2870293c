"""Tile-height sweep of the persistent GEMM (bf_gemm_set_tile_rows 160 / 192 / 224 / 256, 0 = the
per-shape model) on the path's shapes, interleaved in one process, median of 3 rounds; torch's
F.linear (hipBLASLt, plain bf16 output, no residual) beside it for reference only.
usage: gemm_tile_sweep.py [--fp8] [name ...]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from boxfusion_amd import _lib  # noqa: E402

SHAPES = [  # name, M, N, K, act, out_bf16, resid
    ("clip_qkv", 32896, 3840, 1280, None, True, False),
    ("clip_proj", 32896, 1280, 1280, None, False, True),
    ("clip_fc1", 32896, 5120, 1280, "gelu", True, False),
    ("clip_fc2", 32896, 1280, 5120, None, False, True),
    ("clip_outproj", 128, 1024, 1280, None, False, False),
    ("clip_cls_fc1", 128, 5120, 1280, "gelu", True, False),
    ("clip_cls_fc2", 128, 1280, 5120, None, False, True),
    ("cutr_g_qkv", 12800, 2304, 768, None, True, False),
    ("cutr_g_proj", 12800, 768, 768, None, False, True),
    ("cutr_g_fc1", 12800, 3072, 768, "gelu", True, False),
    ("cutr_g_fc2", 12800, 768, 3072, None, False, True),
    ("cutr_w_qkv", 36864, 2304, 768, None, True, False),
    ("cutr_w_proj", 25600, 768, 768, None, False, True),
    ("cutr_w_fc1", 25600, 3072, 768, "gelu", True, False),
    ("cutr_w_fc2", 25600, 768, 3072, None, False, True),
]


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


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    fp8 = "--fp8" in sys.argv
    L = _lib.lib()
    dev = torch.device("cuda")
    heights = [0] if "--auto-only" in sys.argv else [0, 160, 192, 224, 256]
    for name, M, N, K, act, ob, use_resid in SHAPES:
        if args and name not in args:
            continue
        if fp8 and M < 1024:
            continue
        g = torch.Generator(device="cuda").manual_seed(1)
        a = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).bfloat16()
        bias = torch.randn(N, device=dev, generator=g)
        resid = torch.randn(M, N, device=dev, generator=g) if use_resid else None
        out = torch.empty((M, N), device=dev, dtype=torch.bfloat16 if ob else torch.float32)
        if fp8:
            a8, w8 = a.to(_lib.FP8), w.to(_lib.FP8)
            fn = lambda: _lib.gemm_fp8(a8, w8, 0.5, bias, act=act, resid=resid, out=out)
        else:
            fn = lambda: _lib.gemm(a, w, bias, act=act, resid=resid, out=out)
        times = {h: [] for h in heights}
        ref = None
        for rnd in range(3):
            for h in heights:
                _lib.set_knobs(tile_rows=h)
                times[h].append(bench(fn))
                if rnd == 0 and resid is None:
                    fn()
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(ref, out):
                        print(f"  {name}: tile height {h} changed the output", flush=True)
        _lib.set_knobs(tile_rows=0)
        t_lib = (bench(lambda: torch.nn.functional.linear(a, w)) if not fp8 and "--auto-only" not in sys.argv
                 else float("nan"))
        fl = 2.0 * M * N * K
        msg = f"{name:13s} M={M:6d} N={N:5d} K={K:5d}"
        for h in heights:
            us = sorted(times[h])[1]
            msg += f" | {h or 'auto'} {us:7.1f} us {fl / us / 1e6:5.0f} TF"
        msg += f" | torch.linear {t_lib:7.1f} us"
        print(msg, flush=True)


if __name__ == "__main__":
    main()
