"""Stream-K vs tile-parallel persistent GEMM on the path's shapes (bf_gemm_set_streamk).
The stream-K form was measured slower and removed from bf_gemm.hip; this probe
needs a build that still has it and exits otherwise.  python scripts/gemm_streamk_probe.py"""
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
if not hasattr(L, "bf_gemm_set_streamk"):
    raise SystemExit("this build has no stream-K GEMM (measured slower and removed, DESIGN.md section 4)")
SH = [("clip_qkv", 32896, 3840, 1280, None, "bf16"), ("clip_proj", 32896, 1280, 1280, None, "resid"),
      ("clip_fc1", 32896, 5120, 1280, "gelu", "bf16"), ("clip_fc2", 32896, 1280, 5120, None, "resid"),
      ("cutr_qkv", 36864, 2304, 768, None, "bf16"), ("cutr_fc1", 25600, 3072, 768, "gelu", "bf16"),
      ("cutr_fc2", 25600, 768, 3072, None, "resid")]
for name, M, N, K, act, mode in SH:
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.03).bfloat16()
    b = torch.randn(N, device=dev)
    x = torch.randn(M, N, device=dev)
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    f = (lambda: _lib.gemm(a, w, b, act=act, resid=x, out=x)) if mode == "resid" else \
        (lambda: _lib.gemm(a, w, b, act=act, out=o))
    res = {}
    for rnd in range(2):
        for skm in (0, 1):
            L.bf_gemm_set_streamk(skm)
            res.setdefault(skm, []).append(timeit(f))
    L.bf_gemm_set_streamk(0)
    t0, t1 = min(res[0]), min(res[1])
    fl = 2.0 * M * N * K
    print(f"{name:10s} M={M} N={N} K={K}: tile-parallel {t0:7.1f} us ({fl / t0 / 1e6:6.1f} TF/s) | "
          f"stream-K {t1:7.1f} us ({fl / t1 / 1e6:6.1f} TF/s)  {t0 / t1:.3f}x", flush=True)
