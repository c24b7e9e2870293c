"""How fast is hipBLASLt (through torch) on the CLIP GEMM shapes with the epilogues we need?"""
import torch
import torch.nn.functional as F
d = torch.device("cuda")
M = 32896


def bench(fn, flops, name):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1e3
    print(f"{name:40s} {t:7.1f} us  {flops / t / 1e6:7.1f} TF/s", flush=True)


for (N, K, name) in [(3840, 1280, "qkv"), (1280, 1280, "proj"), (5120, 1280, "fc1"), (1280, 5120, "fc2")]:
    A = torch.randn(M, K, device=d).bfloat16()
    W = torch.randn(N, K, device=d).bfloat16()
    b = torch.randn(N, device=d).bfloat16()
    X = torch.randn(M, N, device=d)
    fl = 2 * M * N * K
    bench(lambda: F.linear(A, W, b), fl, f"{name} linear+bias bf16")
    if name == "fc1":
        bench(lambda: F.gelu(F.linear(A, W, b)), fl, f"{name} linear+bias+gelu (2 ops)")
    try:
        bench(lambda: torch.mm(A, W.t(), out_dtype=torch.float32), fl, f"{name} mm out f32")
        bench(lambda: torch.addmm(X, A, W.t(), out_dtype=torch.float32), fl, f"{name} addmm(X) out f32")
    except Exception as e:  # noqa: BLE001
        print(name, "out_dtype:", type(e).__name__, str(e)[:80])
