"""One CLIP ViT-H/14 block on the bench's 128 crops (LN1 -> qkv -> attention -> proj + residual ->
LN2 -> fc1 + GELU -> fc2 + residual), per-kernel HIP-event times, for several builds of
libboxfusion_hip.so loaded side by side (ctypes, RTLD_LOCAL) and run interleaved in one process.

usage: python scripts/probe/clip_block_probe.py [ROUNDS] LIB.so [LIB2.so ...]
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

c_int, c_float, c_void_p, LL = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_longlong
rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 4
paths = [p for p in sys.argv[1:] if not p.isdigit()] or [os.path.join(ROOT, "boxfusion_amd", "libboxfusion_hip.so")]
libs = [ctypes.CDLL(p, mode=os.RTLD_LOCAL) for p in paths]
dev = torch.device("cuda")
torch.manual_seed(0)
N, S, C, H, D, F = 128, 257, 1280, 16, 80, 5120
M = N * S
X0 = torch.randn(M, C, device=dev)
X = X0.clone()
g1, b1 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
wq = (torch.randn(3 * C, C, device=dev) * C ** -0.5).bfloat16()
bq = torch.randn(3 * C, device=dev) * 0.02
wp = (torch.randn(C, C, device=dev) * C ** -0.5).bfloat16()
bp = torch.randn(C, device=dev) * 0.02
w1 = (torch.randn(F, C, device=dev) * C ** -0.5).bfloat16()
bb1 = torch.randn(F, device=dev) * 0.02
w2 = (torch.randn(C, F, device=dev) * F ** -0.5).bfloat16()
bb2 = torch.randn(C, device=dev) * 0.02
LN = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
QKV = torch.empty(M, 3 * C, device=dev, dtype=torch.bfloat16)
O = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
H1 = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)


def st():
    return c_void_p(torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice()))


def P(t):
    return c_void_p(t.data_ptr())


def block(L, ev):
    def mark(i):
        ev[i].record()
    mark(0)
    L.bf_layernorm(P(X), c_int(C), P(g1), P(b1), c_float(1e-5), P(LN), c_int(C), None, c_int(M), c_int(C), st())
    mark(1)
    L.bf_gemm_bf16(P(LN), c_int(C), P(wq), c_int(C), P(bq), None, c_int(0), c_int(0), P(QKV), c_int(3 * C),
                   c_int(1), None, c_int(M), c_int(3 * C), c_int(C), c_int(0), st())
    mark(2)
    L.bf_attention_bf16_omap(P(QKV), c_void_p(QKV.data_ptr() + 2 * C), c_void_p(QKV.data_ptr() + 4 * C), P(O),
                             c_int(N), c_int(H), c_int(S), c_int(S), c_int(D), c_int(3 * C), c_int(3 * C),
                             c_int(3 * C), c_int(C), LL(S * 3 * C), LL(S * 3 * C), LL(S * 3 * C), LL(S * C),
                             c_float(D ** -0.5), None, st())
    mark(3)
    L.bf_gemm_bf16(P(O), c_int(C), P(wp), c_int(C), P(bp), P(X), c_int(C), c_int(0), P(X), c_int(C),
                   c_int(0), None, c_int(M), c_int(C), c_int(C), c_int(0), st())
    mark(4)
    L.bf_layernorm(P(X), c_int(C), P(g1), P(b1), c_float(1e-5), P(LN), c_int(C), None, c_int(M), c_int(C), st())
    mark(5)
    L.bf_gemm_bf16(P(LN), c_int(C), P(w1), c_int(C), P(bb1), None, c_int(0), c_int(0), P(H1), c_int(F),
                   c_int(1), None, c_int(M), c_int(F), c_int(C), c_int(1), st())
    mark(6)
    L.bf_gemm_bf16(P(H1), c_int(F), P(w2), c_int(F), P(bb2), P(X), c_int(C), c_int(0), P(X), c_int(C),
                   c_int(0), None, c_int(M), c_int(C), c_int(F), c_int(0), st())
    mark(7)


names = ["ln1", "qkv", "attn", "proj", "ln2", "fc1", "fc2"]
res = {p: {n: [] for n in names} for p in paths}
attn_cold = {p: [] for p in paths}
for r in range(rounds):
    for L, p in zip(libs, paths):
        X.copy_(X0)
        for it in range(4):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
            block(L, ev)
            torch.cuda.synchronize()
            if it >= 1:
                for i, n in enumerate(names):
                    res[p][n].append(ev[i].elapsed_time(ev[i + 1]) * 1e3)
        # attention from a cold cache (a 512 MB write between the qkv GEMM and the attention)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        flush.fill_(r & 255)
        e0.record()
        L.bf_attention_bf16_omap(P(QKV), c_void_p(QKV.data_ptr() + 2 * C), c_void_p(QKV.data_ptr() + 4 * C), P(O),
                                 c_int(N), c_int(H), c_int(S), c_int(S), c_int(D), c_int(3 * C), c_int(3 * C),
                                 c_int(3 * C), c_int(C), LL(S * 3 * C), LL(S * 3 * C), LL(S * 3 * C), LL(S * C),
                                 c_float(D ** -0.5), None, st())
        e1.record()
        torch.cuda.synchronize()
        attn_cold[p].append(e0.elapsed_time(e1) * 1e3)
    print(f"round {r} done", flush=True)

ref = None
for p in paths:
    tot = 0.0
    line = []
    for n in names:
        v = sorted(res[p][n])
        med = v[len(v) // 2]
        tot += med
        line.append(f"{n} {med:7.1f} (min {v[0]:7.1f})")
    ac = sorted(attn_cold[p])
    print(os.path.basename(os.path.dirname(p)) or p)
    print("   " + " | ".join(line) + f" | block {tot:7.1f} us | attn cold {ac[len(ac) // 2]:7.1f}")
print("attention GF", 4 * S * S * D * H * N / 1e9)
